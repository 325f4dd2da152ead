/*
 * wav.h -- WAV input/output of the offline render path (plain C ABI).
 *
 * Replaces the reference's loader windows_load_wav (wav_reader.h:57-205)
 * and its sample converters (audio.h:66-121):
 *
 *   dsp_wav_parse    host-side RIFF walk of a file image.  64-bit offsets
 *                    (the reference's `unsigned long` sizes and u32 counts
 *                    overflow past 4 GiB); honours fmt chunks longer than 16
 *                    bytes (the reference reads exactly 16 and desyncs,
 *                    wav_reader.h:113) and the pad byte of odd-sized chunks;
 *                    resolves WAVE_FORMAT_EXTENSIBLE (0xFFFE) to its
 *                    sub-format; concatenates every `data` chunk as the
 *                    reference does (wav_reader.h:121-133).
 *   dsp_wav_decode   GPU: interleaved PCM / float payload -> planar float,
 *                    bit-exact with convertInt16/24/32ToFloat + deinterleave
 *                    (int16 and int32 divide by (float)(2^31 - 1) == 2^31,
 *                    int24 divides in double by 2^31 - 1, audio.h:66-110).
 *   dsp_wav_encode   GPU: planar float -> interleaved payload (interleave,
 *                    audio.h:123-133); float32 is exact, PCM rounds half to
 *                    even and clips (the reference has no PCM writer).
 *   dsp_wav_write_header  canonical 44-byte RIFF/WAVE header (46 for
 *                    float, with the cbSize field), RIFF sizes clamped to
 *                    0xFFFFFFFF past 4 GiB.
 */
#ifndef DSPBENCH_WAV_H
#define DSPBENCH_WAV_H

#include <stddef.h>
#include <stdint.h>

#include "dspbench.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DSP_WAV_FORMAT_PCM 1
#define DSP_WAV_FORMAT_FLOAT 3
#define DSP_WAV_FORMAT_EXTENSIBLE 0xFFFE
#define DSP_WAV_MAX_DATA_CHUNKS 8

typedef struct dsp_wav_info {
    uint16_t format;          /* DSP_WAV_FORMAT_PCM or _FLOAT (extensible resolved) */
    uint16_t channels;
    uint32_t sample_rate;
    uint16_t bits_per_sample; /* 16 / 24 / 32 (PCM), 32 (float) */
    uint16_t block_align;     /* bytes per frame = channels * bits / 8 */
    uint64_t frames;          /* samples per channel = data_bytes / block_align */
    uint64_t data_bytes;      /* payload bytes, all data chunks */
    uint32_t n_data_chunks;
    uint64_t data_offset[DSP_WAV_MAX_DATA_CHUNKS]; /* payload byte offsets in the file */
    uint64_t data_size[DSP_WAV_MAX_DATA_CHUNKS];   /* payload bytes of each chunk */
} dsp_wav_info;

/* Parse a file image.  DSP_ERR_INVALID: not RIFF/WAVE, truncated, no fmt or
 * data chunk, or more data chunks than DSP_WAV_MAX_DATA_CHUNKS;
 * DSP_ERR_UNSUPPORTED: a format other than PCM 16/24/32 or float 32
 * (the reference returns Wav_Invalid_Format, wav_reader.h:191-195). */
int dsp_wav_parse(const void *file, uint64_t file_bytes, dsp_wav_info *info);

/* Decode `frames` frames starting at frame `frame0` of the concatenated
 * payload `payload` (info->data_bytes bytes, e.g. gathered from the data
 * chunks) into out[c][0 .. frames), c < info->channels.  With
 * DSP_EXEC_HOST_BUFFERS payload and out are host pointers. */
int dsp_wav_decode(const void *payload, const dsp_wav_info *info, uint64_t frame0,
                   uint64_t frames, float *const *out, const dsp_exec *ex);

/* Encode in[c][0 .. frames) (c < channels) into an interleaved payload of
 * `bits` (16 / 24 / 32 PCM, or 32 float when format = DSP_WAV_FORMAT_FLOAT). */
int dsp_wav_encode(const float *const *in, uint32_t channels, uint64_t frames,
                   uint16_t format, uint16_t bits, void *payload, const dsp_exec *ex);

/* The offline render path end to end from a WAV payload in host memory
 * (the reference's load + convert + render, wav_reader.h:57-205,
 * audio.h:66-121, audio.cpp:13-175): per time chunk the payload bytes cross
 * PCIe, are decoded on the GPU (dsp_wav_decode), rendered (+ the STFT when
 * mag != NULL) with C device channels (file channels past C dropped,
 * missing ones zero), and the render / magnitude rows are copied back into
 * host rows out[c] / mag[c]; streamed as dsp_render_stft_host (dspbench.h). */
int dsp_render_stft_wav(const void *payload, const dsp_wav_info *info, uint32_t C, uint32_t B, float sr,
                        const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window, uint32_t K,
                        float *const *out, float *const *mag, uint64_t ld, uint64_t chunk, const dsp_exec *ex);

/* Write the header for `frames` frames; returns the header size in bytes
 * (44 PCM, 46 float) or a negative dsp_status if cap is too small. */
int dsp_wav_write_header(void *out, uint64_t cap, uint16_t format, uint16_t channels,
                         uint32_t sample_rate, uint16_t bits, uint64_t frames);

#ifdef __cplusplus
}
#endif
#endif
