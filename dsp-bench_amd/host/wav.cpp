// wav.cpp -- RIFF/WAVE parsing and header writing (host side of wav.h).
//
// The chunk walk follows the reference's loader (wav_reader.h:57-205):
// RIFF + WAVE check, then chunks until the end of the file, `fmt ` read,
// every `data` chunk appended, everything else skipped.  Differences, all
// fixes of reference defects documented in SURVEY 8(f):
//   * sizes and offsets are 64-bit (the reference's u32 sample counts and
//     `unsigned long` chunk sizes wrap past 4 GiB);
//   * an fmt chunk longer than 16 bytes (cbSize, WAVE_FORMAT_EXTENSIBLE) is
//     skipped to its end instead of desynchronising the walk
//     (wav_reader.h:113 reads exactly sizeof(Wav_Format) = 16);
//   * odd-sized chunks are followed by their RIFF pad byte;
//   * a data chunk whose size runs past the end of the file (streamed
//     writers leave 0 / 0xFFFFFFFF) is clamped to the bytes present;
//   * WAVE_FORMAT_EXTENSIBLE resolves to the PCM / IEEE-float sub-format.
#include <cstring>

#include "dspbench/wav.h"

namespace {

uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }
uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
void put32(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

// KSDATAFORMAT_SUBTYPE_{PCM,IEEE_FLOAT} = {0000000X-0000-0010-8000-00aa00389b71}
const uint8_t kGuidTail[14] = {0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80,
                               0x00, 0x00, 0xaa, 0x00, 0x38, 0x9b, 0x71};

}  // namespace

extern "C" int dsp_wav_parse(const void *file, uint64_t n, dsp_wav_info *info) {
    if (!file || !info) return DSP_ERR_INVALID;
    std::memset(info, 0, sizeof *info);
    const uint8_t *p = (const uint8_t *)file;
    if (n < 12 || std::memcmp(p, "RIFF", 4) != 0 || std::memcmp(p + 8, "WAVE", 4) != 0)
        return DSP_ERR_INVALID;  // Wav_Not_A_RIFF
    bool have_fmt = false;
    uint16_t fmt = 0;
    uint64_t pos = 12;
    while (pos + 8 <= n) {
        const uint8_t *h = p + pos;
        uint64_t size = le32(h + 4);
        pos += 8;
        const bool is_data = std::memcmp(h, "data", 4) == 0;
        if (pos + size > n) {
            if (!is_data) return DSP_ERR_INVALID;  // truncated non-data chunk
            size = n - pos;
        }
        if (std::memcmp(h, "fmt ", 4) == 0) {
            if (size < 16) return DSP_ERR_INVALID;
            const uint8_t *f = p + pos;
            fmt = le16(f);
            info->channels = le16(f + 2);
            info->sample_rate = le32(f + 4);
            info->bits_per_sample = le16(f + 14);
            if (fmt == DSP_WAV_FORMAT_EXTENSIBLE) {
                if (size < 40 || std::memcmp(f + 26, kGuidTail, 14) != 0) return DSP_ERR_UNSUPPORTED;
                fmt = le16(f + 24);  // sub-format code
            }
            have_fmt = true;
        } else if (is_data) {
            if (info->n_data_chunks == DSP_WAV_MAX_DATA_CHUNKS) return DSP_ERR_INVALID;
            info->data_offset[info->n_data_chunks] = pos;
            info->data_size[info->n_data_chunks] = size;
            info->n_data_chunks++;
            info->data_bytes += size;
        }
        pos += size + (size & 1);
    }
    if (!have_fmt || info->n_data_chunks == 0 || info->channels == 0) return DSP_ERR_INVALID;
    const uint16_t bits = info->bits_per_sample;
    const bool ok = (fmt == DSP_WAV_FORMAT_PCM && (bits == 16 || bits == 24 || bits == 32)) ||
                    (fmt == DSP_WAV_FORMAT_FLOAT && bits == 32);
    if (!ok) return DSP_ERR_UNSUPPORTED;  // Wav_Invalid_Format (wav_reader.h:191-195)
    // a frame must fit the 16-bit nBlockAlign field (found by
    // tests/sanitize/host_fuzz.cpp: 16384 channels x 4 bytes wrapped to 0)
    if ((uint32_t)info->channels * (bits / 8u) > 0xffffu) return DSP_ERR_INVALID;
    info->format = fmt;
    info->block_align = (uint16_t)(info->channels * (bits / 8));
    info->frames = info->data_bytes / info->block_align;
    return DSP_OK;
}

extern "C" int dsp_wav_write_header(void *out, uint64_t cap, uint16_t format, uint16_t channels,
                                    uint32_t sample_rate, uint16_t bits, uint64_t frames) {
    const bool flt = format == DSP_WAV_FORMAT_FLOAT;
    if (!out || channels == 0 || !((flt && bits == 32) ||
                                   (format == DSP_WAV_FORMAT_PCM && (bits == 16 || bits == 24 || bits == 32))))
        return DSP_ERR_INVALID;
    const uint32_t hdr = flt ? 46u : 44u;
    if (cap < hdr) return DSP_ERR_INVALID;
    const uint64_t data = frames * channels * (bits / 8u);
    const uint64_t riff = data + hdr - 8u + (data & 1u);
    uint8_t *h = (uint8_t *)out;
    std::memcpy(h, "RIFF", 4);
    put32(h + 4, riff > 0xffffffffull ? 0xffffffffu : (uint32_t)riff);
    std::memcpy(h + 8, "WAVE", 4);
    std::memcpy(h + 12, "fmt ", 4);
    put32(h + 16, flt ? 18u : 16u);
    put16(h + 20, format);
    put16(h + 22, channels);
    put32(h + 24, sample_rate);
    put32(h + 28, sample_rate * channels * (bits / 8u));
    put16(h + 32, (uint16_t)(channels * (bits / 8u)));
    put16(h + 34, bits);
    uint8_t *d = h + 36;
    if (flt) {
        put16(h + 36, 0);  // cbSize
        d = h + 38;
    }
    std::memcpy(d, "data", 4);
    put32(d + 4, data > 0xffffffffull ? 0xffffffffu : (uint32_t)data);
    return (int)hdr;
}
