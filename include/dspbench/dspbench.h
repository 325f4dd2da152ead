/*
 * dspbench.h -- C ABI of the MI355X offline-render + spectrum path.
 *
 * libdspbench.so exports everything declared here plus every host service of
 * plugin_header.h.  Plain pointers and sizes only; no torch, no C++ types.
 *
 * What each entry point replaces in the reference (odecaux/DSP-Bench):
 *
 *   dsp_render_offline  render_audio called back to back with a fixed block
 *                       size until EOF (audio.cpp:13-175, block pump of
 *                       wasapi_audio.cpp:223-251).  The reference has no
 *                       offline renderer (README.md:16 TODO); semantics are
 *                       exactly those of SURVEY §3.1 (i)-(v), one-shot mode.
 *   dsp_stft_magnitude  windowing -> fft_forward -> pythagore_array per frame
 *                       (dsp.cpp:69-72, 74-103, 166-168) over frames of hop H.
 *   dsp_render_stft     the two above fused: render, keep the render, and
 *                       the spectrum of the rendered signal (headline path).
 *   dsp_ir_analysis     compute_IR (plugin.cpp:17-58) followed by
 *                       fft_perform_and_get_magnitude (dsp.cpp:53-66).
 *   dsp_fft_forward /   fft_forward / fft_reverse (dsp.cpp:74-132) with the
 *   dsp_fft_reverse     same split re/im layout and 1/sqrt(N) scaling.
 *
 * Plugin dispatch: a plugin reaches the GPU as a dsp_plugin.  For the stock
 * plugins whose audio_callback is a per-sample map the `kind` selects a
 * specialised kernel that reads the plugin's own parameter / state blob at
 * the struct offsets the plugin declares (gain_test: Parameters{float gain},
 * IR_test: Parameters{float gain; float step}, static_gain_plugin:
 * State{float gain}).  DSP_PLUGIN_GENERIC runs the plugin's own
 * audio_callback, compiled from its unchanged source to gfx950 code by the
 * module compiler (module.h), through the generic block driver.
 *
 * Errors: every entry point returns DSP_OK (0) or a negative dsp_status.
 * Nothing aborts; HIP errors are mapped to DSP_ERR_HIP and the HIP error
 * string is kept in dsp_last_error().
 */
#ifndef DSPBENCH_H
#define DSPBENCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): dsp_fir_method removed (DSP_EXEC_FIR_DIRECT in dsp_exec.flags
 * selects the direct form), the transport / gather-plan entry points and the
 * dsp_comm layout of shard.h, dsp_callback_facts and the fact-gated block
 * classes of module.h.  A binding written against 1 must not assume those. */
#define DSPBENCH_ABI_VERSION 3

enum dsp_status {
    DSP_OK = 0,
    DSP_ERR_INVALID = -1,     /* bad argument (null pointer, size, alignment) */
    DSP_ERR_HIP = -2,         /* a HIP runtime call failed */
    DSP_ERR_UNSUPPORTED = -3, /* valid request this build does not implement */
    DSP_ERR_NOMEM = -4,       /* device allocation failed */
    DSP_ERR_NO_DEVICE = -5    /* no gfx950 device visible */
};

/* Windows.  Symmetric convention w[n] = a - b cos(2 pi n / (N - 1)), the
 * convention of ippsWinHamming_32f (dsp.cpp:71). */
enum dsp_window {
    DSP_WIN_HAMMING = 0, /* 0.54 / 0.46: reference parity window */
    DSP_WIN_HANN = 1,    /* 0.5 / 0.5: benchmark window (BASELINE cfg 4) */
    DSP_WIN_RECT = 2
};

enum dsp_plugin_kind {
    DSP_PLUGIN_NOOP = 0,        /* test/no_op.cpp */
    DSP_PLUGIN_GAIN = 1,        /* build/gain_test.cpp: out *= params.gain (f32 @0) */
    DSP_PLUGIN_STATIC_GAIN = 2, /* test/static_gain_plugin.cpp: out *= state.gain (f32 @0) */
    DSP_PLUGIN_IR_RAMP = 3,     /* build/IR_test.cpp: out[s] = (float)g_s, g -= step (f32 @0, @4) */
    DSP_PLUGIN_FIR = 4,         /* build-defined cfg 3b: y[n] = sum_k taps[k] x[n-k], params = float taps[T],
                                   T <= 2048; state carries across blocks, so whole files only
                                   (sample_offset 0; shard by channel) */
    DSP_PLUGIN_BIQUAD = 5,      /* build-defined: a cascade of S = params_size / 20 (1..4) direct-form-I
                                   biquads, params = float {b0, b1, b2, a1, a2}[S], y = b0 x + b1 x1 +
                                   b2 x2 - a1 y1 - a2 y2 (plugins/biquad.cpp's section), zero initial
                                   state carried across blocks: whole files only (sample_offset 0;
                                   shard by channel).  Block-parallel (a state scan), fp32 within a
                                   bound of float64, not bit-exact with a serial chain; not in graphs */
    DSP_PLUGIN_GENERIC = 16     /* compiled audio_callback run on the GPU (module) */
};

typedef struct dsp_plugin {
    int32_t kind;          /* dsp_plugin_kind */
    uint32_t params_size;  /* bytes of the Parameters blob */
    const void *params;    /* host pointer to the Parameters blob */
    uint32_t state_size;   /* bytes of the State blob */
    void *state;           /* host pointer to the State blob */
    const void *module;    /* DSP_PLUGIN_GENERIC: dsp_module handle, else NULL */
} dsp_plugin;

/* Execution context (ref has none: single-threaded per audio thread). */
#define DSP_EXEC_HOST_BUFFERS 0x1u /* in/out/mag are host pointers: stage via HBM */
#define DSP_EXEC_SYNC 0x2u         /* synchronise the stream before returning */
#define DSP_EXEC_FIR_DIRECT 0x4u   /* DSP_PLUGIN_FIR: the direct form even when T <= 1025 (default:
                                      FFT overlap-save with 8192-point frames for T <= 1025, the
                                      direct form above) */
#define DSP_EXEC_NO_SPECIALIZE 0x8u /* DSP_PLUGIN_GENERIC: run the plugin's callback on every block.
                                      Default: a plugin whose callback the IR analysis proves to
                                      ignore its input (then one block, the same on every channel)
                                      or to scale it by one factor runs as that block tiled / that
                                      gain in the fused kernels (module.h dsp_callback_facts) */
#define DSP_EXEC_VERIFY_CLASS 0x10u /* DSP_PLUGIN_GENERIC rendered by a block class: afterwards run
                                      the callback on the first, the last and two more blocks of the
                                      call's own input and compare with the rendered rows bit for
                                      bit; on a mismatch render the call again with the callback on
                                      every block.  Reported through dsp_exec.result.  Costs a
                                      stream synchronisation (dsp_render_offline / dsp_render_stft).
                                      A call whose output rows overlap its input rows (in place)
                                      runs the callback on every block instead: the check and a
                                      re-render need the input after the render.  Honoured by
                                      dsp_render_offline and dsp_render_stft, and per chunk by the
                                      chunked (dsp_render_stft_host / _wav) and sharded drivers,
                                      whose result ORs their chunks' bits; dsp_render_loop with
                                      the flag runs the callback on every block (result 0) */
#define DSP_EXEC_SERIAL_STATE 0x20u /* DSP_PLUGIN_GENERIC whose callback writes its State: one chain
                                      of blocks in order on one lane, as the reference's audio thread
                                      runs them (default: speculative segments, module.h
                                      dsp_state_spec_info -- the same bits) */
/* the flags that choose how a call computes (not where its buffers live):
 * the chunked and sharded drivers pass them on to every chunk */
#define DSP_EXEC_METHOD_FLAGS \
    (DSP_EXEC_FIR_DIRECT | DSP_EXEC_NO_SPECIALIZE | DSP_EXEC_VERIFY_CLASS | DSP_EXEC_SERIAL_STATE)

/* dsp_exec.result bits (written when result is not NULL) */
#define DSP_RESULT_CLASS 0x1u      /* a GENERIC plugin ran as its block class */
#define DSP_RESULT_VERIFIED 0x2u   /* DSP_EXEC_VERIFY_CLASS: the checked blocks matched */
#define DSP_RESULT_RERENDERED 0x4u /* DSP_EXEC_VERIFY_CLASS: a checked block differed; the call was
                                      rendered again with the callback on every block */

typedef struct dsp_exec {
    int32_t device;         /* HIP device ordinal; -1 = current device */
    uint32_t flags;         /* DSP_EXEC_* */
    void *stream;           /* hipStream_t; NULL = the legacy default stream */
    uint64_t sample_offset; /* global index of in[c][0] (time-chunk shards);
                               must be a multiple of the block size B */
    uint32_t *result;       /* optional: DSP_RESULT_* of the call (NULL: not reported) */
} dsp_exec;

/* Number of frames of an STFT over L samples: L >= N ? (L - N) / H + 1 : 0. */
uint64_t dsp_stft_frame_count(uint64_t L, uint32_t N, uint32_t H);

/* DSP_PLUGIN_BIQUAD's plan for a cascade (host only, no device): *window =
 * the number of preceding 2048-sample tiles whose end state still reaches a
 * tile's entering state above 2^-48 (1..192: the render sums exactly those, in
 * a fixed order, and is bitwise reproducible run to run), or 0 for a cascade
 * that does not decay that fast (a chained look-back: within the same error
 * bound, not bitwise reproducible).  DSP_ERR_INVALID for a bad blob. */
int dsp_biquad_plan(const float *coef, uint32_t sections, uint32_t *window);

/* Test hooks (not for production use).
 * DSP_DEBUG_BIQUAD_SPIN_LIMIT (set): the sleeps a DSP_PLUGIN_BIQUAD look-back
 *   waits for a preceding tile's words before it gives up (value ~0 restores
 *   the default); a launch in which a wave gave up is rendered again, on the
 *   same stream before the call's later work, as one serial chain per channel
 *   (within the same bound).  0 gives up wherever a word is not there at the
 *   first look.
 * DSP_DEBUG_BIQUAD_REPAIRS (get): launches on the current device rendered
 *   again that way since the last get (read it after the renders finished). */
enum { DSP_DEBUG_BIQUAD_SPIN_LIMIT = 1, DSP_DEBUG_BIQUAD_REPAIRS = 2 };
int dsp_debug_set(int what, uint64_t value);
int dsp_debug_get(int what, uint64_t *value);

/* Offline render, one-shot:
 *   nblocks = ceil(L / B); out[c] holds nblocks * B floats.
 *   Block b: out = file[cursor .. cursor+B) for c < in_channels, zero past
 *   EOF and for c >= in_channels, then audio_callback(out, C, B, sr).
 * in[c] (c < in_channels) hold L floats.  in_channels may be 0 (silence). */
int dsp_render_offline(const float *const *in, uint32_t in_channels, uint64_t L,
                       float *const *out, uint32_t C, uint32_t B, float sr,
                       const dsp_plugin *plugin, const dsp_exec *ex);

/* Offline render, loop mode (render_audio with audio_file_loop set,
 * audio.cpp:100-132): the file wraps -- block b, sample s reads file sample
 * (cursor + b B + s) mod L for c < min(in_channels, C); other channels are
 * zero (audio.cpp:138-141); then audio_callback in place.  Renders nblocks
 * blocks into out[c] (nblocks B floats) and returns the next read cursor,
 * (cursor + nblocks B) mod L, in *cursor_out (may be NULL).  L == 0 with a
 * file is DSP_ERR_INVALID (the reference spins forever, audio.cpp:104).
 * Device buffers only. */
int dsp_render_loop(const float *const *in, uint32_t in_channels, uint64_t L, uint64_t cursor,
                    float *const *out, uint32_t C, uint32_t B, uint64_t nblocks, float sr,
                    const dsp_plugin *plugin, uint64_t *cursor_out, const dsp_exec *ex);

/* STFT magnitude over C planar channels of L samples:
 *   F = dsp_stft_frame_count(L, N, H); mag[c][f * ld + k] = |X_f[k]| / sqrt(N)
 *   for k < K, X_f = DFT_N(w * in[c][f*H .. f*H + N)).
 * K <= N/2 + 1 for real input (K = N/2 + 1 = 4097 at N = 8192), or K = N
 * for the reference's all-bins layout (dsp.cpp:65; mirror |X[N-k]| = |X[k]|).
 * N = 8192 runs the CDNA4 wave-per-frame kernel; other powers of two <= 8192
 * run the generic LDS kernel. */
int dsp_stft_magnitude(const float *const *in, uint32_t C, uint64_t L, uint32_t N,
                       uint32_t H, int32_t window, uint32_t K, float *const *mag,
                       uint64_t ld, const dsp_exec *ex);

/* Render + STFT of the render, fused when the plugin is a per-sample map
 * (NOOP / GAIN / STATIC_GAIN / IR_RAMP) and N = 8192, H % B == 0.
 * Output = dsp_render_offline's out + dsp_stft_magnitude(out, ..., nblocks*B). */
int dsp_render_stft(const float *const *in, uint32_t in_channels, uint64_t L,
                    float *const *out, uint32_t C, uint32_t B, float sr,
                    const dsp_plugin *plugin, uint32_t N, uint32_t H,
                    int32_t window, uint32_t K, float *const *mag, uint64_t ld,
                    const dsp_exec *ex);

/* End to end from host memory: dsp_render_stft (mag != NULL) or
 * dsp_render_offline (mag == NULL) of host rows in[c] (L samples) into host
 * rows out[c] (ceil(L / B) B floats) and mag[c] (F rows of stride ld),
 * streamed through HBM in time chunks of about `chunk` samples (0: one
 * chunk): the upload of chunk t + 1 and the download of chunk t - 1 overlap
 * chunk t's compute (three HIP streams, two device slots).  Pinned host
 * buffers (hipHostMalloc / hipHostRegister) are DMA'd directly, pageable ones
 * staged through pinned slots.  Results equal the device-buffer call bit for
 * bit (lcm(B, H)-aligned chunks with an N - H halo); FIR and GENERIC plugins
 * run as one chunk.  Returns when the host rows are written.  ex->stream is
 * the compute stream. */
int dsp_render_stft_host(const float *const *in, uint32_t in_channels, uint64_t L, float *const *out, uint32_t C,
                         uint32_t B, float sr, const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window,
                         uint32_t K, float *const *mag, uint64_t ld, uint64_t chunk, const dsp_exec *ex);

/* IR analysis: ir_out[c][0..ir_len) = audio_callback(delta) for every
 * channel (plugin.cpp:27-54), then mag[0 .. 4*ir_len) = |FFT_{4 ir_len}(
 * hamming(ir_len) * ir_out[0], zero padded)| / sqrt(4 ir_len) (dsp.cpp:53-66).
 * ir_len = 2048 in the reference (hardcoded_values.h:27). */
int dsp_ir_analysis(const dsp_plugin *plugin, uint32_t C, float sr, uint32_t ir_len,
                    float *const *ir_out, float *mag, const dsp_exec *ex);

/* Complex FFT services (dsp.cpp:74-132): n a power of two <= 8192.
 * forward: re + i*im = DFT(in + 0i) / sqrt(n)
 * reverse: out = Re(IDFT(re + i*im)) / sqrt(n) */
int dsp_fft_forward(const float *in, float *re, float *im, uint32_t n,
                    const dsp_exec *ex);
int dsp_fft_reverse(const float *re, const float *im, float *out, uint32_t n,
                    const dsp_exec *ex);

/* Elementwise services on device buffers (dsp.cpp:171-181, 208-210, 248-250). */
int dsp_gain(const float *in, float *out, float gain, uint64_t n, const dsp_exec *ex);
int dsp_copy(const float *in, float *out, uint64_t n, const dsp_exec *ex);
int dsp_set(float value, float *out, uint64_t n, const dsp_exec *ex);
int dsp_magnitude(const float *re, const float *im, float *out, uint64_t n,
                  const dsp_exec *ex);

/* Display reductions for long-file overviews.
 * minmax: the IR / waveform view's per-pixel extremes (opengl.h:877-890):
 *   vmax[p] = max(-1, max x[s]), vmin[p] = min(+1, min x[s]) over the
 *   samples s with s * pixels / n == p (the reference's initial values; the
 *   index product is 64-bit here, the reference's u32 product wraps).
 * spectrogram: out[p * K + k] = max of mag[f * ld + k] over the frames f
 *   with f * pixels / F == p (0 for an empty column). */
int dsp_minmax_decimate(const float *x, uint64_t n, uint32_t pixels, float *vmax, float *vmin,
                        const dsp_exec *ex);
int dsp_spectrogram_decimate(const float *mag, uint64_t F, uint32_t K, uint64_t ld,
                             uint32_t pixels, float *out, const dsp_exec *ex);

/* Kernel timing: when enabled, every launch of the dominant kernel of
 * dsp_render_stft / dsp_stft_magnitude (the 8192-point wave-per-frame kernel)
 * is bracketed by HIP events on its stream.  dsp_kernel_timing() waits for
 * them, returns the summed duration, the launch count and the algorithmic
 * bytes of those launches, and clears the record.  Enabling
 * creates a stock of events for the current device, and read-out events are
 * reused, so the timed launches do not pay for event creation. */
void dsp_kernel_timing_enable(int on);
int dsp_kernel_timing(double *total_ms, uint64_t *launches, uint64_t *bytes);

/* The 8192-point kernel and its options are fixed at build time.  The A/B
 * and ablation instantiations live in a separate tools build (`make ab`:
 * build/ab/libdspbench_ab.so, which adds dsp_stft_pk_ab_options()); this
 * library has no process-wide kernel selection. */


/* Diagnostics. */
int dsp_abi_version(void);
const char *dsp_status_string(int status);
const char *dsp_last_error(void);
int dsp_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* DSPBENCH_H */
