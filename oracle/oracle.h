/*
 * oracle.h -- CPU restatement of the DSP-Bench hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdspbench.so, the
 * dspbench Python package) links, loads or calls anything under oracle/.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, and only as the checker / the timed CPU baseline.
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the odecaux/DSP-Bench checkout).
 *
 * Pinning: the plugin bodies are pinned by the reference plugins compiled
 * from their own sources (oracle/_ref, see oracle/Makefile) and by the
 * known-answer vectors of test/tests.cpp.  The FFT path
 * (IPP 2021.5.0, a third-party binary absent here) is restated from IPP's
 * documented definitions and pinned by the analytic KATs K4/K5 and by a
 * float64 numpy FFT; no reference test touches dsp.cpp.
 */
#ifndef DSPBENCH_ORACLE_H
#define DSPBENCH_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* audio_callback_t (ref plugin.h:10) */
typedef void (*oracle_callback_t)(void *params, void *state, float **out,
                                  unsigned num_channels, unsigned num_samples,
                                  float sample_rate);

/* Offline render = render_audio (ref audio.cpp:13-175) called back to back
 * with a fixed block size, one-shot mode, until EOF.  Returns
 * the number of blocks rendered = ceil(L/B).  out[c] must hold
 * nblocks*B floats. */
uint64_t oracle_render_offline(const float *const *file, uint32_t file_channels,
                               uint64_t L, float **out, uint32_t C, uint32_t B,
                               float sr, oracle_callback_t cb, void *params,
                               void *state);

/* Loop mode (ref audio.cpp:100-132): render exactly nblocks blocks, wrapping
 * the read cursor.  Returns the final cursor. */
uint64_t oracle_render_loop(const float *const *file, uint32_t file_channels,
                            uint64_t L, uint64_t cursor, float **out, uint32_t C,
                            uint32_t B, uint64_t nblocks, float sr,
                            oracle_callback_t cb, void *params, void *state);

/* Restated stock-plugin callbacks (cross-checked against oracle/_ref). */
void oracle_cb_gain_test(void *params, void *state, float **out, unsigned C,
                         unsigned n, float sr);          /* build/gain_test.cpp:39-58 */
void oracle_cb_static_gain(void *params, void *state, float **out, unsigned C,
                           unsigned n, float sr);        /* test/static_gain_plugin.cpp:27-40 */
void oracle_cb_ir_test(void *params, void *state, float **out, unsigned C,
                       unsigned n, float sr);            /* build/IR_test.cpp:40-60 */
void oracle_cb_no_op(void *params, void *state, float **out, unsigned C,
                     unsigned n, float sr);              /* test/no_op.cpp:14-20 */

/* Windows: 0 = Hamming (ippsWinHamming_32f, ref dsp.cpp:69-72),
 *          1 = Hann (build-defined benchmark window).
 * Symmetric convention w[n] = a - b cos(2 pi n / (N-1)). */
enum { ORACLE_WIN_HAMMING = 0, ORACLE_WIN_HANN = 1, ORACLE_WIN_RECT = 2 };
void oracle_window_f64(int kind, uint32_t n, double *w);
void oracle_window_f32(int kind, uint32_t n, float *w);

/* Complex FFT, split re/im, in place.  dir = -1 forward, +1 inverse.
 * Scaled by 1/sqrt(N) both ways (IPP_FFT_DIV_BY_SQRTN, ref dsp.cpp:87-92). */
void oracle_fft_f64(double *re, double *im, uint32_t n, int dir);
void oracle_fft_f32(float *re, float *im, uint32_t n, int dir);

/* fft_forward (ref dsp.cpp:74-103): real input, zero imaginary part. */
void oracle_fft_forward_f64(const float *in, double *re, double *im, uint32_t n);
/* fft_reverse (ref dsp.cpp:106-132): real part of the scaled inverse. */
void oracle_fft_reverse_f64(const float *re_in, const float *im_in, double *out,
                            uint32_t n);

/* fft_perform_and_get_magnitude (ref dsp.cpp:53-66): Hamming-window the
 * first ir_len samples of ir0, zero-pad to 4*ir_len, FFT, magnitude of all
 * 4*ir_len bins. */
void oracle_ir_magnitude_f64(const float *ir0, uint32_t ir_len, double *mag);

/* STFT magnitude (build-defined composition of a9/a10/a12):
 * frames f = 0..F-1 with F = (L >= N) ? (L-N)/H + 1 : 0, window, FFT, first
 * K bins of |X|/sqrt(N).  mag is F*ld values (row f at mag + f*ld). */
uint64_t oracle_stft_frames(uint64_t L, uint32_t N, uint32_t H);
void oracle_stft_mag_f64(const float *x, uint64_t L, uint32_t N, uint32_t H,
                         int win, uint32_t K, uint64_t ld, double *mag);
/* fp32 version used as the timed CPU baseline (real-input packing, fp32
 * arithmetic with double-accurate twiddles); nthreads <= 0 = all cores. */
void oracle_stft_mag_f32(const float *x, uint64_t L, uint32_t N, uint32_t H,
                         int win, uint32_t K, uint64_t ld, float *mag,
                         int nthreads);
/* The CPU baseline's STFT: radix-4 Stockham real FFT, fp32 (bench.py). */
void oracle_stft_mag_f32_r4(const float *x, uint64_t L, uint32_t N, uint32_t H,
                            int win, uint32_t K, uint64_t ld, float *mag, int nthreads);

/* Parameter normalisation (ref plugin.h:173-233), used by the K6 KATs. */
float    oracle_normalize_int(int32_t lo, int32_t hi, float value);
int32_t  oracle_denormalize_int(int32_t lo, int32_t hi, float nv);
float    oracle_normalize_float(float lo, float hi, int is_log, float value);
float    oracle_denormalize_float(float lo, float hi, int is_log, float nv);
float    oracle_normalize_enum_index(uint32_t num_entries, int32_t index);
uint32_t oracle_denormalize_enum_index(uint32_t num_entries, float nv);

/* WAV sample decode (ref audio.h:66-110 + wav_reader.h:163-199): n
 * interleaved samples of `bits` (16 / 24 / 32 PCM, or 32 with is_float =
 * format 3) at src -> float at dst, then deinterleaved into C planar rows. */
void oracle_pcm_to_float(int bits, int is_float, const void *src, float *dst, uint64_t n);
void oracle_deinterleave(float *const *dst, const float *src, uint64_t frames, uint32_t C);
/* The inverse for the WAV writer (not in the reference, which only renders
 * to the device): float -> PCM with round-half-even and clipping to the
 * integer range, or raw float (bits 32, is_float). */
void oracle_float_to_pcm(int bits, int is_float, const float *src, void *dst, uint64_t n);

/* Display reductions (ref opengl.h:877-890, draw.h:150-160). */
void oracle_minmax_decimate(const float *x, uint64_t n, uint32_t P, float *vmax, float *vmin);
void oracle_spectrogram_decimate(const float *mag, uint64_t F, uint32_t K, uint64_t ld, uint32_t P,
                                 float *out);

/* FIR render (build-defined cfg 3b), float64 accumulation. */
void oracle_fir_f64(const float *x, uint64_t L, const float *h, uint32_t T, double *y, uint64_t Ly);

/* A cascade of S direct-form-I biquads (coef = {b0, b1, b2, a1, a2}[S]) over
 * x zero-padded to Ly samples, zero initial state: y = b0 x + b1 x1 + b2 x2 -
 * a1 y1 - a2 y2 per section (dsp-bench_amd/plugins/biquad.cpp:43-57).
 * _f64: float64 throughout.  _f32: the serial fp32 chain, evaluated left to
 * right as the plugin's source writes it, IEEE (no contraction) -- the CPU
 * baseline of DSP_PLUGIN_BIQUAD.  _bound: per-section inputs' and outputs'
 * magnitude terms, max_n (|b0 v_n| + |b1 v_{n-1}| + |b2 v_{n-2}| + |a1 y_{n-1}|
 * + |a2 y_{n-2}|), written to lmax[S] (float64 run). */
void oracle_biquad_f64(const float *x, uint64_t L, uint64_t Ly, const float *coef, uint32_t S, double *y,
                       double *lmax);
void oracle_biquad_f32(const float *x, uint64_t L, uint64_t Ly, const float *coef, uint32_t S, float *y);

#ifdef __cplusplus
}
#endif
#endif
