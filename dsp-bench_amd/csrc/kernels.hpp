// kernels.hpp -- kernel argument blocks and launchers shared by the HIP
// translation units and the C ABI (capi.cpp).
#pragma once
#include "common.hpp"

struct dsp_module;  // include/dspbench/module.h

namespace dspb {

typedef float v2f __attribute__((ext_vector_type(2)));

struct RenderArgs {
    ChanIn in;
    uint32_t in_ch;
    uint64_t L;      // file samples available from in[c][0]
    ChanOut out;
    uint64_t start;  // first local sample to render
    uint64_t end;    // one past the last (nblocks * B)
    SampleMap map;
    uint64_t goff;   // global index of local sample 0
};

struct Stft8kArgs {
    ChanIn in;           // signal (memory source) or WAV file (fused)
    uint32_t in_ch;      // channels present in `in`
    uint64_t L;          // valid samples in in[c] (file length when fused)
    ChanOut out;         // fused: render output
    ChanOut mag;         // magnitudes, row f at mag[c] + f * ld
    uint64_t F;          // frames per channel
    uint32_t H;          // hop
    uint32_t K;          // bins stored (<= 4097, or 8192 = mirrored all-bins)
    uint64_t ld;         // row stride of mag
    uint32_t valid;      // samples of a frame that exist (8192, or IR length)
    const v2f *win2;     // window as 4096 float2 (w[2m], w[2m+1]), zero past valid
    const v2f *tw;       // T8192[k] = exp(-2 pi i k / 8192), k < 8192
    float scale;         // 1 / sqrt(8192)
    SampleMap map;       // fused render map
    uint64_t goff;       // global sample index of in[c][0] / out[c][0]
    uint64_t *stamps;    // diagnostic builds only (-DDSPB_STAMPS): per-frame phase clocks
    const float4 *wbase; // computed-window variants: (cos, sin) of theta (2 lane), theta (2 lane + 1)
    float wa, wb;        // window w = wa - wb cos(theta n), pre-scaled
    uint64_t tail_end;   // > F H: waves F .. render [F H, tail_end) too (stft_pk PER path), else 0
};

struct GenericFftArgs {
    // input: either split complex (re, im[may be null]) or real frames
    const float *re_in;
    const float *im_in;
    ChanIn sig;          // real frames: signal channels (STFT / IR)
    uint64_t frame_hop;  // samples between frames
    uint32_t valid;      // samples per frame that exist (zero beyond)
    const float *win;    // window (n floats, may be null)
    uint32_t n, log2n;
    int dir;             // -1 forward, +1 inverse
    const v2f *tw;       // T8192
    float scale;
    // output: split complex, real part only, or magnitude rows
    float *re_out;
    float *im_out;
    ChanOut mag;
    uint32_t K;
    uint64_t ld;
    int mode;  // 0: complex->complex, 1: complex->real part, 2: frames->mag
};

int launch_ramp_table(float *table, uint32_t B, float gain, float step, hipStream_t s);
int launch_render(const RenderArgs &A, uint32_t C, bool vec, hipStream_t s);
int launch_render_wrap(const RenderArgs &A, uint32_t C, uint64_t cursor, hipStream_t s);
int module_render(::dsp_module *m, const void *params, uint32_t params_size, const float *const *in,
                  uint32_t in_ch, uint64_t L, float *const *out, uint32_t C, uint32_t B, float sr,
                  uint64_t goff, hipStream_t s, uint32_t flags);
int module_callback_once(::dsp_module *m, const void *params, uint32_t params_size, float *const *bufs, uint32_t C,
                         uint32_t B, float sr, hipStream_t s);
int module_ir(::dsp_module *m, const void *params, uint32_t params_size, float *const *bufs, uint32_t C,
              uint32_t n, float sr, hipStream_t s);
// a stateless plugin's block class for (Parameters, C, B, sr), probed once
// through its own callback and cached in the module (module.cpp)
enum { kSpecNone = 0, kSpecTable = 1, kSpecGain = 2, kSpecGainTable = 3 };
struct ModuleSpec {
    int kind = kSpecNone;
    float gain = 1.f;             // kSpecGain: y = gain x
    const float *table = nullptr; // kSpecTable: the block every block renders (B floats, every channel);
                                  // kSpecGainTable: C rows of B gains, y = x * G[c][position]
    // kSpecTable: the block is an f64 ramp rounded to f32, table[i] =
    // (float)fma(-i, rs, rg0) for every i < B, checked bit for bit on the host
    // (the fused kernels then evaluate it instead of loading the table)
    bool affine = false;
    double rg0 = 0.0, rs = 0.0;
    void *use = nullptr;  // kSpecTable: the hold on the table, released by module_spec_done
};
int module_specialize(::dsp_module *m, const void *params, uint32_t params_size, uint32_t C, uint32_t B, float sr,
                      hipStream_t s, ModuleSpec *out);
// after the launches that read a table class's block (ModuleSpec::use)
int module_spec_done(::dsp_module *m, void *use, hipStream_t s);
void spec_reap(::dsp_module *m);
size_t module_spec_retired(::dsp_module *m);  // tables evicted and not yet freed
struct FirFftArgs {
    ChanIn in;           // input channels
    uint32_t in_ch;
    uint64_t L;          // input samples (zero past)
    ChanOut out;         // render rows, Ly samples
    uint64_t Ly;
    uint64_t F;          // frames = ceil(Ly / 7168)
    const float *H;      // FFT(taps)/16384, lane-major pairs (fir_fft.hip)
    v2f h2048;           // H[2048]
    const v2f *tw;       // T8192 + lane-major stage twiddles (capi.cpp get_tw)
    uint32_t nout;       // fir_pair_kernel: output channels in `out` (set by launch_fir_pair)
};
int launch_fir_fft(const FirFftArgs &A, uint32_t C, hipStream_t s);
// two channels per frame as one complex signal, 4096-point frames, hop 3072
// (C even; F = ceil(Ly / kPairHop); H = SampleMap::pairH; h2048 unused)
constexpr uint32_t kPairHop = 3072;
int launch_fir_pair(const FirFftArgs &A, uint32_t C, hipStream_t s);
int launch_fir(const float *x, uint64_t L, float *y, uint64_t Ly, const float *h8, uint32_t T8,
               bool y_aligned16, hipStream_t s);
// DSP_PLUGIN_BIQUAD (iir.hip): one launch renders C <= 16 channels of Ly
// samples from zero state; tiles of 64 lanes x biquad_lane_samples() samples
struct BiquadArgs {
    ChanIn in;
    uint32_t in_ch;
    uint64_t L;            // file samples (zero past)
    ChanOut out;
    uint64_t Ly;           // rendered samples per channel
    uint32_t C;            // channels of this launch
    uint64_t ntiles_ch;    // biquad_tiles(Ly)
    const float *coef;     // 5 S floats (b0 b1 b2 a1 a2 per section)
    const float *Q;        // 65 D x D: M^(T l)
    const float *P;        // 257 D x D: M^(64 T k)
    uint32_t window;       // W: S_in from the W previous tiles' aggregates (0: inclusive look-back)
    uint64_t *aggw, *inclw;  // per tile, nch D words: epoch << 32 | float bits (aggregate, inclusive)
    uint64_t epoch;        // distinct per launch on one workspace (32 bits used)
    uint32_t spin_limit;   // sleeps a look-back waits before it gives up
    uint32_t *err;         // the stream's workspace word: a wave that gave up writes the epoch
    uint32_t *repairs;     // host-mapped: launches biquad_repair_kernel rendered again (diagnostic)
    uint32_t in_aligned16, out_aligned16;
};
uint64_t biquad_tiles(uint64_t Ly);
uint32_t biquad_lane_samples();
// nch = 2: one wavefront per tile of a channel pair (C even), packed math
int launch_biquad(const BiquadArgs &A, uint32_t sections, uint32_t nch, hipStream_t s);
int launch_minmax(const float *x, uint64_t n, uint32_t P, float *vmax, float *vmin, hipStream_t s);
int launch_spectro(const float *mag, uint64_t F, uint32_t K, uint64_t ld, uint32_t P, float *out,
                   hipStream_t s);
int launch_wav_decode(const uint8_t *payload, uint32_t C, uint16_t bits, bool is_float, uint64_t frame0,
                      uint64_t frames, const ChanOut &out, bool out_aligned16, hipStream_t s);
int launch_wav_encode(uint8_t *payload, uint32_t C, uint16_t bits, bool is_float, uint64_t frames,
                      const ChanOut &in, hipStream_t s);
bool stft8192_pk_per_path(const Stft8kArgs &A, bool fused);
int stft_pk_ab_options();  // A/B option bits of this thread: 0 unless the tools build (stft_pk_ab.hip) set them
int launch_stft8192_pk(const Stft8kArgs &A, uint32_t C, bool fused, int opt, hipStream_t s);
int launch_fft_generic(const GenericFftArgs &A, uint64_t transforms, uint32_t C, hipStream_t s);
int launch_gain(const float *in, float *out, float g, uint64_t n, hipStream_t s);
int launch_set(float v, float *out, uint64_t n, hipStream_t s);
int launch_copy(const float *in, float *out, uint64_t n, hipStream_t s, bool *done);
int launch_upload(float *dst, const float *src, uint64_t n, hipStream_t s);
int launch_impulse(const ChanOut &buf, uint32_t C, uint32_t n, hipStream_t s);
int launch_magnitude(const float *re, const float *im, float *out, uint64_t n, hipStream_t s);

}  // namespace dspb
