// host_services.cpp -- the plugin -> host service surface of plugin_header.h.
//
// The reference registers these symbols by name in its MCJIT
// (compiler.cpp:311-386) and implements them over IPP (dsp.cpp:166-274) and
// libm.  Here they are exported by libdspbench.so so that a plugin compiled
// by the plugin compiler links against them unchanged.
//
// Where they run: plugin code calls them from initialize_state (host, once
// per load) and, for host-dispatched callbacks, from audio_callback.  The
// spectral services fft_forward / fft_reverse go to the GPU (the same
// kernel family as the STFT path, via dsp_fft_forward / dsp_fft_reverse);
// the remaining array helpers are elementwise loops on the caller's host
// buffers -- they are ABI surface, not the hot path.
//
// Behavioural notes kept from the reference:
//  * random_uniform_32_array is a no-op (dsp.cpp:203-205).
//  * log2/log10/to_db are ln * constant (dsp.cpp:226-239), not log2f etc.
//  * add_array / product_array are declared by the reference header but
//    never defined there (link error); here they are defined.
//  * ln_ip_32_array is registered by the reference but missing from its
//    header; exported here too.
//  * allocators return NULL when the arena is full; the plugin compiler's
//    initialize_state_error_wrapper turns that into Runtime_Low_Memory (1)
//    as wrapper_plugin_object.cpp:66-115 does.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "dspbench/dspbench.h"
#include "dspbench/host.h"
#include "dspbench/plugin_header.h"

// ---------------------------------------------------------------------------
// Initializer / arena (ref plugin.h:117-142, memory.h:89-106)
// ---------------------------------------------------------------------------
struct dsp_initializer {
    char *base;
    size_t used;
    size_t capacity;
    int device;  // GPU used by the spectral services
};

extern "C" dsp_initializer *dsp_initializer_create(size_t arena_bytes, int device) {
    dsp_initializer *ini = (dsp_initializer *)std::calloc(1, sizeof(dsp_initializer));
    if (!ini) return nullptr;
    ini->base = (char *)std::calloc(arena_bytes ? arena_bytes : 1, 1);
    if (!ini->base) { std::free(ini); return nullptr; }
    ini->capacity = arena_bytes;
    ini->device = device;
    return ini;
}

extern "C" void dsp_initializer_reset(dsp_initializer *ini) {
    if (ini) { std::memset(ini->base, 0, ini->used); ini->used = 0; }
}

extern "C" size_t dsp_initializer_used(const dsp_initializer *ini) { return ini ? ini->used : 0; }

extern "C" void dsp_initializer_destroy(dsp_initializer *ini) {
    if (!ini) return;
    std::free(ini->base);
    std::free(ini);
}

static void *arena_alloc(void *ctx, size_t bytes) {
    dsp_initializer *ini = (dsp_initializer *)ctx;
    if (!ini) return nullptr;
    const size_t a = (bytes + 15) & ~(size_t)15;  // 16-byte aligned slices
    if (ini->used + a > ini->capacity) return nullptr;
    void *p = ini->base + ini->used;
    ini->used += a;
    return p;
}

extern "C" {

float *allocate_buffer(int num_sample, void *ctx) {
    if (num_sample < 0) return nullptr;
    return (float *)arena_alloc(ctx, sizeof(float) * (size_t)num_sample);
}

float **allocate_buffers(int num_samples, int num_channels, void *ctx) {
    if (num_samples < 0 || num_channels < 0) return nullptr;
    float **ch = (float **)arena_alloc(ctx, sizeof(float *) * (size_t)num_channels);
    if (!ch) return nullptr;
    for (int i = 0; i < num_channels; ++i) {
        ch[i] = allocate_buffer(num_samples, ctx);
        if (!ch[i]) return nullptr;
    }
    return ch;
}

void *allocate_bytes(int num_bytes, void *ctx) {
    if (num_bytes < 0) return nullptr;
    return arena_alloc(ctx, (size_t)num_bytes);
}

// ---- scalar math (ref compiler.cpp:311-350: libm by name) ----
double sin_64(double d) { return std::sin(d); }
double cos_64(double d) { return std::cos(d); }
double tan_64(double d) { return std::tan(d); }
double fabs_64(double d) { return std::fabs(d); }
double pow_64(double a, double b) { return std::pow(a, b); }
double fmod_64(double a, double b) { return std::fmod(a, b); }
double ceil_64(double d) { return std::ceil(d); }
double floor_64(double d) { return std::floor(d); }
double sqrt_64(double d) { return std::sqrt(d); }
double exp_64(double d) { return std::exp(d); }
double log10_64(double d) { return std::log10(d); }
double log_64(double d) { return std::log(d); }
double asin_64(double d) { return std::asin(d); }
double acos_64(double d) { return std::acos(d); }
double atan_64(double d) { return std::atan(d); }
double atan2_64(double a, double b) { return std::atan2(a, b); }
double sinh_64(double d) { return std::sinh(d); }
double cosh_64(double d) { return std::cosh(d); }
double tanh_64(double d) { return std::tanh(d); }

float sin_32(float d) { return std::sin(d); }
float cos_32(float d) { return std::cos(d); }
float tan_32(float d) { return std::tan(d); }
float fabs_32(float d) { return std::fabs(d); }
float pow_32(float a, float b) { return std::pow(a, b); }
float fmod_32(float a, float b) { return std::fmod(a, b); }
float ceil_32(float d) { return std::ceil(d); }
float floor_32(float d) { return std::floor(d); }
float sqrt_32(float d) { return std::sqrt(d); }
float exp_32(float d) { return std::exp(d); }
float log10_32(float d) { return std::log10(d); }
float log_32(float d) { return std::log(d); }
float asin_32(float d) { return std::asin(d); }
float acos_32(float d) { return std::acos(d); }
float atan_32(float d) { return std::atan(d); }
float atan2_32(float a, float b) { return std::atan2(a, b); }
float sinh_32(float d) { return std::sinh(d); }
float cosh_32(float d) { return std::cosh(d); }
float tanh_32(float d) { return std::tanh(d); }

// ---- generators (IPP Tone / Triangle semantics; parity unpinned: IPP absent) ----
static const double kTwoPi = 6.283185307179586476925286766559;

// ippsTone_32f: x[n] = ampl * cos(2 pi freq n + phase); phase advanced by
// 2 pi freq len (mod 2 pi).  freq is normalised (cycles per sample).
void sin_32_array(real32 *out, real32 ampl, real32 freq, i32 n, real32 *phase) {
    double ph = phase ? *phase : 0.0;
    for (i32 i = 0; i < n; ++i) out[i] = (float)(ampl * std::cos(kTwoPi * freq * i + ph));
    if (phase) *phase = (float)std::fmod(ph + kTwoPi * freq * n, kTwoPi);
}

// ippsTriangle_32f with asymmetry h in (-pi, pi): within one period the wave
// falls from +ampl to -ampl over (pi + h) radians and rises back over (pi - h).
static float triangle_at(double ph, double ampl, double h) {
    ph = std::fmod(ph, kTwoPi);
    if (ph < 0) ph += kTwoPi;
    const double fall = M_PI + h;
    if (ph < fall) return (float)(ampl * (1.0 - 2.0 * ph / fall));
    return (float)(ampl * (-1.0 + 2.0 * (ph - fall) / (kTwoPi - fall)));
}

static void triangle_gen(real32 *out, real32 ampl, real32 freq, i32 n, double h, real32 *phase) {
    double ph = phase ? *phase : 0.0;
    for (i32 i = 0; i < n; ++i) out[i] = triangle_at(ph + kTwoPi * freq * i, ampl, h);
    if (phase) *phase = (float)std::fmod(ph + kTwoPi * freq * n, kTwoPi);
}

void triangle_32_array(real32 *out, real32 ampl, real32 freq, i32 n, real32 *phase) {
    triangle_gen(out, ampl, freq, n, 0.0, phase);
}

// ref dsp.cpp:185-192: a saw made from a maximally asymmetric triangle.
void phasor_32_array(real32 *out, real32 ampl, real32 freq, i32 n, real32 *phase) {
    if (phase && *phase == 0.0f) *phase += 0.000005f;
    triangle_gen(out, ampl, freq, n, -M_PI + 0.00000004f, phase);
}

void random_uniform_32_array(real32 *out, i32 n, void *rng) { (void)out; (void)n; (void)rng; }

// ---- array moves ----
// element by element, first to last -- the device build's copy_array
// (plugin_device.h), so a plugin renders the same on both builds even when its
// rows overlap (the reference's ippsCopy_32f leaves overlap undefined); a
// shift right repeats in[0], as it does there
void copy_array(real32 *in, real32 *out, i32 n) {
    volatile real32 *o = out;  // (not turned into memmove, whose overlap semantics differ)
    for (i32 i = 0; i < n; ++i) o[i] = in[i];
}
void set_array(real32 v, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = v; }
void zero_array(real32 *out, i32 n) { if (n > 0) std::memset(out, 0, sizeof(float) * n); }
void add_array(real32 *a, real32 *b, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = a[i] + b[i]; }
void product_array(real32 *a, real32 *b, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = a[i] * b[i]; }

// ---- elementwise (ref dsp.cpp:208-274) ----
static const float kInvLn2 = 1.0f / (float)0.69314718055994530942;
static const float kInvLn10 = 1.0f / (float)2.30258509299404568402;
static const float kDbPerLn = 20.0f / (float)2.30258509299404568402;
static const float kLnPerDb = (float)2.30258509299404568402 / 20.0f;

void gain_32_array(real32 *in, real32 *out, real32 g, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = in[i] * g; }
void dc_offset_32_array(real32 *in, real32 *out, real32 o, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = in[i] + o; }
void sqrt_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::sqrt(in[i]); }
void abs_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::fabs(in[i]); }
void ln_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::log(in[i]); }
void log2_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::log(in[i]) * kInvLn2; }
void log10_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::log(in[i]) * kInvLn10; }
void to_db_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::log(in[i]) * kDbPerLn; }
void from_db_32_array(real32 *in, real32 *out, i32 n) { for (i32 i = 0; i < n; ++i) out[i] = std::exp(in[i] * kLnPerDb); }

void gain_ip_32_array(real32 *io, real32 g, i32 n) { gain_32_array(io, io, g, n); }
void dc_offset_ip_32_array(real32 *io, real32 o, i32 n) { dc_offset_32_array(io, io, o, n); }
void sqrt_ip_32_array(real32 *io, i32 n) { sqrt_32_array(io, io, n); }
void abs_ip_32_array(real32 *io, i32 n) { abs_32_array(io, io, n); }
void ln_ip_32_array(real32 *io, i32 n) { ln_32_array(io, io, n); }
void log2_ip_32_array(real32 *io, i32 n) { log2_32_array(io, io, n); }
void log10_ip_32_array(real32 *io, i32 n) { log10_32_array(io, io, n); }

void pythagore_array(real32 *x, real32 *y, real32 *out, i32 n) {
    for (i32 i = 0; i < n; ++i) out[i] = std::sqrt(x[i] * x[i] + y[i] * y[i]);
}

// ---- spectral services (ref dsp.cpp:69-132) ----
// The FFT "context" is the initializer itself: the GPU plan cache lives in
// libdspbench per device, keyed by order, so any thread may use it.
void *fft_initialize(void *ctx) { return ctx; }

void windowing_hamming(real32 *in, real32 *out, i32 n) {
    if (n <= 0) return;
    if (n == 1) { out[0] = in[0]; return; }
    for (i32 i = 0; i < n; ++i) {
        const double w = 0.54 - 0.46 * std::cos(kTwoPi * (double)i / (double)(n - 1));
        out[i] = in[i] * (float)w;
    }
}

static dsp_exec host_exec(void *ctx) {
    dsp_exec ex{};
    ex.device = ctx ? ((dsp_initializer *)ctx)->device : -1;
    ex.flags = DSP_EXEC_HOST_BUFFERS | DSP_EXEC_SYNC;
    ex.stream = nullptr;
    return ex;
}

// ensure((n & (n-1)) == 0) and order <= MAX_FFT_ORDER (dsp.cpp:79,86): the
// reference aborts; the service reports on stderr and leaves out untouched.
void fft_forward(real32 *in, real32 *re, real32 *im, i32 n, void *ctx) {
    dsp_exec ex = host_exec(ctx);
    int st = dsp_fft_forward(in, re, im, (uint32_t)n, &ex);
    if (st) dsp_host_report("fft_forward", st);
}

void fft_reverse(real32 *re, real32 *im, real32 *out, i32 n, void *ctx) {
    dsp_exec ex = host_exec(ctx);
    int st = dsp_fft_reverse(re, im, out, (uint32_t)n, &ex);
    if (st) dsp_host_report("fft_reverse", st);
}

}  // extern "C"

#include <cstdio>
extern "C" void dsp_host_report(const char *what, int status) {
    std::fprintf(stderr, "dspbench: %s: %s (%s)\n", what, dsp_status_string(status), dsp_last_error());
}
