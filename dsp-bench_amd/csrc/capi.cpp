// capi.cpp -- the extern "C" boundary of libdspbench (include/dspbench/dspbench.h).
//
// Validates arguments, owns the per-device constant tables (twiddles,
// windows: the analogue of the IPP FFT spec / plan cache of dsp.cpp:84-95 and
// IPP_FFT_Context, structs.h:170-178), maps a dsp_plugin onto a kernel and
// launches on the caller's stream.  Fails loudly (negative status) on
// anything it cannot run on the GPU -- there is no CPU path here.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "kernels.hpp"
#include "dspbench/wav.h"

namespace dspb {

static thread_local char g_last_error[512] = "";

void set_last_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char *what) {
    set_last_error("%s: %s", what, hipGetErrorString(e));
    if (e == hipErrorOutOfMemory) return DSP_ERR_NOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return DSP_ERR_NO_DEVICE;
    return DSP_ERR_HIP;
}

static int invalid(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
    va_end(ap);
    return DSP_ERR_INVALID;
}

// ---------------------------------------------------------------------------
// per-device resources
// ---------------------------------------------------------------------------
// A cached device table (FIR taps and spectra, BIQUAD transition powers):
// each call that maps it holds it until its launches are enqueued; the table
// is freed when the cache has evicted it and no call holds it, after the
// device has finished the work already enqueued
typedef std::shared_ptr<float> DevTable;
static DevTable dev_table(float *p, int dev) {
    return DevTable(p, [dev](float *q) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        (void)hipDeviceSynchronize();
        (void)hipFree(q);
        if (prev >= 0) (void)hipSetDevice(prev);
    });
}

struct FirTaps {  // a FIR filter's device taps + overlap-save spectrum
    std::vector<float> taps;
    DevTable dev;
    float h2048r, h2048i;
};

struct IirTab {  // a biquad cascade's coefficients + state-transition powers (biquad_tables)
    std::vector<float> coef;
    DevTable dev;
    uint32_t window;  // biquad_tables' W
};

// the look-back workspace of biquad_scan_kernel, one per (device, stream):
// calls on one stream run in order, so a launch only meets words tagged with
// its own epoch (zeroed at allocation; epochs run 1 .. 2^32 - 1)
struct IirWork {
    uint64_t *aggw = nullptr, *inclw = nullptr;  // cap * 16 words each, one allocation, then the error word
    uint64_t cap = 0;
    uint64_t epoch = 0;
};

struct DeviceRes {
    v2f *tw8192 = nullptr;  // exp(-2 pi i k / 8192), then 896 lane-major stage twiddles
    float4 *wbase = nullptr;  // (cos, sin)(theta 2l), (cos, sin)(theta (2l+1)), theta = 2 pi / 8191
    std::map<std::tuple<int, uint32_t, uint32_t, float>, float *> windows;  // (kind, N, valid, scale)
    std::map<std::pair<void *, int>, std::pair<float *, size_t>> scratch;  // per (stream, slot)
    std::vector<FirTaps> fir;                                  // FIR filters seen (plugin_map)
    std::vector<IirTab> iir;                                   // biquad cascades seen (plugin_map)
    std::map<void *, IirWork> iir_work;                        // per stream
    uint32_t *iir_fb_host = nullptr, *iir_fb_dev = nullptr;  // host-mapped counter of repaired launches
    float *delta = nullptr;  // 2048 floats: 1, 0, 0, ... (compute_IR's impulse, read-only)
};

static std::mutex g_mu;
// (never destroyed: its tables must not be freed after the HIP runtime's own
// teardown at process exit)
static std::map<int, DeviceRes> &g_res = *new std::map<int, DeviceRes>;

static int current_device(int *dev) {
    DSPB_HIP(hipGetDevice(dev));
    return DSP_OK;
}

// RAII: make ex->device current for the call, restore afterwards.
struct DeviceGuard {
    int prev = -1;
    int dev = -1;
    int status = DSP_OK;
    explicit DeviceGuard(const dsp_exec *ex) {
        hipError_t e = hipGetDevice(&prev);
        if (e != hipSuccess) { status = hip_fail(e, "hipGetDevice"); return; }
        dev = prev;
        if (ex && ex->device >= 0 && ex->device != prev) {
            e = hipSetDevice(ex->device);
            if (e != hipSuccess) { status = hip_fail(e, "hipSetDevice"); return; }
            dev = ex->device;
        }
    }
    ~DeviceGuard() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

// A call on a stream that is being captured into a graph cannot make a
// first-use table or scratch allocation (an allocation, a legacy-stream
// launch and a sync would invalidate the capture): it is refused instead, and
// one eager call of the same shape beforehand creates what it needs.
static int refuse_capture(hipStream_t s, const char *what) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
        set_last_error("stream capture: %s is created on first use; make one eager call of this shape on the "
                       "capturing stream first", what);
        return DSP_ERR_INVALID;
    }
    return DSP_OK;
}

// Synchronous upload of a constant table (launch_upload: kernel arguments,
// not a copy -- see render.hip); the tables are shared by every stream of the
// device, so the upload completes before the first use.  (Callers check the
// caller's stream for capture first: refuse_capture.)
static int upload_table(void *dst, const void *src, size_t bytes) {
    if (int st = launch_upload((float *)dst, (const float *)src, bytes / sizeof(float), nullptr)) return st;
    DSPB_HIP(hipStreamSynchronize(nullptr));
    return DSP_OK;
}

static int get_tw(int dev, hipStream_t s, const v2f **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    if (!r.tw8192) {
        if (int st = refuse_capture(s, "the FFT twiddle table")) return st;
        std::vector<v2f> h(8192);
        for (int k = 0; k < 8192; ++k) {
            const double a = -2.0 * M_PI * (double)k / 8192.0;
            h[k] = v2f{(float)std::cos(a), (float)std::sin(a)};
        }
        // exact zeros / ones at the quarter turns
        h[0] = v2f{1.f, 0.f}; h[2048] = v2f{0.f, -1.f};
        h[4096] = v2f{-1.f, 0.f}; h[6144] = v2f{0.f, 1.f};
        // lane-major stage twiddles of the 64 x 64 step (stft_soa.hip):
        // [8192 + 64 (j-1) + l] = T[2 l j], [8192 + 448 + 64 (j-1) + l] = T[16 l j]
        for (int j = 1; j < 8; ++j)
            for (int l = 0; l < 64; ++l) h.push_back(h[(2 * l * j) & 8191]);
        for (int j = 1; j < 8; ++j)
            for (int l = 0; l < 64; ++l) h.push_back(h[(16 * l * j) & 8191]);
        // stft_pk.hip pairs, one float4 per (hi, lane), hi < 4:
        // (re T[16 l hi], re T[16 l (hi + 4)], im T[16 l hi], im T[16 l (hi + 4)])
        for (int hi = 0; hi < 4; ++hi)
            for (int l = 0; l < 64; ++l) {
                const v2f a = h[(16 * l * hi) & 8191], b = h[(16 * l * (hi + 4)) & 8191];
                h.push_back(v2f{a.x, b.x});
                h.push_back(v2f{a.y, b.y});
            }
        v2f *d = nullptr;
        DSPB_HIP(hipMalloc(&d, sizeof(v2f) * h.size()));
        if (int st = upload_table(d, h.data(), sizeof(v2f) * h.size())) {
            (void)hipFree(d);
            return st;
        }
        r.tw8192 = d;
    }
    *out = r.tw8192;
    return DSP_OK;
}

// compute_IR's impulse (plugin.cpp:27-34) as a read-only device buffer: the
// IR render of a map plugin reads it as its file, so no impulse launch
constexpr uint32_t kDeltaLen = 2048;  // the largest ir_len (4 ir_len <= 8192)
static int get_delta(int dev, hipStream_t s, const float **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    if (!r.delta) {
        if (int st = refuse_capture(s, "the impulse buffer")) return st;
        std::vector<float> h(kDeltaLen, 0.0f);
        h[0] = 1.0f;
        float *d = nullptr;
        DSPB_HIP(hipMalloc(&d, sizeof(float) * kDeltaLen));
        if (int st = upload_table(d, h.data(), sizeof(float) * kDeltaLen)) {
            (void)hipFree(d);
            return st;
        }
        r.delta = d;
    }
    *out = r.delta;
    return DSP_OK;
}

// Window of length `valid` (symmetric, ref ippsWinHamming_32f convention)
// zero-padded to N.  Computed in double, rounded once to float.
static int get_window(int dev, hipStream_t s, int kind, uint32_t N, uint32_t valid, const float **out,
                      double scale = 1.0) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    auto key = std::make_tuple(kind, N, valid, (float)scale);
    auto it = r.windows.find(key);
    if (it != r.windows.end()) { *out = it->second; return DSP_OK; }
    if (int st = refuse_capture(s, "a window table")) return st;
    double a = 0.54, b = 0.46;
    if (kind == DSP_WIN_HANN) { a = 0.5; b = 0.5; }
    else if (kind == DSP_WIN_RECT) { a = 1.0; b = 0.0; }
    std::vector<float> h(N, 0.f);
    for (uint32_t n = 0; n < valid; ++n)
        h[n] = valid == 1 ? (float)scale
                          : (float)(scale * (a - b * std::cos(2.0 * M_PI * (double)n / (double)(valid - 1))));
    float *d = nullptr;
    DSPB_HIP(hipMalloc(&d, sizeof(float) * N));
    if (int st = upload_table(d, h.data(), sizeof(float) * N)) {
        (void)hipFree(d);
        return st;
    }
    r.windows[key] = d;
    *out = d;
    return DSP_OK;
}

// stft8192_pk_kernel folds DIV_BY_SQRTN and the 1/2 of the real split into
// the window: 0.5 / sqrt(N)
static float window_prescale(uint32_t N) { return (float)(0.5 / std::sqrt((double)N)); }

// Inputs of the computed-window kernels (stft_soa.hip kOptWinComp): per-lane
// base angles and the (pre-scaled) cosine-window coefficients.
static int set_wincomp(int dev, hipStream_t s, int kind, Stft8kArgs *A) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        DeviceRes &r = g_res[dev];
        if (!r.wbase) {
            if (int st = refuse_capture(s, "the window base angles")) return st;
            std::vector<float4> h(64);
            const double th = 2.0 * M_PI / 8191.0;
            for (int l = 0; l < 64; ++l)
                h[l] = float4{(float)std::cos(th * 2 * l), (float)std::sin(th * 2 * l),
                              (float)std::cos(th * (2 * l + 1)), (float)std::sin(th * (2 * l + 1))};
            float4 *d = nullptr;
            DSPB_HIP(hipMalloc(&d, sizeof(float4) * 64));
            if (int st = upload_table(d, h.data(), sizeof(float4) * 64)) {
                (void)hipFree(d);
                return st;
            }
            r.wbase = d;
        }
        A->wbase = r.wbase;
    }
    double a = 0.54, b = 0.46;
    if (kind == DSP_WIN_HANN) { a = 0.5; b = 0.5; }
    else if (kind == DSP_WIN_RECT) { a = 1.0; b = 0.0; }
    const double sc = window_prescale(8192);
    A->wa = (float)(a * sc);
    A->wb = (float)(b * sc);
    return DSP_OK;
}

// Stream-ordered scratch: calls on one stream are serialised by the stream,
// so one buffer per (device, stream, slot) is enough.  Slots: 0 the IR_test
// block table, 1 loop mode's wrapped file.
static int get_scratch(int dev, hipStream_t s, size_t bytes, float **out, int slot_id = 0) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    auto &slot = r.scratch[std::make_pair((void *)s, slot_id)];
    if (slot.second < bytes) {
        // a stream being captured into a graph cannot allocate or wait: its
        // scratch must exist from an eager call of the same shape first
        if (int st = refuse_capture(s, "the stream's scratch buffer")) return st;
        if (slot.first) {
            DSPB_HIP(hipStreamSynchronize(s));
            DSPB_HIP(hipFree(slot.first));
        }
        slot.first = nullptr;
        slot.second = 0;
        DSPB_HIP(hipMalloc(&slot.first, bytes));
        slot.second = bytes;
    }
    *out = slot.first;
    return DSP_OK;
}

// ---------------------------------------------------------------------------
// optional per-launch timing of the dominant kernel (HIP events on the
// launch stream), read back by dsp_kernel_timing(); used by bench.py
// ---------------------------------------------------------------------------
struct TimedLaunch {
    hipEvent_t start, stop;
    uint64_t bytes;
    int dev;
};
static bool g_timing = false;
// recycled timing events per device (g_mu): a hipEventCreate pair per timed
// launch cost more than the records themselves
static std::map<int, std::vector<hipEvent_t>> g_event_pool;

// A/B and ablation options of stft8192_pk_kernel: 0 in the product library
// (the tools build's stft_pk_ab.hip sets them per thread)
static int pk_options() { return stft_pk_ab_options(); }

// a closed-form IR ramp (plugin_map) leaves the block table unbuilt; every
// fused path but stft_pk's PER path reads it
static int ensure_ramp_table(const SampleMap &m, hipStream_t s) {
    if (m.kind != MapKind::Ramp || m.closed != 1) return DSP_OK;  // 2: the table holds it already
    return launch_ramp_table(const_cast<float *>(m.table), m.B, (float)m.rg0, (float)m.rs, s);
}

static int launch_stft(const Stft8kArgs &A, uint32_t C, bool fused, hipStream_t s) {
    if (fused && !(A.map.closed && stft8192_pk_per_path(A, fused))) {
        const int st = ensure_ramp_table(A.map, s);
        if (st) return st;
    }
    return launch_stft8192_pk(A, C, fused, pk_options(), s);
}

static std::vector<TimedLaunch> g_timed;

// set while a call times its launches as one region (the pipelined GENERIC
// render + STFT): the launches inside record nothing of their own
static thread_local bool tl_timing_outer = false;

static int timing_begin(hipStream_t s, TimedLaunch *t) {
    t->start = t->stop = nullptr;
    if (!g_timing || tl_timing_outer) return DSP_OK;
    DSPB_HIP(hipGetDevice(&t->dev));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto &pool = g_event_pool[t->dev];
        if (pool.size() >= 2) {
            t->start = pool.back();
            pool.pop_back();
            t->stop = pool.back();
            pool.pop_back();
        }
    }
    if (!t->start) {
        DSPB_HIP(hipEventCreate(&t->start));
        DSPB_HIP(hipEventCreate(&t->stop));
    }
    DSPB_HIP(hipEventRecord(t->start, s));
    return DSP_OK;
}

static int timing_end(hipStream_t s, TimedLaunch *t, uint64_t bytes) {
    if (!t->start) return DSP_OK;
    DSPB_HIP(hipEventRecord(t->stop, s));
    t->bytes = bytes;
    std::lock_guard<std::mutex> lk(g_mu);
    g_timed.push_back(*t);
    return DSP_OK;
}

static bool is_pow2(uint64_t n) { return n && !(n & (n - 1)); }
static uint32_t ilog2(uint64_t n) { uint32_t l = 0; while ((1ull << l) < n) ++l; return l; }
static bool aligned(const void *p, size_t a) { return ((uintptr_t)p % a) == 0; }

// ---------------------------------------------------------------------------
// plugin -> sample map
// ---------------------------------------------------------------------------
// FFT(taps zero-padded to 8192) / 16384 in double, laid out for
// fir_fft.hip: for ka < 16 and lane l, 8 floats
//   (Re H[k1], Re H[k2], Im H[k1], Im H[k2], Re H[M-k1], Re H[M-k2], Im H[M-k1], Im H[M-k2])
// with k1 = l + 64 ka, k2 = k1 + 1024, M = 4096; then H[2048] (re, im).
// FFT_n(taps zero-padded) in float64 (iterative radix-2, forward e^-i)
static void taps_spectrum(const float *taps, uint32_t T, int n, std::vector<double> &re, std::vector<double> &im) {
    re.assign(n, 0.0);
    im.assign(n, 0.0);
    for (uint32_t i = 0; i < T; ++i) re[i] = taps[i];
    for (int i = 1, j = 0; i < n; ++i) {  // iterative radix-2, forward (e^-i)
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { std::swap(re[i], re[j]); std::swap(im[i], im[j]); }
    }
    for (int len = 2; len <= n; len <<= 1) {
        const int hlen = len >> 1;
        for (int k = 0; k < hlen; ++k) {
            const double a = -2.0 * M_PI * k / len, wr = std::cos(a), wi = std::sin(a);
            for (int s0 = 0; s0 < n; s0 += len) {
                const double xr = re[s0 + k + hlen] * wr - im[s0 + k + hlen] * wi;
                const double xi = re[s0 + k + hlen] * wi + im[s0 + k + hlen] * wr;
                re[s0 + k + hlen] = re[s0 + k] - xr;
                im[s0 + k + hlen] = im[s0 + k] - xi;
                re[s0 + k] += xr;
                im[s0 + k] += xi;
            }
        }
    }
}

// the 8192-point table of fir_fft_kernel (kOlsHop 7168, one channel per frame)
static void ols_table(const float *taps, uint32_t T, float *out) {
    std::vector<double> re, im;
    taps_spectrum(taps, T, 8192, re, im);
    const double sc = 1.0 / 16384.0;
    for (int ka = 0; ka < 16; ++ka)
        for (int l = 0; l < 64; ++l) {
            const int k1 = l + 64 * ka, k2 = k1 + 1024, m1 = 4096 - k1, m2 = 4096 - k2;
            float *o = out + 8 * (64 * ka + l);
            o[0] = (float)(re[k1] * sc); o[1] = (float)(re[k2] * sc);
            o[2] = (float)(im[k1] * sc); o[3] = (float)(im[k2] * sc);
            o[4] = (float)(re[m1] * sc); o[5] = (float)(re[m2] * sc);
            o[6] = (float)(im[m1] * sc); o[7] = (float)(im[m2] * sc);
        }
    out[8192] = (float)(re[2048] * sc);
    out[8193] = (float)(im[2048] * sc);
}

// the 4096-point table of fir_pair_kernel (two channels as one complex
// signal): H = FFT_4096(taps) / 4096 (the inverse's scale), as float4
// [q][lane] = (Re H[l + 64 q], Re H[l + 64 (q + 32)], Im .., Im ..), the
// pairing of the transform's packed last combine
static void pair_table(const float *taps, uint32_t T, float *out) {
    std::vector<double> re, im;
    taps_spectrum(taps, T, 4096, re, im);
    const double sc = 1.0 / 4096.0;
    for (int q = 0; q < 32; ++q)
        for (int l = 0; l < 64; ++l) {
            const int k0 = l + 64 * q, k1 = k0 + 2048;
            float *o = out + 4 * (64 * q + l);
            o[0] = (float)(re[k0] * sc); o[1] = (float)(re[k1] * sc);
            o[2] = (float)(im[k0] * sc); o[3] = (float)(im[k1] * sc);
        }
}

// IR_test (build/IR_test.cpp:47-58) runs `gain -= step` in double from the
// float parameters.  The sequence is often exact -- every partial result a
// double -- and then table[i] = (float)(gain - i step) is one f64 FMA, with
// no sequential kernel.  This checks that bit for bit against the recurrence
// itself (B host f64 subtractions, cached per parameter set).
static bool ramp_closed_form(float gain, float step, uint32_t B) {
    if (B > (1u << 16)) return false;
    static std::mutex mu;
    static struct { uint32_t g, s, B; bool ok; } last = {0, 0, 0, false};
    uint32_t gb, sb;
    std::memcpy(&gb, &gain, 4);
    std::memcpy(&sb, &step, 4);
    std::lock_guard<std::mutex> lk(mu);
    if (last.B == B && last.g == gb && last.s == sb) return last.ok;
    double g = gain;
    const double s = step;
    bool ok = true;
    for (uint32_t i = 0; i < B && ok; ++i) {
        const double c = std::fma(-(double)i, s, (double)gain);
        ok = std::memcmp(&c, &g, sizeof(double)) == 0;
        g -= s;
    }
    last = {gb, sb, B, ok};
    return ok;
}

constexpr uint32_t kIirPairSections = 2;  // cascades of >= this many sections: channel pairs per wave

// DSP_PLUGIN_BIQUAD (iir.hip): the cascade's zero-input state transition over
// T = biquad_lane_samples() samples, M (D x D, D = 2 S, state = (y1, y2) per
// section; section k's x history is section k-1's y history), simulated in
// float64 from each unit state, then its powers:
//   [5 S coefficients, padded to 20][M^l, l = 0..64][M^(64 k), k = 0..256]
// Returns W, the number of preceding tiles (of 64 T samples) whose aggregate
// reaches a tile's entering state with a weight ||M^(64 k)||_inf above 2^-48
// (every later power below it too): 1..256, or 0 when the transition does not
// decay that fast (then the kernel's inclusive look-back).
static uint32_t biquad_tables(const float *cf, uint32_t S, std::vector<float> &h) {
    const int D = 2 * (int)S, T = (int)biquad_lane_samples();
    std::vector<double> M((size_t)D * D);
    for (int j = 0; j < D; ++j) {
        double Y1[4], Y2[4], X1[4], X2[4];
        for (int k = 0; k < (int)S; ++k) {
            Y1[k] = (2 * k == j) ? 1.0 : 0.0;
            Y2[k] = (2 * k + 1 == j) ? 1.0 : 0.0;
        }
        for (int k = 0; k < (int)S; ++k) {
            X1[k] = k ? Y1[k - 1] : 0.0;
            X2[k] = k ? Y2[k - 1] : 0.0;
        }
        for (int n = 0; n < T; ++n) {
            double v = 0.0;
            for (int k = 0; k < (int)S; ++k) {
                const float *c = cf + 5 * k;
                const double y = (double)c[0] * v + (double)c[1] * X1[k] + (double)c[2] * X2[k] -
                                 (double)c[3] * Y1[k] - (double)c[4] * Y2[k];
                X2[k] = X1[k];
                X1[k] = v;
                Y2[k] = Y1[k];
                Y1[k] = y;
                v = y;
            }
        }
        for (int k = 0; k < (int)S; ++k) {
            M[(size_t)(2 * k) * D + j] = Y1[k];
            M[(size_t)(2 * k + 1) * D + j] = Y2[k];
        }
    }
    auto mul = [D](const std::vector<double> &a, const std::vector<double> &b) {
        std::vector<double> r((size_t)D * D, 0.0);
        for (int i = 0; i < D; ++i)
            for (int k = 0; k < D; ++k)
                for (int j = 0; j < D; ++j) r[(size_t)i * D + j] += a[(size_t)i * D + k] * b[(size_t)k * D + j];
        return r;
    };
    std::vector<double> I((size_t)D * D, 0.0);
    for (int i = 0; i < D; ++i) I[(size_t)i * D + i] = 1.0;
    h.assign(20 + (65 + 257) * (size_t)D * D, 0.f);
    for (uint32_t q = 0; q < 5 * S; ++q) h[q] = cf[q];
    std::vector<double> Q = I;
    float *o = h.data() + 20;
    for (int l = 0; l <= 64; ++l) {
        for (int q = 0; q < D * D; ++q) o[(size_t)l * D * D + q] = (float)Q[q];
        Q = mul(M, Q);
    }
    std::vector<double> Pm = I, step = I;
    for (int l = 0; l < 64; ++l) step = mul(M, step);  // M^64 in float64
    o += (size_t)65 * D * D;
    uint32_t W = 0;  // the last k <= 256 whose weight is above the cut, + 1
    bool finite = true;
    for (int k = 0; k <= 256; ++k) {
        double nrm = 0.0;
        for (int i = 0; i < D; ++i) {
            double row = 0.0;
            for (int j = 0; j < D; ++j) row += std::fabs(Pm[(size_t)i * D + j]);
            nrm = std::max(nrm, row);
        }
        finite = finite && std::isfinite(nrm);
        if (nrm > std::ldexp(1.0, -48)) W = (uint32_t)k + 1;
        for (int q = 0; q < D * D; ++q) o[(size_t)k * D * D + q] = (float)Pm[q];
        Pm = mul(step, Pm);
    }
    // decayed within the table: the weights of the last 64 powers are all below the cut
    return (finite && W <= 192) ? std::max<uint32_t>(W, 1) : 0u;
}

// sleeps a BIQUAD look-back waits for a predecessor's words before it gives
// up (a legitimate wait is a few rounds: a tile waits only for waves
// dispatched before it); the launch is then rendered again serially
// (iir.hip biquad_repair_kernel, on the same stream)
constexpr uint32_t kIirSpinLimit = 1u << 16;
static std::atomic<uint32_t> g_iir_spin_limit{kIirSpinLimit};

// takes the stream's workspace for one launch (a fresh epoch) and launches,
// under one lock: launches on a stream are enqueued in epoch order
static int iir_launch(int dev, hipStream_t s, BiquadArgs *A, uint32_t sections, uint32_t nch) {
    const uint64_t tiles = (uint64_t)(A->C / nch) * A->ntiles_ch;
    {   // every launch takes a fresh epoch: a graph replay would reuse it
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
            set_last_error("stream capture: a BIQUAD render cannot be captured (its look-back state is per launch)");
            return DSP_ERR_INVALID;
        }
    }
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    if (!r.iir_fb_host) {
        if (int st = refuse_capture(s, "the BIQUAD repair counter")) return st;
        void *p = nullptr;
        DSPB_HIP(hipHostMalloc(&p, 64, hipHostMallocMapped));
        r.iir_fb_host = (uint32_t *)p;
        *r.iir_fb_host = 0;
        void *d = nullptr;
        DSPB_HIP(hipHostGetDevicePointer(&d, p, 0));
        r.iir_fb_dev = (uint32_t *)d;
    }
    IirWork &w = r.iir_work[(void *)s];
    if (w.cap < tiles) {
        if (int st = refuse_capture(s, "the BIQUAD look-back workspace")) return st;
        if (w.aggw) {
            DSPB_HIP(hipStreamSynchronize(s));
            DSPB_HIP(hipFree(w.aggw));
            w = IirWork{};
        }
        const uint64_t cap = std::max<uint64_t>(tiles, 1024);
        const size_t bytes = (2 * cap * 16 + 1) * sizeof(uint64_t);  // 16 words: a channel pair's 2 x 8
        void *p = nullptr;
        DSPB_HIP(hipMalloc(&p, bytes));
        DSPB_HIP(hipMemsetAsync(p, 0, bytes, s));
        w.aggw = (uint64_t *)p;
        w.inclw = w.aggw + cap * 16;
        w.cap = cap;
    }
    A->aggw = w.aggw;
    A->inclw = w.inclw;
    A->err = (uint32_t *)(w.inclw + w.cap * 16);
    A->repairs = r.iir_fb_dev;
    A->spin_limit = g_iir_spin_limit.load(std::memory_order_relaxed);
    w.epoch = w.epoch % 0xffffffffull + 1;
    A->epoch = w.epoch;
    if (int st = launch_biquad(*A, sections, nch, s)) return st;
    return DSP_OK;
}

// *table: a hold on the call's cached device table (FIR / BIQUAD), kept by
// the caller until the call's launches are enqueued
static int plugin_map(const dsp_plugin *p, uint32_t B, int dev, hipStream_t s, SampleMap *m, float sr,
                      uint32_t flags, DevTable *table) {
    m->kind = MapKind::Noop;
    m->fir_direct = (flags & DSP_EXEC_FIR_DIRECT) ? 1u : 0u;
    m->a = 1.f;
    m->table = nullptr;
    m->B = B;
    m->b_mask = is_pow2(B) ? B - 1 : 0;
    m->taps = nullptr;
    m->ntaps8 = 0;
    m->iir_tab = nullptr;
    m->sections = 0;
    m->iir_window = 0;
    m->module = nullptr;
    m->gparams = nullptr;
    m->gparams_size = 0;
    m->sr = sr;
    m->closed = 0;
    m->rg0 = m->rs = 0.0;
    if (!p) return DSP_OK;  // no plugin loaded: the file plays through (audio.cpp:144)
    float v0 = 0.f, v1 = 0.f;
    switch (p->kind) {
    case DSP_PLUGIN_NOOP:
        return DSP_OK;
    case DSP_PLUGIN_GAIN:  // build/gain_test.cpp: Parameters{float gain}
        if (!p->params || p->params_size < 4) return invalid("GAIN plugin needs a 4-byte params blob");
        std::memcpy(&v0, p->params, 4);
        m->kind = MapKind::Gain;
        m->a = v0;
        return DSP_OK;
    case DSP_PLUGIN_STATIC_GAIN:  // test/static_gain_plugin.cpp: State{float gain}
        if (!p->state || p->state_size < 4) return invalid("STATIC_GAIN plugin needs a 4-byte state blob");
        std::memcpy(&v0, p->state, 4);
        m->kind = MapKind::Gain;
        m->a = v0;
        return DSP_OK;
    case DSP_PLUGIN_IR_RAMP: {  // build/IR_test.cpp: Parameters{float gain; float step}
        if (!p->params || p->params_size < 8) return invalid("IR_RAMP plugin needs an 8-byte params blob");
        std::memcpy(&v0, p->params, 4);
        std::memcpy(&v1, (const char *)p->params + 4, 4);
        float *table = nullptr;
        int st = get_scratch(dev, s, sizeof(float) * B, &table);
        if (st) return st;
        m->kind = MapKind::Ramp;
        m->table = table;
        m->rg0 = (double)v0;
        m->rs = (double)v1;
        m->closed = ramp_closed_form(v0, v1, B) ? 1u : 0u;
        // closed form: the table is built only by ensure_ramp_table, for the
        // kernels that read it
        if (!m->closed) return launch_ramp_table(table, B, v0, v1, s);
        return DSP_OK;
    }
    case DSP_PLUGIN_FIR: {  // build-defined cfg 3b: Parameters{float taps[T]}
        const uint32_t T = p->params_size / 4;
        if (!p->params || T == 0 || p->params_size % 4 || T > 2048)
            return invalid("FIR plugin needs 1..2048 float taps as its params blob");
        const uint32_t T8 = (T + 15) & ~15u;  // zero-padded to 16 (fir.hip)
        // device copy: [taps, T8 floats][overlap-save H table, 8192 + 2 floats],
        // cached per device by the taps' bytes (the host FFT and the upload
        // happen once per filter, not once per render)
        std::vector<float> key((const float *)p->params, (const float *)p->params + T);
        float h2048[2] = {0.f, 0.f};
        {
            std::lock_guard<std::mutex> lk(g_mu);
            DeviceRes &r = g_res[dev];
            const FirTaps *ft = nullptr;
            for (auto &e : r.fir)
                if (e.taps == key) { ft = &e; break; }
            if (!ft) {
                if (int st = refuse_capture(s, "a FIR filter's device taps")) return st;
                // [taps, T8][8192-point table, 8194 (+ 2 pad)][4096-point pair table, 8192]
                std::vector<float> h(T8 + 8196 + 8192, 0.f);
                std::memcpy(h.data(), key.data(), 4 * (size_t)T);
                if (T <= 1025) {
                    ols_table(h.data(), T, h.data() + T8);
                    pair_table(h.data(), T, h.data() + T8 + 8196);
                }
                float *d = nullptr;
                DSPB_HIP(hipMalloc(&d, sizeof(float) * h.size()));
                if (int st = upload_table(d, h.data(), sizeof(float) * h.size())) {
                    (void)hipFree(d);
                    return st;
                }
                if (r.fir.size() >= 8) r.fir.erase(r.fir.begin());  // small LRU-ish cap (freed once unheld)
                r.fir.push_back(FirTaps{key, dev_table(d, dev), h[T8 + 8192], h[T8 + 8193]});
                ft = &r.fir.back();
            }
            *table = ft->dev;  // held by the call (copied under the lock)
            h2048[0] = ft->h2048r;
            h2048[1] = ft->h2048i;
        }
        float *tp = table->get();
        m->kind = MapKind::Fir;
        m->taps = tp;
        m->ntaps8 = T8;
        m->ntaps = T;
        m->olsH = tp + T8;
        m->pairH = tp + T8 + 8196;  // 16-byte aligned: T8 and 8196 are multiples of 4
        m->olsH2048[0] = h2048[0];
        m->olsH2048[1] = h2048[1];
        return DSP_OK;
    }
    case DSP_PLUGIN_BIQUAD: {  // build-defined: Parameters{float coef[5 S]}, S = 1..4 sections
        const uint32_t S = p->params_size / 20;
        if (!p->params || S == 0 || S > 4 || p->params_size % 20)
            return invalid("BIQUAD plugin needs 1..4 sections of 5 floats (b0 b1 b2 a1 a2) as its params blob");
        std::vector<float> key((const float *)p->params, (const float *)p->params + 5 * S);
        for (float v : key)
            if (!std::isfinite(v)) return invalid("BIQUAD coefficients must be finite");
        uint32_t window = 0;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            DeviceRes &r = g_res[dev];
            const IirTab *it = nullptr;
            for (auto &e : r.iir)
                if (e.coef == key) { it = &e; break; }
            if (!it) {
                if (int st = refuse_capture(s, "a BIQUAD cascade's state-transition tables")) return st;
                std::vector<float> h;
                const uint32_t W = biquad_tables(key.data(), S, h);
                float *d = nullptr;
                DSPB_HIP(hipMalloc(&d, sizeof(float) * h.size()));
                if (int st = upload_table(d, h.data(), sizeof(float) * h.size())) {
                    (void)hipFree(d);
                    return st;
                }
                if (r.iir.size() >= 8) r.iir.erase(r.iir.begin());  // as the FIR cache (freed once unheld)
                r.iir.push_back(IirTab{key, dev_table(d, dev), W});
                it = &r.iir.back();
            }
            *table = it->dev;  // held by the call (copied under the lock)
            window = it->window;
        }
        m->kind = MapKind::Biquad;
        m->iir_tab = table->get();
        m->sections = S;
        m->iir_window = window;
        return DSP_OK;
    }
    case DSP_PLUGIN_GENERIC:  // the plugin's own audio_callback, compiled for gfx950 (module.h)
        if (!p->module) return invalid("GENERIC plugin needs a loaded dsp_module");
        m->kind = MapKind::Generic;
        m->module = const_cast<void *>(p->module);
        m->gparams = p->params;
        m->gparams_size = p->params_size;
        m->gflags = flags;
        return DSP_OK;
    default:
        return invalid("unknown plugin kind %d", p->kind);
    }
}

// whether any input row [in[c], in[c] + L) overlaps any output row [out[c'], out[c'] + Lr)
static bool rows_overlap(const float *const *in, uint32_t in_ch, uint64_t L, const float *const *out, uint32_t C,
                         uint64_t Lr) {
    for (uint32_t a = 0; a < in_ch; ++a)
        for (uint32_t b = 0; b < C; ++b) {
            const uintptr_t i0 = reinterpret_cast<uintptr_t>(in[a]), o0 = reinterpret_cast<uintptr_t>(out[b]);
            if (L && Lr && i0 < o0 + 4 * Lr && o0 < i0 + 4 * L) return true;
        }
    return false;
}

// A GENERIC plugin with a known block class (module.h dsp_module_block_class)
// runs as that map: its own callback's block as a table, or its gain.
// in_place: the call renders over its own input; with DSP_EXEC_VERIFY_CLASS
// the callback then runs on every block, since the check needs the input
// after the render (and a re-render would need it whole)
// a table class's block held by a call: released (an event after the call's
// launches on its stream) when the call returns, so an evicted table is freed
// only after every launch that reads it
struct SpecHold {
    ::dsp_module *m = nullptr;
    void *use = nullptr;
    hipStream_t s = nullptr;
    DevTable table;  // the call's FIR / BIQUAD table (plugin_map)
    ~SpecHold() {
        if (use) (void)module_spec_done(m, use, s);
    }
};

static int specialize_generic(SampleMap *m, uint32_t C, uint32_t B, hipStream_t s, const dsp_exec *ex,
                              bool in_place, SpecHold *hold) {
    if (m->kind != MapKind::Generic || (ex && (ex->flags & DSP_EXEC_NO_SPECIALIZE))) return DSP_OK;
    if (in_place && ex && (ex->flags & DSP_EXEC_VERIFY_CLASS)) return DSP_OK;
    ModuleSpec sp;
    int st = module_specialize((::dsp_module *)m->module, m->gparams, m->gparams_size, C, B, m->sr, s, &sp);
    if (st) return st;
    hold->m = (::dsp_module *)m->module;
    hold->use = sp.use;
    hold->s = s;
    if (sp.kind == kSpecTable) {
        m->kind = MapKind::Ramp;  // value = table[(global sample) mod B]
        m->table = sp.table;
        m->closed = 0;
        if (sp.affine) {  // ... = (float)fma(-i, rs, rg0), checked against every table value
            m->closed = 2;  // (the table is the callback's own block: nothing to build)
            m->rg0 = sp.rg0;
            m->rs = sp.rs;
        }
    } else if (sp.kind == kSpecGain) {
        m->kind = MapKind::Gain;
        m->a = sp.gain;
    } else if (sp.kind == kSpecGainTable) {
        m->kind = MapKind::GainTable;  // value = x * table[c B + (global sample) mod B]
        m->table = sp.table;
        m->closed = 0;
    }
    return DSP_OK;
}

// DSP_EXEC_VERIFY_CLASS: after a GENERIC plugin rendered by its block class,
// run its callback on blocks of the call's own input -- the first, the last
// and two more (a hash of the call's length and offset) -- as render_audio
// hands them over (audio.cpp:13-175: the file, zeros past EOF and for the
// channels the file lacks), and compare with the rendered rows bit for bit.
// *ok = false on any difference.  Synchronises the stream.
static int verify_class(const SampleMap &orig, const float *const *in, uint32_t in_ch, uint64_t L,
                        float *const *out, uint32_t C, uint32_t B, uint64_t goff, hipStream_t s, bool *ok) {
    *ok = true;
    const uint64_t nb = (L + B - 1) / B;
    if (nb == 0) return DSP_OK;
    uint64_t pick[4] = {0, nb - 1, 0, 0};
    uint64_t h = (L * 0x9e3779b97f4a7c15ull) ^ (goff + 0x632be59bd9b4e019ull);
    for (int i = 2; i < 4; ++i) {
        h ^= h >> 29;
        h *= 0xbf58476d1ce4e5b9ull;
        h ^= h >> 32;
        pick[i] = h % nb;
    }
    const uint64_t n = (uint64_t)C * B;
    float *d = nullptr;
    DSPB_HIP(hipMalloc(&d, sizeof(float) * n));
    struct Free {
        float *p;
        ~Free() { (void)hipFree(p); }
    } fr{d};
    std::vector<float> blk(n), got(n), want(n);
    for (uint64_t b : pick) {
        const uint64_t i0 = b * B;
        const uint64_t m = L > i0 ? std::min<uint64_t>(B, L - i0) : 0;  // file samples in the block
        std::fill(blk.begin(), blk.end(), 0.f);
        for (uint32_t c = 0; c < std::min(in_ch, C); ++c)
            if (m) DSPB_HIP(hipMemcpyAsync(blk.data() + (uint64_t)c * B, in[c] + i0, m * sizeof(float),
                                           hipMemcpyDeviceToHost, s));
        for (uint32_t c = 0; c < C; ++c)
            DSPB_HIP(hipMemcpyAsync(got.data() + (uint64_t)c * B, out[c] + i0, (uint64_t)B * sizeof(float),
                                    hipMemcpyDeviceToHost, s));
        DSPB_HIP(hipStreamSynchronize(s));
        DSPB_HIP(hipMemcpyAsync(d, blk.data(), sizeof(float) * n, hipMemcpyHostToDevice, s));
        std::vector<float *> rows(C);
        for (uint32_t c = 0; c < C; ++c) rows[c] = d + (uint64_t)c * B;
        if (int st = module_callback_once((::dsp_module *)orig.module, orig.gparams, orig.gparams_size, rows.data(),
                                          C, B, orig.sr, s))
            return st;
        DSPB_HIP(hipMemcpyAsync(want.data(), d, sizeof(float) * n, hipMemcpyDeviceToHost, s));
        DSPB_HIP(hipStreamSynchronize(s));
        if (std::memcmp(want.data(), got.data(), sizeof(float) * n) != 0) {
            *ok = false;
            set_last_error("DSP_EXEC_VERIFY_CLASS: block %llu rendered by the block class differs from the "
                           "plugin's callback; rendered again with the callback",
                           (unsigned long long)b);
            return DSP_OK;
        }
    }
    return DSP_OK;
}

static void set_result(const dsp_exec *ex, uint32_t bits) {
    if (ex && ex->result) *ex->result = bits;
}

// ---------------------------------------------------------------------------
// host-buffer staging (DSP_EXEC_HOST_BUFFERS)
// ---------------------------------------------------------------------------
struct Staged {
    std::vector<float *> dev;
    ~Staged() {
        for (float *p : dev)
            if (p) (void)hipFree(p);
    }
    int alloc(size_t n_floats, float **out) {
        float *p = nullptr;
        if (n_floats == 0) n_floats = 1;
        DSPB_HIP(hipMalloc(&p, n_floats * sizeof(float)));
        dev.push_back(p);
        *out = p;
        return DSP_OK;
    }
};

static hipStream_t stream_of(const dsp_exec *ex) { return ex ? (hipStream_t)ex->stream : nullptr; }
static bool host_mode(const dsp_exec *ex) { return ex && (ex->flags & DSP_EXEC_HOST_BUFFERS); }
static uint64_t goff_of(const dsp_exec *ex) { return ex ? ex->sample_offset : 0; }

static int finish(const dsp_exec *ex) {
    if (ex && (ex->flags & (DSP_EXEC_SYNC | DSP_EXEC_HOST_BUFFERS)))
        DSPB_HIP(hipStreamSynchronize(stream_of(ex)));
    return DSP_OK;
}

// ---------------------------------------------------------------------------
// core device-pointer implementations
// ---------------------------------------------------------------------------
static int render_device(const float *const *in, uint32_t in_ch, uint64_t L, float *const *out,
                         uint32_t C, uint32_t B, const SampleMap &map, uint64_t start,
                         uint64_t goff, hipStream_t s) {
    const uint64_t nblocks = (L + B - 1) / B;
    const uint64_t end = nblocks * B;
    if (map.kind == MapKind::Generic) {
        if (start != 0) return invalid("GENERIC render: the fused tail path does not apply");
        return module_render((::dsp_module *)map.module, map.gparams, map.gparams_size, in, in_ch, L, out, C, B,
                             map.sr, goff, s, map.gflags);
    }
    if (map.kind == MapKind::Biquad) {  // the cascade from zero state at the start of the file
        if (start != 0 || goff != 0) return invalid("BIQUAD render: whole files only (sample_offset 0)");
        int dev = 0;
        DSPB_HIP(hipGetDevice(&dev));
        const uint32_t S = map.sections, D = 2 * S;
        // channel pairs in one wavefront (packed math) from kIirPairSections
        // sections on; an odd last channel on its own
        const bool pairs = S >= kIirPairSections;
        for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
            const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
            const uint32_t np = pairs ? cn & ~1u : 0;
            for (int part = 0; part < 2; ++part) {
                const uint32_t first = part ? np : 0, count = part ? cn - np : np, nch = part ? 1 : 2;
                if (!count) continue;
                BiquadArgs A{};
                A.in_aligned16 = A.out_aligned16 = 1;
                for (uint32_t j = 0; j < count; ++j) {
                    const uint32_t c = c0 + first + j;
                    A.out.p[j] = out[c];
                    A.out_aligned16 &= aligned(out[c], 16) ? 1u : 0u;
                    if (c < in_ch) {
                        A.in.p[j] = in[c];
                        A.in_ch = j + 1;
                        A.in_aligned16 &= aligned(in[c], 16) ? 1u : 0u;
                    }
                }
                A.L = L;
                A.Ly = end;
                A.C = count;
                A.ntiles_ch = biquad_tiles(end);
                A.coef = map.iir_tab;
                A.Q = map.iir_tab + 20;
                A.P = A.Q + (size_t)65 * D * D;
                A.window = map.iir_window;
                if (int st = iir_launch(dev, s, &A, S, nch)) return st;
            }
        }
        return DSP_OK;
    }
    if (map.kind == MapKind::Fir) {  // convolution from the start of the file
        if (start != 0 || goff != 0) return invalid("FIR render: whole files only (sample_offset 0)");
        if (map.ntaps <= 1025 && !map.fir_direct) {
            // overlap-save: channel pairs as one complex signal (fir_pair_kernel,
            // 4096-point frames); an odd last channel on its own
            // (fir_fft_kernel, 8192-point real frames)
            const v2f *tw = nullptr;
            int dev = 0;
            DSPB_HIP(hipGetDevice(&dev));
            int st = get_tw(dev, s, &tw);
            if (st) return st;
            for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
                const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
                const uint32_t np = cn & ~1u;  // (kMaxChannels is even)
                if (np) {
                    FirFftArgs A{};
                    for (uint32_t j = 0; j < np; ++j) {
                        A.out.p[j] = out[c0 + j];
                        if (c0 + j < in_ch) {
                            A.in.p[j] = in[c0 + j];
                            A.in_ch = j + 1;
                        }
                    }
                    A.L = L;
                    A.Ly = end;
                    A.tw = tw;
                    A.F = (end + kPairHop - 1) / kPairHop;
                    A.H = map.pairH;
                    if ((st = launch_fir_pair(A, np, s))) return st;
                }
                if (cn & 1) {
                    const uint32_t c = c0 + cn - 1;
                    FirFftArgs A{};
                    A.out.p[0] = out[c];
                    if (c < in_ch) {
                        A.in.p[0] = in[c];
                        A.in_ch = 1;
                    }
                    A.L = L;
                    A.Ly = end;
                    A.F = (end + 7167) / 7168;
                    A.H = map.olsH;
                    A.h2048 = v2f{map.olsH2048[0], map.olsH2048[1]};
                    A.tw = tw;
                    if ((st = launch_fir_fft(A, 1, s))) return st;
                }
            }
            return DSP_OK;
        }
        for (uint32_t c = 0; c < C; ++c) {
            int st = launch_fir(c < in_ch ? in[c] : nullptr, L, out[c], end, map.taps, map.ntaps8,
                                aligned(out[c], 16), s);
            if (st) return st;
        }
        return DSP_OK;
    }
    for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
        const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
        RenderArgs A{};
        bool vec = (start % 4) == 0;
        A.in_ch = 0;
        for (uint32_t j = 0; j < cn; ++j) {
            A.out.p[j] = out[c0 + j];
            vec = vec && aligned(out[c0 + j], 16);
            if (c0 + j < in_ch) {
                A.in.p[j] = in[c0 + j];
                A.in_ch = j + 1;
                vec = vec && aligned(in[c0 + j], 16);
            }
        }
        A.L = L;
        A.start = start;
        A.end = end;
        A.map = map;
        if (map.kind == MapKind::GainTable) A.map.table += (uint64_t)c0 * map.B;  // this group's rows
        A.goff = goff;
        int st = launch_render(A, cn, vec, s);
        if (st) return st;
    }
    return DSP_OK;
}

static int check_stft_args(uint32_t N, uint32_t H, uint32_t K, uint64_t ld, int32_t window) {
    if (window != DSP_WIN_HAMMING && window != DSP_WIN_HANN && window != DSP_WIN_RECT)
        return invalid("window=%d is not a DSP_WIN_* kind", window);
    if (!is_pow2(N) || N < 4 || N > 8192) return invalid("N=%u must be a power of two in [4, 8192]", N);
    if (H == 0) return invalid("hop H must be > 0");
    if (K == 0 || (K > N / 2 + 1 && K != N)) return invalid("K=%u must be <= N/2+1 or == N", K);
    if (ld < K) return invalid("ld=%llu < K=%u", (unsigned long long)ld, K);
    return DSP_OK;
}

static int stft_device(const float *const *in, uint32_t C, uint64_t L, uint32_t N, uint32_t H,
                       int window, uint32_t K, float *const *mag, uint64_t ld, int dev,
                       hipStream_t s) {
    const uint64_t F = dsp_stft_frame_count(L, N, H);
    if (F == 0) return DSP_OK;
    const v2f *tw = nullptr;
    const float *win = nullptr;
    int st = get_tw(dev, s, &tw);
    if (st) return st;
    bool fast = (N == 8192) && (H % 2 == 0);
    for (uint32_t c = 0; c < C; ++c) fast = fast && aligned(in[c], 8);
    st = get_window(dev, s, window, N, N, &win, fast ? window_prescale(N) : 1.0);
    if (st) return st;
    for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
        const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
        if (fast) {
            Stft8kArgs A{};
            for (uint32_t j = 0; j < cn; ++j) {
                A.in.p[j] = in[c0 + j];
                A.mag.p[j] = mag[c0 + j];
            }
            A.in_ch = cn;
            A.L = L;
            A.F = F;
            A.H = H;
            A.K = K;
            A.ld = ld;
            A.valid = N;
            A.win2 = reinterpret_cast<const v2f *>(win);
            A.tw = tw;
            A.scale = (float)(1.0 / std::sqrt((double)N));
            if ((st = set_wincomp(dev, s, window, &A))) return st;
            TimedLaunch tl{};
            if ((st = timing_begin(s, &tl))) return st;
            st = launch_stft(A, cn, false, s);
            if (st) return st;
            // algorithmic bytes: frame input read once per hop + magnitudes
            st = timing_end(s, &tl, (uint64_t)cn * F * ((uint64_t)H * 4 + (uint64_t)K * 4));
        } else {
            GenericFftArgs A{};
            for (uint32_t j = 0; j < cn; ++j) {
                A.sig.p[j] = in[c0 + j];
                A.mag.p[j] = mag[c0 + j];
            }
            A.frame_hop = H;
            A.valid = N;
            A.win = win;
            A.n = N;
            A.log2n = ilog2(N);
            A.dir = -1;
            A.tw = tw;
            A.scale = (float)(1.0 / std::sqrt((double)N));
            A.K = K;
            A.ld = ld;
            A.mode = 2;
            st = launch_fft_generic(A, F, cn, s);
        }
        if (st) return st;
    }
    return DSP_OK;
}

// GENERIC render + STFT: the plugin's own callback renders the whole file
// (module.cpp, the LDS-blocks driver), then the memory-source STFT reads the
// render back, both on the caller's stream.  Measured against the
// alternatives: chunks pipelined through the Infinity Cache on
// two streams, and three kernels fusing the callback with the FFT, were all
// slower -- a plugin callback runs serially over its block, and the LDS that
// holds blocks in flight is the same LDS the FFT's transposes need.
static int generic_render_stft(const float *const *in, uint32_t in_ch, uint64_t L, float *const *out, uint32_t C,
                               uint32_t B, const SampleMap &map, uint32_t N, uint32_t H, int window, uint32_t K,
                               float *const *mag, uint64_t ld, uint64_t goff, int dev, hipStream_t s) {
    const uint64_t Lr = (L + B - 1) / B * B;
    int st = module_render((::dsp_module *)map.module, map.gparams, map.gparams_size, in, in_ch, L, out, C, B,
                           map.sr, goff, s, map.gflags);
    return st ? st : stft_device(out, C, Lr, N, H, window, K, mag, ld, dev, s);
}

}  // namespace dspb

using namespace dspb;

// ===========================================================================
// extern "C"
// ===========================================================================
extern "C" {

int dsp_abi_version(void) { return DSPBENCH_ABI_VERSION; }



void dsp_kernel_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_timing = on != 0;
    // a stock of events for the current device, created here rather than
    // between the launches being timed
    int dev = 0;
    if (g_timing && hipGetDevice(&dev) == hipSuccess) {
        auto &pool = g_event_pool[dev];
        while (pool.size() < 1024) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            pool.push_back(e);
        }
    }
}

int dsp_kernel_timing(double *total_ms, uint64_t *launches, uint64_t *bytes) {
    std::vector<TimedLaunch> v;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        v.swap(g_timed);
    }
    double ms = 0.0;
    uint64_t b = 0;
    for (auto &t : v) {
        float e = 0.f;
        DSPB_HIP(hipEventSynchronize(t.stop));
        DSPB_HIP(hipEventElapsedTime(&e, t.start, t.stop));
        ms += e;
        b += t.bytes;
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto &t : v) {
            g_event_pool[t.dev].push_back(t.stop);
            g_event_pool[t.dev].push_back(t.start);
        }
    }
    if (total_ms) *total_ms = ms;
    if (launches) *launches = v.size();
    if (bytes) *bytes = b;
    return DSP_OK;
}

const char *dsp_last_error(void) { return g_last_error; }

const char *dsp_status_string(int s) {
    switch (s) {
    case DSP_OK: return "ok";
    case DSP_ERR_INVALID: return "invalid argument";
    case DSP_ERR_HIP: return "HIP runtime error";
    case DSP_ERR_UNSUPPORTED: return "unsupported";
    case DSP_ERR_NOMEM: return "out of device memory";
    case DSP_ERR_NO_DEVICE: return "no device";
    default: return "unknown status";
    }
}

int dsp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int dsp_debug_set(int what, uint64_t value) {
    if (what != DSP_DEBUG_BIQUAD_SPIN_LIMIT) return invalid("dsp_debug_set: unknown hook %d", what);
    g_iir_spin_limit.store(value > 0xffffffffull ? kIirSpinLimit : (uint32_t)value);
    return DSP_OK;
}

int dsp_debug_get(int what, uint64_t *value) {
    if (what != DSP_DEBUG_BIQUAD_REPAIRS || !value) return invalid("dsp_debug_get: unknown hook %d", what);
    int dev = 0;
    if (int st = current_device(&dev)) return st;
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceRes &r = g_res[dev];
    *value = 0;
    if (r.iir_fb_host) {
        *value = __atomic_exchange_n(r.iir_fb_host, 0u, __ATOMIC_SEQ_CST);
    }
    return DSP_OK;
}

int dsp_biquad_plan(const float *coef, uint32_t sections, uint32_t *window) {
    if (!coef || !window || sections == 0 || sections > 4) return invalid("dsp_biquad_plan: 1..4 sections");
    for (uint32_t q = 0; q < 5 * sections; ++q)
        if (!std::isfinite(coef[q])) return invalid("BIQUAD coefficients must be finite");
    std::vector<float> h;
    *window = biquad_tables(coef, sections, h);
    return DSP_OK;
}

uint64_t dsp_stft_frame_count(uint64_t L, uint32_t N, uint32_t H) {
    if (N == 0 || H == 0 || L < N) return 0;
    return (L - N) / H + 1;
}

int dsp_render_offline(const float *const *in, uint32_t in_channels, uint64_t L,
                       float *const *out, uint32_t C, uint32_t B, float sr,
                       const dsp_plugin *plugin, const dsp_exec *ex) {
    // (only a GENERIC plugin reads the sample rate)
    if (B == 0) return invalid("block size B must be > 0");
    if (C == 0) return DSP_OK;
    if (!out) return invalid("out is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!out[c]) return invalid("out[%u] is NULL", c);
    if (in_channels && !in) return invalid("in is NULL");
    for (uint32_t c = 0; c < in_channels; ++c)
        if (!in[c]) return invalid("in[%u] is NULL", c);
    if (ex && ex->sample_offset % B) return invalid("sample_offset must be a multiple of B");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t nblocks = (L + B - 1) / B;
    const uint64_t Lr = nblocks * B;

    std::vector<const float *> din(in_channels);
    std::vector<float *> dout(C);
    Staged stage;
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < in_channels; ++c) {
            float *d;
            int st = stage.alloc(L, &d);
            if (st) return st;
            DSPB_HIP(hipMemcpyAsync(d, in[c], L * sizeof(float), hipMemcpyHostToDevice, s));
            din[c] = d;
        }
        for (uint32_t c = 0; c < C; ++c) {
            int st = stage.alloc(Lr, &dout[c]);
            if (st) return st;
        }
    } else {
        for (uint32_t c = 0; c < in_channels; ++c) din[c] = in[c];
        for (uint32_t c = 0; c < C; ++c) dout[c] = out[c];
    }
    SpecHold hold;  // released after the call's launches
    SampleMap map;
    int st = plugin_map(plugin, B, g.dev, s, &map, sr, ex ? ex->flags : 0, &hold.table);
    if (st) return st;
    const SampleMap orig = map;
    if ((st = specialize_generic(&map, C, B, s, ex, rows_overlap(din.data(), in_channels, L, dout.data(), C, Lr), &hold)))
        return st;
    TimedLaunch tl{};
    if ((st = timing_begin(s, &tl))) return st;
    st = render_device(din.data(), in_channels, L, dout.data(), C, B, map, 0, goff_of(ex), s);
    if (st) return st;
    {   // algorithmic bytes: file read (unless the map ignores its input) + render write
        uint64_t bytes = (uint64_t)C * Lr * 4;
        if (map.kind != MapKind::Ramp) bytes += (uint64_t)std::min(in_channels, C) * L * 4;
        if ((st = timing_end(s, &tl, bytes))) return st;
    }
    if (orig.kind == MapKind::Generic && map.kind != MapKind::Generic) {
        uint32_t res = DSP_RESULT_CLASS;
        if (ex && (ex->flags & DSP_EXEC_VERIFY_CLASS)) {
            bool ok = true;
            if ((st = verify_class(orig, din.data(), in_channels, L, dout.data(), C, B, goff_of(ex), s, &ok))) return st;
            res |= ok ? DSP_RESULT_VERIFIED : DSP_RESULT_RERENDERED;
            if (!ok && (st = render_device(din.data(), in_channels, L, dout.data(), C, B, orig, 0, goff_of(ex), s)))
                return st;
        }
        set_result(ex, res);
    } else {
        set_result(ex, 0);
    }
    if (host_mode(ex))
        for (uint32_t c = 0; c < C; ++c)
            DSPB_HIP(hipMemcpyAsync(out[c], dout[c], Lr * sizeof(float), hipMemcpyDeviceToHost, s));
    return finish(ex);
}

int dsp_render_loop(const float *const *in, uint32_t in_channels, uint64_t L, uint64_t cursor,
                    float *const *out, uint32_t C, uint32_t B, uint64_t nblocks, float sr,
                    const dsp_plugin *plugin, uint64_t *cursor_out, const dsp_exec *ex) {
    if (B == 0) return invalid("block size B must be > 0");
    if (in_channels && L == 0) return invalid("loop mode over an empty file (the reference spins forever, audio.cpp:104)");
    if (in_channels && cursor >= L) return invalid("cursor %llu past the file (L = %llu)", (unsigned long long)cursor,
                                                   (unsigned long long)L);
    if (cursor_out) *cursor_out = in_channels ? (uint64_t)((cursor + (unsigned __int128)nblocks * B) % L) : cursor;
    if (C == 0 || nblocks == 0) return DSP_OK;
    if (!out) return invalid("out is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!out[c]) return invalid("out[%u] is NULL", c);
    if (in_channels && !in) return invalid("in is NULL");
    for (uint32_t c = 0; c < in_channels; ++c)
        if (!in[c]) return invalid("in[%u] is NULL", c);
    if (host_mode(ex)) return invalid("dsp_render_loop: device buffers only");
    if (ex && ex->sample_offset % B) return invalid("sample_offset must be a multiple of B");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t Lr = nblocks * B;
    SpecHold hold;  // released after the call's launches
    SampleMap map;
    int st = plugin_map(plugin, B, g.dev, s, &map, sr, ex ? ex->flags : 0, &hold.table);
    if (st) return st;
    // DSP_EXEC_VERIFY_CLASS: loop mode renders with the callback on every
    // block (as an in-place call does) rather than a class it would not check
    const bool verify = ex && (ex->flags & DSP_EXEC_VERIFY_CLASS);
    const MapKind before = map.kind;
    if ((st = specialize_generic(&map, C, B, s, ex, verify, &hold))) return st;
    set_result(ex, before == MapKind::Generic && map.kind != MapKind::Generic ? DSP_RESULT_CLASS : 0u);
    if ((st = ensure_ramp_table(map, s))) return st;
    const uint32_t in_ch = std::min(in_channels, C);  // channels_to_write (audio.cpp:66)
    auto wrap = [&](const float *const *src, float *const *dst, uint32_t nc, const SampleMap &m) -> int {
        for (uint32_t c0 = 0; c0 < nc; c0 += kMaxChannels) {
            const uint32_t cn = (nc - c0) < (uint32_t)kMaxChannels ? (nc - c0) : kMaxChannels;
            RenderArgs A{};
            for (uint32_t j = 0; j < cn; ++j) {
                A.out.p[j] = dst[c0 + j];
                if (c0 + j < in_ch) {
                    A.in.p[j] = src[c0 + j];
                    A.in_ch = j + 1;
                }
            }
            A.L = L;
            A.start = 0;
            A.end = Lr;
            A.map = m;
            if (m.kind == MapKind::GainTable) A.map.table += (uint64_t)c0 * m.B;  // this group's rows
            A.goff = goff_of(ex);
            if (int e = launch_render_wrap(A, cn, cursor, s)) return e;
        }
        return DSP_OK;
    };
    if (map.kind == MapKind::Noop || map.kind == MapKind::Gain || map.kind == MapKind::Ramp ||
        map.kind == MapKind::GainTable)
        return (st = wrap(in, out, C, map)) ? st : finish(ex);
    // FIR / GENERIC: the wrapped file is materialised (the plugin's block
    // stream), then rendered as a one-shot file of nblocks B samples
    float *tmp = nullptr;
    if (in_ch) {
        if ((st = get_scratch(g.dev, s, sizeof(float) * Lr * in_ch, &tmp, 1))) return st;
        std::vector<float *> rows(in_ch);
        for (uint32_t c = 0; c < in_ch; ++c) rows[c] = tmp + (uint64_t)c * Lr;
        SampleMap id{};
        id.kind = MapKind::Noop;
        id.B = B;
        if ((st = wrap(in, rows.data(), in_ch, id))) return st;
        std::vector<const float *> crow(rows.begin(), rows.end());
        st = render_device(crow.data(), in_ch, Lr, out, C, B, map, 0, goff_of(ex), s);
    } else {
        st = render_device(nullptr, 0, Lr, out, C, B, map, 0, goff_of(ex), s);
    }
    return st ? st : finish(ex);
}

int dsp_stft_magnitude(const float *const *in, uint32_t C, uint64_t L, uint32_t N, uint32_t H,
                       int32_t window, uint32_t K, float *const *mag, uint64_t ld,
                       const dsp_exec *ex) {
    int st = check_stft_args(N, H, K, ld, window);
    if (st) return st;
    if (C == 0) return DSP_OK;
    if (!in || !mag) return invalid("in / mag is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!in[c] || !mag[c]) return invalid("in[%u] / mag[%u] is NULL", c, c);
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t F = dsp_stft_frame_count(L, N, H);
    std::vector<const float *> din(C);
    std::vector<float *> dmag(C);
    Staged stage;
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < C; ++c) {
            float *d;
            if ((st = stage.alloc(L, &d))) return st;
            DSPB_HIP(hipMemcpyAsync(d, in[c], L * sizeof(float), hipMemcpyHostToDevice, s));
            din[c] = d;
            if ((st = stage.alloc(F * ld, &dmag[c]))) return st;
        }
    } else {
        for (uint32_t c = 0; c < C; ++c) { din[c] = in[c]; dmag[c] = mag[c]; }
    }
    st = stft_device(din.data(), C, L, N, H, window, K, dmag.data(), ld, g.dev, s);
    if (st) return st;
    if (host_mode(ex) && F)
        for (uint32_t c = 0; c < C; ++c)
            DSPB_HIP(hipMemcpyAsync(mag[c], dmag[c], F * ld * sizeof(float), hipMemcpyDeviceToHost, s));
    return finish(ex);
}

int dsp_render_stft(const float *const *in, uint32_t in_channels, uint64_t L,
                    float *const *out, uint32_t C, uint32_t B, float sr,
                    const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window,
                    uint32_t K, float *const *mag, uint64_t ld, const dsp_exec *ex) {

    if (B == 0) return invalid("block size B must be > 0");
    int st = check_stft_args(N, H, K, ld, window);
    if (st) return st;
    if (C == 0) return DSP_OK;
    if (!out || !mag) return invalid("out / mag is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!out[c] || !mag[c]) return invalid("out[%u] / mag[%u] is NULL", c, c);
    if (in_channels && !in) return invalid("in is NULL");
    for (uint32_t c = 0; c < in_channels; ++c)
        if (!in[c]) return invalid("in[%u] is NULL", c);
    if (ex && ex->sample_offset % B) return invalid("sample_offset must be a multiple of B");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t nblocks = (L + B - 1) / B;
    const uint64_t Lr = nblocks * B;
    const uint64_t F = dsp_stft_frame_count(Lr, N, H);

    std::vector<const float *> din(in_channels);
    std::vector<float *> dout(C), dmag(C);
    Staged stage;
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < in_channels; ++c) {
            float *d;
            if ((st = stage.alloc(L, &d))) return st;
            DSPB_HIP(hipMemcpyAsync(d, in[c], L * sizeof(float), hipMemcpyHostToDevice, s));
            din[c] = d;
        }
        for (uint32_t c = 0; c < C; ++c) {
            if ((st = stage.alloc(Lr, &dout[c]))) return st;
            if ((st = stage.alloc(F * ld, &dmag[c]))) return st;
        }
    } else {
        for (uint32_t c = 0; c < in_channels; ++c) din[c] = in[c];
        for (uint32_t c = 0; c < C; ++c) { dout[c] = out[c]; dmag[c] = mag[c]; }
    }
    SpecHold hold;  // released after the call's launches
    SampleMap map;
    if ((st = plugin_map(plugin, B, g.dev, s, &map, sr, ex ? ex->flags : 0, &hold.table))) return st;
    const SampleMap orig = map;
    if ((st = specialize_generic(&map, C, B, s, ex, rows_overlap(din.data(), in_channels, L, dout.data(), C, Lr), &hold)))
        return st;
    const uint64_t goff = goff_of(ex);
    set_result(ex, orig.kind == MapKind::Generic && map.kind != MapKind::Generic ? DSP_RESULT_CLASS : 0u);

    bool fused = (N == 8192) && (H % 128 == 0) && (H <= N) && (goff % 2 == 0) && F > 0 &&
                 map.kind != MapKind::Fir && map.kind != MapKind::Generic && map.kind != MapKind::Biquad;
    for (uint32_t c = 0; c < C; ++c) fused = fused && aligned(dout[c], 8);
    for (uint32_t c = 0; c < in_channels; ++c) fused = fused && aligned(din[c], 8);

    if (!fused && map.kind == MapKind::Generic) {
        // the plugin's own callback, then the STFT (generic_render_stft), timed
        // as one region: file read + render write + magnitude write
        TimedLaunch tl{};
        if ((st = timing_begin(s, &tl))) return st;
        tl_timing_outer = true;
        st = generic_render_stft(din.data(), in_channels, L, dout.data(), C, B, map, N, H, window, K, dmag.data(),
                                 ld, goff, g.dev, s);
        tl_timing_outer = false;
        if (st) return st;
        const uint64_t bytes = (uint64_t)std::min(in_channels, C) * L * 4 + (uint64_t)C * Lr * 4 +
                               (uint64_t)C * F * K * 4;
        if ((st = timing_end(s, &tl, bytes))) return st;
    } else if (!fused) {
        st = render_device(din.data(), in_channels, L, dout.data(), C, B, map, 0, goff, s);
        if (st) return st;
        st = stft_device(dout.data(), C, Lr, N, H, window, K, dmag.data(), ld, g.dev, s);
        if (st) return st;
    } else {
        const v2f *tw = nullptr;
        const float *win = nullptr;
        if ((st = get_tw(g.dev, s, &tw))) return st;
        if ((st = get_window(g.dev, s, window, N, N, &win, window_prescale(N)))) return st;
        bool tail_in_kernel = false;
        for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
            const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
            Stft8kArgs A{};
            A.in_ch = 0;
            for (uint32_t j = 0; j < cn; ++j) {
                A.out.p[j] = dout[c0 + j];
                A.mag.p[j] = dmag[c0 + j];
                if (c0 + j < in_channels) {
                    A.in.p[j] = din[c0 + j];
                    A.in_ch = j + 1;
                }
            }
            A.L = L;
            A.F = F;
            A.H = H;
            A.K = K;
            A.ld = ld;
            A.valid = N;
            A.win2 = reinterpret_cast<const v2f *>(win);
            A.tw = tw;
            A.scale = (float)(1.0 / std::sqrt((double)N));
            if ((st = set_wincomp(g.dev, s, window, &A))) return st;
            A.map = map;
            if (map.kind == MapKind::GainTable) A.map.table += (uint64_t)c0 * map.B;  // this group's rows
            A.goff = goff;
            // the PER kernel also renders the tail no frame owns
            if (stft8192_pk_per_path(A, true)) A.tail_end = Lr, tail_in_kernel = true;
            TimedLaunch tl{};
            if ((st = timing_begin(s, &tl))) return st;
            if ((st = launch_stft(A, cn, true, s))) return st;
            // algorithmic bytes: render write 4 B + magnitudes 4 K/H B
            // per hop sample, plus the file read when the map uses its input
            const uint64_t hop_samples = (uint64_t)cn * F * H;
            uint64_t bytes = hop_samples * 4 + (uint64_t)cn * F * K * 4;
            if (map.kind != MapKind::Ramp) bytes += (uint64_t)A.in_ch * F * H * 4;
            if (A.tail_end) bytes += (uint64_t)cn * (A.tail_end - F * (uint64_t)H) * 4;
            if ((st = timing_end(s, &tl, bytes))) return st;
        }
        // the render tail no frame owns: [F*H, Lr)
        if (!tail_in_kernel) {
            st = render_device(din.data(), in_channels, L, dout.data(), C, B, map, F * (uint64_t)H, goff, s);
            if (st) return st;
        }
    }
    if (orig.kind == MapKind::Generic && map.kind != MapKind::Generic && ex && (ex->flags & DSP_EXEC_VERIFY_CLASS)) {
        bool ok = true;
        if ((st = verify_class(orig, din.data(), in_channels, L, dout.data(), C, B, goff, s, &ok))) return st;
        set_result(ex, DSP_RESULT_CLASS | (ok ? DSP_RESULT_VERIFIED : DSP_RESULT_RERENDERED));
        if (!ok && (st = generic_render_stft(din.data(), in_channels, L, dout.data(), C, B, orig, N, H, window, K,
                                             dmag.data(), ld, goff, g.dev, s)))
            return st;
    }
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < C; ++c) {
            DSPB_HIP(hipMemcpyAsync(out[c], dout[c], Lr * sizeof(float), hipMemcpyDeviceToHost, s));
            if (F)
                DSPB_HIP(hipMemcpyAsync(mag[c], dmag[c], F * ld * sizeof(float),
                                        hipMemcpyDeviceToHost, s));
        }
    }
    return finish(ex);
}

int dsp_ir_analysis(const dsp_plugin *plugin, uint32_t C, float sr, uint32_t ir_len,
                    float *const *ir_out, float *mag, const dsp_exec *ex) {
    if (C == 0 || ir_len == 0) return invalid("C and ir_len must be > 0");
    if (!is_pow2(ir_len) || 4ull * ir_len > 8192) return invalid("4*ir_len must be a power of two <= 8192");
    if (!ir_out || !mag) return invalid("ir_out / mag is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!ir_out[c]) return invalid("ir_out[%u] is NULL", c);
    if (plugin && plugin->kind == DSP_PLUGIN_GENERIC && C > (uint32_t)kMaxChannels)
        return invalid("GENERIC plugin: IR analysis of 1..%d channels", kMaxChannels);
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint32_t n = 4 * ir_len;
    std::vector<float *> dir(C);
    float *dmag = mag;
    Staged stage;
    int st;
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < C; ++c)
            if ((st = stage.alloc(ir_len, &dir[c]))) return st;
        if ((st = stage.alloc(n, &dmag))) return st;
    } else {
        for (uint32_t c = 0; c < C; ++c) dir[c] = ir_out[c];
    }
    // compute_IR (plugin.cpp:27-34): IR[c] = delta, then one callback of ir_len
    SampleMap map;
    DevTable table;  // held until the call's launches are enqueued
    if ((st = plugin_map(plugin, ir_len, g.dev, s, &map, sr, ex ? ex->flags : 0, &table))) return st;
    if (map.kind == MapKind::Generic) {  // the impulse in place, a fresh scratch State, one callback
        for (uint32_t c0 = 0; c0 < C; c0 += kMaxChannels) {
            const uint32_t cn = (C - c0) < (uint32_t)kMaxChannels ? (C - c0) : kMaxChannels;
            ChanOut imp{};
            for (uint32_t j = 0; j < cn; ++j) imp.p[j] = dir[c0 + j];
            if ((st = launch_impulse(imp, cn, ir_len, s))) return st;
        }
        if ((st = module_ir((::dsp_module *)map.module, map.gparams, map.gparams_size, dir.data(), C, ir_len, sr, s)))
            return st;
    } else {  // map plugins: render the read-only impulse into IR[c], one launch
        const float *delta;
        if ((st = get_delta(g.dev, s, &delta))) return st;
        std::vector<const float *> cin(C, delta);
        if ((st = render_device(cin.data(), C, ir_len, dir.data(), C, ir_len, map, 0, 0, s))) return st;
    }

    // fft_perform_and_get_magnitude (dsp.cpp:53-66): channel 0 only
    const v2f *tw = nullptr;
    const float *win = nullptr;
    if ((st = get_tw(g.dev, s, &tw))) return st;
    const bool fast_ir = n == 8192 && aligned(dir[0], 8);
    if ((st = get_window(g.dev, s, DSP_WIN_HAMMING, n, ir_len, &win, fast_ir ? window_prescale(n) : 1.0)))
        return st;
    if (fast_ir) {
        Stft8kArgs A{};
        A.in.p[0] = dir[0];
        A.in_ch = 1;
        A.L = ir_len;
        A.mag.p[0] = dmag;
        A.F = 1;
        A.H = n;
        A.K = n;  // all bins, as the reference stores them (dsp.cpp:65)
        A.ld = n;
        A.valid = ir_len;
        A.win2 = reinterpret_cast<const v2f *>(win);
        A.tw = tw;
        A.scale = (float)(1.0 / std::sqrt((double)n));
        if ((st = launch_stft(A, 1, false, s))) return st;
    } else {
        GenericFftArgs A{};
        A.sig.p[0] = dir[0];
        A.frame_hop = 0;
        A.valid = ir_len;
        A.win = win;
        A.n = n;
        A.log2n = ilog2(n);
        A.dir = -1;
        A.tw = tw;
        A.scale = (float)(1.0 / std::sqrt((double)n));
        A.mag.p[0] = dmag;
        A.K = n;
        A.ld = n;
        A.mode = 2;
        if ((st = launch_fft_generic(A, 1, 1, s))) return st;
    }
    if (host_mode(ex)) {
        for (uint32_t c = 0; c < C; ++c)
            DSPB_HIP(hipMemcpyAsync(ir_out[c], dir[c], ir_len * sizeof(float), hipMemcpyDeviceToHost, s));
        DSPB_HIP(hipMemcpyAsync(mag, dmag, n * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    return finish(ex);
}

static int fft_service(const float *re_in, const float *im_in, float *re_out, float *im_out,
                       uint32_t n, int dir, const dsp_exec *ex) {
    if (!is_pow2(n) || n < 2 || n > 8192) return invalid("n=%u must be a power of two in [2, 8192]", n);
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const v2f *tw = nullptr;
    int st = get_tw(g.dev, s, &tw);
    if (st) return st;
    Staged stage;
    const float *dre = re_in, *dim = im_in;
    float *dro = re_out, *dio = im_out;
    if (host_mode(ex)) {
        float *a, *b;
        if ((st = stage.alloc(n, &a))) return st;
        DSPB_HIP(hipMemcpyAsync(a, re_in, n * sizeof(float), hipMemcpyHostToDevice, s));
        dre = a;
        if (im_in) {
            if ((st = stage.alloc(n, &b))) return st;
            DSPB_HIP(hipMemcpyAsync(b, im_in, n * sizeof(float), hipMemcpyHostToDevice, s));
            dim = b;
        }
        if ((st = stage.alloc(n, &dro))) return st;
        if (im_out && (st = stage.alloc(n, &dio))) return st;
    }
    GenericFftArgs A{};
    A.re_in = dre;
    A.im_in = dim;
    A.n = n;
    A.log2n = ilog2(n);
    A.dir = dir;
    A.tw = tw;
    A.scale = (float)(1.0 / std::sqrt((double)n));
    A.re_out = dro;
    A.im_out = dio;
    A.mode = im_out ? 0 : 1;
    if ((st = launch_fft_generic(A, 1, 1, s))) return st;
    if (host_mode(ex)) {
        DSPB_HIP(hipMemcpyAsync(re_out, dro, n * sizeof(float), hipMemcpyDeviceToHost, s));
        if (im_out)
            DSPB_HIP(hipMemcpyAsync(im_out, dio, n * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    return finish(ex);
}

int dsp_fft_forward(const float *in, float *re, float *im, uint32_t n, const dsp_exec *ex) {
    if (!in || !re || !im) return invalid("fft_forward: NULL buffer");
    return fft_service(in, nullptr, re, im, n, -1, ex);
}

int dsp_fft_reverse(const float *re, const float *im, float *out, uint32_t n, const dsp_exec *ex) {
    if (!re || !im || !out) return invalid("fft_reverse: NULL buffer");
    return fft_service(re, im, out, nullptr, n, +1, ex);
}

int dsp_gain(const float *in, float *out, float gain, uint64_t n, const dsp_exec *ex) {
    if (!in || !out) return invalid("NULL buffer");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    int st = launch_gain(in, out, gain, n, stream_of(ex));
    return st ? st : finish(ex);
}

int dsp_copy(const float *in, float *out, uint64_t n, const dsp_exec *ex) {
    if (!in || !out) return invalid("NULL buffer");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    bool done = false;
    if (!host_mode(ex)) {
        const int st = launch_copy(in, out, n, stream_of(ex), &done);
        if (st) return st;
    }
    if (!done) DSPB_HIP(hipMemcpyAsync(out, in, n * sizeof(float), hipMemcpyDeviceToDevice, stream_of(ex)));
    return finish(ex);
}

int dsp_set(float value, float *out, uint64_t n, const dsp_exec *ex) {
    if (!out) return invalid("NULL buffer");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    // the runtime's 32-bit memset with the value's bit pattern: 6.5 TB/s
    // against 6.0 for the float4 kernel (profiles/r02_elementwise_bw.txt)
    if (!host_mode(ex) && n) {
        uint32_t bits;
        std::memcpy(&bits, &value, 4);
        DSPB_HIP(hipMemsetD32Async((hipDeviceptr_t)out, (int)bits, n, stream_of(ex)));
        return finish(ex);
    }
    int st = launch_set(value, out, n, stream_of(ex));
    return st ? st : finish(ex);
}

int dsp_magnitude(const float *re, const float *im, float *out, uint64_t n, const dsp_exec *ex) {
    if (!re || !im || !out) return invalid("NULL buffer");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    int st = launch_magnitude(re, im, out, n, stream_of(ex));
    return st ? st : finish(ex);
}

// ---------------------------------------------------------------------------
// WAV payload decode / encode (wav.h)
// ---------------------------------------------------------------------------
static int wav_fmt_ok(uint16_t format, uint16_t bits) {
    return (format == DSP_WAV_FORMAT_PCM && (bits == 16 || bits == 24 || bits == 32)) ||
           (format == DSP_WAV_FORMAT_FLOAT && bits == 32);
}

int dsp_wav_decode(const void *payload, const dsp_wav_info *info, uint64_t frame0, uint64_t frames,
                   float *const *out, const dsp_exec *ex) {
    if (!info || !wav_fmt_ok(info->format, info->bits_per_sample)) return invalid("bad dsp_wav_info format");
    const uint32_t C = info->channels;
    if (C == 0 || C > (uint32_t)kMaxChannels) return invalid("channels must be 1..%d", kMaxChannels);
    if (frame0 > info->frames || frames > info->frames - frame0) return invalid("frame range past the payload");
    if (frames == 0) return DSP_OK;
    if (!payload || !out) return invalid("NULL buffer");
    for (uint32_t c = 0; c < C; ++c)
        if (!out[c]) return invalid("out[%u] is NULL", c);
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t ba = (uint64_t)C * (info->bits_per_sample / 8u);
    const uint8_t *src = (const uint8_t *)payload;
    uint64_t f0 = frame0;
    ChanOut o{};
    Staged stage;
    if (host_mode(ex)) {
        float *d;
        int st = stage.alloc((frames * ba + 3) / 4, &d);
        if (st) return st;
        DSPB_HIP(hipMemcpyAsync(d, src + frame0 * ba, frames * ba, hipMemcpyHostToDevice, s));
        src = (const uint8_t *)d;
        f0 = 0;
        for (uint32_t c = 0; c < C; ++c)
            if ((st = stage.alloc(frames, &o.p[c]))) return st;
    } else {
        for (uint32_t c = 0; c < C; ++c) o.p[c] = out[c];
    }
    bool al = true;
    for (uint32_t c = 0; c < C; ++c) al = al && aligned(o.p[c], 16);
    int st = launch_wav_decode(src, C, info->bits_per_sample, info->format == DSP_WAV_FORMAT_FLOAT, f0,
                               frames, o, al, s);
    if (st) return st;
    if (host_mode(ex))
        for (uint32_t c = 0; c < C; ++c)
            DSPB_HIP(hipMemcpyAsync(out[c], o.p[c], frames * sizeof(float), hipMemcpyDeviceToHost, s));
    return finish(ex);
}

int dsp_wav_encode(const float *const *in, uint32_t C, uint64_t frames, uint16_t format, uint16_t bits,
                   void *payload, const dsp_exec *ex) {
    if (!wav_fmt_ok(format, bits)) return invalid("unsupported WAV sample format");
    if (C == 0 || C > (uint32_t)kMaxChannels) return invalid("channels must be 1..%d", kMaxChannels);
    if (frames == 0) return DSP_OK;
    if (!in || !payload) return invalid("NULL buffer");
    for (uint32_t c = 0; c < C; ++c)
        if (!in[c]) return invalid("in[%u] is NULL", c);
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const uint64_t bytes = frames * C * (bits / 8u);
    uint8_t *dst = (uint8_t *)payload;
    ChanOut i{};
    Staged stage;
    if (host_mode(ex)) {
        float *d;
        int st = stage.alloc((bytes + 3) / 4, &d);
        if (st) return st;
        dst = (uint8_t *)d;
        for (uint32_t c = 0; c < C; ++c) {
            if ((st = stage.alloc(frames, &i.p[c]))) return st;
            DSPB_HIP(hipMemcpyAsync(i.p[c], in[c], frames * sizeof(float), hipMemcpyHostToDevice, s));
        }
    } else {
        for (uint32_t c = 0; c < C; ++c) i.p[c] = const_cast<float *>(in[c]);
    }
    int st = launch_wav_encode(dst, C, bits, format == DSP_WAV_FORMAT_FLOAT, frames, i, s);
    if (st) return st;
    if (host_mode(ex)) DSPB_HIP(hipMemcpyAsync(payload, dst, bytes, hipMemcpyDeviceToHost, s));
    return finish(ex);
}

// ---------------------------------------------------------------------------
// display reductions
// ---------------------------------------------------------------------------
int dsp_minmax_decimate(const float *x, uint64_t n, uint32_t pixels, float *vmax, float *vmin,
                        const dsp_exec *ex) {
    if (pixels == 0) return DSP_OK;
    if (!vmax || !vmin || (n && !x)) return invalid("NULL buffer");
    if (pixels > (1u << 24) || n >= (1ull << 39)) return invalid("pixels <= 2^24 and n < 2^39");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const float *dx = x;
    float *dmax = vmax, *dmin = vmin;
    Staged stage;
    if (host_mode(ex)) {
        float *t;
        int st;
        if ((st = stage.alloc(n, &t))) return st;
        if (n) DSPB_HIP(hipMemcpyAsync(t, x, n * sizeof(float), hipMemcpyHostToDevice, s));
        dx = t;
        if ((st = stage.alloc(pixels, &dmax)) || (st = stage.alloc(pixels, &dmin))) return st;
    }
    int st = launch_minmax(dx, n, pixels, dmax, dmin, s);
    if (st) return st;
    if (host_mode(ex)) {
        DSPB_HIP(hipMemcpyAsync(vmax, dmax, pixels * sizeof(float), hipMemcpyDeviceToHost, s));
        DSPB_HIP(hipMemcpyAsync(vmin, dmin, pixels * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    return finish(ex);
}

int dsp_spectrogram_decimate(const float *mag, uint64_t F, uint32_t K, uint64_t ld, uint32_t pixels,
                             float *out, const dsp_exec *ex) {
    if (pixels == 0 || K == 0) return DSP_OK;
    if (!out || (F && !mag)) return invalid("NULL buffer");
    if (ld < K) return invalid("ld < K");
    if (pixels > (1u << 24) || F >= (1ull << 39)) return invalid("pixels <= 2^24 and F < 2^39");
    DeviceGuard g(ex);
    if (g.status) return g.status;
    hipStream_t s = stream_of(ex);
    const float *dm = mag;
    float *dout = out;
    Staged stage;
    if (host_mode(ex)) {
        float *t;
        int st;
        const uint64_t nin = F ? (F - 1) * ld + K : 0;
        if ((st = stage.alloc(nin, &t))) return st;
        if (nin) DSPB_HIP(hipMemcpyAsync(t, mag, nin * sizeof(float), hipMemcpyHostToDevice, s));
        dm = t;
        if ((st = stage.alloc((uint64_t)pixels * K, &dout))) return st;
    }
    int st = launch_spectro(dm, F, K, ld, pixels, dout, s);
    if (st) return st;
    if (host_mode(ex))
        DSPB_HIP(hipMemcpyAsync(out, dout, (uint64_t)pixels * K * sizeof(float), hipMemcpyDeviceToHost, s));
    return finish(ex);
}

}  // extern "C"
