// iir.hip -- DSP_PLUGIN_BIQUAD: a cascade of S <= 4 biquad sections over a
// whole file, block-parallel.
//
// Each section is the direct-form-I difference equation of our stateful
// example plugin (plugins/biquad.cpp:43-57, the callback the reference's audio
// thread runs block after block, audio.cpp:160-165):
//
//   y[n] = b0 x[n] + b1 x[n-1] + b2 x[n-2] - a1 y[n-1] - a2 y[n-2]
//
// section k's input is section k-1's output, every history starts at zero
// (initialize_state's State s = {}) and is carried across blocks, so the
// render of ceil(L/B) blocks is the cascade run over the zero-padded file --
// whatever B is.  A serial chain per channel would leave the chip idle (one
// lane per channel), so the recurrence is split the way a linear scan is:
//
//   state s = (y1, y2) of every section, D = 2 S values.  Over T samples with
//   zero input the cascade maps s to M s (M = M_T, D x D), and over a run of
//   input from state s it ends in M s + e, where e is the end state of the same
//   run started from s = 0 (section 1's x history is the file itself, known).
//
// One wavefront owns a tile of 64 T samples of one channel, lane l the T
// samples [l T, (l + 1) T):
//   1. the tile is staged through LDS (coalesced 16-byte loads) into each
//      lane's registers; pass 1 runs the cascade from s = 0 -> e_l;
//   2. a Kogge-Stone scan over the lanes with the powers M^(T 2^j) gives
//      E_l = sum_{m <= l} M^(T (l - m)) e_m (the tile's state at the end of
//      lane l, tile entered at s = 0); E_63 is the tile's aggregate;
//   3. the tile publishes its aggregate; the state entering it is
//      S_in = sum_k M^(64 T k) agg_(i-1-k).  For a filter whose transition
//      decays (every stable one the host finds decaying within 256 tiles),
//      the sum stops at the W tiles whose weight exceeds 2^-48 (lane k reads
//      tile k + 1 back): only aggregates, a fixed summation order, the same
//      bits every run.  Otherwise (W = 0) a decoupled look-back: predecessors'
//      aggregates are combined back to the first that holds an inclusive state,
//      and every tile publishes its own inclusive state E_63 + M^(64 T) S_in;
//   4. lane l starts from E_(l-1) + M^(T l) S_in and runs the cascade again
//      over its registers (pass 2), the real outputs, out through LDS.
// So every sample is read once and written once from HBM (8 B per sample).
// Tile g is the wave's place in launch order, so a tile only ever waits for
// tiles of waves dispatched before it.  The wait is bounded anyway
// (A.spin_limit sleeps): a wave that gives up writes the launch's epoch into
// its stream's error word, and biquad_repair_kernel, launched behind every
// scan on the same stream, then renders the launch again as one serial chain
// per channel -- the call never returns stale words as audio, whatever the
// dispatch order or the other work on the GPU.
//
// Arithmetic: fp32, each section as fma(-a1, y1, fma(-a2, y2, fma(b2, x2,
// fma(b1, x1, b0 x)))); the matrix powers come from float64 (capi.cpp
// biquad_tables).  Not bit-exact with a serial fp32 chain (nor is the serial
// chain with the reference's -ffast-math build of the same source): the
// parity bar is a bound against float64 derived from the filter's own
// impulse responses (tests/test_gpu_biquad.py).
#include "kernels.hpp"

namespace dspb {

constexpr int kIirT = 32;             // samples per lane
constexpr int kIirTile = 64 * kIirT;  // samples per wavefront (tile)
constexpr int kIirWaves = 4;          // wavefronts per workgroup
constexpr int kIirLdsStride = kIirT + 1;  // floats per lane chunk in LDS (conflict-free column reads)
typedef float f4 __attribute__((ext_vector_type(4)));

// a lane's values for NCH channels at once: float (one channel per wave) or
// a VGPR pair (a channel pair per wave: every section step one v_pk_fma_f32)
template <int NCH> struct Lanes;
template <> struct Lanes<1> {
    typedef float V;
    static __device__ __forceinline__ V splat(float x) { return x; }
    static __device__ __forceinline__ V fma(V a, V b, V c) { return __builtin_fmaf(a, b, c); }
    static __device__ __forceinline__ float get(V v, int) { return v; }
    static __device__ __forceinline__ void set(V &v, int, float x) { v = x; }
    static __device__ __forceinline__ V shfl_up(V v, uint32_t d) { return __shfl_up(v, d); }
    static __device__ __forceinline__ V shfl(V v, int l) { return __shfl(v, l); }
    static __device__ __forceinline__ V shfl_xor(V v, int m) { return __shfl_xor(v, m); }
};
template <> struct Lanes<2> {
    typedef v2f V;
    static __device__ __forceinline__ V splat(float x) { return V{x, x}; }
    static __device__ __forceinline__ V fma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
    static __device__ __forceinline__ float get(V v, int k) { return k ? v.y : v.x; }
    static __device__ __forceinline__ void set(V &v, int k, float x) {
        if (k) v.y = x;
        else v.x = x;
    }
    static __device__ __forceinline__ V shfl_up(V v, uint32_t d) { return V{__shfl_up(v.x, d), __shfl_up(v.y, d)}; }
    static __device__ __forceinline__ V shfl(V v, int l) { return V{__shfl(v.x, l), __shfl(v.y, l)}; }
    static __device__ __forceinline__ V shfl_xor(V v, int m) { return V{__shfl_xor(v.x, m), __shfl_xor(v.y, m)}; }
};

template <int S, int NCH>
struct Cascade {
    static constexpr int D = 2 * S;
    typedef Lanes<NCH> LN;
    typedef typename LN::V V;
    V b0[S], b1[S], b2[S], na1[S], na2[S];

    __device__ explicit Cascade(const float *cf) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
            b0[k] = LN::splat(cf[5 * k]);
            b1[k] = LN::splat(cf[5 * k + 1]);
            b2[k] = LN::splat(cf[5 * k + 2]);
            na1[k] = LN::splat(-cf[5 * k + 3]);
            na2[k] = LN::splat(-cf[5 * k + 4]);
        }
    }

    // runs the cascade over x[0..T) from state st (y1, y2 per section; the x
    // history of section k > 0 is section k - 1's (y1, y2)); section 1's x
    // history is (xh1, xh2).  st ends as the state after x[T-1].  kWrite:
    // x[n] becomes the last section's output.
    template <bool kWrite>
    __device__ __forceinline__ void run(V (&x)[kIirT], V xh1, V xh2, V (&st)[D]) const {
        V X1[S], X2[S], Y1[S], Y2[S];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            Y1[k] = st[2 * k];
            Y2[k] = st[2 * k + 1];
            X1[k] = k ? st[2 * k - 2] : xh1;
            X2[k] = k ? st[2 * k - 1] : xh2;
        }
#pragma unroll
        for (int n = 0; n < kIirT; ++n) {
            V v = x[n];
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const V acc = LN::fma(b2[k], X2[k], LN::fma(b1[k], X1[k], b0[k] * v));
                const V y = LN::fma(na1[k], Y1[k], LN::fma(na2[k], Y2[k], acc));
                X2[k] = X1[k];
                X1[k] = v;
                Y2[k] = Y1[k];
                Y1[k] = y;
                v = y;
            }
            if (kWrite) x[n] = v;
        }
#pragma unroll
        for (int k = 0; k < S; ++k) {
            st[2 * k] = Y1[k];
            st[2 * k + 1] = Y2[k];
        }
    }
};

// r = m v for a D x D row-major matrix in memory
template <int D, int NCH>
__device__ __forceinline__ void matvec(const float *m, const typename Lanes<NCH>::V (&v)[D],
                                       typename Lanes<NCH>::V (&r)[D]) {
    typedef Lanes<NCH> LN;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        typename LN::V a = LN::splat(0.f);
#pragma unroll
        for (int j = 0; j < D; ++j) a = LN::fma(LN::splat(m[i * D + j]), v[j], a);
        r[i] = a;
    }
}

// NCH = 2: a wavefront owns the same 2048 samples of a channel pair (lane
// values are VGPR pairs, every recurrence step a packed FMA: half the VALU
// of two single-channel tiles); the tile's words hold both channels' states
template <int S, bool kChain, int NCH>
__global__ __launch_bounds__(256) void biquad_scan_kernel(BiquadArgs A) {
    constexpr int D = 2 * S;
    typedef Lanes<NCH> LN;
    typedef typename LN::V V;
    __shared__ float lds[kIirWaves][64 * kIirLdsStride];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    float *buf = lds[wave];

    // tile g = the wave's place in launch order: workgroups are dispatched in
    // increasing id, so a tile's predecessors belong to waves already running
    // or done (the waits are bounded anyway)
    const uint32_t U = A.C / NCH;  // channel units (pairs) of the launch
    const uint64_t g = (uint64_t)blockIdx.x * kIirWaves + wave;
    if (g >= (uint64_t)U * A.ntiles_ch) return;
    const uint32_t u = (uint32_t)(g % U);
    const uint64_t ti = g / U;
    const uint64_t base = ti * kIirTile;  // first sample of the tile in the channel

    // 1. stage each channel of the unit through LDS: 16-byte loads, element e
    // of the tile -> lane chunk e / T, then into the lane's registers
    V xr[kIirT], h1 = LN::splat(0.f), h2 = LN::splat(0.f);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        const uint32_t c = u * NCH + (uint32_t)ch;
        const float *x = c < A.in_ch ? A.in.p[c] : nullptr;
        const uint64_t lim = (x && A.L > base) ? A.L - base : 0;  // file samples in or after the tile
        if (lim >= (uint64_t)kIirTile && A.in_aligned16) {
            const f4 *x4 = reinterpret_cast<const f4 *>(x + base);
            f4 v[kIirTile / 256];
#pragma unroll
            for (int k = 0; k < kIirTile / 256; ++k) v[k] = __builtin_nontemporal_load(x4 + k * 64 + lane);
#pragma unroll
            for (int k = 0; k < kIirTile / 256; ++k) {
                const uint32_t e = k * 256 + lane * 4;
                float *d = buf + (e / kIirT) * kIirLdsStride + e % kIirT;
                d[0] = v[k].x, d[1] = v[k].y, d[2] = v[k].z, d[3] = v[k].w;
            }
        } else {
            for (uint32_t e = lane; e < (uint32_t)kIirTile; e += 64)
                buf[(e / kIirT) * kIirLdsStride + e % kIirT] = e < lim ? x[base + e] : 0.f;
        }
        // section 1's x history at the tile start: the file's two samples before it
        float a1 = 0.f, a2 = 0.f;
        if (lane == 0 && x) {
            if (base >= 1 && base - 1 < A.L) a1 = x[base - 1];
            if (base >= 2 && base - 2 < A.L) a2 = x[base - 2];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int n = 0; n < kIirT; ++n) LN::set(xr[n], ch, buf[lane * kIirLdsStride + n]);
        if (lane > 0) {
            a1 = buf[(lane - 1) * kIirLdsStride + kIirT - 1];
            a2 = buf[(lane - 1) * kIirLdsStride + kIirT - 2];
        }
        LN::set(h1, ch, a1);
        LN::set(h2, ch, a2);
        // (the next channel overwrites the tile: LDS ops of a wave complete in order)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    // pass 1: from state 0
    const Cascade<S, NCH> cs(A.coef);
    V E[D];
#pragma unroll
    for (int r = 0; r < D; ++r) E[r] = LN::splat(0.f);
    cs.template run<false>(xr, h1, h2, E);

    // 2. scan over the lanes: E_l = sum_{m <= l} M^(T (l - m)) e_m
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t d = 1u << j;
        V t[D], r[D];
#pragma unroll
        for (int q = 0; q < D; ++q) t[q] = LN::shfl_up(E[q], d);
        matvec<D, NCH>(A.Q + (size_t)d * D * D, t, r);
        if (lane >= d) {
#pragma unroll
            for (int q = 0; q < D; ++q) E[q] += r[q];
        }
    }
    V agg[D];
#pragma unroll
    for (int q = 0; q < D; ++q) agg[q] = LN::shfl(E[q], 63);

    // 3. the state entering the tile.  A tile's aggregate (and, in the
    // chained mode, its inclusive state) is published as NCH D self-validating
    // 64-bit words (launch tag << 32 | float bits), each one relaxed atomic
    // store at device scope: a reader takes a value only when all its words
    // carry this launch's tag -- no flag, so no release / acquire (no L2
    // write-back or invalidate) on either side
    constexpr int NW = NCH * D;  // words per tile
    V Sin[D];
#pragma unroll
    for (int q = 0; q < D; ++q) Sin[q] = LN::splat(0.f);
    const uint64_t tag = A.epoch << 32;
    auto publish = [&](uint64_t *words, const V (&v)[D]) {
        float mine = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) mine = lane == (uint32_t)w ? LN::get(v[w / NCH], w % NCH) : mine;
        if (lane < (uint32_t)NW)
            __hip_atomic_store(words + g * NW + lane, tag | __float_as_uint(mine), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // the words of tile gj: true when all carry this launch's tag
    auto fetch = [&](const uint64_t *words, uint64_t gj, V (&v)[D]) {
        bool ok = true;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint64_t t = __hip_atomic_load(const_cast<uint64_t *>(words) + gj * NW + w, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            ok = ok && (t & 0xffffffff00000000ull) == tag;
            LN::set(v[w / NCH], w % NCH, __uint_as_float((uint32_t)t));
        }
        return ok;
    };
    uint32_t spins = 0;
    auto give_up = [&]() {  // bounded; the launch is then rendered again (biquad_repair_kernel)
        if (++spins <= A.spin_limit) {
            __builtin_amdgcn_s_sleep(1);
            return false;
        }
        if (lane == 0) __hip_atomic_store(A.err, (uint32_t)A.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
    };
    publish(A.aggw, agg);
    if constexpr (!kChain) {
        // a filter whose transition decays: S_in = sum_{k < W} M^(64 T k)
        // agg_(i-1-k), every older tile's weight being below 2^-48 (the host
        // picked W).  Aggregates only, summed in a fixed order: no chain of
        // inclusive states, and the same bits on every run.
        for (uint32_t k0 = 0; k0 < A.window && (uint64_t)k0 < ti; k0 += 64) {
            const uint32_t k = k0 + lane;
            const bool valid = k < A.window && (uint64_t)k < ti;
            const uint64_t gj = valid ? (ti - 1 - k) * U + u : 0;
            V v[D], w[D];
            for (;;) {
                const bool ok = !valid || fetch(A.aggw, gj, v);
                if (__ballot(!ok) == 0 || give_up()) break;
            }
#pragma unroll
            for (int q = 0; q < D; ++q) v[q] = valid ? v[q] : LN::splat(0.f);
            matvec<D, NCH>(A.P + (size_t)(valid ? k : 0) * D * D, v, w);
#pragma unroll
            for (int q = 0; q < D; ++q) {
                V a = w[q];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) a += LN::shfl_xor(a, o);
                Sin[q] += a;
            }
        }
    } else {
        // a filter that does not decay within the table (W = 0): decoupled
        // look-back, predecessors' aggregates back to the first one holding an
        // inclusive state; this tile then publishes its own
        float mult[D * D];  // M^(64 T (i - 1 - jbase)), the window's weight
#pragma unroll
        for (int q = 0; q < D * D; ++q) mult[q] = (q % (D + 1)) == 0 ? 1.f : 0.f;
        int64_t jbase = (int64_t)ti - 1;
        while (jbase >= 0) {
            const int64_t jj = jbase - (int64_t)lane;
            const uint64_t gj = jj >= 0 ? (uint64_t)jj * U + u : 0;
            V v[D], w[D];
            uint32_t state = 2;  // before the channel's first tile: an inclusive zero
#pragma unroll
            for (int q = 0; q < D; ++q) v[q] = LN::splat(0.f);
            if (jj >= 0) state = fetch(A.inclw, gj, v) ? 2u : fetch(A.aggw, gj, v) ? 1u : 0u;
            const uint64_t incl = __ballot(state == 2);
            const uint64_t ready = __ballot(state != 0);
            const uint32_t first = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
            const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
            if ((ready & need) != need) {
                if (give_up()) break;
                continue;
            }
#pragma unroll
            for (int q = 0; q < D; ++q) v[q] = (lane <= first && jj >= 0) ? v[q] : LN::splat(0.f);
            matvec<D, NCH>(A.P + (size_t)lane * D * D, v, w);  // M^(64 T lane) v
#pragma unroll
            for (int q = 0; q < D; ++q) {
                V a = w[q];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) a += LN::shfl_xor(a, o);
                w[q] = a;
            }
#pragma unroll
            for (int q = 0; q < D; ++q) {
                V a = Sin[q];
#pragma unroll
                for (int j = 0; j < D; ++j) a = LN::fma(LN::splat(mult[q * D + j]), w[j], a);
                Sin[q] = a;
            }
            if (first < 64) break;
            // next window: weight by M^(64 T 64) more
            float nm[D * D];
            const float *p64 = A.P + (size_t)64 * D * D;
#pragma unroll
            for (int i = 0; i < D; ++i)
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < D; ++k) a = __builtin_fmaf(mult[i * D + k], p64[k * D + j], a);
                    nm[i * D + j] = a;
                }
#pragma unroll
            for (int q = 0; q < D * D; ++q) mult[q] = nm[q];
            jbase -= 64;
        }
        V inc[D], r[D];  // agg + M^(64 T) S_in
        matvec<D, NCH>(A.P + (size_t)D * D, Sin, r);
#pragma unroll
        for (int q = 0; q < D; ++q) inc[q] = agg[q] + r[q];
        publish(A.inclw, inc);
    }

    // 4. lane l from E_(l-1) + M^(T l) S_in, over its own samples
    V s0[D];
    {
        V r[D];
        matvec<D, NCH>(A.Q + (size_t)lane * D * D, Sin, r);
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const V prev = LN::shfl_up(E[q], 1);
            s0[q] = (lane ? prev : LN::splat(0.f)) + r[q];
        }
    }
    cs.template run<true>(xr, h1, h2, s0);
    const uint64_t ny = A.Ly > base ? A.Ly - base : 0;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
        for (int n = 0; n < kIirT; ++n) buf[lane * kIirLdsStride + n] = LN::get(xr[n], ch);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float *y = A.out.p[u * NCH + (uint32_t)ch];
        if (ny >= (uint64_t)kIirTile && A.out_aligned16) {
            f4 *y4 = reinterpret_cast<f4 *>(y + base);
#pragma unroll
            for (int k = 0; k < kIirTile / 256; ++k) {
                const uint32_t e = k * 256 + lane * 4;
                const float *sp = buf + (e / kIirT) * kIirLdsStride + e % kIirT;
                __builtin_nontemporal_store(f4{sp[0], sp[1], sp[2], sp[3]}, y4 + k * 64 + lane);
            }
        } else {
            for (uint32_t e = lane; e < (uint32_t)kIirTile && e < ny; e += 64)
                y[base + e] = buf[(e / kIirT) * kIirLdsStride + e % kIirT];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Behind every scan on its stream: when a wave of that launch gave up its
// look-back (the error word holds the launch's epoch -- epochs are unique per
// launch on a workspace, so no reset is needed), render the launch again as
// one serial chain per channel (a workgroup per channel: the wave stages a
// tile through LDS, lane 0 runs the cascade over it), the same difference
// equation within the same bound.  Otherwise one load and out.
template <int S>
__global__ __launch_bounds__(64) void biquad_repair_kernel(BiquadArgs A) {
    if (__hip_atomic_load(A.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint32_t)A.epoch) return;
    __shared__ float buf[kIirTile];
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    if (c == 0 && lane == 0) __hip_atomic_fetch_add(A.repairs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const float *x = c < A.in_ch ? A.in.p[c] : nullptr;
    float *y = A.out.p[c];
    const Cascade<S, 1> cs(A.coef);
    float st[2 * S], h1 = 0.f, h2 = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * S; ++q) st[q] = 0.f;
    for (uint64_t base = 0; base < A.Ly; base += kIirTile) {
        for (uint32_t e = lane; e < (uint32_t)kIirTile; e += 64) buf[e] = (x && base + e < A.L) ? x[base + e] : 0.f;
        __syncthreads();
        if (lane == 0) {
            for (int k0 = 0; k0 < kIirTile; k0 += kIirT) {
                float v[kIirT];
#pragma unroll
                for (int n = 0; n < kIirT; ++n) v[n] = buf[k0 + n];
                const float n1 = v[kIirT - 1], n2 = v[kIirT - 2];  // the next run's x history
                cs.template run<true>(v, h1, h2, st);
                h1 = n1;
                h2 = n2;
#pragma unroll
                for (int n = 0; n < kIirT; ++n) buf[k0 + n] = v[n];
            }
        }
        __syncthreads();
        for (uint32_t e = lane; e < (uint32_t)kIirTile && base + e < A.Ly; e += 64) y[base + e] = buf[e];
        __syncthreads();
    }
}

uint64_t biquad_tiles(uint64_t Ly) { return (Ly + kIirTile - 1) / kIirTile; }
uint32_t biquad_lane_samples() { return kIirT; }

int launch_biquad(const BiquadArgs &A, uint32_t sections, uint32_t nch, hipStream_t s) {
    if (nch != 1 && nch != 2) return DSP_ERR_INVALID;
    if (A.C == 0 || A.C % nch || A.C > (uint32_t)kMaxChannels) return DSP_ERR_INVALID;
    const uint64_t waves = (uint64_t)(A.C / nch) * A.ntiles_ch;
    if (waves == 0) return DSP_OK;
    const uint64_t groups = (waves + kIirWaves - 1) / kIirWaves;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    const dim3 grid((uint32_t)groups), blk(256);
    const bool chain = A.window == 0;
#define DSPB_BQ(SS, CH, NC) hipLaunchKernelGGL((biquad_scan_kernel<SS, CH, NC>), grid, blk, 0, s, A)
    switch ((sections * 2 + (chain ? 1 : 0)) * 2 + (nch - 1)) {
    case 4: DSPB_BQ(1, false, 1); break;
    case 5: DSPB_BQ(1, false, 2); break;
    case 6: DSPB_BQ(1, true, 1); break;
    case 7: DSPB_BQ(1, true, 2); break;
    case 8: DSPB_BQ(2, false, 1); break;
    case 9: DSPB_BQ(2, false, 2); break;
    case 10: DSPB_BQ(2, true, 1); break;
    case 11: DSPB_BQ(2, true, 2); break;
    case 12: DSPB_BQ(3, false, 1); break;
    case 13: DSPB_BQ(3, false, 2); break;
    case 14: DSPB_BQ(3, true, 1); break;
    case 15: DSPB_BQ(3, true, 2); break;
    case 16: DSPB_BQ(4, false, 1); break;
    case 17: DSPB_BQ(4, false, 2); break;
    case 18: DSPB_BQ(4, true, 1); break;
    case 19: DSPB_BQ(4, true, 2); break;
    default: return DSP_ERR_INVALID;
    }
#undef DSPB_BQ
    DSPB_HIP(hipGetLastError());
    const dim3 rgrid(A.C), rblk(64);
    switch (sections) {
    case 1: hipLaunchKernelGGL((biquad_repair_kernel<1>), rgrid, rblk, 0, s, A); break;
    case 2: hipLaunchKernelGGL((biquad_repair_kernel<2>), rgrid, rblk, 0, s, A); break;
    case 3: hipLaunchKernelGGL((biquad_repair_kernel<3>), rgrid, rblk, 0, s, A); break;
    default: hipLaunchKernelGGL((biquad_repair_kernel<4>), rgrid, rblk, 0, s, A); break;
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}


}  // namespace dspb
