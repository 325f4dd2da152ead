// fft_device.hpp -- register-level FFT building blocks for CDNA4 (wave64).
#pragma once
#include "kernels.hpp"
#include "twiddles.inc"

namespace dspb {

// Phase clocks for the diagnostic build (tools/stamps.hip): lane 0 of each
// wave records s_memtime at phase boundaries.  Compiled out otherwise.
#ifdef DSPB_STAMPS
#define DSPB_STAMP(A, f, lane, i)                                                         \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        uint64_t t_;                                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        if ((lane) == 0) (A).stamps[(f) * 8 + (i)] = t_;                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)
#else
#define DSPB_STAMP(A, f, lane, i) do { } while (0)
#endif

__device__ __forceinline__ v2f cmul(v2f a, v2f b) {
    return v2f{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ v2f mul_negi(v2f a) { return v2f{a.y, -a.x}; }

// Forward DFT4 in place: (a, b, c, d) <- (X0, X1, X2, X3).
__device__ __forceinline__ void dft4(v2f &a, v2f &b, v2f &c, v2f &d) {
    v2f t0 = a + c, t1 = a - c, t2 = b + d, t3 = b - d;
    v2f m3 = mul_negi(t3);
    a = t0 + t2;
    c = t0 - t2;
    b = t1 + m3;
    d = t1 - m3;
}

// Forward DFT8 on u[0..7], natural order in and out (radix-2 over DFT4s).
__device__ __forceinline__ void dft8(v2f &u0, v2f &u1, v2f &u2, v2f &u3, v2f &u4,
                                     v2f &u5, v2f &u6, v2f &u7) {
    v2f e0 = u0, e1 = u2, e2 = u4, e3 = u6;
    v2f o0 = u1, o1 = u3, o2 = u5, o3 = u7;
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    const float r = 0x1.6a09e6p-1f;  // 1/sqrt(2)
    v2f w1 = v2f{(o1.x + o1.y) * r, (o1.y - o1.x) * r};   // W8^1 o1
    v2f w2 = mul_negi(o2);                                // W8^2 o2
    v2f w3 = v2f{(o3.y - o3.x) * r, -(o3.x + o3.y) * r};  // W8^3 o3
    u0 = e0 + o0; u4 = e0 - o0;
    u1 = e1 + w1; u5 = e1 - w1;
    u2 = e2 + w2; u6 = e2 - w2;
    u3 = e3 + w3; u7 = e3 - w3;
}

// Register index holding X[k] after dft64 (base-8 digit reversal).
__host__ __device__ constexpr int perm64(int k) { return 8 * (k & 7) + (k >> 3); }

__device__ __forceinline__ v2f twiddle64(v2f a, int m) {
    if (m == 0) return a;
    if (m == 16) return mul_negi(a);
    return cmul(a, v2f{kW64_re[m], kW64_im[m]});
}

// Forward 64-point DFT of v[0..63] (natural order in); X[k] ends in
// v[perm64(k)].  8 x 8 decomposition: k = k1 + 8 k2, b = 8 b1 + b2.
__device__ __forceinline__ void dft64(v2f (&v)[64]) {
#pragma unroll
    for (int b2 = 0; b2 < 8; ++b2) {
        __builtin_amdgcn_sched_barrier(0);  // bound the live range: one DFT8 at a time
        dft8(v[b2], v[8 + b2], v[16 + b2], v[24 + b2], v[32 + b2], v[40 + b2],
             v[48 + b2], v[56 + b2]);
    }
    // now y[b2][k1] sits at v[8 k1 + b2]
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1)
#pragma unroll
        for (int b2 = 1; b2 < 8; ++b2) v[8 * k1 + b2] = twiddle64(v[8 * k1 + b2], b2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
        __builtin_amdgcn_sched_barrier(0);
        dft8(v[8 * k1], v[8 * k1 + 1], v[8 * k1 + 2], v[8 * k1 + 3], v[8 * k1 + 4],
             v[8 * k1 + 5], v[8 * k1 + 6], v[8 * k1 + 7]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // X[k1 + 8 k2] at v[8 k1 + k2]
}

__device__ __forceinline__ void lds_fence() {
    // LDS ops of one wave complete in order; the clobber stops the compiler
    // from moving loads above the other lanes' stores.
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float bperm(uint32_t byte_addr, float x) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute((int)byte_addr, __float_as_int(x)));
}

// Forward 32-point DFT of v[0..31] (natural order in); X[k] ends in
// v[perm32(k)].  8 x 4 decomposition: k = k1 + 8 k2, j = 4 j1 + j2.
__host__ __device__ constexpr int perm32(int k) { return 4 * (k & 7) + (k >> 3); }

__device__ __forceinline__ void dft32(v2f (&v)[32]) {
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) {
        __builtin_amdgcn_sched_barrier(0);
        dft8(v[j2], v[4 + j2], v[8 + j2], v[12 + j2], v[16 + j2], v[20 + j2], v[24 + j2],
             v[28 + j2]);
    }
    // y[j2][k1] at v[4 k1 + j2]; twiddle W32^(j2 k1) = W64^(2 j2 k1)
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1)
#pragma unroll
        for (int j2 = 1; j2 < 4; ++j2) v[4 * k1 + j2] = twiddle64(v[4 * k1 + j2], 2 * j2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
        __builtin_amdgcn_sched_barrier(0);
        dft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // X[k1 + 8 k2] at v[4 k1 + k2]
}

enum { kSrcMemory = 0, kSrcRender = 1 };
// which bins a frame stores: all k <= 4096 (K = 4097), K = 8192 with the
// mirrored upper half (reference layout, dsp.cpp:65), or any K < 4097
enum { kKHalf = 0, kKMirror = 1, kKPartial = 2 };

__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
    // Blocks b, b+8, b+16 ... are dealt to one XCD; give them consecutive
    // logical indices (bijective for any nwg; speed only, never correctness).
    const uint32_t xcd = bid & 7u, q = nwg >> 3, r = nwg & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace dspb
