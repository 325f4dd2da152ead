// fft_soa.hpp -- scalar (structure-of-arrays) complex FFT building blocks.
// Complex values are two scalar registers; -i, conjugation and negation are
// free (renames / source modifiers).  Used by the kernels built with
// -fno-slp-vectorize (stft_soa.hip, stft_pair_soa.hip).
#pragma once
#include "fft_device.hpp"

namespace dspb {

struct cx {
    float r, i;
};
__device__ __forceinline__ cx operator+(cx a, cx b) { return cx{a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cx operator-(cx a, cx b) { return cx{a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cx mulc(cx a, float c, float s) {  // a * (c + i s)
    return cx{__builtin_fmaf(a.r, c, -a.i * s), __builtin_fmaf(a.r, s, a.i * c)};
}
__device__ __forceinline__ cx mulc(cx a, cx w) { return mulc(a, w.r, w.i); }
__device__ __forceinline__ cx negi(cx a) { return cx{a.i, -a.r}; }  // -i a

__device__ __forceinline__ void sdft4(cx &a, cx &b, cx &c, cx &d) {
    const cx t0 = a + c, t1 = a - c, t2 = b + d, t3 = negi(b - d);
    a = t0 + t2;
    c = t0 - t2;
    b = t1 + t3;
    d = t1 - t3;
}

__device__ __forceinline__ void sdft8(cx &u0, cx &u1, cx &u2, cx &u3, cx &u4, cx &u5, cx &u6,
                                      cx &u7) {
    cx e0 = u0, e1 = u2, e2 = u4, e3 = u6;
    cx o0 = u1, o1 = u3, o2 = u5, o3 = u7;
    sdft4(e0, e1, e2, e3);
    sdft4(o0, o1, o2, o3);
    const float r = 0x1.6a09e6p-1f;
    const cx w1 = cx{(o1.r + o1.i) * r, (o1.i - o1.r) * r};
    const cx w2 = negi(o2);
    const cx w3 = cx{(o3.i - o3.r) * r, -(o3.r + o3.i) * r};
    u0 = e0 + o0; u4 = e0 - o0;
    u1 = e1 + w1; u5 = e1 - w1;
    u2 = e2 + w2; u6 = e2 - w2;
    u3 = e3 + w3; u7 = e3 - w3;
}

__device__ __forceinline__ cx stw64(cx a, int m) {  // a * W64^m, m compile-time
    if (m == 0) return a;
    if (m == 16) return negi(a);
    if (m == 32) return cx{-a.r, -a.i};
    if (m == 48) return cx{-a.i, a.r};
    return mulc(a, kW64_re[m], kW64_im[m]);
}

// 64-point DFT, natural order in, X[k] at v[perm64(k)] out (8 x 8).
// BAR: pin one DFT8 at a time (bounds register pressure, costs ILP).
template <bool BAR = true>
__device__ __forceinline__ void sdft64(cx (&v)[64]) {
#pragma unroll
    for (int b2 = 0; b2 < 8; ++b2) {
        if (BAR) __builtin_amdgcn_sched_barrier(0);
        sdft8(v[b2], v[8 + b2], v[16 + b2], v[24 + b2], v[32 + b2], v[40 + b2], v[48 + b2],
              v[56 + b2]);
    }
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1)
#pragma unroll
        for (int b2 = 1; b2 < 8; ++b2) v[8 * k1 + b2] = stw64(v[8 * k1 + b2], b2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
        if (BAR) __builtin_amdgcn_sched_barrier(0);
        sdft8(v[8 * k1], v[8 * k1 + 1], v[8 * k1 + 2], v[8 * k1 + 3], v[8 * k1 + 4],
              v[8 * k1 + 5], v[8 * k1 + 6], v[8 * k1 + 7]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// 32-point DFT, natural order in, X[k] at v[perm32(k)] out (8 x 4).
__device__ __forceinline__ void sdft32(cx (&v)[32]) {
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) {
        __builtin_amdgcn_sched_barrier(0);
        sdft8(v[j2], v[4 + j2], v[8 + j2], v[12 + j2], v[16 + j2], v[20 + j2], v[24 + j2],
              v[28 + j2]);
    }
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1)
#pragma unroll
        for (int j2 = 1; j2 < 4; ++j2) v[4 * k1 + j2] = stw64(v[4 * k1 + j2], 2 * j2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
        __builtin_amdgcn_sched_barrier(0);
        sdft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

}  // namespace dspb
