// fft_x2.hpp -- FFT building blocks on TWO FRAMES AT ONCE.
//
// A cx2 holds the same complex element of two different frames:
//   r = (Re frame0, Re frame1), i = (Im frame0, Im frame1)
// so every complex operation is a pair of v_pk_*_f32 instructions that do
// useful work in both halves, and -i / conjugation / negation are register
// renames plus neg modifiers -- no v_mov / v_xor to re-pair halves.  On
// CDNA4 a wave issues about one VALU instruction per 4 cycles packed or not
// (PMC-measured), so this halves the issue cost of the transform.
#pragma once
#include "fft_device.hpp"

namespace dspb {

struct cx2 {
    v2f r, i;
};
__device__ __forceinline__ cx2 operator+(cx2 a, cx2 b) { return cx2{a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cx2 operator-(cx2 a, cx2 b) { return cx2{a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cx2 negi(cx2 a) { return cx2{a.i, -a.r}; }  // -i a
// a * (c + i s), c and s the same for both frames
__device__ __forceinline__ cx2 mulc2(cx2 a, float c, float s) {
    return cx2{a.r * c - a.i * s, a.r * s + a.i * c};
}

__device__ __forceinline__ void x2dft4(cx2 &a, cx2 &b, cx2 &c, cx2 &d) {
    const cx2 t0 = a + c, t1 = a - c, t2 = b + d, t3 = negi(b - d);
    a = t0 + t2;
    c = t0 - t2;
    b = t1 + t3;
    d = t1 - t3;
}

// PRE4: the two DFT4s (evens u0 u2 u4 u6, odds u1 u3 u5 u7, in place) are
// done already (the windowed periodic frames: stft_pk.hpp x2dft4_win)
template <bool PRE4 = false>
__device__ __forceinline__ void x2dft8(cx2 &u0, cx2 &u1, cx2 &u2, cx2 &u3, cx2 &u4, cx2 &u5,
                                       cx2 &u6, cx2 &u7) {
    cx2 e0 = u0, e1 = u2, e2 = u4, e3 = u6;
    cx2 o0 = u1, o1 = u3, o2 = u5, o3 = u7;
    if constexpr (!PRE4) {
        x2dft4(e0, e1, e2, e3);
        x2dft4(o0, o1, o2, o3);
    }
    const float r = 0x1.6a09e6p-1f;
    const cx2 w1 = cx2{(o1.r + o1.i) * r, (o1.i - o1.r) * r};
    const cx2 w2 = negi(o2);
    const cx2 w3 = cx2{(o3.i - o3.r) * r, -((o3.r + o3.i) * r)};
    u0 = e0 + o0; u4 = e0 - o0;
    u1 = e1 + w1; u5 = e1 - w1;
    u2 = e2 + w2; u6 = e2 - w2;
    u3 = e3 + w3; u7 = e3 - w3;
}

__device__ __forceinline__ cx2 x2tw64(cx2 a, int m) {  // a * W64^m, m compile-time
    if (m == 0) return a;
    if (m == 16) return negi(a);
    if (m == 32) return cx2{-a.r, -a.i};
    if (m == 48) return cx2{-a.i, a.r};
    return mulc2(a, kW64_re[m], kW64_im[m]);
}

// (a + W64^M x, a - W64^M x) with W64^M factored as c (1 + i tan) or
// s (cot + i) (twiddles.inc kW64_lf_*): two FMAs for x times the unit-free
// factor, four for the butterfly with the scale folded in -- 6 instructions
// instead of a complex multiply (4) and the add/sub (4).  M % 16 == 0: adds.
template <int M>
__device__ __forceinline__ void x2bfly(cx2 &a, cx2 &x) {
    constexpr int m = M & 63;
    if constexpr (m % 16 == 0) {
        cx2 t = x;
        if constexpr (m == 16) t = negi(x);
        if constexpr (m == 32) t = cx2{-x.r, -x.i};
        if constexpr (m == 48) t = cx2{-x.i, x.r};
        const cx2 s = a;
        a = s + t;
        x = s - t;
    } else {
        const float f = kW64_lf_f[m], c = kW64_lf_s[m];
        v2f ur, ui;
        if constexpr ((m + 8) % 32 <= 16) {  // W = c (1 + i tan)
            ur = x.r - v2f{f, f} * x.i;
            ui = x.i + v2f{f, f} * x.r;
        } else {  // W = s (cot + i)
            ur = v2f{f, f} * x.r - x.i;
            ui = v2f{f, f} * x.i + x.r;
        }
        const v2f cc = v2f{c, c};
        const cx2 s = a;
        a = cx2{s.r + cc * ur, s.i + cc * ui};
        x = cx2{s.r - cc * ur, s.i - cc * ui};
    }
}

// DFT4 of (a, W^{2K} b, W^{4K} c, W^{6K} d), W = W64, as four factored
// butterflies: (t0, t1) = a +- W^{4K} c, (h2, h3) = b +- W^{4K} d, then
// X0/X2 = t0 +- W^{2K} h2, X1/X3 = t1 +- W^{2K+16} h3 (W^16 = -i).
// 24 instructions for K with nontrivial twiddles instead of 28.
template <int K>
__device__ __forceinline__ void x2dft4_tw(cx2 &a, cx2 &b, cx2 &c, cx2 &d) {
    x2bfly<4 * K>(a, c);
    x2bfly<4 * K>(b, d);
    x2bfly<2 * K>(a, b);
    x2bfly<2 * K + 16>(c, d);
    const cx2 x1 = c, x2 = b;  // positions: a = X0, b = X1, c = X2, d = X3
    b = x1;
    c = x2;
}

template <int K1 = 0, bool BAR = true>
__device__ __forceinline__ void x2dft32_stage2(cx2 (&v)[32]) {
    if constexpr (K1 < 8) {
        if (BAR) __builtin_amdgcn_sched_barrier(0);
        x2dft4_tw<K1>(v[4 * K1], v[4 * K1 + 1], v[4 * K1 + 2], v[4 * K1 + 3]);
        x2dft32_stage2<K1 + 1, BAR>(v);
    }
}

// 32-point DFT, natural order in, X[k] at v[perm32(k)] out (8 x 4).
// BAR: pin one DFT8 / DFT4 at a time (bounds register pressure, costs ILP).
// PRE4: the DFT8s' first DFT4s are done (x2dft8<true>).
template <bool BAR = true, bool PRE4 = false>
__device__ __forceinline__ void x2dft32(cx2 (&v)[32]) {
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) {
        if (BAR) __builtin_amdgcn_sched_barrier(0);
        x2dft8<PRE4>(v[j2], v[4 + j2], v[8 + j2], v[12 + j2], v[16 + j2], v[20 + j2], v[24 + j2],
                     v[28 + j2]);
    }
    x2dft32_stage2<0, BAR>(v);
    __builtin_amdgcn_sched_barrier(0);
}

}  // namespace dspb
