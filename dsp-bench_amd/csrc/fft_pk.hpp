// fft_pk.hpp -- packed (two independent sub-transforms per VGPR pair)
// 4096-point complex FFT for one wavefront, forward or inverse, as used by
// the 8192-point real STFT (stft_pk.hip) and the overlap-save FIR
// (fir_fft.hip).  See stft_pk.hip for the derivation of the layout.
#pragma once
#include "fft_soa.hpp"
#include "fft_x2.hpp"

namespace dspb {

// both halves: a * w
__device__ __forceinline__ cx2 cmul2(cx2 a, cx2 w) {
    return cx2{a.r * w.r - a.i * w.i, a.r * w.i + a.i * w.r};
}
// (c + i s) broadcast times both halves of w
__device__ __forceinline__ cx2 cmulb(cx c, cx2 w) {
    return cx2{c.r * w.r - c.i * w.i, c.r * w.i + c.i * w.r};
}

// radix-2 DIT combine of a transformed pair: halves (E[k], O[k]) at
// a[perm32(k)] -> (Y[k], Y[k+32]) as scalars
__device__ __forceinline__ void combine64(const cx2 (&a)[32], cx (&yp)[32], cx (&ym)[32]) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const cx2 p = a[perm32(k)];
        const cx e = cx{p.r.x, p.i.x};
        const cx t = stw64(cx{p.r.y, p.i.y}, k);
        yp[k] = e + t;
        ym[k] = e - t;
    }
}

// the same combine, packed: y[k] = (Y[k], Y[k+32]) as one cx2.  W64^K is
// factored as c (1 + i tan) or s (cot + i) (kW64_lf_*, |tan|, |cot| <= 1):
// the odd half times the unit-free factor is two scalar FMAs, and the scale
// rides in the butterfly, one v_pk_fma per part: (e, e) + (u, u) * (c, -c).
// 4 instructions per nontrivial K instead of 6 (a full complex multiply
// before the butterfly).
template <int K>
__device__ __forceinline__ cx2 combine1(cx2 p) {
    v2f tr, ti;  // (u, u), splats of one scalar
    v2f pm = v2f{1.f, -1.f};
    if constexpr (K == 0) {
        tr = v2f{p.r.y, p.r.y};
        ti = v2f{p.i.y, p.i.y};
    } else if constexpr (K == 16) {  // t = -i O = (O.i, -O.r)
        tr = v2f{p.i.y, p.i.y};
        ti = -v2f{p.r.y, p.r.y};
    } else {
        const float f = kW64_lf_f[K];
        const float orr = p.r.y, oi = p.i.y;
        float ur, ui;
        if constexpr ((K + 8) % 32 <= 16) {  // W = c (1 + i tan)
            ur = __builtin_fmaf(-f, oi, orr);
            ui = __builtin_fmaf(f, orr, oi);
        } else {  // W = s (cot + i)
            ur = __builtin_fmaf(f, orr, -oi);
            ui = __builtin_fmaf(f, oi, orr);
        }
        tr = v2f{ur, ur};
        ti = v2f{ui, ui};
        pm = v2f{kW64_lf_s[K], -kW64_lf_s[K]};
    }
    return cx2{tr * pm + v2f{p.r.x, p.r.x}, ti * pm + v2f{p.i.x, p.i.x}};
}
template <int K = 0>
__device__ __forceinline__ void combine64p(const cx2 (&a)[32], cx2 (&y)[32]) {
    if constexpr (K < 32) {
        y[K] = combine1<K>(a[perm32(K)]);
        combine64p<K + 1>(a, y);
    }
}

template <bool INV>
__device__ __forceinline__ cx2 conj2(cx2 a) {
    if constexpr (INV) return cx2{a.r, -a.i};
    return a;
}
template <bool INV>
__device__ __forceinline__ cx conj1(cx a) {
    if constexpr (INV) return cx{a.r, -a.i};
    return a;
}

// DFT32 of both halves; INV: the unnormalised inverse, conj(DFT(conj(x)))
// (PRE4: forward, the first DFT4s done by the caller)
template <bool BAR, bool INV, bool PRE4 = false>
__device__ __forceinline__ void x2dft32_dir(cx2 (&v)[32]) {
    static_assert(!(INV && PRE4), "PRE4: forward only");
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = conj2<INV>(v[j]);
    x2dft32<BAR, PRE4>(v);
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = conj2<INV>(v[j]);
}

// combine of the inverse: (E, O) -> (E + W64^-k O, E - W64^-k O), through
// the same conjugation identity
template <bool INV, int K = 0>
__device__ __forceinline__ void combine64p_dir(const cx2 (&a)[32], cx2 (&y)[32]) {
    if constexpr (K < 32) {
        y[K] = conj2<INV>(combine1<K>(conj2<INV>(a[perm32(K)])));
        combine64p_dir<INV, K + 1>(a, y);
    }
}
template <bool INV>
__device__ __forceinline__ void combine64_dir(const cx2 (&a)[32], cx (&yp)[32], cx (&ym)[32]) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const cx2 p = conj2<INV>(a[perm32(k)]);
        const cx e = cx{p.r.x, p.i.x};
        const cx t = stw64(cx{p.r.y, p.i.y}, k);
        yp[k] = conj1<INV>(e + t);
        ym[k] = conj1<INV>(e - t);
    }
}

// The transpose of fft4096_pk_front through a 64 x 33 tile (8.4 KB per wave
// instead of 16.6 KB) in four passes of 32 floats per lane:
//   pass x: every lane writes its row's columns 0..31 (the .x halves);
//           lane d reads column d & 31, rows 32 (d >= 32) + a, a < 32 -> X[a]
//   pass y: the same with columns 32..63 (.y halves) -> Y[a]
//   then v_permlane32_swap(X[a], Y[a]) trades the upper lanes' X for the
//   lower lanes' Y: every lane holds its own column, rows 0..31 in X and
//   rows 32..63 in Y (32 swaps per component, no pass holds more than the
//   frame's 128 VGPRs).
__device__ __forceinline__ void transpose_pl(const cx2 (&Q)[32], float *lds, uint32_t lane, cx2 (&R)[32]) {
    const uint32_t wrow = lane * 33u;                           // this lane's row
    const uint32_t rcol = (lane & 32u) * 33u + (lane & 31u);    // rows 32 (d >= 32) + a, column d & 31
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        float X[32], Yv[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) lds[wrow + k] = c ? Q[k].i.x : Q[k].r.x;
        lds_fence();
#pragma unroll
        for (int a = 0; a < 32; ++a) X[a] = lds[rcol + 33u * a];
        lds_fence();
#pragma unroll
        for (int k = 0; k < 32; ++k) lds[wrow + k] = c ? Q[k].i.y : Q[k].r.y;
        lds_fence();
#pragma unroll
        for (int a = 0; a < 32; ++a) Yv[a] = lds[rcol + 33u * a];
        lds_fence();
#pragma unroll
        for (int a = 0; a < 32; ++a) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(X[a]), __float_as_uint(Yv[a]), false,
                                                            false);
            X[a] = __uint_as_float(r[0]);
            Yv[a] = __uint_as_float(r[1]);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const v2f lo2 = v2f{X[2 * j], X[2 * j + 1]}, hi2 = v2f{Yv[2 * j], Yv[2 * j + 1]};
            if (c) {
                R[j].i = lo2;
                R[16 + j].i = hi2;
            } else {
                R[j].r = lo2;
                R[16 + j].r = hi2;
            }
        }
    }
}

// 4096-point complex FFT of one wavefront.  In: P[j] = (u[2j], u[2j+1]),
// u[r] = element l + 64 r of this lane l (r is the register index).  Out:
// U[l + 64 q] = zp[q] (q < 32), zm[q - 32] -- forward: Z = DFT(u), inverse
// (INV): the unnormalised inverse.  tlo[j] = W4096^(l j), thp[h] =
// (W4096^(8 l h), W4096^(8 l (h + 4))); lds = this wave's 64 x 65 tile.
// Everything up to the last combine: R holds the second DFT64's even/odd
// DFT32 halves (combine64p / combine64_dir finish it).
// PL: the transpose goes through transpose_pl's 64 x 33 tile.
// HOOK: called once the transpose's last LDS read has completed (the tile
// is free from there on; the A/B kernel stft8192_mem_pf_kernel, stft_pk_ab.hip,
// prefetches into it).
struct NoHook {
    __device__ void operator()() const {}
};
template <bool INV, bool BAR_DFT, bool BAR_TW, bool PL = false, bool AB_NOXP = false, typename HOOK = NoHook,
          bool PRE4 = false>
__device__ __forceinline__ void fft4096_pk_front(cx2 (&P)[32], float *lds, const cx (&tlo)[8], const cx2 (&thp)[4],
                                                 uint32_t lane, cx2 (&R)[32], const HOOK &hook = HOOK{}) {
    // DFT64 over the register index: even/odd DFT32 in the halves, combine
    // (PRE4: P holds the first DFT4s' outputs already)
    x2dft32_dir<BAR_DFT, INV, PRE4>(P);
    cx2 Q[32];  // Q[k] = (Y[k], Y[k+32]) * (W4096^(+-l k), W4096^(+-l (k+32)))
    {
        cx2 Y[32];
        combine64p_dir<INV>(P, Y);
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (BAR_TW) __builtin_amdgcn_sched_barrier(0);
            const int lo = k & 7, hi = k >> 3;
            const cx2 w = lo ? cmulb(tlo[lo], thp[hi]) : thp[hi];
            Q[k] = cmul2(Y[k], conj2<INV>(w));
        }
    }
    // transpose through LDS: row l, column kb -> column l, row a
    // R[j] = (t[2j], t[2j+1]), t[a] = row a of column l
    if constexpr (PL) {
        transpose_pl(Q, lds, lane, R);
        x2dft32_dir<BAR_DFT, INV>(R);
        return;
    }
    if constexpr (AB_NOXP) {  // ablation only (wrong results): the transpose's cost
#pragma unroll
        for (int j = 0; j < 32; ++j) R[j] = Q[j];
        x2dft32_dir<BAR_DFT, INV>(R);
        return;
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        lds[lane * 65u + k] = Q[k].r.x;
        lds[lane * 65u + k + 32] = Q[k].r.y;
    }
    lds_fence();
#pragma unroll
    for (int j = 0; j < 32; ++j) R[j].r = v2f{lds[(2 * j) * 65 + lane], lds[(2 * j + 1) * 65 + lane]};
    lds_fence();
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        lds[lane * 65u + k] = Q[k].i.x;
        lds[lane * 65u + k + 32] = Q[k].i.y;
    }
    lds_fence();
#pragma unroll
    for (int j = 0; j < 32; ++j) R[j].i = v2f{lds[(2 * j) * 65 + lane], lds[(2 * j + 1) * 65 + lane]};
    if constexpr (!__is_same(HOOK, NoHook)) {
        lds_fence();
        hook();
    }
    // DFT64 over the other index (its combine is the caller's)
    x2dft32_dir<BAR_DFT, INV>(R);
}

template <bool INV, bool BAR_DFT = true, bool BAR_TW = true, bool PL = false>
__device__ __forceinline__ void fft4096_pk(cx2 (&P)[32], float *lds, const cx (&tlo)[8], const cx2 (&thp)[4],
                                           uint32_t lane, cx (&zp)[32], cx (&zm)[32]) {
    cx2 R[32];
    fft4096_pk_front<INV, BAR_DFT, BAR_TW, PL>(P, lds, tlo, thp, lane, R);
    combine64_dir<INV>(R, zp, zm);
}

// The same transform with a packed last combine: Y2[q] = (U[l + 64 q],
// U[l + 64 (q + 32)]) in the halves of one cx2 (forward only) -- 6 packed
// instructions per pair instead of 8 scalar ones.
template <bool BAR_DFT = true, bool BAR_TW = true, bool AB_NOXP = false, typename HOOK = NoHook, bool PRE4 = false>
__device__ __forceinline__ void fft4096_pk_y2(cx2 (&P)[32], float *lds, const cx (&tlo)[8], const cx2 (&thp)[4],
                                              uint32_t lane, cx2 (&Y2)[32], const HOOK &hook = HOOK{}) {
    cx2 R[32];
    fft4096_pk_front<false, BAR_DFT, BAR_TW, false, AB_NOXP, HOOK, PRE4>(P, lds, tlo, thp, lane, R, hook);
    combine64p(R, Y2);
}

// Low-footprint forward transform for 3 waves per SIMD.  The stage
// twiddles are loaded after the first DFT32s (tw = get_tw's table: T8192,
// then the lane-major rows) instead of living in 30 VGPRs from the kernel's
// start, and the transpose is transpose_pl's, so 12 waves per CU fit in the
// LDS.  Output as fft4096_pk_y2.
template <bool BAR_DFT = true>
__device__ __forceinline__ void fft4096_pk_y2_lo(cx2 (&P)[32], float *lds, const v2f *tw, uint32_t lane,
                                                 cx2 (&Y2)[32]) {
    x2dft32_dir<BAR_DFT, false>(P);
    cx2 Q[32];
    {
        cx tlo[8];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            const v2f a = (tw + 8192u + 64u * (uint32_t)(j - 1))[lane];
            tlo[j] = cx{a.x, a.y};
        }
        const float4 *tp4 = reinterpret_cast<const float4 *>(tw + 8192u + 896u);
        cx2 Y[32];
        combine64p(P, Y);
#pragma unroll
        for (int hi = 0; hi < 4; ++hi) {
            const float4 t = tp4[64u * (uint32_t)hi + lane];
            const cx2 th = cx2{v2f{t.x, t.y}, v2f{t.z, t.w}};
#pragma unroll
            for (int lo = 0; lo < 8; ++lo) {
                __builtin_amdgcn_sched_barrier(0);
                const int k = lo + 8 * hi;
                const cx2 w = lo ? cmulb(tlo[lo], th) : th;
                Q[k] = cmul2(Y[k], w);
            }
        }
    }
    cx2 R[32];
    transpose_pl(Q, lds, lane, R);
    x2dft32_dir<BAR_DFT, false>(R);
    combine64p(R, Y2);
}

}  // namespace dspb
