// fir_fft.hip -- FIR render by FFT overlap-save, one wavefront per
// 8192-sample frame (cfg 3b at the HBM roof instead of the FP32 roof).
//
// Frame f covers input samples [f H - 1024, f H + 7168), H = 7168; its
// circular convolution with the taps (T <= 1025) equals the linear one at
// frame positions n >= 1024, so it owns outputs [f H, (f + 1) H).  Per frame:
//
//   forward   the 8192-point real FFT of stft_pk.hip (packed 4096-point
//             complex FFT + paired real split): X1 = 2 X[k], X2 = conj 2 X[M-k]
//   multiply  Y = X * H, H = FFT(taps zero-padded) / 16384 (the inverse's
//             1/4096, the two real-split halvings; a power of two: exact)
//   inverse   the split run backwards on the same lane pairs --
//             Z'[k] = E + i O, Z'[M-k] = conj E + i conj O with
//             E = Y[k] + conj Y[M-k], O = (Y[k] - conj Y[M-k]) W8192^-k --
//             the M-k half sent back to its owner lane with ds_bpermute,
//             then the packed 4096-point inverse (fft4096_pk<true>)
//   store     y[2m] = Re z'[m], y[2m+1] = Im z'[m] for m >= 512 (non-temporal:
//             the render is written once)
//
// tools/olsave_model.py is the numpy model of exactly this index math.
#include "fft_pk.hpp"

namespace dspb {

constexpr uint32_t kOlsHop = 7168;    // outputs per frame
constexpr uint32_t kOlsHist = 1024;   // history samples per frame (T - 1 <= 1024)

// twiddles for the 4096-point passes; `salt` is an opaque zero so that the
// second load (for the inverse) is not merged with the first and the
// compiler does not keep 30 VGPRs of twiddles live across the whole frame
__device__ __forceinline__ void load_stage_tw(const v2f *tw, uint32_t lane, uint32_t salt, cx (&tlo)[8],
                                              cx2 (&thp)[4]) {
    const v2f *t = tw + salt;
#pragma unroll
    for (int j = 1; j < 8; ++j) {
        const v2f a = (t + 8192u + 64u * (uint32_t)(j - 1))[lane];
        tlo[j] = cx{a.x, a.y};
    }
    const float4 *tp4 = reinterpret_cast<const float4 *>(t + 8192u + 896u);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const float4 q = tp4[64u * (uint32_t)h + lane];
        thp[h] = cx2{v2f{q.x, q.y}, v2f{q.z, q.w}};
    }
}

// EDGE: frames that reach before sample 0 or past L (bounds-checked loads);
// interior frames run the EDGE = false instantiation
// hs: the block's LDS copy of H, [2 ka + h][lane] float4 (kernel prologue)
template <bool EDGE>
__device__ __forceinline__ void fir_fft_frame(const FirFftArgs &A, uint64_t f, uint32_t ch, float *lds,
                                              const float4 *hs, uint32_t lane) {
    const int64_t fs = (int64_t)(f * kOlsHop) - (int64_t)kOlsHist;  // even
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    cx tlo[8];
    cx2 thp[4];
    load_stage_tw(A.tw, lane, 0u, tlo, thp);

    // ---- frame: v[b] = (x[fs + 2l + 128b], x[fs + 2l + 128b + 1]), zero outside [0, L)
    cx2 P[32];
    {
        cx v[64];
        if constexpr (!EDGE) {
            if (x != nullptr) {
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const v2f t = reinterpret_cast<const v2f *>(x + fs + 128 * b)[lane];
                    v[b] = cx{t.x, t.y};
                }
            } else {  // a channel the file does not have: silence
#pragma unroll
                for (int b = 0; b < 64; ++b) v[b] = cx{0.f, 0.f};
            }
        } else {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const int64_t s = fs + 2 * (int64_t)lane + 128 * b;
                v[b] = cx{(x && s >= 0 && (uint64_t)s < A.L) ? x[s] : 0.f,
                          (x && s + 1 >= 0 && (uint64_t)(s + 1) < A.L) ? x[s + 1] : 0.f};
            }
        }
#pragma unroll
        for (int j = 0; j < 32; ++j)
            P[j] = cx2{v2f{v[2 * j].r, v[2 * j + 1].r}, v2f{v[2 * j].i, v[2 * j + 1].i}};
    }

    cx zp[32], zm[32];
    fft4096_pk<false, false, false, true>(P, lds, tlo, thp, lane, zp, zm);

    // ---- split, H multiply, inverse split, paired over (ka, ka + 16) --------
    const uint32_t src = ((64u - lane) & 63u) * 4u;
    const bool l0 = lane == 0;
    const v2f wl2 = A.tw[lane];  // W8192^l
    const cx wl = cx{wl2.x, wl2.y};
    // own Z'[l + 64 ka] (ka < 32) and, received from lane 64 - l, Z'[l + 64 ka']
    // (ka' = 32 + q): lane 64 - l computes it as its Z'[M - k] at ka = 31 - q
    // and it is sent in the same iteration; lane 0 (which pairs with itself,
    // shifted by one register) is fixed up after the loop
    cx zk[32], zr[32];
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) {
        const cx a0 = ka == 0 ? zp[0] : zm[32 - ka], b0 = zm[31 - ka];
        const cx a1 = zm[16 - ka], b1 = zm[15 - ka];
        const cx s0 = cx{l0 ? a0.r : b0.r, l0 ? a0.i : b0.i};
        const cx s1 = cx{l0 ? a1.r : b1.r, l0 ? a1.i : b1.i};
        const cx2 Pp = cx2{v2f{bperm(src, s0.r), bperm(src, s1.r)}, v2f{bperm(src, s0.i), bperm(src, s1.i)}};
        const cx2 Z = cx2{v2f{zp[ka].r, zp[ka + 16].r}, v2f{zp[ka].i, zp[ka + 16].i}};
        const cx2 E = cx2{Z.r + Pp.r, Z.i - Pp.i};
        const cx2 D = cx2{Z.r - Pp.r, Z.i + Pp.i};
        const cx2 tw = cmulb(wl, cx2{v2f{kW128_re[ka], kW128_re[ka + 16]}, v2f{kW128_im[ka], kW128_im[ka + 16]}});
        const cx2 T = cmul2(negi(D), tw);
        const cx2 X1 = E + T;  // 2 X[k]
        const cx2 X2 = E - T;  // conj 2 X[M - k]
        const float4 ha = hs[(2u * ka) * 64u + lane], hb = hs[(2u * ka + 1u) * 64u + lane];
        const cx2 Hk = cx2{v2f{ha.x, ha.y}, v2f{ha.z, ha.w}};
        const cx2 HMk = cx2{v2f{hb.x, hb.y}, v2f{hb.z, hb.w}};
        const cx2 Yk = cmul2(X1, Hk);
        const cx2 YMk = cmul2(cx2{X2.r, -X2.i}, HMk);
        const cx2 E2 = cx2{Yk.r + YMk.r, Yk.i - YMk.i};                           // Y[k] + conj Y[M-k]
        const cx2 O2 = cmul2(cx2{Yk.r - YMk.r, Yk.i + YMk.i}, cx2{tw.r, -tw.i});  // (..) W^-k
        const cx2 Zk = cx2{E2.r - O2.i, E2.i + O2.r};                            // E + i O
        const cx2 ZMk = cx2{E2.r + O2.i, O2.r - E2.i};                           // conj E + i conj O
        zk[ka] = cx{Zk.r.x, Zk.i.x};
        zk[ka + 16] = cx{Zk.r.y, Zk.i.y};
        zr[31 - ka] = cx{bperm(src, ZMk.r.x), bperm(src, ZMk.i.x)};
        zr[15 - ka] = cx{bperm(src, ZMk.r.y), bperm(src, ZMk.i.y)};
    }
    // lane 0 received its own Z'[M - k] of ka = 31 - q at q; it needs the one of
    // ka = 32 - q, i.e. what landed at q - 1, and at q = 0 the self-paired
    // bin k = 2048: Z[2048] = zm[0], 2 X[2048] = 2 conj Z, Z'[2048] = 2 conj Y
    {
        const cx Z = zm[0];
        const cx Y = mulc(cx{2.f * Z.r, -2.f * Z.i}, A.h2048.x, A.h2048.y);
#pragma unroll
        for (int q = 31; q >= 1; --q) zr[q] = cx{l0 ? zr[q - 1].r : zr[q].r, l0 ? zr[q - 1].i : zr[q].i};
        zr[0] = cx{l0 ? 2.f * Y.r : zr[0].r, l0 ? -2.f * Y.i : zr[0].i};
    }

    // ---- inverse 4096-point FFT over the register index ka -------------------
    cx2 Q[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const cx u0 = 2 * j < 32 ? zk[2 * j] : zr[2 * j - 32];
        const cx u1 = 2 * j + 1 < 32 ? zk[2 * j + 1] : zr[2 * j + 1 - 32];
        Q[j] = cx2{v2f{u0.r, u1.r}, v2f{u0.i, u1.i}};
    }
    cx yp[32], ym[32];
    {
        uint32_t salt = 0u;
        asm volatile("" : "+s"(salt));
        load_stage_tw(A.tw, lane, salt, tlo, thp);
    }
    fft4096_pk<true, false, false, true>(Q, lds, tlo, thp, lane, yp, ym);

    // ---- outputs: m = l + 64 b, b >= 8 -> y[f H + 2l + 128 (b - 8)] ----------
    float *o = A.out.p[ch];
    const uint64_t ob = f * kOlsHop + 2u * lane;
    if (f * kOlsHop + kOlsHop <= A.Ly) {
#pragma unroll
        for (int b = 8; b < 64; ++b) {
            const cx z = b < 32 ? yp[b] : ym[b - 32];
            __builtin_nontemporal_store(v2f{z.r, z.i}, reinterpret_cast<v2f *>(o + ob + 128u * (uint32_t)(b - 8)));
        }
    } else {
#pragma unroll
        for (int b = 8; b < 64; ++b) {
            const cx z = b < 32 ? yp[b] : ym[b - 32];
            const uint64_t i = ob + 128u * (uint32_t)(b - 8);
            if (i < A.Ly) o[i] = z.r;
            if (i + 1 < A.Ly) o[i + 1] = z.i;
        }
    }
}

// one launch for all frames: a wave takes the bounds-checked path only for
// frame 0 and the frames at or past fe (a wave-uniform branch), so the few
// edge frames overlap the interior ones instead of running as serial
// single-wave launches
// LDS per block: four 64 x 33 transpose tiles (transpose_pl) and the
// filter's spectrum H (32 KB), staged once per block -- the split reads H
// from LDS instead of waiting on L2 -- 66.5 KB, as with 64 x 65 tiles alone.
__global__ __launch_bounds__(256, 2) void fir_fft_kernel(FirFftArgs A, uint64_t fe) {
    __shared__ __attribute__((aligned(16))) float lds_all[4][64 * 33];
    __shared__ float4 hs[2048];
    {  // global H: [ka][lane][h] float4 -> LDS [2 ka + h][lane]
        const float4 *H4 = reinterpret_cast<const float4 *>(A.H);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t g = threadIdx.x + 256u * (uint32_t)i;
            const uint32_t ka = g >> 7, ln = (g & 127u) >> 1, h = g & 1u;
            hs[(2u * ka + h) * 64u + ln] = H4[g];
        }
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ch = blockIdx.y;
    const uint64_t f = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (f >= A.F) return;
    if (f == 0 || f >= fe) fir_fft_frame<true>(A, f, ch, lds_all[wave], hs, lane);
    else fir_fft_frame<false>(A, f, ch, lds_all[wave], hs, lane);
}

// interior frames: [1, fe) with (f H - 1024) + 8192 <= L; the rest is edge
static uint64_t interior_end(const FirFftArgs &A) {
    uint64_t fe = 1;
    if (A.L + kOlsHist >= 8192u && A.in_ch > 0) fe = (A.L + kOlsHist - 8192u) / kOlsHop + 1;
    if (fe > A.F) fe = A.F;
    if (fe < 1) fe = 1;
    return fe;
}

// ---------------------------------------------------------------------------
// Two channels per frame (fir_pair_kernel).  The taps are real, so the
// convolution of u = x0 + i x1 is conv(x0, h) + i conv(x1, h): one complex
// 4096-point frame carries a channel pair, no real split (no partner
// exchange) in either direction.  Frame f covers input [f P - 1024,
// f P + 3072), P = kPairHop = 3072, and owns outputs [f P, (f + 1) P):
//
//   load      u[l + 64 r] (lane l, register r) = x0[s] + i x1[s],
//             s = f P - 1024 + l + 64 r, zero outside [0, L) and for a
//             channel the file lacks; P[j] = (u[2j], u[2j+1])
//   forward   the packed 4096-point FFT with its packed last combine:
//             (Z[l + 64 q], Z[l + 64 (q + 32)]) in one cx2
//   multiply  by (H[l + 64 q], H[l + 64 (q + 32)]), H = FFT_4096(taps) /
//             4096 (the inverse's scale, a power of 2), then re-paired
//             (v_pk_mov_b32) as the inverse's input pairs (Z'[2j], Z'[2j+1])
//   inverse   the same transform, conjugated twiddles: y[l + 64 q]
//   store     out0[f P + l + 64 (q - 16)] = Re y, out1[..] = Im y, q >= 16
//
// Per output sample: two 4096-point transforms per 6144 outputs instead of
// two 4096-point transforms plus the split per 7168 (fir_fft_kernel): 3,100
// VALU per frame against 4,050 (PMC), 7.5% faster on cfg 3b
// (profiles/r03_fir_pair_ab.txt).  An odd last channel keeps fir_fft_kernel.
template <bool EDGE>
__device__ __forceinline__ void fir_pair_frame(const FirFftArgs &A, uint64_t f, uint32_t c0, float *lds,
                                               const float4 *hs, uint32_t lane) {
    const int64_t fs = (int64_t)(f * kPairHop) - (int64_t)kOlsHist;
    const float *x0 = c0 < A.in_ch ? A.in.p[c0] : nullptr;
    const float *x1 = c0 + 1 < A.in_ch ? A.in.p[c0 + 1] : nullptr;

    cx tlo[8];
    cx2 thp[4];
    load_stage_tw(A.tw, lane, 0u, tlo, thp);

    cx2 P[32];
    if constexpr (!EDGE) {
        // interior: both channels present (the launch sends pairs with a
        // missing channel down the EDGE path)
        // wave-uniform bases, 32-bit lane offsets (the global saddr form)
        const float *b0 = x0 + fs, *b1 = x1 + fs;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t o = lane + 128u * (uint32_t)j;
            P[j] = cx2{v2f{b0[o], b0[o + 64u]}, v2f{b1[o], b1[o + 64u]}};
        }
    } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int64_t s0 = fs + (int64_t)lane + 128 * j, s1 = s0 + 64;
            const bool in0 = s0 >= 0 && (uint64_t)s0 < A.L, in1 = s1 >= 0 && (uint64_t)s1 < A.L;
            P[j] = cx2{v2f{(x0 && in0) ? x0[s0] : 0.f, (x0 && in1) ? x0[s1] : 0.f},
                       v2f{(x1 && in0) ? x1[s0] : 0.f, (x1 && in1) ? x1[s1] : 0.f}};
        }
    }

    // forward, packed last combine: Y2[q] = (Z[l + 64 q], Z[l + 64 (q + 32)]);
    // times H in the same pairing (hs[q][lane]); re-paired as the inverse's
    // input Q[j] = (Z'[l + 64 (2j)], Z'[l + 64 (2j + 1)])
    cx2 Q[32];
    {
        cx2 R[32], Y2[32];
        fft4096_pk_front<false, false, false, true>(P, lds, tlo, thp, lane, R);
        combine64p(R, Y2);
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const float4 h = hs[64u * (uint32_t)q + lane];
            Y2[q] = cmul2(Y2[q], cx2{v2f{h.x, h.y}, v2f{h.z, h.w}});
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int r0 = 2 * j, r1 = 2 * j + 1;  // Z'[l + 64 r] = r < 32 ? Y2[r].x : Y2[r - 32].y
            const cx2 a = Y2[r0 & 31], b = Y2[r1 & 31];
            // one v_pk_mov_b32 per part: (a.lo, b.lo) or (a.hi, b.hi)
            if (r0 < 32) {
                asm("v_pk_mov_b32 %0, %1, %2 op_sel:[0,0]" : "=v"(Q[j].r) : "v"(a.r), "v"(b.r));
                asm("v_pk_mov_b32 %0, %1, %2 op_sel:[0,0]" : "=v"(Q[j].i) : "v"(a.i), "v"(b.i));
            } else {
                asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,1]" : "=v"(Q[j].r) : "v"(a.r), "v"(b.r));
                asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,1]" : "=v"(Q[j].i) : "v"(a.i), "v"(b.i));
            }
        }
    }

    {
        uint32_t salt = 0u;
        asm volatile("" : "+s"(salt));
        load_stage_tw(A.tw, lane, salt, tlo, thp);
    }
    // inverse, packed last combine: y[l + 64 q] = q < 32 ? yp[q] : ym[q - 32]
    cx yp[32], ym[32];
    {
        cx2 R[32], Y2[32];
        fft4096_pk_front<true, false, false, true>(Q, lds, tlo, thp, lane, R);
        combine64p_dir<true>(R, Y2);
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            yp[q] = cx{Y2[q].r.x, Y2[q].i.x};
            ym[q] = cx{Y2[q].r.y, Y2[q].i.y};
        }
    }

    // a channel the file lacks renders exact zeros (its imaginary part holds
    // the rounding of the other channel's transform, not silence)
    const uint32_t c1 = c0 + 1;
    const bool two = c1 < A.nout;  // (wave-uniform)
    // the lane index through an opaque copy: the stores' offsets are formed
    // here, not hoisted to the kernel's start and held across the frame (250 -> 214 VGPRs)
    asm volatile("" : "+v"(lane));
    float *o0 = A.out.p[c0] + f * kPairHop;
    float *o1 = two ? A.out.p[c1] + f * kPairHop : o0;
    if (f * kPairHop + kPairHop <= A.Ly) {
        if (two && x1) {
#pragma unroll
            for (int q = 16; q < 64; ++q) {
                const cx z = q < 32 ? yp[q] : ym[q - 32];
                const uint32_t o = lane + 64u * (uint32_t)(q - 16);
                __builtin_nontemporal_store(z.r, o0 + o);
                __builtin_nontemporal_store(z.i, o1 + o);
            }
        } else {
#pragma unroll
            for (int q = 16; q < 64; ++q) {
                const cx z = q < 32 ? yp[q] : ym[q - 32];
                const uint32_t o = lane + 64u * (uint32_t)(q - 16);
                __builtin_nontemporal_store(z.r, o0 + o);
                if (two) __builtin_nontemporal_store(0.f, o1 + o);
            }
        }
    } else {
        const uint64_t n = A.Ly - f * kPairHop;
#pragma unroll
        for (int q = 16; q < 64; ++q) {
            const cx z = q < 32 ? yp[q] : ym[q - 32];
            const uint32_t o = lane + 64u * (uint32_t)(q - 16);
            if (o < n) {
                o0[o] = z.r;
                if (two) o1[o] = x1 ? z.i : 0.f;
            }
        }
    }
}

// grid (frame groups of 4, channel pairs); LDS: four 64 x 33 tiles and H
// (32 KB), as fir_fft_kernel
__global__ __launch_bounds__(256, 2) void fir_pair_kernel(FirFftArgs A, uint64_t fe) {
    __shared__ __attribute__((aligned(16))) float lds_all[4][64 * 33];
    __shared__ float4 hs[2048];
    {
        const float4 *H4 = reinterpret_cast<const float4 *>(A.H);
#pragma unroll
        for (int i = 0; i < 8; ++i) hs[threadIdx.x + 256u * (uint32_t)i] = H4[threadIdx.x + 256u * (uint32_t)i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t c0 = 2u * blockIdx.y;
    const uint64_t f = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (f >= A.F) return;
    if (f == 0 || f >= fe || c0 + 1 >= A.in_ch) fir_pair_frame<true>(A, f, c0, lds_all[wave], hs, lane);
    else fir_pair_frame<false>(A, f, c0, lds_all[wave], hs, lane);
}

int launch_fir_pair(const FirFftArgs &A, uint32_t C, hipStream_t s) {
    if (A.F == 0 || C == 0) return DSP_OK;
    // interior frames: [1, fe) with (f P - 1024) + 4096 <= L
    uint64_t fe = 1;
    if (A.L >= kPairHop) fe = (A.L - kPairHop) / kPairHop + 1;
    if (fe > A.F) fe = A.F;
    if (fe < 1) fe = 1;
    const uint64_t groups = (A.F + 3) / 4;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    FirFftArgs B = A;
    B.nout = C;
    hipLaunchKernelGGL(fir_pair_kernel, dim3((uint32_t)groups, (C + 1) / 2), dim3(256), 0, s, B, fe);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_fir_fft(const FirFftArgs &A, uint32_t C, hipStream_t s) {
    if (A.F == 0 || C == 0) return DSP_OK;
    const uint64_t fe = interior_end(A);
    const uint64_t groups = (A.F + 3) / 4;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    hipLaunchKernelGGL(fir_fft_kernel, dim3((uint32_t)groups, C), dim3(256), 0, s, A, fe);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
