// stft_soa.hip -- 8192-point STFT kernel, one wavefront per frame, scalar
// (structure-of-arrays) arithmetic.
//
// Same 64 x 64 four-step transform as stft8192_kernel (spectral.hip), written
// for the CDNA4 VALU as it is actually priced (PMC: ~4 cycles per VALU
// instruction, packed or not): complex values live as two scalar registers,
// so multiplying by -i, conjugating and swapping halves are register
// renames / source modifiers instead of v_mov + v_xor pairs, and the
// translation unit is built with -fno-slp-vectorize so nothing is re-packed.
//
// Further savings over the packed kernel:
//   * the window table is pre-scaled by 0.5/sqrt(N) (both the IPP
//     DIV_BY_SQRTN scale and the 1/2 of the real-input split), so no
//     per-bin scale multiply;
//   * the real-input split produces X[k] and X[M-k] from ONE (E, W^k O)
//     pair: X[k] = E + T, X[M-k] = conj(E - T) -- half the partner fetches
//     (ds_bpermute), twiddles and products; lane 0 pairs within its own
//     registers (column 0) and adds the self-paired bin k = 2048.
#include "fft_soa.hpp"
#include "frame_load.hpp"

namespace dspb {

// OPT bits (A/B-selectable, see dsp_stft_soa_options):
//   kOptNoBar      no scheduling barriers inside the DFT64 passes
//   kOptPrefetchTw stage twiddles from the lane-major table, issued first
//   kOptWinComp    window computed from per-lane base angles (no table loads)
//   kOptLdsTable   IR ramp table staged through the wave's LDS tile (pow2 B
//                  <= 4096): 2 coalesced loads per lane instead of 64 gathers
enum { kOptNoBar = 1, kOptPrefetchTw = 2, kOptWinComp = 4, kOptLdsTable = 8 };
// Phase ablation for the diagnostic build (tools/stamps.hip): skip pieces
// to price them.  DSPB_ABLATE is 0 in every shipped build.
#ifndef DSPB_ABLATE
#define DSPB_ABLATE 0
#endif
enum { kAbLoad = 1, kAbWindow = 2, kAbDft1 = 4, kAbTw = 8, kAbLds = 16, kAbDft2 = 32, kAbSplit = 64 };
// default for the A/B-switchable headline shapes (tools/ab_soa.py, MI355X:
// fused 0.73 -> 0.65 ms, memory 0.78 -> 0.71 ms per stereo hour vs 0);
// other shapes run kSoaKmOpt (no computed window: partial frames allowed)
[[maybe_unused]] constexpr int kSoaDefaultOpt = kOptPrefetchTw | kOptWinComp | kOptLdsTable;
constexpr int kSoaKmOpt = kOptLdsTable;

template <int SRC, int KM, MapKind MK, bool POW2, int OPT>
__global__ __launch_bounds__(256, 2) void stft8192_soa_kernel(Stft8kArgs A) {
    __shared__ __attribute__((aligned(16))) float lds_all[4][64 * 65];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ch = blockIdx.y;
    const uint64_t f = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (f >= A.F) return;  // whole wave leaves; nothing below waits on other waves
    float *lds = lds_all[wave];
    DSPB_STAMP(A, f, lane, 0);
    const uint64_t fs = f * (uint64_t)A.H;
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    // twiddle factors W4096^(a lo), W4096^(8 a hi) for step 3 (early: their
    // L2 latency then hides under the frame load and the first DFT)
    cx tlo[8], thi[8];
    if constexpr (OPT & kOptPrefetchTw) {
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            // lane-major copies (capi.cpp get_tw): one coalesced 512-B row each
            const v2f a = (A.tw + 8192u + 64u * (uint32_t)(j - 1))[lane];
            const v2f b = (A.tw + 8192u + 448u + 64u * (uint32_t)(j - 1))[lane];
            tlo[j] = cx{a.x, a.y};
            thi[j] = cx{b.x, b.y};
        }
    }
    float4 wbase = float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (OPT & kOptWinComp) wbase = A.wbase[lane];

    // ---- 1. load (+ fused render), window (pre-scaled by 0.5/sqrt N) ------
    cx v[64];
    if constexpr (SRC == kSrcMemory) {
        if (A.valid >= 8192u) {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const v2f t = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
                v[b] = cx{t.x, t.y};
            }
        } else {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint32_t s = 2u * lane + 128u * (uint32_t)b;
                v2f t = v2f{0.f, 0.f};
                if (s < A.valid) t = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
                v[b] = cx{t.x, t.y};
            }
        }
    } else if (DSPB_ABLATE & kAbLoad) {
#pragma unroll
        for (int b = 0; b < 64; ++b) v[b] = cx{(float)lane * 1e-3f + b, (float)b * 1e-3f - lane};
    } else {
        if constexpr ((OPT & kOptLdsTable) && MK == MapKind::Ramp && POW2) {
            if (A.map.B >= 4u && A.map.B <= 4096u) {
                lds_table_frame(A, lds, fs, lane, v);
            } else {
                s_render_frame<MK, POW2>(A, x, fs, lane, v);
            }
        } else {
            s_render_frame<MK, POW2>(A, x, fs, lane, v);
        }
        float *o = A.out.p[ch] + fs;
#pragma unroll
        for (int b = 0; b < 64; ++b)
            if (128u * (uint32_t)b < A.H)
                reinterpret_cast<v2f *>(o + 128u * (uint32_t)b)[lane] = v2f{v[b].r, v[b].i};
    }
    if constexpr (DSPB_ABLATE & kAbWindow) {
    } else if constexpr (OPT & kOptWinComp) {
        // w(n) = wa - wb cos(theta n), n = 2 lane + e + 128 b:
        // cos(alpha_e + beta_b) = C_e cos(beta_b) - S_e sin(beta_b)
#pragma unroll
        for (int b = 0; b < 64; ++b) {
            const float t0 = __builtin_fmaf(wbase.x, kWinB_c[b], -wbase.y * kWinB_s[b]);
            const float t1 = __builtin_fmaf(wbase.z, kWinB_c[b], -wbase.w * kWinB_s[b]);
            v[b] = cx{v[b].r * __builtin_fmaf(-A.wb, t0, A.wa), v[b].i * __builtin_fmaf(-A.wb, t1, A.wa)};
        }
    } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int b = 16 * g; b < 16 * g + 16; ++b) {
                const v2f w = (A.win2 + 64u * (uint32_t)b)[lane];
                v[b] = cx{v[b].r * w.x, v[b].i * w.y};
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    DSPB_STAMP(A, f, lane, 1);
    // ---- 2. DFT64 over b -------------------------------------------------
    if (!(DSPB_ABLATE & kAbDft1)) sdft64<!(OPT & kOptNoBar)>(v);
    DSPB_STAMP(A, f, lane, 2);

    // ---- 3. twiddle W4096^(a kb) = W^(a lo) W^(8 a hi), kb = lo + 8 hi ------
    {
        if constexpr (!(OPT & kOptPrefetchTw)) {
#pragma unroll
            for (int j = 1; j < 8; ++j) {
                const v2f a = A.tw[2u * lane * (uint32_t)j];
                const v2f b = A.tw[16u * lane * (uint32_t)j];
                tlo[j] = cx{a.x, a.y};
                thi[j] = cx{b.x, b.y};
            }
        }
#pragma unroll
        for (int hi = 0; hi < 8; ++hi) {
            if (DSPB_ABLATE & kAbTw) break;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int lo = 0; lo < 8; ++lo) {
                const int kb = lo + 8 * hi;
                if (kb == 0) continue;
                const cx w = lo ? (hi ? mulc(tlo[lo], thi[hi]) : tlo[lo]) : thi[hi];
                v[perm64(kb)] = mulc(v[perm64(kb)], w);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    DSPB_STAMP(A, f, lane, 3);
    // ---- 4. transpose through LDS, in place (re, then im) ----------------
    if constexpr (!(DSPB_ABLATE & kAbLds)) {
#pragma unroll
    for (int kb = 0; kb < 64; ++kb) lds[lane * 65u + kb] = v[perm64(kb)].r;
    lds_fence();
#pragma unroll
    for (int a = 0; a < 64; ++a) v[a].r = lds[a * 65 + lane];
    lds_fence();
#pragma unroll
    for (int kb = 0; kb < 64; ++kb) lds[lane * 65u + kb] = v[perm64(kb)].i;
    lds_fence();
#pragma unroll
    for (int a = 0; a < 64; ++a) v[a].i = lds[a * 65 + lane];
    }

    DSPB_STAMP(A, f, lane, 4);
    // ---- 5. DFT64 over a: Z[lane + 64 ka] at v[perm64(ka)] --------------
    if (!(DSPB_ABLATE & kAbDft2)) sdft64<!(OPT & kOptNoBar)>(v);
    DSPB_STAMP(A, f, lane, 5);

    // ---- 6. paired real split: (k, M-k), k = lane + 64 ka, ka < 32 -----------
    float *mrow = A.mag.p[ch] + f * A.ld;
    if constexpr (DSPB_ABLATE & kAbSplit) {
#pragma unroll
        for (int ka = 0; ka < 64; ++ka) (mrow + 64u * (uint32_t)ka)[lane] = v[ka].r + v[ka].i;
        DSPB_STAMP(A, f, lane, 6);
        return;
    }
    const uint32_t src = ((64u - lane) & 63u) * 4u;
    const bool l0 = lane == 0;
    const v2f wl2 = A.tw[lane];  // W8192^lane
    const cx wl = cx{wl2.x, wl2.y};
#pragma unroll
    for (int ka = 0; ka < 32; ++ka) {
        if ((ka & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const cx zp = v[perm64(63 - ka)];
        const float tr = bperm(src, zp.r), ti = bperm(src, zp.i);
        // lane 0 (column 0): Z[M - 64 ka] = its own Z[64 ((64 - ka) & 63)]
        const cx own = v[perm64((64 - ka) & 63)];
        const cx P = cx{l0 ? own.r : tr, l0 ? own.i : ti};
        const cx Z = v[perm64(ka)];
        const cx E = cx{Z.r + P.r, Z.i - P.i};  // 2 E   (P conjugated)
        const cx D = cx{Z.r - P.r, Z.i + P.i};  // 2 i O
        const cx tw = ka == 0 ? wl : mulc(wl, kW128_re[ka], kW128_im[ka]);  // W8192^k
        const cx T = mulc(negi(D), tw);         // 2 W^k O
        const cx X1 = E + T;                    // 2 X[k]
        const cx X2 = E - T;                    // 2 conj X[M - k]
        const float m1 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X1.r, X1.r, X1.i * X1.i));
        const float m2 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X2.r, X2.r, X2.i * X2.i));
        const uint32_t k1 = lane + 64u * (uint32_t)ka;  // < 2048
        const uint32_t k2 = 4096u - k1;                 // > 2048 (4096 at k1 = 0)
        if constexpr (KM == kKPartial) {
            if (k1 < A.K) mrow[k1] = m1;
            if (k2 < A.K) mrow[k2] = m2;
        } else {
            (mrow + 64u * (uint32_t)ka)[lane] = m1;
            (mrow + 4096u - 64u * (uint32_t)ka)[-(int)lane] = m2;
            if constexpr (KM == kKMirror) {
                // |X[8192 - k]| = |X[k]|: bins 4096..8191 (k1 = 0 rewrites bin 0)
                mrow[k1 == 0 ? 0u : 8192u - k1] = m1;
                (mrow + 4096u + 64u * (uint32_t)ka)[lane] = m2;
            }
        }
    }
    if (l0) {  // the self-paired bin k = 2048: |X| = 2 |Z[2048]| (scaled)
        const cx Z = v[perm64(32)];
        const float m = 2.f * __builtin_amdgcn_sqrtf(__builtin_fmaf(Z.r, Z.r, Z.i * Z.i));
        if (KM != kKPartial || 2048u < A.K) mrow[2048] = m;
        if (KM == kKMirror) mrow[6144] = m;
    }
    DSPB_STAMP(A, f, lane, 6);
}

template <int SRC, MapKind MK, bool POW2, int OPT>
static void launch_soa_km(int km, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, POW2, OPT>), grid, dim3(256), 0, s, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKMirror, MK, POW2, OPT>), grid, dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKPartial, MK, POW2, OPT>), grid, dim3(256), 0, s, A);
}

// the headline shapes (IR_test-fused and memory-source, 4097 bins) can run
// every OPT combination for A/B; everything else runs kSoaDefaultOpt
template <int SRC, MapKind MK>
static void launch_soa_ab(int opt, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    switch (opt & 14) {
    case 0: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 0>), grid, dim3(256), 0, s, A); break;
    case 2: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 2>), grid, dim3(256), 0, s, A); break;
    case 4: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 4>), grid, dim3(256), 0, s, A); break;
    case 6: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 6>), grid, dim3(256), 0, s, A); break;
    case 8: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 8>), grid, dim3(256), 0, s, A); break;
    case 10: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 10>), grid, dim3(256), 0, s, A); break;
    case 12: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 12>), grid, dim3(256), 0, s, A); break;
    default: hipLaunchKernelGGL((stft8192_soa_kernel<SRC, kKHalf, MK, true, 14>), grid, dim3(256), 0, s, A); break;
    }
}

// A.win2 must hold the window pre-scaled by 0.5 / sqrt(8192); with
// kOptWinComp also A.wbase / A.wa / A.wb (valid == 8192 only).
int launch_stft8192_soa(const Stft8kArgs &A, uint32_t C, bool fused, int opt, hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    const uint64_t groups = (A.F + 3) / 4;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)groups, C);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    // computed window: full frames only (the twiddle prefetch is a loss
    // without it: too many loads in flight)
    if (A.valid < 8192u || !A.wbase) opt &= ~(kOptWinComp | kOptPrefetchTw);
    constexpr int D = kSoaKmOpt;
    if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_soa_km<kSrcRender, MapKind::Noop, true, D>(km, grid, stream, A); break;
        case MapKind::Gain: launch_soa_km<kSrcRender, MapKind::Gain, true, D>(km, grid, stream, A); break;
        case MapKind::Ramp:
            if (pow2 && km == kKHalf) launch_soa_ab<kSrcRender, MapKind::Ramp>(opt, grid, stream, A);
            else if (pow2) launch_soa_km<kSrcRender, MapKind::Ramp, true, D>(km, grid, stream, A);
            else launch_soa_km<kSrcRender, MapKind::Ramp, false, D>(km, grid, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else if (km == kKHalf) {
        launch_soa_ab<kSrcMemory, MapKind::Noop>(opt, grid, stream, A);
    } else {
        launch_soa_km<kSrcMemory, MapKind::Noop, true, D>(km, grid, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
