// stft_pair_soa.hip -- 8192-point STFT, TWO WAVEFRONTS PER FRAME, scalar
// (structure-of-arrays) arithmetic.
//
// The work split of stft_pair.hip (32 complex points per lane, 64 VGPRs of
// data, four waves per SIMD; 64-point column DFTs split over the lane pair
// (c, c+32) with one v_permlane32_swap radix-2 step; 64 x 64 transpose
// through 16.6 KB of LDS; stage-2 columns paired with their real-split
// partner 64 - kb in slot c ^ 16) combined with the arithmetic of
// stft_soa.hip (scalar complex, no re-packing, window pre-scaled by
// 0.5/sqrt(N), real split producing X[k] and X[M-k] from one (E, W^k O)).
//
// Register map (r = 0..31, h = lane half):
//   after a column DFT, v[perm32(r)] holds output index
//   (r & 15) + 16 h + 32 (r >> 4)
#include "fft_soa.hpp"

namespace dspb {

__device__ __forceinline__ uint32_t colmap2s(uint32_t w, uint32_t c) {
    if (w == 0) return c < 16 ? c : (c == 16 ? 32u : 80u - c);
    return c < 16 ? 16u + c : 64u - c;
}

__device__ __forceinline__ float swap_lo(float a, float b, float *nb) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    *nb = __uint_as_float(r[1]);
    return __uint_as_float(r[0]);
}

// 64-point column DFT over a lane pair: v holds input index 2 j + h.
__device__ __forceinline__ void sdft64_pair(cx (&v)[32], uint32_t h) {
    sdft32(v);
    if (h) {  // odd half: O'[k'] = W64^k' O[k']
#pragma unroll
        for (int k = 1; k < 32; ++k) v[perm32(k)] = stw64(v[perm32(k)], k);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        cx &lo = v[perm32(q)], &hi = v[perm32(q + 16)];
        cx e, o;
        e.r = swap_lo(lo.r, hi.r, &o.r);  // lanes 32-63 of lo <-> lanes 0-31 of hi
        e.i = swap_lo(lo.i, hi.i, &o.i);
        lo = e + o;
        hi = e - o;
    }
}

template <MapKind MK, bool POW2>
__device__ __forceinline__ cx render_pair_s(const Stft8kArgs &A, const float *x, uint64_t fs,
                                            uint32_t s) {
    const uint64_t li = fs + s;
    if constexpr (MK == MapKind::Ramp) {
        const float *T = A.map.table;
        const uint64_t gi = A.goff + li;
        if constexpr (POW2) {
            const v2f t = *reinterpret_cast<const v2f *>(T + ((uint32_t)gi & A.map.b_mask));
            return cx{t.x, t.y};
        } else {
            const uint32_t p = (uint32_t)(gi % A.map.B);
            const uint32_t q = (p + 1 == A.map.B) ? 0u : p + 1;
            return cx{T[p], T[q]};
        }
    } else {
        cx b;
        if (x != nullptr && li + 1 < A.L) {
            const v2f t = *reinterpret_cast<const v2f *>(x + li);
            b = cx{t.x, t.y};
        } else {
            b = cx{(x && li < A.L) ? x[li] : 0.f, 0.f};
        }
        if constexpr (MK == MapKind::Gain) b = cx{b.r * A.map.a, b.i * A.map.a};
        return b;
    }
}

template <int SRC, int KM, MapKind MK, bool POW2>
__global__ __launch_bounds__(128, 4) void stft8192_pair_soa_kernel(Stft8kArgs A) {
    __shared__ float tile[64 * 65];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t c = l & 31u, h = l >> 5;
    const uint32_t ch = blockIdx.y;
    const uint64_t f = xcd_remap(blockIdx.x, gridDim.x);
    if (f >= A.F) return;  // uniform over the workgroup
    const uint64_t fs = f * (uint64_t)A.H;
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    // ---- load: z index m = m0 + 128 j ------------------------------------
    const uint32_t m0 = c + 32u * w + 64u * h;
    cx v[32];
    if constexpr (SRC == kSrcMemory) {
        if (A.valid >= 8192u) {
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const v2f t = reinterpret_cast<const v2f *>(x + fs + 256u * j)[m0];
                v[j] = cx{t.x, t.y};
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                v2f t = v2f{0.f, 0.f};
                if (2u * (m0 + 128u * j) < A.valid) t = reinterpret_cast<const v2f *>(x + fs + 256u * j)[m0];
                v[j] = cx{t.x, t.y};
            }
        }
    } else {
        float *o = A.out.p[ch] + fs;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t s = 2u * (m0 + 128u * j);
            v[j] = render_pair_s<MK, POW2>(A, x, fs, s);
            if (s < A.H) *reinterpret_cast<v2f *>(o + s) = v2f{v[j].r, v[j].i};
        }
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const v2f wv = (A.win2 + 128u * j)[m0];
        v[j] = cx{v[j].r * wv.x, v[j].i * wv.y};
    }

    // ---- stage 1 ----------------------------------------------------------
    sdft64_pair(v, h);
    {
        const uint32_t a = c + 32u * w;
        const v2f w32v = A.tw[64u * a];
        const cx w32 = cx{w32v.x, w32v.y};
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const v2f t = A.tw[2u * a * (uint32_t)q + 32u * a * h];  // W4096^(a (q + 16 h))
            const cx wq = cx{t.x, t.y};
            v[perm32(q)] = mulc(v[perm32(q)], wq);
            v[perm32(q + 16)] = mulc(v[perm32(q + 16)], mulc(wq, w32));
        }
    }

    // ---- transpose through LDS: tile[kb][a] --------------------------------
    {
        const uint32_t a = c + 32u * w;
        const uint32_t kbase = 16u * h;
        const uint32_t kb2 = colmap2s(w, c);
#pragma unroll
        for (int r = 0; r < 32; ++r) tile[(kbase + (r & 15) + 32 * (r >> 4)) * 65u + a] = v[perm32(r)].r;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j].r = tile[kb2 * 65u + 2u * j + h];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 32; ++r) tile[(kbase + (r & 15) + 32 * (r >> 4)) * 65u + a] = v[perm32(r)].i;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j].i = tile[kb2 * 65u + 2u * j + h];
    }

    // ---- stage 2 ----------------------------------------------------------
    sdft64_pair(v, h);

    // ---- paired real split: 16 pairs (k, M - k) per lane ----------------------
    const uint32_t kb = colmap2s(w, c);
    const bool self_col = (w == 0) && (c == 0 || c == 16);
    const uint32_t paddr = ((self_col ? c : (c ^ 16u)) + 32u * (1u - h)) * 4u;
    const bool col0 = (w == 0) && (c == 0);
    const v2f wl2 = A.tw[kb + 1024u * h];  // W8192^(kb + 1024 h)
    const cx wl = cx{wl2.x, wl2.y};
    float *mrow = A.mag.p[ch] + f * A.ld;
    const cx own0 = v[perm32(0)], own16 = v[perm32(16)];
    cx prev = own0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if ((r & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const cx zp = v[perm32(31 - r)];
        const cx t = cx{bperm(paddr, zp.r), bperm(paddr, zp.i)};
        // column 0 pairs inside itself, shifted by one register (see stft_pair.hip)
        const cx p0 = r == 0 ? (h ? own16 : own0) : prev;
        const cx P = cx{col0 ? p0.r : t.r, col0 ? p0.i : t.i};
        prev = t;
        const cx Z = v[perm32(r)];
        const cx E = cx{Z.r + P.r, Z.i - P.i};
        const cx D = cx{Z.r - P.r, Z.i + P.i};
        const cx tw = r == 0 ? wl : mulc(wl, kW128_re[r], kW128_im[r]);  // W8192^k
        const cx T = mulc(negi(D), tw);
        const cx X1 = E + T, X2 = E - T;
        const float m1 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X1.r, X1.r, X1.i * X1.i));
        const float m2 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X2.r, X2.r, X2.i * X2.i));
        const uint32_t k1 = kb + 64u * ((uint32_t)r + 16u * h);
        const uint32_t k2 = 4096u - k1;
        if constexpr (KM == kKPartial) {
            if (k1 < A.K) mrow[k1] = m1;
            if (k2 < A.K) mrow[k2] = m2;
        } else {
            mrow[k1] = m1;
            mrow[k2] = m2;
            if constexpr (KM == kKMirror) {
                mrow[k1 == 0 ? 0u : 8192u - k1] = m1;
                mrow[8192u - k2] = m2;
            }
        }
    }
    if (col0 && h == 0) {  // self-paired bin 2048 = Z[64 * 32] at (h 0, r 16)
        const float m = 2.f * __builtin_amdgcn_sqrtf(__builtin_fmaf(own16.r, own16.r, own16.i * own16.i));
        if (KM != kKPartial || 2048u < A.K) mrow[2048] = m;
        if (KM == kKMirror) mrow[6144] = m;
    }
}

template <int SRC, MapKind MK, bool POW2>
static void launch_pair_soa_km(int km, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_pair_soa_kernel<SRC, kKHalf, MK, POW2>), grid, dim3(128), 0, s, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_pair_soa_kernel<SRC, kKMirror, MK, POW2>), grid, dim3(128), 0, s, A);
    else
        hipLaunchKernelGGL((stft8192_pair_soa_kernel<SRC, kKPartial, MK, POW2>), grid, dim3(128), 0, s, A);
}

// A.win2 must hold the window pre-scaled by 0.5 / sqrt(8192).
int launch_stft8192_pair_soa(const Stft8kArgs &A, uint32_t C, bool fused, hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    if (A.F > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)A.F, C);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_pair_soa_km<kSrcRender, MapKind::Noop, true>(km, grid, stream, A); break;
        case MapKind::Gain: launch_pair_soa_km<kSrcRender, MapKind::Gain, true>(km, grid, stream, A); break;
        case MapKind::Ramp:
            if (pow2) launch_pair_soa_km<kSrcRender, MapKind::Ramp, true>(km, grid, stream, A);
            else launch_pair_soa_km<kSrcRender, MapKind::Ramp, false>(km, grid, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else {
        launch_pair_soa_km<kSrcMemory, MapKind::Noop, true>(km, grid, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
