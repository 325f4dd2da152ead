// stft_pair2.hip -- 8192-point STFT, TWO FRAMES PER WORKGROUP OF TWO WAVES,
// the two frames packed into the halves of each VGPR pair.
//
// Work split as stft_pair_soa.hip (lane (wave w, slot c, half h) owns 32
// complex points of column a = c + 32 w; the 64-point column DFT is split
// over the lane pair (c, c+32) with one v_permlane32_swap radix-2 step;
// 64 x 64 transpose through LDS; stage-2 column kb and its real-split
// partner 64 - kb in slots c and c ^ 16 of one wave), but every register
// holds the same element of frames f0 = 2 g and f1 = 2 g + 1 (fft_x2.hpp):
// the transform of two frames costs one instruction stream.  Twiddles, the
// window and all index arithmetic are shared by the two frames.
//
// Register map (r = 0..31, h = lane half): after a column DFT, v[perm32(r)]
// holds output index (r & 15) + 16 h + 32 (r >> 4).
#include "fft_x2.hpp"

namespace dspb {

__device__ __forceinline__ uint32_t colmap2x(uint32_t w, uint32_t c) {
    if (w == 0) return c < 16 ? c : (c == 16 ? 32u : 80u - c);
    return c < 16 ? 16u + c : 64u - c;
}

__device__ __forceinline__ float swap32(float a, float b, float *nb) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    *nb = __uint_as_float(r[1]);
    return __uint_as_float(r[0]);
}

__device__ __forceinline__ v2f swap32v(v2f a, v2f b, v2f *nb) {
    float ox, oy;
    const float ex = swap32(a.x, b.x, &ox);
    const float ey = swap32(a.y, b.y, &oy);
    *nb = v2f{ox, oy};
    return v2f{ex, ey};
}

// 64-point column DFT over a lane pair: v holds input index 2 j + h.
__device__ __forceinline__ void x2dft64_pair(cx2 (&v)[32], uint32_t h) {
    x2dft32(v);
    if (h) {  // odd half: O'[k'] = W64^k' O[k']
#pragma unroll
        for (int k = 1; k < 32; ++k) v[perm32(k)] = x2tw64(v[perm32(k)], k);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        cx2 &lo = v[perm32(q)], &hi = v[perm32(q + 16)];
        cx2 e, o;
        e.r = swap32v(lo.r, hi.r, &o.r);  // lanes 32-63 of lo <-> lanes 0-31 of hi
        e.i = swap32v(lo.i, hi.i, &o.i);
        lo = e + o;
        hi = e - o;
    }
}

template <MapKind MK, bool POW2>
__device__ __forceinline__ v2f render_x2(const Stft8kArgs &A, const float *x, uint64_t li) {
    // samples li, li + 1 of the rendered signal (local index)
    if constexpr (MK == MapKind::Ramp) {
        const float *T = A.map.table;
        const uint64_t gi = A.goff + li;
        if constexpr (POW2) {
            return *reinterpret_cast<const v2f *>(T + ((uint32_t)gi & A.map.b_mask));
        } else {
            const uint32_t p = (uint32_t)(gi % A.map.B);
            const uint32_t q = (p + 1 == A.map.B) ? 0u : p + 1;
            return v2f{T[p], T[q]};
        }
    } else {
        v2f b;
        if (x != nullptr && li + 1 < A.L) {
            b = *reinterpret_cast<const v2f *>(x + li);
        } else {
            b = v2f{(x && li < A.L) ? x[li] : 0.f, 0.f};
        }
        if constexpr (MK == MapKind::Gain) b = b * A.map.a;
        return b;
    }
}

template <int SRC, int KM, MapKind MK, bool POW2>
__global__ __launch_bounds__(128, 2) void stft8192_pair2_kernel(Stft8kArgs A) {
    __shared__ v2f tile[64 * 65];  // one component of both frames' 64 x 64 transpose
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t c = l & 31u, h = l >> 5;
    const uint32_t ch = blockIdx.y;
    const uint64_t f0 = 2ull * xcd_remap(blockIdx.x, gridDim.x);
    if (f0 >= A.F) return;  // uniform over the workgroup
    const bool has1 = f0 + 1 < A.F;      // odd F: the last group computes f0 twice
    const uint64_t f1 = has1 ? f0 + 1 : f0;
    const uint64_t fs0 = f0 * (uint64_t)A.H, fs1 = f1 * (uint64_t)A.H;
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    // ---- load both frames: z index m = m0 + 128 j --------------------------
    const uint32_t m0 = c + 32u * w + 64u * h;
    cx2 v[32];
    if constexpr (SRC == kSrcMemory) {
        const bool full = A.valid >= 8192u;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t s = 2u * (m0 + 128u * j);
            v2f a = v2f{0.f, 0.f}, b = v2f{0.f, 0.f};
            if (full || s < A.valid) {
                a = *reinterpret_cast<const v2f *>(x + fs0 + s);
                b = *reinterpret_cast<const v2f *>(x + fs1 + s);
            }
            v[j] = cx2{v2f{a.x, b.x}, v2f{a.y, b.y}};
        }
    } else {
        float *o = A.out.p[ch];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t s = 2u * (m0 + 128u * j);
            const v2f a = render_x2<MK, POW2>(A, x, fs0 + s);
            const v2f b = render_x2<MK, POW2>(A, x, fs1 + s);
            if (s < A.H) {  // each frame owns the render of its hop
                *reinterpret_cast<v2f *>(o + fs0 + s) = a;
                if (has1) *reinterpret_cast<v2f *>(o + fs1 + s) = b;
            }
            v[j] = cx2{v2f{a.x, b.x}, v2f{a.y, b.y}};
        }
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const v2f wv = (A.win2 + 128u * j)[m0];  // pre-scaled by 0.5/sqrt(N)
        v[j] = cx2{v[j].r * wv.x, v[j].i * wv.y};
    }

    // ---- stage 1 ----------------------------------------------------------
    x2dft64_pair(v, h);
    {
        const uint32_t a = c + 32u * w;
        const v2f w32 = A.tw[64u * a];  // W4096^(32 a)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const v2f wq = A.tw[2u * a * (uint32_t)q + 32u * a * h];  // W4096^(a (q + 16 h))
            const v2f wq2 = v2f{wq.x * w32.x - wq.y * w32.y, wq.x * w32.y + wq.y * w32.x};
            v[perm32(q)] = mulc2(v[perm32(q)], wq.x, wq.y);
            v[perm32(q + 16)] = mulc2(v[perm32(q + 16)], wq2.x, wq2.y);
        }
    }

    // ---- transpose through LDS: tile[kb][a], re then im ----------------------
    {
        const uint32_t a = c + 32u * w;
        const uint32_t kbase = 16u * h;
        const uint32_t kb2 = colmap2x(w, c);
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
    x2dft64_pair(v, h);

    // ---- paired real split: 16 pairs (k, M - k) per lane, both frames -------
    const uint32_t kb = colmap2x(w, c);
    const bool self_col = (w == 0) && (c == 0 || c == 16);
    const uint32_t paddr = ((self_col ? c : (c ^ 16u)) + 32u * (1u - h)) * 4u;
    const bool col0 = (w == 0) && (c == 0);
    const v2f wl = A.tw[kb + 1024u * h];  // W8192^(kb + 1024 h)
    float *mrow0 = A.mag.p[ch] + f0 * A.ld;
    float *mrow1 = A.mag.p[ch] + f1 * A.ld;
    const cx2 own0 = v[perm32(0)], own16 = v[perm32(16)];
    cx2 prev = own0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if ((r & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const cx2 zp = v[perm32(31 - r)];
        cx2 t;
        t.r.x = bperm(paddr, zp.r.x);
        t.r.y = bperm(paddr, zp.r.y);
        t.i.x = bperm(paddr, zp.i.x);
        t.i.y = bperm(paddr, zp.i.y);
        const cx2 p0 = r == 0 ? (h ? own16 : own0) : prev;
        const cx2 P = col0 ? p0 : t;  // column 0 pairs inside itself, shifted by one
        prev = t;
        const cx2 Z = v[perm32(r)];
        const cx2 E = cx2{Z.r + P.r, Z.i - P.i};
        const cx2 D = cx2{Z.r - P.r, Z.i + P.i};
        v2f tw = wl;  // W8192^k, k = kb + 64 (r + 16 h)
        if (r) tw = v2f{wl.x * kW128_re[r] - wl.y * kW128_im[r], wl.x * kW128_im[r] + wl.y * kW128_re[r]};
        const cx2 T = mulc2(negi(D), tw.x, tw.y);
        const cx2 X1 = E + T, X2 = E - T;
        const v2f q1 = X1.r * X1.r + X1.i * X1.i;
        const v2f q2 = X2.r * X2.r + X2.i * X2.i;
        const v2f m1 = v2f{__builtin_amdgcn_sqrtf(q1.x), __builtin_amdgcn_sqrtf(q1.y)};
        const v2f m2 = v2f{__builtin_amdgcn_sqrtf(q2.x), __builtin_amdgcn_sqrtf(q2.y)};
        const uint32_t k1 = kb + 64u * ((uint32_t)r + 16u * h);
        const uint32_t k2 = 4096u - k1;
        if constexpr (KM == kKPartial) {
            if (k1 < A.K) { mrow0[k1] = m1.x; if (has1) mrow1[k1] = m1.y; }
            if (k2 < A.K) { mrow0[k2] = m2.x; if (has1) mrow1[k2] = m2.y; }
        } else {
            mrow0[k1] = m1.x;
            mrow0[k2] = m2.x;
            if (has1) {
                mrow1[k1] = m1.y;
                mrow1[k2] = m2.y;
            }
            if constexpr (KM == kKMirror) {
                const uint32_t k1m = k1 == 0 ? 0u : 8192u - k1;
                mrow0[k1m] = m1.x;
                mrow0[8192u - k2] = m2.x;
                if (has1) {
                    mrow1[k1m] = m1.y;
                    mrow1[8192u - k2] = m2.y;
                }
            }
        }
    }
    if (col0 && h == 0) {  // self-paired bin 2048 = Z[64 * 32] at (h 0, r 16)
        const v2f q = own16.r * own16.r + own16.i * own16.i;
        const float ma = 2.f * __builtin_amdgcn_sqrtf(q.x), mb = 2.f * __builtin_amdgcn_sqrtf(q.y);
        if (KM != kKPartial || 2048u < A.K) {
            mrow0[2048] = ma;
            if (has1) mrow1[2048] = mb;
        }
        if (KM == kKMirror) {
            mrow0[6144] = ma;
            if (has1) mrow1[6144] = mb;
        }
    }
}

template <int SRC, MapKind MK, bool POW2>
static void launch_pair2_km(int km, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_pair2_kernel<SRC, kKHalf, MK, POW2>), grid, dim3(128), 0, s, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_pair2_kernel<SRC, kKMirror, MK, POW2>), grid, dim3(128), 0, s, A);
    else
        hipLaunchKernelGGL((stft8192_pair2_kernel<SRC, kKPartial, MK, POW2>), grid, dim3(128), 0, s, A);
}

// A.win2 must hold the window pre-scaled by 0.5 / sqrt(8192).
int launch_stft8192_pair2(const Stft8kArgs &A, uint32_t C, bool fused, hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    const uint64_t groups = (A.F + 1) / 2;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)groups, C);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_pair2_km<kSrcRender, MapKind::Noop, true>(km, grid, stream, A); break;
        case MapKind::Gain: launch_pair2_km<kSrcRender, MapKind::Gain, true>(km, grid, stream, A); break;
        case MapKind::Ramp:
            if (pow2) launch_pair2_km<kSrcRender, MapKind::Ramp, true>(km, grid, stream, A);
            else launch_pair2_km<kSrcRender, MapKind::Ramp, false>(km, grid, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else {
        launch_pair2_km<kSrcMemory, MapKind::Noop, true>(km, grid, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
