// stft_pair.hip -- 8192-point STFT kernel, TWO WAVEFRONTS PER FRAME.
//
// Same transform as stft8192_kernel (spectral.hip): the real frame is packed
// as 4096 complex points z[m] = x[2m] + i x[2m+1] and transformed by a
// 64 x 64 four-step FFT, then split into the 4097 real-input bins.  The
// difference is the work split, chosen for occupancy on CDNA4:
//
//   * a 128-thread workgroup owns one frame; lane (wave w, slot c, half h)
//     holds 32 complex points (64 VGPRs instead of 128), so four waves fit
//     per SIMD (16 per CU) and hide each other's HBM / LDS latency;
//   * each 64-point column DFT is split over a lane pair (c, c+32): a
//     32-point DFT in registers per lane, then one radix-2 step whose
//     exchange is v_permlane32_swap (lanes 0-31 <-> 32-63, no LDS);
//   * the 64 x 64 transpose between the two stages goes through 16.6 KB of
//     LDS (one component at a time, row stride 65 floats: conflict-free
//     ds_write_b32, at most 2-way ds_read_b32);
//   * stage-2 columns are assigned so that column kb and its real-split
//     partner 64 - kb sit in the same wave (slots c and c ^ 16): the
//     partner value Z[M - k] is one ds_bpermute away.
//
// Index bookkeeping (r = register group index 0..31, h = half):
//   stage-1 column   a  = c + 32 w,   b = 2 j + h           (j = 0..31)
//   after combine    kb = (r & 15) + 16 h + 32 (r >> 4)     at v[perm32(r)]
//   stage-2 column   kb' = colmap2(w, c), a = 2 j + h
//   after combine    ka = (r & 15) + 16 h + 32 (r >> 4)     -> Z[kb' + 64 ka]
#include "fft_device.hpp"

namespace dspb {

// Stage-2 column of slot c in wave w.  Wave 0: {0..15, 32, 63..49};
// wave 1: {16..31, 48..33}.  The partner column 64 - kb lives in slot c ^ 16
// (columns 0 and 32 are their own partners).
__device__ __forceinline__ uint32_t colmap2(uint32_t w, uint32_t c) {
    if (w == 0) return c < 16 ? c : (c == 16 ? 32u : 80u - c);
    return c < 16 ? 16u + c : 64u - c;
}

// Radix-2 combine across the lane halves: on entry lanes 0-31 hold E[k'],
// lanes 32-63 hold O'[k'] = W64^k' O[k'] in v[perm32(k')]; on exit lane half
// h holds X[kb] for kb = (r & 15) + 16 h + 32 (r >> 4) at v[perm32(r)].
__device__ __forceinline__ void combine_halves(v2f (&v)[32]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        v2f &lo = v[perm32(q)], &hi = v[perm32(q + 16)];
        // upper half of `lo` <-> lower half of `hi`
        auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo.x), __float_as_uint(hi.x),
                                                   false, false);
        auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo.y), __float_as_uint(hi.y),
                                                   false, false);
        const v2f e = v2f{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
        const v2f o = v2f{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
        lo = e + o;
        hi = e - o;
    }
}

// 64-point column DFT split over the lane pair: v holds b = 2 j + h, j = 0..31.
__device__ __forceinline__ void dft64_pair(v2f (&v)[32], uint32_t h) {
    dft32(v);
    if (h) {  // odd-b half: O'[k'] = W64^k' O[k']
#pragma unroll
        for (int k = 1; k < 32; ++k) v[perm32(k)] = twiddle64(v[perm32(k)], k);
    }
    combine_halves(v);
}

template <MapKind MK, bool POW2>
__device__ __forceinline__ v2f render_pair(const Stft8kArgs &A, const float *x, uint64_t fs,
                                           uint32_t s) {
    // one float2 of the rendered frame at frame sample s (even)
    const uint64_t li = fs + s;
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
        if constexpr (MK == MapKind::Gain) b *= A.map.a;
        return b;
    }
}

template <int SRC, int KM, MapKind MK, bool POW2>
__global__ __launch_bounds__(128, 4) void stft8192_pair_kernel(Stft8kArgs A) {
    __shared__ float tile[64 * 65];  // one component of the 64 x 64 transpose
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t c = l & 31u, h = l >> 5;
    const uint32_t ch = blockIdx.y;
    const uint64_t f = xcd_remap(blockIdx.x, gridDim.x);
    if (f >= A.F) return;  // uniform over the workgroup: no barrier is left waiting
    const uint64_t fs = f * (uint64_t)A.H;
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    // ---- load: z index m = m0 + 128 j  (a = c + 32 w, b = 2 j + h) -------
    const uint32_t m0 = c + 32u * w + 64u * h;
    v2f v[32];
    if constexpr (SRC == kSrcMemory) {
        if (A.valid >= 8192u) {  // uniform: the whole frame exists
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = reinterpret_cast<const v2f *>(x + fs + 256u * j)[m0];
        } else {  // IR analysis: only the first `valid` samples exist, zero pad
#pragma unroll
            for (int j = 0; j < 32; ++j)
                v[j] = 2u * (m0 + 128u * j) < A.valid
                           ? reinterpret_cast<const v2f *>(x + fs + 256u * j)[m0]
                           : v2f{0.f, 0.f};
        }
    } else {
        float *o = A.out.p[ch] + fs;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t s = 2u * (m0 + 128u * j);
            v[j] = render_pair<MK, POW2>(A, x, fs, s);
            if (s < A.H) *reinterpret_cast<v2f *>(o + s) = v[j];  // this frame owns [fs, fs+H)
        }
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] *= (A.win2 + 128u * j)[m0];

    // ---- stage 1: 64-point DFTs over b, column a = c + 32 w --------------
    dft64_pair(v, h);

    // ---- twiddle W4096^(a kb) = T8192[2 a kb] ----------------------------
    {
        const uint32_t a = c + 32u * w;
        const v2f w32 = A.tw[64u * a];  // W4096^(32 a)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const v2f wq = A.tw[2u * a * (uint32_t)q + 32u * a * h];  // W4096^(a (q + 16 h))
            v[perm32(q)] = cmul(v[perm32(q)], wq);
            v[perm32(q + 16)] = cmul(v[perm32(q + 16)], cmul(wq, w32));
        }
    }

    // ---- transpose: tile[kb][a], re then im -------------------------------
    {
        const uint32_t a = c + 32u * w;
        const uint32_t kbase = 16u * h;
        const uint32_t kb2 = colmap2(w, c);  // stage-2 column of this lane
#pragma unroll
        for (int r = 0; r < 32; ++r)
            tile[(kbase + (r & 15) + 32 * (r >> 4)) * 65u + a] = v[perm32(r)].x;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j].x = tile[kb2 * 65u + 2u * j + h];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 32; ++r)
            tile[(kbase + (r & 15) + 32 * (r >> 4)) * 65u + a] = v[perm32(r)].y;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j].y = tile[kb2 * 65u + 2u * j + h];
    }

    // ---- stage 2: 64-point DFTs over a, column kb' --------------------------
    dft64_pair(v, h);

    // ---- real-input split, magnitude, store ---------------------------------
    const uint32_t kb = colmap2(w, c);
    const bool self_col = (w == 0) && (c == 0 || c == 16);
    const uint32_t pl = (self_col ? c : (c ^ 16u)) + 32u * (1u - h);  // partner lane
    const uint32_t paddr = pl * 4u;
    const bool col0 = (w == 0) && (c == 0);
    const v2f wl = A.tw[kb + 1024u * h];  // W8192^(kb + 1024 h)
    float *mrow = A.mag.p[ch] + f * A.ld;
    const v2f own0 = v[perm32(0)], own16 = v[perm32(16)];
    v2f prev = own0;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        if ((r & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const v2f zp = v[perm32(31 - r)];
        v2f t;
        t.x = bperm(paddr, zp.x);
        t.y = bperm(paddr, zp.y);
        v2f P = t;
        if (col0) {  // column 0 pairs with itself, shifted by one (see header)
            if (r == 0) P = h ? own16 : own0;
            else if (r == 16) P = h ? own0 : own16;
            else P = prev;
        }
        prev = t;
        const v2f Z = v[perm32(r)];
        const v2f cp = v2f{P.x, -P.y};
        const v2f E = Z + cp;  // 2 E
        const v2f D = Z - cp;  // 2 i O
        const v2f O = v2f{D.y, -D.x};
        const int kc = (r & 15) + 32 * (r >> 4);
        const v2f tw = kc == 0 ? wl : cmul(wl, v2f{kW128_re[kc], kW128_im[kc]});
        const v2f X = E + cmul(tw, O);  // 2 X[k]
        const float m = __builtin_amdgcn_sqrtf(X.x * X.x + X.y * X.y) * (0.5f * A.scale);
        const uint32_t k = kb + 64u * ((uint32_t)(r & 15) + 16u * h + 32u * (uint32_t)(r >> 4));
        if constexpr (KM == kKPartial) {
            if (k < A.K) mrow[k] = m;
        } else {
            mrow[k] = m;
            if constexpr (KM == kKMirror) mrow[k == 0 ? 0u : 8192u - k] = m;
        }
    }
    if (col0 && h == 0 && (KM != kKPartial || A.K > 4096u))
        mrow[4096] = __builtin_fabsf(own0.x - own0.y) * A.scale;  // Nyquist: Re Z0 - Im Z0
}

template <int SRC, MapKind MK, bool POW2>
static void launch_pair_km(int km, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_pair_kernel<SRC, kKHalf, MK, POW2>), grid, dim3(128), 0, s, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_pair_kernel<SRC, kKMirror, MK, POW2>), grid, dim3(128), 0, s, A);
    else
        hipLaunchKernelGGL((stft8192_pair_kernel<SRC, kKPartial, MK, POW2>), grid, dim3(128), 0, s, A);
}

int launch_stft8192_pair(const Stft8kArgs &A, uint32_t C, bool fused, hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    if (A.F > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)A.F, C);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_pair_km<kSrcRender, MapKind::Noop, true>(km, grid, stream, A); break;
        case MapKind::Gain: launch_pair_km<kSrcRender, MapKind::Gain, true>(km, grid, stream, A); break;
        case MapKind::Ramp:
            if (pow2) launch_pair_km<kSrcRender, MapKind::Ramp, true>(km, grid, stream, A);
            else launch_pair_km<kSrcRender, MapKind::Ramp, false>(km, grid, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else {
        launch_pair_km<kSrcMemory, MapKind::Noop, true>(km, grid, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
