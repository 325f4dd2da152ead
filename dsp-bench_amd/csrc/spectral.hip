// spectral.hip -- CDNA4 kernels for the windowed-FFT / magnitude path.
//
// Replaces the IPP pipeline of the reference (dsp.cpp:53-132, 166-168):
//   windowing_hamming (ippsWinHamming_32f)  -> fused into the frame load
//   fft_forward (ippsFFTFwd_CToC_32f, DIV_BY_SQRTN) -> register/LDS FFT
//   pythagore_array (ippsMagnitude_32f)     -> fused into the store
//
// Two kernels:
//
//  * stft8192_kernel -- the hot one.  ONE WAVEFRONT PER 8192-POINT FRAME.
//    The real frame is packed as 4096 complex points z[m] = x[2m] + i x[2m+1]
//    and transformed with a 64 x 64 four-step FFT that maps onto wave64:
//      1. lane a holds z[a + 64 b], b = 0..63 (coalesced float2 loads: one
//         wave instruction = 512 contiguous bytes), window applied on load;
//      2. 64-point DFT over b in registers (8 x 8, constant twiddles);
//      3. twiddle W4096^(a kb) (double-accurate table, L1/L2 resident);
//      4. transpose 64 x 64 through LDS (row stride 65 -> conflict-free
//         ds_write_b32 / ds_read_b32), no workgroup barrier: the exchange
//         is wave-private;
//      5. 64-point DFT over a in registers -> Z[kb + 64 ka] on lane kb;
//      6. real-input split X[k] = E + W8192^k O with the partner Z[M-k]
//         fetched lane-to-lane by ds_bpermute, |X|/sqrt(N), coalesced store.
//    Four waves (four consecutive frames) per 256-thread workgroup, blockIdx
//    remapped so consecutive frame groups share an XCD (their 50 % overlap
//    is then an L2 hit).  Optionally fused with a per-sample render map
//    (gain_test / static_gain / IR_test / no_op): the render of the frame's
//    hop is stored from the same registers, so the rendered signal is
//    written once and never re-read.
//
//  * fft_generic_kernel -- one workgroup per transform, radix-2 Stockham in
//    LDS, any power of two <= 8192, forward or inverse.  Serves
//    fft_forward / fft_reverse (plugin services), STFTs with N != 8192 and
//    IR analyses with other IR lengths.  Latency-bound by nature.
#include "kernels.hpp"
#include "fft_device.hpp"

namespace dspb {






// Fused render source: the frame's 8192 samples are produced by the
// per-sample plugin map (render.hip's rule) instead of read back from HBM.
template <MapKind MK, bool POW2>
__device__ __forceinline__ void render_frame(const Stft8kArgs &A, const float *x, uint64_t fs,
                                             uint32_t lane, v2f (&v)[64]) {
    const uint64_t gbase = A.goff + fs;  // global index of the frame's sample 0
    if constexpr (MK == MapKind::Ramp) {
        const float *T = A.map.table;    // IR_test ramp, one block long
        if constexpr (POW2) {            // B >= 2: (p & mask) is even, p + 1 in range
            const uint32_t p0 = (uint32_t)gbase + 2u * lane;
#pragma unroll
            for (int b = 0; b < 64; ++b)
                v[b] = *reinterpret_cast<const v2f *>(T + ((p0 + 128u * (uint32_t)b) & A.map.b_mask));
        } else {
            const uint32_t Bn = A.map.B;
            uint32_t p = (uint32_t)((gbase + 2u * lane) % Bn);
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint32_t q = (p + 1 == Bn) ? 0u : p + 1;
                v[b] = v2f{T[p], T[q]};
                p += 128u;
                while (p >= Bn) p -= Bn;
            }
        }
    } else {
        if (x != nullptr && fs + 8192u <= A.L) {  // wave-uniform: whole frame inside the file
#pragma unroll
            for (int b = 0; b < 64; ++b)
                v[b] = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
        } else {  // EOF inside the frame (or no file channel): zero past L
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint64_t li = fs + 2u * lane + 128u * (uint32_t)b;
                v[b] = v2f{(x && li < A.L) ? x[li] : 0.f, (x && li + 1 < A.L) ? x[li + 1] : 0.f};
            }
        }
        if constexpr (MK == MapKind::Gain) {
#pragma unroll
            for (int b = 0; b < 64; ++b) v[b] *= A.map.a;  // one fp32 multiply per sample
        }
    }
}

template <int SRC, bool FULL, int KM, MapKind MK = MapKind::Noop, bool POW2 = true>
__global__ __launch_bounds__(256, 2) void stft8192_kernel(Stft8kArgs A) {
    __shared__ float lds_all[4][64 * 65];
    const uint32_t lane = threadIdx.x & 63u;
    // wave index made provably uniform so frame addresses live in SGPRs
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t c = blockIdx.y;
    const uint64_t f = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (f >= A.F) return;  // whole wave leaves; no workgroup barrier below
    float *lds = lds_all[wave];

    const uint64_t fs = f * (uint64_t)A.H;  // first sample of the frame (local)
    const float *x = (c < A.in_ch) ? A.in.p[c] : nullptr;

    // ---- 1. load (+ fused render) + window --------------------------------
    v2f v[64];
    if constexpr (SRC == kSrcMemory) {
#pragma unroll
        for (int b = 0; b < 64; ++b) {
            if (FULL || 2u * lane + 128u * (uint32_t)b < A.valid)
                v[b] = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
            else
                v[b] = v2f{0.f, 0.f};
        }
    } else {
        render_frame<MK, POW2>(A, x, fs, lane, v);
        // this frame owns the render of its hop [fs, fs + H)
        float *o = A.out.p[c] + fs;
#pragma unroll
        for (int b = 0; b < 64; ++b)
            if (128u * (uint32_t)b < A.H) reinterpret_cast<v2f *>(o + 128u * (uint32_t)b)[lane] = v[b];
    }
    // window, in groups of 16 so the window loads (L2-resident table) do not
    // all become live at once next to the 128 data registers
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b = 16 * g; b < 16 * g + 16; ++b) v[b] *= (A.win2 + 64u * (uint32_t)b)[lane];
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- 2. DFT64 over b -------------------------------------------------
    dft64(v);

    // ---- 3. twiddle W4096^(a kb) = T8192[2 a kb] --------------------------
    {
        v2f tlo[8], thi[8];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            tlo[j] = A.tw[2u * lane * (uint32_t)j];
            thi[j] = A.tw[16u * lane * (uint32_t)j];
        }
#pragma unroll
        for (int hi = 0; hi < 8; ++hi) {
            __builtin_amdgcn_sched_barrier(0);  // one group of 8 twiddles live at a time
#pragma unroll
            for (int lo = 0; lo < 8; ++lo) {
                const int kb = lo + 8 * hi;
                if (kb == 0) continue;
                const v2f w = lo ? (hi ? cmul(tlo[lo], thi[hi]) : tlo[lo]) : thi[hi];
                v[perm64(kb)] = cmul(v[perm64(kb)], w);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    // ---- 4. transpose through LDS, in place: re first, then im ----------
    // After the re pass v[a].x is the new re while every v[.].y still holds
    // the old im, so one 64-entry register array suffices.
#pragma unroll
    for (int kb = 0; kb < 64; ++kb) lds[lane * 65u + kb] = v[perm64(kb)].x;
    lds_fence();
#pragma unroll
    for (int a = 0; a < 64; ++a) v[a].x = lds[a * 65 + lane];
    lds_fence();
#pragma unroll
    for (int kb = 0; kb < 64; ++kb) lds[lane * 65u + kb] = v[perm64(kb)].y;
    lds_fence();
#pragma unroll
    for (int a = 0; a < 64; ++a) v[a].y = lds[a * 65 + lane];

    // ---- 5. DFT64 over a: Z[lane + 64 ka] at v[perm64(ka)] --------------
    dft64(v);

    // ---- 6. real split, magnitude, store ---------------------------------
    float *mrow = A.mag.p[c] + f * A.ld;
    const uint32_t src = ((64u - lane) & 63u) * 4u;
    const v2f z0 = v[perm64(0)];
    const v2f wl = A.tw[lane];  // W8192^lane
    v2f prev = z0;
#pragma unroll
    for (int ka = 0; ka < 64; ++ka) {
        if ((ka & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        const v2f zp = v[perm64(63 - ka)];
        v2f t;
        t.x = bperm(src, zp.x);
        t.y = bperm(src, zp.y);
        // lane 0 pairs with itself: Z[(-64 ka) mod 4096] = what lane 0
        // fetched one step earlier (Z[0] at ka = 0).
        const v2f P = (lane == 0) ? (ka == 0 ? z0 : prev) : t;
        prev = t;
        const v2f Z = v[perm64(ka)];
        const v2f cp = v2f{P.x, -P.y};
        const v2f E = 0.5f * (Z + cp);
        const v2f D = 0.5f * (Z - cp);
        const v2f O = v2f{D.y, -D.x};
        const v2f tw = ka == 0 ? wl : cmul(wl, v2f{kW128_re[ka], kW128_im[ka]});  // W8192^k
        const v2f X = E + cmul(tw, O);
        // v_sqrt_f32 (1 ulp): the correctly rounded libm expansion costs ~20 VALU
        const float m = __builtin_amdgcn_sqrtf(X.x * X.x + X.y * X.y) * A.scale;
        if constexpr (KM == kKPartial) {
            const uint32_t k = lane + 64u * (uint32_t)ka;
            if (k < A.K) (mrow + 64u * (uint32_t)ka)[lane] = m;
        } else {
            (mrow + 64u * (uint32_t)ka)[lane] = m;  // k < 4096 always stored
            if constexpr (KM == kKMirror) {
                // |X[8192 - k]| = |X[k]|; lane 0 of ka = 0 writes bin 0 twice
                float *mp = mrow + (8192u - 64u * (uint32_t)ka) - lane;
                (ka == 0 && lane == 0 ? mrow : mp)[0] = m;
            }
        }
    }
    if (lane == 0 && (KM != kKPartial || A.K > 4096u))
        mrow[4096] = __builtin_fabsf(z0.x - z0.y) * A.scale;
}

// ---------------------------------------------------------------------------
// Generic radix-2 Stockham FFT in LDS: one workgroup per transform.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void fft_generic_kernel(GenericFftArgs A) {
    extern __shared__ __attribute__((aligned(16))) v2f smem[];
    const uint32_t n = A.n, half = n >> 1;
    v2f *buf0 = smem, *buf1 = smem + n;
    const uint64_t f = blockIdx.x;
    const uint32_t c = blockIdx.y;

    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        v2f z;
        if (A.mode == 2) {
            float xv = 0.f;
            if (i < A.valid) xv = A.sig.p[c][f * A.frame_hop + i];
            z = v2f{xv * (A.win ? A.win[i] : 1.f), 0.f};
        } else {
            z = v2f{A.re_in[i], A.im_in ? A.im_in[i] : 0.f};
        }
        buf0[i] = z;
    }
    __syncthreads();
    const uint32_t tstride_base = 8192u / n;  // W_n^k = T8192[k * 8192/n]
    for (uint32_t ns = 1, lg = 0; ns < n; ns <<= 1, ++lg) {
        for (uint32_t j = threadIdx.x; j < half; j += blockDim.x) {
            const uint32_t k = j & (ns - 1);
            // W_{2 ns}^k = W_n^{k n / (2 ns)}
            const uint32_t ti = (k << (A.log2n - lg - 1)) * tstride_base;
            v2f w = A.tw[ti];
            if (A.dir > 0) w.y = -w.y;
            const v2f a = buf0[j];
            const v2f b = cmul(buf0[j + half], w);
            const uint32_t o = ((j >> lg) << (lg + 1)) + k;
            buf1[o] = a + b;
            buf1[o + ns] = a - b;
        }
        __syncthreads();
        v2f *t = buf0; buf0 = buf1; buf1 = t;
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const v2f z = buf0[i] * A.scale;
        if (A.mode == 0) {
            A.re_out[i] = z.x;
            A.im_out[i] = z.y;
        } else if (A.mode == 1) {
            A.re_out[i] = z.x;
        } else if (i < A.K) {
            A.mag.p[c][f * A.ld + i] = __builtin_sqrtf(z.x * z.x + z.y * z.y);
        }
    }
}

// ---------------------------------------------------------------------------
// launchers (called from capi.cpp)
// ---------------------------------------------------------------------------
template <int SRC, bool FULL, MapKind MK, bool POW2>
static void launch_km(int km, dim3 grid, dim3 block, hipStream_t stream, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_kernel<SRC, FULL, kKHalf, MK, POW2>), grid, block, 0, stream, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_kernel<SRC, FULL, kKMirror, MK, POW2>), grid, block, 0, stream, A);
    else
        hipLaunchKernelGGL((stft8192_kernel<SRC, FULL, kKPartial, MK, POW2>), grid, block, 0, stream, A);
}

int launch_stft8192(const Stft8kArgs &A, uint32_t C, bool fused, bool full,
                    hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    const uint64_t groups = (A.F + 3) / 4;
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)groups, C), block(256);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_km<kSrcRender, true, MapKind::Noop, true>(km, grid, block, stream, A); break;
        case MapKind::Gain: launch_km<kSrcRender, true, MapKind::Gain, true>(km, grid, block, stream, A); break;
        case MapKind::Ramp:
            if (pow2) launch_km<kSrcRender, true, MapKind::Ramp, true>(km, grid, block, stream, A);
            else launch_km<kSrcRender, true, MapKind::Ramp, false>(km, grid, block, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else if (full) {
        launch_km<kSrcMemory, true, MapKind::Noop, true>(km, grid, block, stream, A);
    } else {
        launch_km<kSrcMemory, false, MapKind::Noop, true>(km, grid, block, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_fft_generic(const GenericFftArgs &A, uint64_t transforms, uint32_t C,
                       hipStream_t stream) {
    if (transforms == 0 || C == 0) return DSP_OK;
    if (transforms > 0x7fffffffull) return DSP_ERR_INVALID;
    const size_t smem = 2u * A.n * sizeof(v2f);
    DSPB_HIP(hipFuncSetAttribute((const void *)fft_generic_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    dim3 grid((uint32_t)transforms, C), block(256);
    hipLaunchKernelGGL(fft_generic_kernel, grid, block, smem, stream, A);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
