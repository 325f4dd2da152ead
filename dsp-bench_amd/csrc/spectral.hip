// spectral.hip -- the generic LDS FFT of the windowed-FFT / magnitude path.
//
// fft_generic_kernel: one workgroup per transform, radix-2 Stockham in LDS,
// any power of two <= 8192, forward or inverse.  It serves fft_forward /
// fft_reverse (the plugin services, dsp.cpp:74-132, split re/im with
// DIV_BY_SQRTN), STFTs with N != 8192 and IR analyses with other IR lengths
// (windowing_hamming -> FFT -> pythagore_array, dsp.cpp:53-72, 166-168).
// These are latency-bound single frames or small batches.  The 8192-point
// hot path is stft8192_pk_kernel (stft_pk.hpp).
#include "kernels.hpp"
#include "fft_device.hpp"

namespace dspb {

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
// launcher (called from capi.cpp)
// ---------------------------------------------------------------------------
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
