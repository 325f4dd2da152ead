// display.hip -- overview reductions for long files.
//
// minmax_decimate: the IR / waveform view's per-pixel (max, min), restating
// opengl.h:877-890 -- every pixel starts at {max = -1, min = +1} and sample
// s belongs to pixel s * P / n (64-bit here; the reference's u32 product
// wraps for long files).  Pixel p owns the contiguous samples
// [ceil(p n / P), ceil((p + 1) n / P)), so one workgroup reduces one pixel's
// run of samples: a streaming HBM read.
//
// spectrogram_decimate: columns of a long STFT for an overview image,
// out[p][k] = max over the frames of column p of |X_f[k]| (the reference
// draws one 4096-bin spectrum, draw.h:150-160; this is its long-file form).
#include "kernels.hpp"

namespace dspb {

__device__ __forceinline__ uint64_t first_of(uint64_t p, uint64_t n, uint64_t P) {
    return (p * n + P - 1) / P;
}

__global__ __launch_bounds__(256) void minmax_kernel(const float *x, uint64_t n, uint32_t P, float *vmax,
                                                     float *vmin) {
    __shared__ float smax[256], smin[256];
    for (uint32_t p = blockIdx.x; p < P; p += gridDim.x) {
        const uint64_t s0 = first_of(p, n, P), s1 = first_of(p + 1ull, n, P);
        float mx = -1.f, mn = 1.f;  // the reference's initial values
        uint64_t s = s0;
        // scalar head up to 16-B alignment, float4 body, scalar tail
        const uint64_t a = ((s0 + 3) & ~3ull) < s1 ? ((s0 + 3) & ~3ull) : s1;
        for (uint64_t i = s + threadIdx.x; i < a; i += blockDim.x) {
            mx = fmaxf(mx, x[i]);
            mn = fminf(mn, x[i]);
        }
        s = a;
        const uint64_t nv = (s1 - s) / 4;
        const float4 *x4 = reinterpret_cast<const float4 *>(x + s);
        for (uint64_t i = threadIdx.x; i < nv; i += blockDim.x) {
            const float4 v = x4[i];
            mx = fmaxf(fmaxf(mx, v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
            mn = fminf(fminf(mn, v.x), fminf(v.y, fminf(v.z, v.w)));
        }
        for (uint64_t i = s + 4 * nv + threadIdx.x; i < s1; i += blockDim.x) {
            mx = fmaxf(mx, x[i]);
            mn = fminf(mn, x[i]);
        }
        smax[threadIdx.x] = mx;
        smin[threadIdx.x] = mn;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) {
                smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + w]);
                smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + w]);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            vmax[p] = smax[0];
            vmin[p] = smin[0];
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void spectro_kernel(const float *mag, uint64_t F, uint32_t K, uint64_t ld,
                                                      uint32_t P, float *out) {
    const uint32_t k = blockIdx.y * blockDim.x + threadIdx.x;
    if (k >= K) return;
    for (uint32_t p = blockIdx.x; p < P; p += gridDim.x) {
        const uint64_t f0 = first_of(p, F, P), f1 = first_of(p + 1ull, F, P);
        float m = 0.f;
        for (uint64_t f = f0; f < f1; ++f) m = fmaxf(m, mag[f * ld + k]);
        out[(uint64_t)p * K + k] = m;
    }
}

int launch_minmax(const float *x, uint64_t n, uint32_t P, float *vmax, float *vmin, hipStream_t s) {
    if (P == 0) return DSP_OK;
    const uint32_t g = P < 65535u ? P : 65535u;
    hipLaunchKernelGGL(minmax_kernel, dim3(g), dim3(256), 0, s, x, n, P, vmax, vmin);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_spectro(const float *mag, uint64_t F, uint32_t K, uint64_t ld, uint32_t P, float *out,
                   hipStream_t s) {
    if (P == 0 || K == 0) return DSP_OK;
    const uint32_t g = P < 65535u ? P : 65535u;
    hipLaunchKernelGGL(spectro_kernel, dim3(g, (K + 255) / 256), dim3(256), 0, s, mag, F, K, ld, P, out);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
