// tools/valu_probe.hip -- VALU issue-rate probe: independent v_add_f32 or
// v_pk_add_f32 chains, k waves per SIMD, no memory in the loop.
// Build with -fno-slp-vectorize, or the scalar chains get packed.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(256) void probe(float *out, int iters, float a) {
    if constexpr (PK) {
        v2f x[8];
        for (int i = 0; i < 8; ++i) x[i] = v2f{a + i, a - i};
        const v2f d = v2f{a, a * 0.5f};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = x[i] + d;
        }
        float s = 0;
        for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        float x[8];
        for (int i = 0; i < 8; ++i) x[i] = a + i;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = x[i] + a;
        }
        float s = 0;
        for (int i = 0; i < 8; ++i) s += x[i];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 1024 * 64 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 4096;
    for (int pk = 0; pk < 2; ++pk) {
        for (int wps : {1, 2, 4, 8}) {
            // 256 threads = 4 waves = one per SIMD; wps blocks per CU
            dim3 grid(256 * wps);
            float ms = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (pk) hipLaunchKernelGGL(probe<true>, grid, dim3(256), 0, 0, out, iters, 1e-7f);
                else hipLaunchKernelGGL(probe<false>, grid, dim3(256), 0, 0, out, iters, 1e-7f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            const double instr_per_wave = (double)iters * 128;  // VALU adds per wave
            const double ns_per_instr_simd = ms * 1e6 / (instr_per_wave * wps);
            std::printf("%s waves/SIMD=%d  %.3f ms  %.3f ns per VALU instr per SIMD (%.2f cycles @2.4GHz)\n",
                        pk ? "v_pk_add_f32" : "v_add_f32  ", wps, ms, ns_per_instr_simd, ns_per_instr_simd * 2.4);
        }
    }
    return 0;
}
