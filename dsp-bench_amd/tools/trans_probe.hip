// tools/trans_probe.hip -- what a v_sqrt_f32 costs a wave beside packed FMAs.
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/trans_probe.hip -o /tmp/trans_probe
//
// Each wave runs R rounds of 8 independent chains and times itself with
// s_memtime (shader clock cycles): only v_pk_fma_f32, only v_sqrt_f32, and
// 7 pk_fma + 1 sqrt per chain step (does the transcendental issue beside the
// packed math or in its place?).  One to four waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(unsigned long long *cyc, float *out, int rounds, float a) {
    v2f x[8];
    float y[8];
    for (int i = 0; i < 8; ++i) {
        x[i] = v2f{a + i, a - i};
        y[i] = 1.0f + a * i;
    }
    const v2f m = v2f{0.999f, 0.998f}, c = v2f{a, a * 0.5f};
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
                for (int k = 0; k < (MODE == 0 ? 8 : 7); ++k) x[i] = x[i] * m + c;
            }
            if constexpr (MODE == 1) {
#pragma unroll
                for (int k = 0; k < 8; ++k) y[i] = __builtin_amdgcn_sqrtf(y[i] + 1.0f);
            }
            if constexpr (MODE == 2) y[i] = __builtin_amdgcn_sqrtf(y[i] + 1.0f);
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y + y[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int wps) {
    const int rounds = 2048, blocks = 256 * wps;
    unsigned long long *cyc;
    float *out;
    hipMalloc(&cyc, blocks * 4 * sizeof(unsigned long long));
    hipMalloc(&out, blocks * 256 * sizeof(float));
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, cyc, out, rounds, 1e-7f);
    hipDeviceSynchronize();
    unsigned long long h[4096];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks * 4; ++i) avg += (double)h[i];
    avg /= blocks * 4;
    // instructions per wave: 64 per round (8 chains x 8 steps), plus the sqrt's add in modes 1 / 2
    const double per = rounds * 64.0;
    std::printf("%-28s waves/SIMD=%d  %.2f cycles per chain step (of 8 per round x 8 chains)\n", name, wps, avg / per);
    hipFree(cyc);
    hipFree(out);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<0>("8 v_pk_fma", w);
        run<1>("8 (v_add + v_sqrt)", w);
        run<2>("7 v_pk_fma + 1 (add+sqrt)", w);
    }
    return 0;
}
