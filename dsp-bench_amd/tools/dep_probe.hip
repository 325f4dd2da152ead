// tools/dep_probe.hip -- issue cost of DEPENDENT packed FP32 math on gfx950.
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/dep_probe.hip -o tools/dep_probe
//
// Each wave runs rounds of NCH independent v_pk_fma_f32 chains, interleaved
// (chain 0 step, chain 1 step, ...), and times itself with s_memtime: with
// NCH = 1 every instruction waits for the previous one, so the cycles per
// instruction are the dependent-issue latency; with enough chains, the
// issue rate.  One and two waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

template <int NCH>
__global__ __launch_bounds__(256) void probe(unsigned long long *cyc, float *out, int rounds, float a) {
    v2f x[NCH];
    for (int i = 0; i < NCH; ++i) x[i] = v2f{a + i, a - i};
    const v2f m = v2f{0.999f, 0.998f}, c = v2f{a, a * 0.5f};
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int k = 0; k < 64 / NCH; ++k) {
#pragma unroll
            for (int i = 0; i < NCH; ++i) x[i] = x[i] * m + c;
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0;
    for (int i = 0; i < NCH; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int NCH>
void run(int wps) {
    const int rounds = 2048, blocks = 256 * wps;
    unsigned long long *cyc;
    float *out;
    (void)hipMalloc(&cyc, blocks * 4 * sizeof(unsigned long long));
    (void)hipMalloc(&out, blocks * 256 * sizeof(float));
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(probe<NCH>, dim3(blocks), dim3(256), 0, 0, cyc, out, rounds, 1e-7f);
    (void)hipDeviceSynchronize();
    static unsigned long long h[8192];
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks * 4; ++i) avg += (double)h[i];
    avg /= blocks * 4;
    std::printf("chains=%2d waves/SIMD=%d  %.2f cycles per v_pk_fma_f32 per wave\n", NCH, wps, avg / (rounds * 64.0));
    (void)hipFree(cyc);
    (void)hipFree(out);
}

int main() {
    for (int w : {1, 2}) {
        run<1>(w);
        run<2>(w);
        run<4>(w);
        run<8>(w);
    }
    return 0;
}
