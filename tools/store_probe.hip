// tools/store_probe.hip -- HBM write-pattern probe for the headline kernel's
// stores, without its FFT.  Every "frame wave" writes what stft8192_pk_kernel
// writes for one frame: 4096 render floats (16 KB, contiguous) and one
// 4097-float magnitude row at mag + f * ld.  Variants change the store width,
// the row layout (ld), the magnitude lane order and a compute delay between
// the two bursts (s_sleep, standing in for the FFT), at the kernel's own
// occupancy (66.5 KB LDS per 4-wave block -> 2 waves per SIMD).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_probe.hip -o build/store_probe
//   ./build/store_probe            (prints one line per variant, GB/s of 8 TB/s)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
    const uint32_t xcd = bid & 7u, q = nwg >> 3, r = nwg & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

struct Args {
    float *out[2];
    float *mag[2];
    uint64_t F;
    uint32_t ld;
    uint32_t delay;  // s_sleep 64 iterations (each ~64 x 64 cycles)
};

// RW: 2 = dwordx2 render stores (the kernel), 4 = dwordx4
// MAG: 0 = the kernel's dword pieces (forward + reversed), 1 = LDS-staged
//      16-byte pieces, 2 = dwordx4 straight (row must be 16 B aligned: ld % 4 == 0)
// NT: render stores non-temporal
template <int RW, int MAG, bool NT>
__global__ __launch_bounds__(256, 2) void probe(Args A) {
    __shared__ __attribute__((aligned(16))) float lds_all[4][64 * 65];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ch = blockIdx.y;
    const uint64_t f = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (f >= A.F) return;
    float *lds = lds_all[wave];
    const float v = (float)lane * 0.25f + (float)f;
    float *o = A.out[ch] + f * 4096u;
    if constexpr (RW == 2) {
#pragma unroll
        for (int b = 0; b < 32; ++b) {
            v2f t = v2f{v + b, v - b};
            if constexpr (NT) __builtin_nontemporal_store(t, reinterpret_cast<v2f *>(o + 128u * b) + lane);
            else reinterpret_cast<v2f *>(o + 128u * b)[lane] = t;
        }
    } else {
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            v4f t = v4f{v + b, v - b, v * b, v + 2 * b};
            if constexpr (NT) __builtin_nontemporal_store(t, reinterpret_cast<v4f *>(o + 256u * b) + lane);
            else reinterpret_cast<v4f *>(o + 256u * b)[lane] = t;
        }
    }
    for (uint32_t i = 0; i < A.delay; ++i) __builtin_amdgcn_s_sleep(64);
    float *mrow = A.mag[ch] + f * A.ld;
    if constexpr (MAG == 0) {
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) {
            mrow[64u * kk + lane] = v + kk;
            mrow[4096u - 64u * kk - lane] = v - kk;
        }
        if (lane == 0) mrow[2048] = v;
    } else if constexpr (MAG == 1) {
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) {
            lds[64u * kk + lane] = v + kk;
            lds[4096u - 64u * kk - lane] = v - kk;
        }
        if (lane == 0) lds[2048] = v;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 q = reinterpret_cast<const float4 *>(lds)[64 * i + lane];
            *reinterpret_cast<f4u *>(mrow + 256u * i + 4u * lane) = f4u{q.x, q.y, q.z, q.w};
        }
        if (lane == 0) mrow[4096] = lds[4096];
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            reinterpret_cast<float4 *>(mrow + 256u * i)[lane] = float4{v + i, v - i, v, v * i};
        if (lane == 0) mrow[4096] = v;
    }
}

__global__ void fill4(float4 *p, uint64_t n4) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = float4{1.f, 2.f, 3.f, 4.f};
}

template <typename K>
static float timeit(K launch, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) launch();
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const uint64_t F = 84372, L = F * 4096u;
    const uint32_t ldmax = 4224;
    // one allocation: the render rows, then the magnitude rows (the fill
    // probe below writes the same byte count from the start of it)
    const uint64_t total = 2 * L + 2 * F * (uint64_t)ldmax;  // floats
    float *out;
    CK(hipMalloc(&out, total * 4));
    float *mag = out + 2 * L;
    Args A;
    A.out[0] = out; A.out[1] = out + L;
    A.mag[0] = mag; A.mag[1] = mag + F * ldmax;
    A.F = F;
    const double bytes = 2.0 * F * (4096 + 4097) * 4;
    dim3 grid((uint32_t)((F + 3) / 4), 2);
    auto line = [&](const char *name, float ms) {
        printf("%-44s %8.4f ms  %7.1f GB/s  %5.1f%%\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
        fflush(stdout);
    };
    {
        const uint64_t n4 = (uint64_t)(bytes / 16);
        if (n4 * 4 > total) { fprintf(stderr, "fill exceeds the buffer\n"); return 1; }
        line("fill float4 grid-stride (same bytes)", timeit([&] { fill4<<<4096, 256>>>((float4 *)out, n4); }));
    }
    struct V { const char *name; int rw, mag; bool nt; uint32_t ld; };
    const V vs[] = {
        {"kernel: x2 NT render, dword mag, ld 4097", 2, 0, true, 4097},
        {"x2 cached render, dword mag, ld 4097", 2, 0, false, 4097},
        {"x4 NT render, dword mag, ld 4097", 4, 0, true, 4097},
        {"x4 cached render, dword mag, ld 4097", 4, 0, false, 4097},
        {"x2 NT render, LDS x4 mag, ld 4097", 2, 1, true, 4097},
        {"x4 NT render, LDS x4 mag, ld 4097", 4, 1, true, 4097},
        {"x2 NT render, dword mag, ld 4100", 2, 0, true, 4100},
        {"x4 NT render, x4 mag, ld 4100", 4, 2, true, 4100},
        {"x4 NT render, x4 mag, ld 4128", 4, 2, true, 4128},
        {"x4 cached render, x4 mag, ld 4128", 4, 2, false, 4128},
        {"x2 NT render, dword mag, ld 4128", 2, 0, true, 4128},
    };
    for (uint32_t delay : {0u, 4u}) {
        A.delay = delay;
        printf("-- compute delay %u x s_sleep(64)\n", delay);
        for (const V &v : vs) {
            A.ld = v.ld;
            float ms = 0;
#define P(rw, m, nt) ms = timeit([&] { probe<rw, m, nt><<<grid, 256>>>(A); })
            if (v.rw == 2 && v.mag == 0 && v.nt) P(2, 0, true);
            else if (v.rw == 2 && v.mag == 0) P(2, 0, false);
            else if (v.rw == 4 && v.mag == 0 && v.nt) P(4, 0, true);
            else if (v.rw == 4 && v.mag == 0) P(4, 0, false);
            else if (v.rw == 2 && v.mag == 1) P(2, 1, true);
            else if (v.rw == 4 && v.mag == 1) P(4, 1, true);
            else if (v.rw == 4 && v.mag == 2 && v.nt) P(4, 2, true);
            else P(4, 2, false);
#undef P
            CK(hipGetLastError());
            line(v.name, ms);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
