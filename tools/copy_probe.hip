// tools/copy_probe.hip -- streaming-kernel shapes for the gain render (cfg 2:
// y = x * g over 2 x 28.8 M floats, 460.8 MB per pass), timed back to back.
//   hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o tools/copy_probe && ./tools/copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// (a) grid-stride, U float4 per lane in flight, capped grid (the current render_vec_kernel)
template <int U, bool NT>
__global__ __launch_bounds__(256) void gs(const float4 *x, float4 *y, uint64_t n4, float g) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; q + (U - 1) * stride < n4; q += U * stride) {
        float4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = x[q + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 v = make_float4(r[u].x * g, r[u].y * g, r[u].z * g, r[u].w * g);
            if (NT) __builtin_nontemporal_store(v.x, &y[q + u * stride].x), __builtin_nontemporal_store(v.y, &y[q + u * stride].y),
                    __builtin_nontemporal_store(v.z, &y[q + u * stride].z), __builtin_nontemporal_store(v.w, &y[q + u * stride].w);
            else y[q + u * stride] = v;
        }
    }
    for (; q < n4; q += stride) y[q] = make_float4(x[q].x * g, x[q].y * g, x[q].z * g, x[q].w * g);
}

typedef float f4v __attribute__((ext_vector_type(4)));
// (b) one tile of 256 * U float4 per block, no loop, grid = n4 / (256 U)
template <int U, bool NT, bool NTL>
__global__ __launch_bounds__(256) void tile(const f4v *x, f4v *y, uint64_t n4, float g) {
    const uint64_t base = (uint64_t)blockIdx.x * 256u * U + threadIdx.x;
    f4v r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t i = base + 256u * u;
        if (i < n4) r[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t i = base + 256u * u;
        if (i < n4) {
            const f4v v = r[u] * g;
            if (NT) __builtin_nontemporal_store(v, y + i);
            else y[i] = v;
        }
    }
}

int main() {
    const uint64_t n = 2ull * 28800000ull, n4 = n / 4;
    // NB = 6 input/output buffer pairs used in rotation (2.76 GB): no pass finds
    // its input in the 256 MiB Infinity Cache (one pair: NT stores leave the
    // 230 MB input resident and the "HBM" rate exceeds 8 TB/s)
    const int NB = 6;
    float *xs[NB], *ys[NB];
    for (int b = 0; b < NB; ++b) {
        CK(hipMalloc(&xs[b], n * 4));
        CK(hipMalloc(&ys[b], n * 4));
        CK(hipMemset(xs[b], 0, n * 4));
    }
    float *x = xs[0], *y = ys[0];
    int cur = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto rot = [&] {
        cur = (cur + 1) % NB;
        x = xs[cur];
        y = ys[cur];
    };
    auto run = [&](const char *name, auto launch0) -> int {
        auto launch = [&] { rot(); launch0(); };
        for (int i = 0; i < 50; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int it = 200;
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-34s %8.2f us  %6.3f TB/s\n", name, us, n * 8.0 / (us * 1e-6) / 1e12);
        return 0;
    };
    const float g = 0.2f;
#define xv reinterpret_cast<const f4v *>(x)
#define yv reinterpret_cast<f4v *>(y)
#define x4 reinterpret_cast<const float4 *>(x)
#define y4 reinterpret_cast<float4 *>(y)
    for (int rep = 0; rep < 2; ++rep) {
        if (rep == 1) {  // one buffer pair: the cache-resident case
            for (int b = 1; b < NB; ++b) xs[b] = xs[0], ys[b] = ys[0];
            printf("-- one buffer pair (input can stay in the Infinity Cache)\n");
        }
        run("gs U4 grid 2048", [&] { hipLaunchKernelGGL((gs<4, false>), dim3(2048), dim3(256), 0, 0, x4, y4, n4, g); });
        run("gs U4 grid 4096", [&] { hipLaunchKernelGGL((gs<4, false>), dim3(4096), dim3(256), 0, 0, x4, y4, n4, g); });
        run("gs U8 grid 2048", [&] { hipLaunchKernelGGL((gs<8, false>), dim3(2048), dim3(256), 0, 0, x4, y4, n4, g); });
        run("gs U4 grid 2048 NT", [&] { hipLaunchKernelGGL((gs<4, true>), dim3(2048), dim3(256), 0, 0, x4, y4, n4, g); });
        auto tl = [&](auto kern, int U) {
            const uint32_t gr = (uint32_t)((n4 + 256u * U - 1) / (256u * U));
            hipLaunchKernelGGL(kern, dim3(gr), dim3(256), 0, 0, xv, yv, n4, g);
        };
        run("tile U4", [&] { tl(tile<4, false, false>, 4); });
        run("tile U8", [&] { tl(tile<8, false, false>, 8); });
        run("tile U16", [&] { tl(tile<16, false, false>, 16); });
        run("tile U4 NT store", [&] { tl(tile<4, true, false>, 4); });
        run("tile U8 NT store", [&] { tl(tile<8, true, false>, 8); });
        run("tile U8 NT load+store", [&] { tl(tile<8, true, true>, 8); });
        run("tile U16 NT store", [&] { tl(tile<16, true, false>, 16); });
    }
    return 0;
}
