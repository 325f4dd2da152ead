// tools/d2h_probe.hip -- device -> pinned host copies: which engine, at what
// rate, and what they cost a kernel running beside them.
//
//   hipcc --offload-arch=gfx950 -O2 tools/d2h_probe.hip -o tools/d2h_probe -lhsa-runtime64
//   ./tools/d2h_probe [MiB]
//
// A "busy" loop (200 launches of an HBM read + write kernel, 4096 workgroups
// each, standing in for the pipeline's chunk kernels) is timed alone and with
// a D2H copy of MiB in flight on another stream, the copy made by
//   memcpy   hipMemcpyAsync (CLR's choice: a blit kernel on the CUs)
//   kernelG  our copy kernel with G workgroups (non-temporal 16-byte stores
//            straight into the pinned host buffer)
//   sdma     hsa_amd_memory_async_copy_on_engine on an SDMA engine
// and H2D (hipMemcpyAsync, SDMA) + D2H of each kind at once (duplex).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)
#define HK(x)                                                                    \
    do {                                                                         \
        hsa_status_t s_ = (x);                                                   \
        if (s_ != HSA_STATUS_SUCCESS) {                                          \
            fprintf(stderr, "%s:%d %s: hsa status 0x%x\n", __FILE__, __LINE__, #x, s_); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

__global__ void busy(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        v.x = v.x * 1.0001f + 1.f;
        b[i] = v;
    }
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void d2h_kernel(f4 *__restrict__ dst, const f4 *__restrict__ src, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        f4 v0 = src[i], v1 = src[i + stride], v2 = src[i + 2 * stride], v3 = src[i + 3 * stride];
        __builtin_nontemporal_store(v0, dst + i);
        __builtin_nontemporal_store(v1, dst + i + stride);
        __builtin_nontemporal_store(v2, dst + i + 2 * stride);
        __builtin_nontemporal_store(v3, dst + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(src[i], dst + i);
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? atoi(argv[1]) : 256;
    const size_t bytes = mib << 20, n4 = bytes / 16;
    float4 *d_src, *d_dst, *ba, *bb, *h_dst, *h_src;
    const size_t busy_n = (64u << 20) / 16;
    CK(hipMalloc(&d_src, bytes));
    CK(hipMalloc(&d_dst, bytes));
    CK(hipMalloc(&ba, busy_n * 16));
    CK(hipMalloc(&bb, busy_n * 16));
    CK(hipHostMalloc(&h_dst, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h_src, bytes, hipHostMallocDefault));
    CK(hipMemset(d_src, 1, bytes));
    CK(hipMemset(ba, 0, busy_n * 16));
    std::memset((void *)h_src, 2, bytes);
    hipStream_t sa, sb, sc;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));

    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    uint32_t mask = 0;
    HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask));
    uint32_t pref = 0;
    (void)hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pref);
    printf("SDMA engines free for D2H: mask 0x%x, preferred 0x%x\n", mask, pref);
    uint32_t mask_up = 0, pref_up = 0;
    (void)hsa_amd_memory_copy_engine_status(g_gpu, g_cpu, &mask_up);
    (void)hsa_amd_memory_get_preferred_copy_engine(g_gpu, g_cpu, &pref_up);
    printf("SDMA engines free for H2D: mask 0x%x, preferred 0x%x\n", mask_up, pref_up);
    if (argc > 2) return 0;  // masks only
    hsa_amd_sdma_engine_id_t eng = (hsa_amd_sdma_engine_id_t)(pref & mask ? (pref & mask & -(pref & mask)) : (mask & -mask));
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));

    auto busy_loop = [&] {
        for (int i = 0; i < 200; ++i) busy<<<4096, 256, 0, sa>>>(ba, bb, busy_n);
    };
    auto d2h_memcpy = [&] { CK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, sb)); };
    int G = 0;
    auto d2h_kernel_ = [&] { d2h_kernel<<<G, 256, 0, sb>>>((f4 *)h_dst, (const f4 *)d_src, n4); };
    auto d2h_sdma = [&] {
        hsa_signal_store_screlease(sig, 1);
        HK(hsa_amd_memory_async_copy_on_engine(h_dst, g_cpu, d_src, g_gpu, bytes, 0, nullptr, sig, eng, true));
    };
    auto wait_d2h = [&](bool sdma) {
        if (sdma) hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        else CK(hipStreamSynchronize(sb));
    };
    auto h2d = [&] { CK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, sc)); };

    // warm everything
    busy_loop();
    d2h_memcpy();
    G = 64;
    d2h_kernel_();
    d2h_sdma();
    wait_d2h(true);
    h2d();
    CK(hipDeviceSynchronize());

    auto t = clk::now();
    busy_loop();
    CK(hipStreamSynchronize(sa));
    const double busy_ms = ms_since(t);
    printf("busy loop alone: %.3f ms\n", busy_ms);

    struct Kind {
        const char *name;
        int G;  // 0: memcpy, -1: sdma
    };
    std::vector<Kind> kinds = {{"memcpy", 0}, {"kernel8", 8}, {"kernel16", 16}, {"kernel32", 32},
                               {"kernel64", 64}, {"kernel128", 128}, {"kernel256", 256}, {"sdma", -1}};
    for (const Kind &k : kinds) {
        G = k.G;
        auto issue = [&] {
            if (k.G == 0) d2h_memcpy();
            else if (k.G > 0) d2h_kernel_();
            else d2h_sdma();
        };
        // D2H alone
        t = clk::now();
        issue();
        wait_d2h(k.G < 0);
        const double alone = ms_since(t);
        // D2H with the busy loop
        t = clk::now();
        issue();
        busy_loop();
        CK(hipStreamSynchronize(sa));
        const double busy_with = ms_since(t);
        wait_d2h(k.G < 0);
        const double copy_with = ms_since(t);
        // H2D + D2H at once
        t = clk::now();
        h2d();
        issue();
        wait_d2h(k.G < 0);
        CK(hipStreamSynchronize(sc));
        const double duplex = ms_since(t);
        printf("%-10s D2H alone %6.1f GB/s | with busy: busy %.3f ms (x%.2f), copy %.3f ms | H2D+D2H %6.1f GB/s total\n",
               k.name, bytes / alone / 1e6, busy_with, busy_with / busy_ms, copy_with, 2 * bytes / duplex / 1e6);
    }
    t = clk::now();
    h2d();
    CK(hipStreamSynchronize(sc));
    printf("H2D alone (hipMemcpyAsync) %6.1f GB/s\n", bytes / ms_since(t) / 1e6);
    hsa_signal_destroy(sig);
    return 0;
}
