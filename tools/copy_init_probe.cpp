// Cold-process cost of the first host->device copy, by kind of source
// buffer (the tables the library uploads on its first call are ~77 KB).
//   hipcc --offload-arch=gfx950 -O2 tools/copy_init_probe.cpp -o tools/copy_init_probe
//   for m in 0 1 2 3; do tools/copy_init_probe $m; done
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void poke(float *d, float v) { d[threadIdx.x] = v; }

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t n = 80000;
    double t0 = now_ms();
    (void)hipFree(nullptr);
    printf("mode %d  runtime init %.3f ms\n", mode, now_ms() - t0);
    float *d = nullptr;
    (void)hipMalloc(&d, 1 << 20);
    t0 = now_ms();
    poke<<<1, 64>>>(d, 1.f);
    (void)hipDeviceSynchronize();
    printf("  first kernel           %.3f ms\n", now_ms() - t0);
    std::vector<float> h(n / 4, 1.f);
    if (mode == 0) {
        t0 = now_ms();
        (void)hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
        printf("  first pageable 80 KB   %.3f ms\n", now_ms() - t0);
    } else if (mode == 1) {
        float *p = nullptr;
        t0 = now_ms();
        (void)hipHostMalloc(&p, n, 0);
        printf("  hipHostMalloc 80 KB    %.3f ms\n", now_ms() - t0);
        memcpy(p, h.data(), n);
        t0 = now_ms();
        (void)hipMemcpy(d, p, n, hipMemcpyHostToDevice);
        printf("  first pinned 80 KB     %.3f ms\n", now_ms() - t0);
    } else if (mode == 2) {
        t0 = now_ms();
        (void)hipMemcpy(d, h.data(), 1024, hipMemcpyHostToDevice);
        printf("  first pageable 1 KB    %.3f ms\n", now_ms() - t0);
    } else if (mode == 3) {
        hipStream_t s;
        (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        t0 = now_ms();
        (void)hipMemcpyAsync(d, h.data(), n, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
        printf("  first async pageable   %.3f ms\n", now_ms() - t0);
    }
    t0 = now_ms();
    (void)hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
    printf("  later pageable 80 KB   %.3f ms\n", now_ms() - t0);
    t0 = now_ms();
    (void)hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost);
    printf("  later D2H 80 KB        %.3f ms\n", now_ms() - t0);
    (void)hipFree(d);
    return 0;
}
