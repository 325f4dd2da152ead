// tools/stamps.hip -- DIAGNOSTIC build of the SoA STFT kernel with phase
// clocks (-DDSPB_STAMPS).  Never linked into libdspbench; its timings are
// for phase SHARES only (the stamps themselves fence the schedule).
//   build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -DDSPB_STAMPS
//          -I../include -Icsrc tools/stamps.hip -o build/stamps
//   ablation set: bash tools/build_ablation.sh <opt>  (build/stamps_ab<mask>)
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstdlib>

#ifndef STAMP_OPT
#define STAMP_OPT 0
#endif
#include "stft_soa.hip"

namespace dspb {
void set_last_error(const char *, ...) {}
int hip_fail(hipError_t e, const char *what) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    return DSP_ERR_HIP;
}
}  // namespace dspb

using namespace dspb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const uint64_t L = 48000ull * 3600;  // 1 h @ 48 kHz
    const uint32_t C = 2, B = 512, H = 4096, N = 8192;
    uint64_t F = (L - N) / H + 1;
    if (argc > 1) F = std::min<uint64_t>(F, strtoull(argv[1], nullptr, 10));
    float *out[2], *mag[2], *table, *win;
    v2f *tw;
    uint64_t *stamps;
    for (int c = 0; c < 2; ++c) {
        CK(hipMalloc(&out[c], L * 4));
        CK(hipMalloc(&mag[c], F * 4097 * 4));
    }
    std::vector<float> ht(B);
    double g = 0.9f;
    for (uint32_t i = 0; i < B; ++i) { ht[i] = (float)g; g -= (double)0.002f; }
    CK(hipMalloc(&table, B * 4));
    CK(hipMemcpy(table, ht.data(), B * 4, hipMemcpyHostToDevice));
    std::vector<v2f> htw(8192);
    for (int k = 0; k < 8192; ++k) htw[k] = v2f{(float)cos(-2 * M_PI * k / 8192), (float)sin(-2 * M_PI * k / 8192)};
    for (int j = 1; j < 8; ++j)  // lane-major stage twiddles (as capi.cpp get_tw)
        for (int l = 0; l < 64; ++l) htw.push_back(htw[(2 * l * j) & 8191]);
    for (int j = 1; j < 8; ++j)
        for (int l = 0; l < 64; ++l) htw.push_back(htw[(16 * l * j) & 8191]);
    CK(hipMalloc(&tw, htw.size() * 8));
    CK(hipMemcpy(tw, htw.data(), htw.size() * 8, hipMemcpyHostToDevice));
    std::vector<float4> hb(64);
    const double th = 2.0 * M_PI / 8191.0;
    for (int l = 0; l < 64; ++l)
        hb[l] = float4{(float)cos(th * 2 * l), (float)sin(th * 2 * l), (float)cos(th * (2 * l + 1)),
                       (float)sin(th * (2 * l + 1))};
    float4 *wbase;
    CK(hipMalloc(&wbase, 64 * sizeof(float4)));
    CK(hipMemcpy(wbase, hb.data(), 64 * sizeof(float4), hipMemcpyHostToDevice));
    std::vector<float> hw(N);
    for (uint32_t n = 0; n < N; ++n) hw[n] = (float)(0.5 / sqrt(8192.0) * (0.5 - 0.5 * cos(2 * M_PI * n / (N - 1))));
    CK(hipMalloc(&win, N * 4));
    CK(hipMemcpy(win, hw.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&stamps, F * 8 * 8 * C));

    Stft8kArgs A{};
    A.in_ch = 0;
    A.L = L;
    for (int c = 0; c < 2; ++c) { A.out.p[c] = out[c]; A.mag.p[c] = mag[c]; }
    A.F = F; A.H = H; A.K = 4097; A.ld = 4097; A.valid = N;
    A.win2 = reinterpret_cast<const v2f *>(win);
    A.tw = tw;
    A.wbase = wbase;
    A.wa = (float)(0.5 * 0.5 / sqrt(8192.0));
    A.wb = A.wa;
    A.map.kind = MapKind::Ramp; A.map.table = table; A.map.B = B; A.map.b_mask = B - 1;
    A.stamps = stamps;
    dim3 grid((uint32_t)((F + 3) / 4), 1);  // one channel: stamps indexed by frame
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((stft8192_soa_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, STAMP_OPT>), grid, dim3(256), 0, 0, A);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
    }
    std::vector<uint64_t> hs(F * 8);
    CK(hipMemcpy(hs.data(), stamps, F * 8 * 8, hipMemcpyDeviceToHost));
    const char *names[6] = {"load+window", "dft64 #1", "twiddle", "transpose", "dft64 #2", "split+store"};
    double sum[6] = {0}, tot = 0;
    uint64_t tmin = ~0ull, tmax = 0;
    for (uint64_t f = 0; f < F; ++f) {
        const uint64_t *t = &hs[f * 8];
        for (int i = 0; i < 6; ++i) sum[i] += (double)(t[i + 1] - t[i]);
        tot += (double)(t[6] - t[0]);
        tmin = std::min(tmin, t[0]);
        tmax = std::max(tmax, t[6]);
    }
    std::printf("kernel %.4f ms (1 channel, %llu frames, stamped build)\n", ms, (unsigned long long)F);
    std::printf("mean wave lifetime %.0f cycles; span %llu cycles\n", tot / F, (unsigned long long)(tmax - tmin));
    for (int i = 0; i < 6; ++i) std::printf("  %-12s %8.0f cycles  %5.1f %%\n", names[i], sum[i] / F, 100.0 * sum[i] / tot);
    return 0;
}
