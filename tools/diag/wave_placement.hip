// wave_placement.hip -- where the SPI puts the waves of the speculative
// segment kernel's workgroups: a grid of 2 x CUs workgroups of
// 256 threads with ~76 KB of LDS each (two per CU, as dspb_seg_c2b512), every
// wave recording (XCC_ID, HW_ID).  Prints, per CU, which SIMD wave 0 of each
// of its workgroups landed on: the callback lanes of a segment round live in
// wave 0, so two workgroups whose wave 0 share a SIMD share its VALU issue.
// Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/wave_placement tools/diag/wave_placement.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256) void place(unsigned *out, unsigned spins) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = 0.f;
    if ((threadIdx.x & 63u) == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = hw;
        out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = xcc;
    }
    for (unsigned i = 0; i < spins; ++i) __builtin_amdgcn_s_sleep(127);  // stay resident together
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned G = 2 * cus, lds = 75 * 1024;
    unsigned *d;
    (void)hipMalloc(&d, G * 4 * 2 * sizeof(unsigned));
    (void)hipFuncSetAttribute((const void *)place, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(place, dim3(G), dim3(256), lds, 0, d, 2000u);
    (void)hipDeviceSynchronize();
    std::vector<unsigned> h(G * 8);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // per CU: the SIMD of each wave of each workgroup
    std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<std::pair<unsigned, std::vector<unsigned>>>> cu;
    for (unsigned b = 0; b < G; ++b) {
        std::vector<unsigned> simd;
        unsigned key_hw = h[2 * (b * 4)], xcc = h[2 * (b * 4) + 1] & 0xf;
        for (int w = 0; w < 4; ++w) simd.push_back((h[2 * (b * 4 + w)] >> 4) & 3);
        const unsigned cuid = (key_hw >> 8) & 0xf, sh = (key_hw >> 12) & 1, se = (key_hw >> 13) & 7;
        cu[{xcc, se, sh, cuid}].push_back({b, simd});
    }
    unsigned same = 0, pairs = 0, n = 0;
    for (auto &e : cu) {
        if (n++ < 6) {
            std::printf("xcc %u se %u sh %u cu %2u:", std::get<0>(e.first), std::get<1>(e.first), std::get<2>(e.first),
                        std::get<3>(e.first));
            for (auto &w : e.second) std::printf("  wg %4u simd[w0..3] = %u %u %u %u", w.first, w.second[0], w.second[1],
                                                 w.second[2], w.second[3]);
            std::printf("\n");
        }
        if (e.second.size() == 2) {
            ++pairs;
            same += e.second[0].second[0] == e.second[1].second[0];
        }
    }
    std::printf("{\"cus_seen\": %zu, \"cus_with_two_workgroups\": %u, \"wave0_on_the_same_simd\": %u}\n", cu.size(), pairs,
                same);
    return 0;
}
