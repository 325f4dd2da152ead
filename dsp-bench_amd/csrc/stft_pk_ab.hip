// stft_pk_ab.hip -- the A/B and ablation instantiations of
// stft8192_pk_kernel (stft_pk.hpp options, dsp_stft_soa_options >> 4): the
// headline shape (IR_test, B = 512), the memory-source kPkMemAos path and the
// persistent LDS-prefetch memory kernel (kPkMemPf, stft8192_mem_pf_kernel).
// Kept in their own code object: loaded only when an option is selected.
#include "stft_pk.hpp"

namespace dspb {

// Memory-source STFT (4097 bins, computed window, H = 4096, every frame
// whole) on a persistent grid: wave w takes units u = w, w + W, ... of the
// (channel, frame) sequence, and while frame u's second DFT64 and real split
// run, the first hop of frame u + W travels into the wave's LDS tile (free
// once the transpose's reads are done) as 16 global_load_lds_dwordx4.  At the
// next frame only the second hop is loaded into VGPRs -- the first hop of
// the neighbouring wave's frame, fetched into L2 one frame earlier.  The
// arithmetic is stft8192_pk_kernel's MSOA path, instruction for instruction.
__device__ __forceinline__ void pf_hop(const float *src, float *lds, uint32_t lane) {
    typedef __attribute__((address_space(3))) float lfloat;
    typedef __attribute__((address_space(3))) void lvoid;
    lfloat *l3 = (lfloat *)lds;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_global_load_lds((const void *)(src + 256u * (uint32_t)i + 4u * lane), (lvoid *)(l3 + 256 * i),
                                         16, 0, 0);
}

template <int OPT = 0>
__global__ __launch_bounds__(256, 2) void stft8192_mem_pf_kernel(Stft8kArgs A, uint32_t nch) {
    __shared__ __attribute__((aligned(16))) float lds_all[4][64 * 65];
    __shared__ float4 wuv[4][64];  // the lane's window coefficients, read back per frame
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * 4u;
    const uint64_t U = A.F * nch;
    uint64_t u = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u + wave;
    if (u >= U) return;
    float *lds = lds_all[wave];
    cx tlo[8];
    cx2 thp[4];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
        const v2f a = (A.tw + 8192u + 64u * (uint32_t)(j - 1))[lane];
        tlo[j] = cx{a.x, a.y};
    }
    {
        const float4 *tp4 = reinterpret_cast<const float4 *>(A.tw + 8192u + 896u);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const float4 t = tp4[64u * (uint32_t)h + lane];
            thp[h] = cx2{v2f{t.x, t.y}, v2f{t.z, t.w}};
        }
    }
    {
        const float4 wbase = A.wbase[lane];
        wuv[wave][lane] = float4{A.wb * wbase.x, A.wb * wbase.y, A.wb * wbase.z, A.wb * wbase.w};
    }
    // (channel, frame) of unit u, stepped by W without a division per frame
    // (host: F C < 2^32)
    const uint32_t F = (uint32_t)A.F, Wn = (uint32_t)W;
    uint32_t c = (uint32_t)u / F, f = (uint32_t)u - c * F;
    pf_hop(A.in.p[c] + (uint64_t)f * 4096u, lds, lane);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the first frame's first hop
    for (;;) {
        const float *x = A.in.p[c] + (uint64_t)f * 4096u;
        uint32_t cn = c, fn = f + Wn;
        while (fn >= F) {  // wave-uniform
            fn -= F;
            ++cn;
        }
        // opaque per frame: the window stays computed inside the loop (hoisted,
        // its 128 values would spill)
        // (an LDS read: kept in VGPRs they spill, and the reload's vmcnt(0)
        // would wait for the previous frame's stores)
        const float4 wl4 = wuv[wave][lane];
        float ue = wl4.x, ve = wl4.y, uo = wl4.z, vo = wl4.w;
        asm volatile("" : "+v"(ue), "+v"(ve), "+v"(uo), "+v"(vo));
        // likewise the stage twiddles (their products) and the split's table
#pragma unroll
        for (int j = 1; j < 8; ++j) asm volatile("" : "+v"(tlo[j].r), "+v"(tlo[j].i));
#pragma unroll
        for (int h = 0; h < 4; ++h) asm volatile("" : "+v"(thp[h].r), "+v"(thp[h].i));
        const v2f *tw = A.tw;
        asm volatile("" : "+s"(tw));
        cx2 P[32];
        // the second hop from global (in flight while the first is read from LDS)
        v2f ga[16], gb[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            ga[j] = reinterpret_cast<const v2f *>(x + 4096u + 256u * (uint32_t)j)[lane];
            gb[j] = reinterpret_cast<const v2f *>(x + 4096u + 256u * (uint32_t)j + 128u)[lane];
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const v2f C = v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}, S = v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]};
            const v2f we = (v2f{ve, ve} * S + v2f{A.wa, A.wa}) - v2f{ue, ue} * C;
            const v2f wo = (v2f{vo, vo} * S + v2f{A.wa, A.wa}) - v2f{uo, uo} * C;
            v2f a, b;
            if (j < 16) {
                a = reinterpret_cast<const v2f *>(lds + 256u * (uint32_t)j)[lane];
                b = reinterpret_cast<const v2f *>(lds + 256u * (uint32_t)j + 128u)[lane];
            } else {
                a = ga[j - 16];
                b = gb[j - 16];
            }
            P[j] = cx2{v2f{a.x, b.x} * we, v2f{a.y, b.y} * wo};
        }
        const uint64_t un = u + W;
        const bool more = un < U;
        cx2 Y2[32];
        fft4096_pk_y2<true, true>(P, lds, tlo, thp, lane, Y2, [&]() {
            if (more) pf_hop(A.in.p[cn] + (uint64_t)fn * 4096u, lds, lane);
        });
        // the prefetch lands before the split's stores are issued, so the
        // wait below covers it alone
        __builtin_amdgcn_s_waitcnt(0x0f70);
        split_y2<kKHalf, true>(Y2, A.mag.p[c] + f * A.ld, A.K, tw, lane, lds);
        if (!more) break;
        u = un;
        c = cn;
        f = fn;
    }
}


// Memory-source STFT with the hops staged once per workgroup (A/B, opt
// kPkMemHop): the four waves of a workgroup take frames f0 .. f0 + 3, which
// span five hops; wave w copies hop w (wave 0 also hop 4) from HBM into LDS
// with 16 global_load_lds_dwordx4, and after a barrier every wave reads its
// two hops from LDS instead of loading 32 KB per frame (half of it the
// neighbour's hop again, from L2).  A second barrier frees the 80 KB for the
// transpose tiles.  The arithmetic is stft8192_pk_kernel's MSOA path.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stft8192_mem_hop_kernel(Stft8kArgs A) {
    __shared__ __attribute__((aligned(16))) float lds_all[5 * 4096];  // 5 hops, then 4 tiles of 64 x 65
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ch = blockIdx.y;
    const uint64_t f0 = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * 4u;
    const uint32_t nf = (uint32_t)(A.F - f0 < 4u ? A.F - f0 : 4u);  // frames of this group, >= 1
    const float *x = A.in.p[ch];
    if (wave <= nf) pf_hop(x + (f0 + wave) * 4096u, lds_all + wave * 4096u, lane);
    if (wave == 0 && nf == 4) pf_hop(x + (f0 + 4u) * 4096u, lds_all + 4u * 4096u, lane);
    cx tlo[8];
    cx2 thp[4];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
        const v2f a = (A.tw + 8192u + 64u * (uint32_t)(j - 1))[lane];
        tlo[j] = cx{a.x, a.y};
    }
    {
        const float4 *tp4 = reinterpret_cast<const float4 *>(A.tw + 8192u + 896u);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const float4 t = tp4[64u * (uint32_t)h + lane];
            thp[h] = cx2{v2f{t.x, t.y}, v2f{t.z, t.w}};
        }
    }
    const float4 wbase = A.wbase[lane];
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's hop copies have landed
    __syncthreads();
    cx2 P[32];
    if (wave < nf) {
        const float *fr = lds_all + wave * 4096u;
        const float ue = A.wb * wbase.x, ve = A.wb * wbase.y, uo = A.wb * wbase.z, vo = A.wb * wbase.w;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const v2f C = v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}, S = v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]};
            const v2f we = (v2f{ve, ve} * S + v2f{A.wa, A.wa}) - v2f{ue, ue} * C;
            const v2f wo = (v2f{vo, vo} * S + v2f{A.wa, A.wa}) - v2f{uo, uo} * C;
            const v2f a = reinterpret_cast<const v2f *>(fr + 256u * (uint32_t)j)[lane];
            const v2f b = reinterpret_cast<const v2f *>(fr + 256u * (uint32_t)j + 128u)[lane];
            P[j] = cx2{v2f{a.x, b.x} * we, v2f{a.y, b.y} * wo};
        }
    }
    __syncthreads();  // every frame is in VGPRs: the LDS holds the transpose tiles from here
    if (wave >= nf) return;
    float *lds = lds_all + wave * (64u * 65u);
    cx2 Y2[32];
    fft4096_pk_y2<false, false>(P, lds, tlo, thp, lane, Y2);
    split_y2<kKHalf, false>(Y2, A.mag.p[ch] + (f0 + wave) * A.ld, A.K, A.tw, lane, lds);
}

static int launch_mem_hop(const Stft8kArgs &A, uint32_t C, hipStream_t stream) {
    // H = 4096, whole frames, 4097 bins, 16-byte rows (the kernel's addressing)
    if (A.H != 4096u || A.valid < 8192u || A.K != 4097u || !A.wbase || A.in_ch < C) return DSP_ERR_INVALID;
    for (uint32_t c = 0; c < C; ++c)
        if (reinterpret_cast<uintptr_t>(A.in.p[c]) & 15u) return DSP_ERR_INVALID;
    const uint64_t groups = (A.F + 3) / 4;
    hipLaunchKernelGGL(stft8192_mem_hop_kernel, dim3((uint32_t)groups, C), dim3(256), 0, stream, A);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

static int launch_mem_pf(const Stft8kArgs &A, uint32_t C, hipStream_t stream) {
    // H = 4096 and whole frames only (the kernel's addressing)
    if (A.H != 4096u || A.valid < 8192u || A.K != 4097u || !A.wbase) return DSP_ERR_INVALID;
    int dev = 0, cus = 0;
    DSPB_HIP(hipGetDevice(&dev));
    DSPB_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t units = A.F * C, groups = (units + 3) / 4;
    const uint32_t g = (uint32_t)(groups < 2ull * (uint64_t)cus ? groups : 2ull * (uint64_t)cus);
    hipLaunchKernelGGL(stft8192_mem_pf_kernel<0>, dim3(g), dim3(256), 0, stream, A, C);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

static int launch_pk_ab(const Stft8kArgs &A, bool fused, int opt, dim3 grid_default, hipStream_t stream) {
    // the variants below are four-wave workgroups; grid_default is sized for kPkWpb
    const dim3 grid((grid_default.x * kPkWpb + 3) / 4, grid_default.y);
    if (!fused) {  // kPkMemAos
        hipLaunchKernelGGL((stft8192_pk_kernel<kSrcMemory, kKHalf, MapKind::Noop, true, true, 0, kPkMemAos>), grid,
                           dim3(256), 0, stream, A);
        DSPB_HIP(hipGetLastError());
        return DSP_OK;
    }
    if (opt & kPkOcc3) {
        switch (opt & ~kPkOcc3) {
        case 0:
            hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, 4, 0, 3>), grid,
                               dim3(256), 0, stream, A);
            break;
        case kPkRenderCached:
            hipLaunchKernelGGL(
                (stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, 4, kPkRenderCached, 3>), grid,
                dim3(256), 0, stream, A);
            break;
        case kPkAbNoRender | kPkAbNoMag:
            hipLaunchKernelGGL(
                (stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, 4, kPkAbNoRender | kPkAbNoMag, 3>),
                grid, dim3(256), 0, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
        DSPB_HIP(hipGetLastError());
        return DSP_OK;
    }
    if (opt & kPkW1) {  // one-wave workgroups, as the product's PER kernel: one group per frame
        const uint64_t tail = A.tail_end > A.F * A.H ? (A.tail_end - A.F * A.H + A.H - 1) / A.H : 0;
        const dim3 g1((uint32_t)(A.F + tail), grid_default.y);
        switch (opt) {
#define DSPB_PK_W1(o)                                                                                            \
    case (o):                                                                                                    \
        hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, 4, (o)>), g1, dim3(64), \
                           0, stream, A);                                                                        \
        break
            DSPB_PK_W1(kPkPerOpt | kPkMagStage);
            DSPB_PK_W1(kPkPerOpt | kPkMagStage | kPkNtMag);
            DSPB_PK_W1(kPkPerOpt | kPkNtMag);
            DSPB_PK_W1(kPkPerOpt | kPkRenderCached);
#undef DSPB_PK_W1
        default: return DSP_ERR_INVALID;
        }
        DSPB_HIP(hipGetLastError());
        return DSP_OK;
    }
    switch (opt) {
#define DSPB_PK_CASE(o)                                                                                     \
    case (o):                                                                                               \
        hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, 4, (o)>), grid, \
                           dim3(256), 0, stream, A);                                                        \
        break
        DSPB_PK_CASE(kPkNoBarDft);
        DSPB_PK_CASE(kPkNoBarTw);
        DSPB_PK_CASE(kPkNoBarSplit);
        DSPB_PK_CASE(kPkNoBarDft | kPkNoBarTw | kPkNoBarSplit);
        DSPB_PK_CASE(kPkRenderCached);
        DSPB_PK_CASE(kPkMagStage);
        DSPB_PK_CASE(kPkMagStage | kPkRenderCached);
        DSPB_PK_CASE(kPkMagStage | kPkNtMag);
        DSPB_PK_CASE(kPkNtMag);
        DSPB_PK_CASE(kPkNoRemap);
        DSPB_PK_CASE(kPkAbNoXpose);
        DSPB_PK_CASE(kPkAbNoXpose | kPkAbNoRender | kPkAbNoMag);
        DSPB_PK_CASE(kPkOldSplit);
        DSPB_PK_CASE(kPkOldSplit | kPkRenderCached);
        DSPB_PK_CASE(kPkOldSplit | kPkNtMag);
        DSPB_PK_CASE(kPkOldSplit | kPkRenderCached | kPkNtMag);
        DSPB_PK_CASE(kPkMagLds);
        DSPB_PK_CASE(kPkMagLds | kPkRenderCached);
        DSPB_PK_CASE(kPkMagLds | kPkNtMag);
        DSPB_PK_CASE(kPkMagLds | kPkRenderCached | kPkNtMag);
        DSPB_PK_CASE(kPkAbNoRender);
        DSPB_PK_CASE(kPkAbNoMag);
        DSPB_PK_CASE(kPkAbNoRender | kPkAbNoMag);
#undef DSPB_PK_CASE
    default: return DSP_ERR_INVALID;
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

// the product's weak hooks (stft_pk.hip), defined here for the tools build
bool stft_pk_ab_dispatch(const Stft8kArgs &A, uint32_t C, bool fused, int opt, dim3 grid, hipStream_t stream,
                         int *st) {
    if (fused) {
        *st = launch_pk_ab(A, fused, opt, grid, stream);
        return true;
    }
    if (opt & kPkMemPf) *st = launch_mem_pf(A, C, stream);
    else if (opt & kPkMemHop) *st = launch_mem_hop(A, C, stream);
    else if (opt & kPkMemAos) *st = launch_pk_ab(A, fused, opt, grid, stream);
    else return false;
    return true;
}

// A/B and ablation options of stft8192_pk_kernel (stft_pk.hpp kPk* bits),
// thread local: a thread's A/B switch never changes another thread's kernel
static thread_local int g_pk_ab_opt = 0;
int stft_pk_ab_options() { return g_pk_ab_opt; }

}  // namespace dspb

extern "C" int dsp_stft_pk_ab_options(int opt) {
    const int old = dspb::g_pk_ab_opt;
    if (opt >= 0 && opt <= 0x3fffff) dspb::g_pk_ab_opt = opt;
    return old;
}
