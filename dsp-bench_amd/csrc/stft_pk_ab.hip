// stft_pk_ab.hip -- the A/B and ablation instantiations of
// stft8192_pk_kernel (stft_pk.hpp options, dsp_stft_soa_options >> 4): the
// headline shape (IR_test, B = 512) and the memory-source kPkMemAos path.
// Kept in their own code object: loaded only when an option is selected.
#include "stft_pk.hpp"

namespace dspb {

int launch_mem_pf(const Stft8kArgs &A, uint32_t C, hipStream_t stream) {
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

int launch_pk_ab(const Stft8kArgs &A, bool fused, int opt, dim3 grid_default, hipStream_t stream) {
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

}  // namespace dspb
