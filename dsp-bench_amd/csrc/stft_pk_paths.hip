// stft_pk_paths.hip -- stft8192_pk_kernel (stft_pk.hpp) for the fused
// NOOP / GAIN / non-PER IR_test renders and for the STFT of a signal in HBM.
#include "stft_pk.hpp"

namespace dspb {

template <int SRC, MapKind MK, bool POW2, bool WINC>
static void launch_pk_km(int km, dim3 grid, hipStream_t s, const Stft8kArgs &A) {
    if (km == kKHalf)
        hipLaunchKernelGGL((stft8192_pk_kernel<SRC, kKHalf, MK, POW2, WINC>), grid, dim3(64 * kPkWpb), 0, s, A);
    else if (km == kKMirror)
        hipLaunchKernelGGL((stft8192_pk_kernel<SRC, kKMirror, MK, POW2, WINC>), grid, dim3(64 * kPkWpb), 0, s, A);
    else
        hipLaunchKernelGGL((stft8192_pk_kernel<SRC, kKPartial, MK, POW2, WINC>), grid, dim3(64 * kPkWpb), 0, s, A);
}

int launch_pk_paths(const Stft8kArgs &A, bool fused, int km, bool pow2, bool winc, dim3 grid, hipStream_t stream) {
    if (fused && winc) {
        // full frames, 4097 bins: the window computed by angle addition
        // instead of 64 float2 loads per frame (the fused gain STFT: 0.807 ->
        // 0.756 ms per stereo hour, profiles/r02_gain_winc_ab.txt)
        switch (A.map.kind) {
        case MapKind::Noop:
            hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Noop, true, true>), grid,
                               dim3(64 * kPkWpb), 0, stream, A);
            break;
        case MapKind::Gain:
            hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Gain, true, true>), grid,
                               dim3(64 * kPkWpb), 0, stream, A);
            break;
        case MapKind::Ramp:
            if (pow2)
                hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true>), grid,
                                   dim3(64 * kPkWpb), 0, stream, A);
            else
                hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, false, true>), grid,
                                   dim3(64 * kPkWpb), 0, stream, A);
            break;
        case MapKind::GainTable:
            if (pow2)
                hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::GainTable, true, true>), grid,
                                   dim3(64 * kPkWpb), 0, stream, A);
            else
                hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::GainTable, false, true>), grid,
                                   dim3(64 * kPkWpb), 0, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else if (fused) {
        switch (A.map.kind) {
        case MapKind::Noop: launch_pk_km<kSrcRender, MapKind::Noop, true, false>(km, grid, stream, A); break;
        case MapKind::Gain: launch_pk_km<kSrcRender, MapKind::Gain, true, false>(km, grid, stream, A); break;
        case MapKind::Ramp:
            if (pow2) launch_pk_km<kSrcRender, MapKind::Ramp, true, false>(km, grid, stream, A);
            else launch_pk_km<kSrcRender, MapKind::Ramp, false, false>(km, grid, stream, A);
            break;
        case MapKind::GainTable:
            if (pow2) launch_pk_km<kSrcRender, MapKind::GainTable, true, false>(km, grid, stream, A);
            else launch_pk_km<kSrcRender, MapKind::GainTable, false, false>(km, grid, stream, A);
            break;
        default: return DSP_ERR_INVALID;
        }
    } else if (winc) {
        hipLaunchKernelGGL((stft8192_pk_kernel<kSrcMemory, kKHalf, MapKind::Noop, true, true>), grid, dim3(64 * kPkWpb), 0,
                           stream, A);
    } else {
        launch_pk_km<kSrcMemory, MapKind::Noop, true, false>(km, grid, stream, A);
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
