// stft_pk.hip -- the 8192-point STFT dispatcher and the fused IR_test
// kernels of the headline (PER path); the kernel is in stft_pk.hpp.
#include "stft_pk.hpp"

namespace dspb {

// Host -> device upload of the library's small constant tables through
// kernel arguments.  The first hipMemcpy of more than a few KB in a process,
// pageable or pinned, costs 7-8 ms (copy-engine start-up,
// tools/copy_init_probe.cpp; 0.02 ms afterwards) and was most of a cold
// call; ~4 KB of kernel arguments per launch costs microseconds.  Here, in
// the headline's translation unit, so that a cold headline call loads one
// code object.
constexpr uint32_t kUploadFloats = 960;
struct UploadChunk {
    uint32_t n;
    float v[kUploadFloats];
};
__global__ void upload_kernel(float *dst, UploadChunk c) {
    for (uint32_t i = threadIdx.x; i < c.n; i += blockDim.x) dst[i] = c.v[i];
}
int launch_upload(float *dst, const float *src, uint64_t n, hipStream_t s) {
    UploadChunk c;
    for (uint64_t off = 0; off < n; off += kUploadFloats) {
        c.n = (uint32_t)(n - off < kUploadFloats ? n - off : kUploadFloats);
        for (uint32_t i = 0; i < c.n; ++i) c.v[i] = src[off + i];
        hipLaunchKernelGGL(upload_kernel, dim3(1), dim3(256), 0, s, dst + off, c);
        DSPB_HIP(hipGetLastError());
    }
    return DSP_OK;
}

// true when launch_stft8192_pk runs the PER kernel for these arguments --
// the fused path that evaluates a closed-form IR ramp itself and renders the
// tail past the last frame's hop (A.tail_end)
bool stft8192_pk_per_path(const Stft8kArgs &A, bool fused) {
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    const bool winc = A.valid >= 8192u && A.wbase != nullptr && km == kKHalf;
    return fused && A.map.kind == MapKind::Ramp && pow2 && winc && A.map.B <= 2048u;
}

// A.win2: the window pre-scaled by 0.5 / sqrt(8192); the computed window
// (A.wbase, A.wa, A.wb) serves the full-frame 4097-bin shapes.
int launch_stft8192_pk(const Stft8kArgs &A, uint32_t C, bool fused, int opt, hipStream_t stream) {
    if (A.F == 0 || C == 0) return DSP_OK;
    // PER path: extra waves for the render tail [F H, tail_end)
    const uint64_t tail = A.tail_end > A.F * A.H ? (A.tail_end - A.F * A.H + A.H - 1) / A.H : 0;
    if (tail && !stft8192_pk_per_path(A, fused)) return DSP_ERR_INVALID;
    const uint64_t groups = (A.F + tail + kPkWpb - 1) / kPkWpb;  // workgroups of the default kernels
    if (groups > 0x7fffffffull) return DSP_ERR_INVALID;
    dim3 grid((uint32_t)groups, C);
    const int km = A.K == 4097u ? kKHalf : (A.K == 8192u ? kKMirror : kKPartial);
    const bool pow2 = A.map.b_mask != 0 && A.map.B >= 2;
    const bool winc = A.valid >= 8192u && A.wbase != nullptr && km == kKHalf;
    if (fused && A.map.kind == MapKind::Ramp && pow2 && winc) {
        // period of the block table in units of 128 samples
        const uint32_t per = A.map.B <= 128u ? 1u : A.map.B / 128u;
        if (per == 4 && opt) {  // A/B at the headline shape (the tools build only: stft_pk_ab.hip)
            int st = DSP_OK;
            if (stft_pk_ab_dispatch(A, C, fused, opt, grid, stream, &st)) return st;
        }
#define DSPB_PK_PER(p) \
    hipLaunchKernelGGL((stft8192_pk_kernel<kSrcRender, kKHalf, MapKind::Ramp, true, true, p, kPkPerOpt>), grid_per, \
                       dim3(64 * kPkPerWpb), 0, stream, A)
        const uint64_t groups_per = (A.F + tail + kPkPerWpb - 1) / kPkPerWpb;
        if (groups_per > 0x7fffffffull) return DSP_ERR_INVALID;
        const dim3 grid_per((uint32_t)groups_per, C);
        switch (per) {
        case 1: DSPB_PK_PER(1); break;
        case 2: DSPB_PK_PER(2); break;
        case 4: DSPB_PK_PER(4); break;
        case 8: DSPB_PK_PER(8); break;
        case 16: DSPB_PK_PER(16); break;
        default: DSPB_PK_PER(0); break;
        }
#undef DSPB_PK_PER
        DSPB_HIP(hipGetLastError());
        return DSP_OK;
    }
    if (opt && !fused && winc) {  // memory-source A/B variants (the tools build only)
        int st = DSP_OK;
        if (stft_pk_ab_dispatch(A, C, fused, opt, grid, stream, &st)) return st;
    }
    return launch_pk_paths(A, fused, km, pow2, winc, grid, stream);
}

// The product library has no A/B variants: these weak definitions stand
// unless the tools build (make ab) links stft_pk_ab.hip, which defines both.
__attribute__((weak)) bool stft_pk_ab_dispatch(const Stft8kArgs &, uint32_t, bool, int, dim3, hipStream_t, int *) {
    return false;
}
__attribute__((weak)) int stft_pk_ab_options() { return 0; }

}  // namespace dspb
