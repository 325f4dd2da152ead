// common.hpp -- shared definitions for the CDNA4 kernels of libdspbench.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dspbench/dspbench.h"

namespace dspb {

constexpr int kMaxChannels = 16;  // channels per launch; the C ABI loops above this

// Channel pointer tables passed by value as kernel arguments.
struct ChanIn {
    const float *p[kMaxChannels];
};
struct ChanOut {
    float *p[kMaxChannels];
};

// Per-sample plugin maps that the render / fused kernels specialise on.
// `table` is the IR_test ramp (B floats) computed on the device by
// ramp_table_kernel, or (GainTable) C rows of B gains, a GENERIC plugin's
// per-(channel, position) gains; Gain uses the scalar `a`.
enum class MapKind : int { Noop = 0, Gain = 1, Ramp = 3, Fir = 4, Generic = 5, Biquad = 6, GainTable = 7 };

struct SampleMap {
    MapKind kind;
    float a;             // gain (Gain)
    const float *table;  // ramp table (Ramp)
    uint32_t B;          // block size
    uint32_t b_mask;     // B - 1 when B is a power of two, else 0
    const float *taps;   // FIR taps, zero-padded to ntaps8 = ceil(T/16)*16 (Fir; not a per-sample map)
    uint32_t ntaps8;
    uint32_t ntaps;      // Fir: real tap count (<= 1025 runs overlap-save)
    uint32_t fir_direct; // Fir: the caller asked for the direct form (DSP_EXEC_FIR_DIRECT)
    const float *olsH;   // Fir: FFT(taps)/16384 in fir_fft.hip's lane-major pair layout
    float olsH2048[2];   // Fir: H[2048]/16384
    const float *pairH;  // Fir: FFT_4096(taps)/4096 in fir_pair_kernel's layout (fir_fft.hip)
    const float *iir_tab; // Biquad: [5 S coefficients, padded to 20][M^(T l), l <= 64][M^(64 T k), k <= 256]
    uint32_t sections;   // Biquad: S (1..4)
    uint32_t iir_window; // Biquad: tiles of aggregates that reach a tile's state (0: inclusive look-back)
    void *module;        // Generic: the dsp_module running the plugin's own audio_callback
    const void *gparams; // Generic: host Parameters blob
    uint32_t gparams_size;
    float sr;            // sample rate handed to the callback (Generic)
    uint32_t gflags;     // Generic: the call's DSP_EXEC_* method flags (DSP_EXEC_SERIAL_STATE)
    // Ramp: table[i] = (float)(gain - i step) in closed form when the host
    // verified that IR_test's sequential f64 recurrence is exact for these
    // parameters and this B (capi.cpp ramp_closed_form); the table is then
    // only built for kernels that still read it (closed = 1); closed = 2: a
    // GENERIC plugin's block table (module.cpp affine_ramp) that the same
    // closed form reproduces bit for bit -- the table exists already
    uint32_t closed;
    double rg0, rs;
};

__device__ __forceinline__ float ramp_value(const SampleMap &m, uint32_t q) {
    return (float)__fma_rn(-(double)q, m.rs, m.rg0);
}

__device__ __forceinline__ uint32_t block_pos(const SampleMap &m, uint64_t gi) {
    return m.b_mask ? (uint32_t)(gi & m.b_mask) : (uint32_t)(gi % m.B);
}

// out = callback(file sample) for one sample at global index gi.
// `base` is already 0 past EOF / for channels the file lacks.
__device__ __forceinline__ float apply_map(const SampleMap &m, float base, uint64_t gi) {
    switch (m.kind) {
    case MapKind::Gain:
        return base * m.a;  // single fp32 multiply: bit-exact vs gain_test
    case MapKind::Ramp:
        return m.closed ? ramp_value(m, block_pos(m, gi)) : m.table[block_pos(m, gi)];
    case MapKind::GainTable:  // `table` is this channel's row of B gains: one fp32 multiply
        return base * m.table[block_pos(m, gi)];
    default:
        return base;
    }
}

}  // namespace dspb

// Host-side error plumbing shared by the C ABI translation units.
namespace dspb {
void set_last_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
}  // namespace dspb

#define DSPB_HIP(call)                                                 \
    do {                                                               \
        hipError_t _e = (call);                                        \
        if (_e != hipSuccess) return ::dspb::hip_fail(_e, #call);      \
    } while (0)
