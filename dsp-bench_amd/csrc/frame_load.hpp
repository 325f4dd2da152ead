// frame_load.hpp -- the rendered samples of one 8192-point frame, for the
// one-wave-per-frame kernels (stft_soa.hip, stft_pk.hip).
//
// Lane l gets v[b] = (x[2l + 128b], x[2l + 128b + 1]) of the frame starting
// at local sample fs, where x is the signal after the plugin's sample map:
//   Ramp (IR_test, ref build/IR_test.cpp:40-60): table[(global sample) mod B]
//   Gain / Noop: the input (zero past EOF or for missing channels) * gain.
//   GainTable: the input * G[ch][(global sample) mod B] (a GENERIC plugin's
//   per-(channel, position) gains, module.cpp kSpecGainTable).
#pragma once
#include "fft_soa.hpp"

namespace dspb {

template <MapKind MK, bool POW2>
__device__ __forceinline__ void s_render_frame(const Stft8kArgs &A, const float *x, uint64_t fs,
                                               uint32_t lane, cx (&v)[64], uint32_t ch = 0) {
    const uint64_t gbase = A.goff + fs;
    if constexpr (MK == MapKind::Ramp) {
        const float *T = A.map.table;
        if constexpr (POW2) {
            const uint32_t p0 = (uint32_t)gbase + 2u * lane;
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const v2f t =
                    *reinterpret_cast<const v2f *>(T + ((p0 + 128u * (uint32_t)b) & A.map.b_mask));
                v[b] = cx{t.x, t.y};
            }
        } else {
            const uint32_t Bn = A.map.B;
            uint32_t p = (uint32_t)((gbase + 2u * lane) % Bn);
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint32_t q = (p + 1 == Bn) ? 0u : p + 1;
                v[b] = cx{T[p], T[q]};
                p += 128u;
                while (p >= Bn) p -= Bn;
            }
        }
    } else {
        if (x != nullptr && fs + 8192u <= A.L) {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const v2f t = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
                v[b] = cx{t.x, t.y};
            }
        } else {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint64_t li = fs + 2u * lane + 128u * (uint32_t)b;
                v[b] = cx{(x && li < A.L) ? x[li] : 0.f, (x && li + 1 < A.L) ? x[li + 1] : 0.f};
            }
        }
        if constexpr (MK == MapKind::Gain) {
#pragma unroll
            for (int b = 0; b < 64; ++b) v[b] = cx{v[b].r * A.map.a, v[b].i * A.map.a};
        }
        if constexpr (MK == MapKind::GainTable) {  // x * G[ch][(global sample) mod B]
            const float *T = A.map.table + (uint64_t)ch * A.map.B;
            if constexpr (POW2) {
                const uint32_t p0 = (uint32_t)gbase + 2u * lane;
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const v2f t =
                        *reinterpret_cast<const v2f *>(T + ((p0 + 128u * (uint32_t)b) & A.map.b_mask));
                    v[b] = cx{v[b].r * t.x, v[b].i * t.y};
                }
            } else {
                const uint32_t Bn = A.map.B;
                uint32_t p = (uint32_t)((gbase + 2u * lane) % Bn);
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const uint32_t q = (p + 1 == Bn) ? 0u : p + 1;
                    v[b] = cx{v[b].r * T[p], v[b].i * T[q]};
                    p += 128u;
                    while (p >= Bn) p -= Bn;
                }
            }
        }
    }
}

// IR ramp from a block table staged in the wave's LDS tile (pow2 B, 4 <= B
// <= 4096): two coalesced float4 loads per lane (B = 512) instead of 64
// scattered 8-byte gathers; the tile is free until the transpose.
__device__ __forceinline__ void lds_table_frame(const Stft8kArgs &A, float *lds, uint64_t fs,
                                                uint32_t lane, cx (&v)[64]) {
    const uint32_t q4 = A.map.B >> 2;  // float4s in the table
    const float4 *T4 = reinterpret_cast<const float4 *>(A.map.table);
    // groups of 4 float4 per lane: all loads of a group in flight
    // together (B = 512 is one group, half of it masked off)
    for (uint32_t g = 0; 256u * g < q4; ++g) {
        float4 t4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = lane + 64u * (4u * g + (uint32_t)u);
            t4[u] = T4[i < q4 ? i : 0u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = lane + 64u * (4u * g + (uint32_t)u);
            if (i < q4) reinterpret_cast<float4 *>(lds)[i] = t4[u];
        }
    }
    lds_fence();
    const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
#pragma unroll
    for (int b = 0; b < 64; ++b) {
        const v2f t = *reinterpret_cast<const v2f *>(
            lds + ((p0 + 128u * (uint32_t)b) & A.map.b_mask));
        v[b] = cx{t.x, t.y};
    }
}

// the gain table's row of this channel (pow2 B, 4 <= B <= 4096) staged in the
// wave's LDS tile like lds_table_frame, then x * G[(global sample) mod B]:
// two coalesced float4 loads per lane at B = 512 instead of 64 scattered
// 8-byte gathers beside the frame's own loads
__device__ __forceinline__ void lds_gain_table_frame(const Stft8kArgs &A, float *lds, const float *x, uint64_t fs,
                                                     uint32_t lane, cx (&v)[64], uint32_t ch) {
    const uint32_t q4 = A.map.B >> 2;  // float4s in the row
    const float4 *T4 = reinterpret_cast<const float4 *>(A.map.table + (uint64_t)ch * A.map.B);
    for (uint32_t g = 0; 256u * g < q4; ++g) {
        float4 t4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = lane + 64u * (4u * g + (uint32_t)u);
            t4[u] = T4[i < q4 ? i : 0u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = lane + 64u * (4u * g + (uint32_t)u);
            if (i < q4) reinterpret_cast<float4 *>(lds)[i] = t4[u];
        }
    }
    s_render_frame<MapKind::Noop, true>(A, x, fs, lane, v);
    lds_fence();
    const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
#pragma unroll
    for (int b = 0; b < 64; ++b) {
        const v2f t = *reinterpret_cast<const v2f *>(lds + ((p0 + 128u * (uint32_t)b) & A.map.b_mask));
        v[b] = cx{v[b].r * t.x, v[b].i * t.y};
    }
}

// pow2 B <= 512: the lane's samples 2 lane + 128 b (+1) meet at most four
// positions of the row, (p0 + 128 b) mod B depends on b mod 4 only, so the
// lane keeps its 4 gain pairs in registers -- four 8-byte loads from a 2 KB
// row and no LDS traffic
__device__ __forceinline__ void reg_gain_table_frame(const Stft8kArgs &A, const float *x, uint64_t fs,
                                                     uint32_t lane, cx (&v)[64], uint32_t ch) {
    const float *T = A.map.table + (uint64_t)ch * A.map.B;
    const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
    v2f t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = *reinterpret_cast<const v2f *>(T + ((p0 + 128u * (uint32_t)j) & A.map.b_mask));
    s_render_frame<MapKind::Noop, true>(A, x, fs, lane, v);
#pragma unroll
    for (int b = 0; b < 64; ++b) v[b] = cx{v[b].r * t[b & 3].x, v[b].i * t[b & 3].y};
}

}  // namespace dspb
