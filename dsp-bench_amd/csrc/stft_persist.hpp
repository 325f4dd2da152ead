// stft_persist.hpp -- the fused IR_test render + STFT of the headline (the
// PER path of stft8192_pk_kernel) on a persistent grid: one 8-wave workgroup
// per CU, every wave walks units u = w, w + W, ... of the (channel, frame)
// sequence with the frame's arithmetic of stft8192_pk_kernel<..., PER, ...>.
//
// What a persistent wave saves per frame, against one wave per frame:
//   - the constants a wave loads before its frame (stage twiddles, window
//     base angles, the split's W8192^l: ~8.7 KB per frame from L2) are
//     loaded once per wave and stay in the VGPRs they occupy anyway;
//   - WTAB: the window is read from a table in LDS, (we, wo) of register
//     pair j as one ds_read_b128, instead of 4 packed FMAs per pair from
//     the lane's base angles (128 VALU per frame).  The Hann / Hamming
//     window of the kernel is symmetric about 8191 / 2, so the table holds
//     pairs j < 16 (16 KB) and pair j >= 16 of lane l is pair 31 - j of
//     lane 63 - l with its four values reversed.
#pragma once
#include "stft_pk.hpp"

namespace dspb {

// tail render of the PER kernel: [fs, tail_end) for a wave past the last frame
__device__ __forceinline__ void per_tail_render(const Stft8kArgs &A, uint32_t ch, uint64_t fs, uint32_t lane) {
    if (fs >= A.tail_end) return;
    const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
    float *o = A.out.p[ch] + fs;
    const uint64_t n = A.tail_end - fs;
#pragma unroll 4
    for (uint32_t b = 0; b < 32u; ++b) {  // H = 4096
        const uint32_t e = 128u * b + 2u * lane;  // even: tail_end is a multiple of B >= 2
        if (e < n) {
            const uint32_t q = (p0 + 128u * b) & A.map.b_mask;
            const v2f t = A.map.closed ? v2f{ramp_value(A.map, q), ramp_value(A.map, q + 1)}
                                       : v2f{A.map.table[q], A.map.table[q + 1]};
            reinterpret_cast<v2f *>(o + 128u * b)[lane] = t;
        }
    }
}

constexpr uint32_t kPersistWaves = 8;

template <int PER, bool WTAB>
__global__ __launch_bounds__(64 * kPersistWaves) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stft8192_per_persist_kernel(Stft8kArgs A, uint32_t Fx, uint32_t U) {
    __shared__ __attribute__((aligned(16))) float lds_all[kPersistWaves][64 * 65];
    __shared__ float4 wtab[WTAB ? 1024 : 1];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (WTAB) {
        // entry (l, j), j < 16: (w[n], w[n + 128], w[n + 1], w[n + 129]), n = 2 l + 256 j,
        // w(m) = wa - wb cos(2 pi m / 8191) in double, rounded once
        const double th = 2.0 * 3.14159265358979323846 / 8191.0;
        const double wa = (double)A.wa, wb = (double)A.wb;
        for (uint32_t e = threadIdx.x; e < 1024u; e += 64u * kPersistWaves) {
            const uint32_t n = 2u * (e & 63u) + 256u * (e >> 6);
            wtab[e] = float4{(float)(wa - wb * cos(th * (double)n)), (float)(wa - wb * cos(th * (double)(n + 128u))),
                             (float)(wa - wb * cos(th * (double)(n + 1u))),
                             (float)(wa - wb * cos(th * (double)(n + 129u)))};
        }
        __syncthreads();
    }
    const uint32_t W = gridDim.x * kPersistWaves;
    uint32_t u = blockIdx.x * kPersistWaves + wave;
    if (u >= U) return;
    float *lds = lds_all[wave];

    // constants of every frame, loaded once
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
    float ue = 0.f, ve = 0.f, uo = 0.f, vo = 0.f;
    if constexpr (!WTAB) {
        const float4 wbase = A.wbase[lane];
        ue = A.wb * wbase.x;
        ve = A.wb * wbase.y;
        uo = A.wb * wbase.z;
        vo = A.wb * wbase.w;
    }
    uint32_t c = u / Fx, f = u - c * Fx;
    for (;;) {
        // opaque per frame: loop-invariant products (the stage twiddles
        // tlo x thp, the window) would otherwise be hoisted and spill
#pragma unroll
        for (int j = 1; j < 8; ++j) asm volatile("" : "+v"(tlo[j].r), "+v"(tlo[j].i));
#pragma unroll
        for (int h = 0; h < 4; ++h) asm volatile("" : "+v"(thp[h].r), "+v"(thp[h].i));
        asm volatile("" : "+v"(ue), "+v"(ve), "+v"(uo), "+v"(vo));
        uint32_t wl = lane;  // the window table's lane offsets, opaque likewise
        asm volatile("" : "+v"(wl));
        const uint64_t fs = (uint64_t)f * 4096u;
        if (f >= A.F) {
            per_tail_render(A, c, fs, lane);
        } else {
            constexpr int NJ = PER >= 2 ? PER / 2 : 1;
            cx2 X[NJ];
            const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
            const float *T = A.map.table;
            if (A.map.closed) {
#pragma unroll
                for (int jj = 0; jj < NJ; ++jj) {
                    const uint32_t q0 = (p0 + 256u * jj) & A.map.b_mask;
                    const uint32_t q1 = (p0 + 256u * jj + (PER >= 2 ? 128u : 0u)) & A.map.b_mask;
                    X[jj] = cx2{v2f{ramp_value(A.map, q0), ramp_value(A.map, q1)},
                                v2f{ramp_value(A.map, q0 + 1), ramp_value(A.map, q1 + 1)}};
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < NJ; ++jj) {
                    const uint32_t q0 = (p0 + 256u * jj) & A.map.b_mask;
                    const uint32_t q1 = (p0 + 256u * jj + (PER >= 2 ? 128u : 0u)) & A.map.b_mask;
                    X[jj] = cx2{v2f{T[q0], T[q1]}, v2f{T[q0 + 1], T[q1 + 1]}};
                }
            }
            {  // the render output: sample pairs of column b repeat with period PER
                float *o = A.out.p[c] + fs;
                v2f st[PER >= 2 ? PER : 1];
#pragma unroll
                for (int b = 0; b < (PER >= 2 ? PER : 1); ++b) st[b] = v2f{X[b / 2].r[b & 1], X[b / 2].i[b & 1]};
#pragma unroll
                for (int b = 0; b < 32; ++b)  // H = 4096 (the launch's condition)
                    __builtin_nontemporal_store(st[b % (PER >= 2 ? PER : 1)],
                                                reinterpret_cast<v2f *>(o + 128u * (uint32_t)b) + lane);
            }
            cx2 P[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                v2f we, wo;
                if constexpr (WTAB) {
                    if (j < 16) {
                        const float4 e = wtab[64u * (uint32_t)j + wl];
                        we = v2f{e.x, e.y};
                        wo = v2f{e.z, e.w};
                    } else {  // pair 31 - j of lane 63 - l, reversed
                        const float4 e = wtab[64u * (uint32_t)(31 - j) + (63u - wl)];
                        we = v2f{e.w, e.z};
                        wo = v2f{e.y, e.x};
                    }
                } else {
                    const v2f C = v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}, S = v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]};
                    we = (v2f{ve, ve} * S + v2f{A.wa, A.wa}) - v2f{ue, ue} * C;
                    wo = (v2f{vo, vo} * S + v2f{A.wa, A.wa}) - v2f{uo, uo} * C;
                }
                const cx2 xj = X[j % NJ];
                P[j] = cx2{xj.r * we, xj.i * wo};
            }
            cx2 Y2[32];
            fft4096_pk_y2<false, false>(P, lds, tlo, thp, lane, Y2);
            split_y2<kKHalf, false>(Y2, A.mag.p[c] + (uint64_t)f * A.ld, A.K, A.tw, lane, lds);
        }
        u += W;
        if (u >= U) break;
        f += W;
        while (f >= Fx) {  // wave-uniform
            f -= Fx;
            ++c;
        }
    }
}

// the PER launch on the persistent grid (fused IR_test, pow2 B <= 2048,
// computed-window shape); DSP_ERR_INVALID when the unit count does not fit
template <bool WTAB>
int launch_per_persist(const Stft8kArgs &A, uint32_t C, uint32_t per, uint64_t tail, hipStream_t s) {
    const uint64_t Fx = A.F + tail, U = Fx * C;
    if (U >= 0x80000000ull || A.H != 4096u) return DSP_ERR_INVALID;
    int dev = 0, cus = 0;
    DSPB_HIP(hipGetDevice(&dev));
    DSPB_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t need = (U + kPersistWaves - 1) / kPersistWaves;
    const uint32_t g = (uint32_t)(need < (uint64_t)cus ? need : (uint64_t)cus);
#define DSPB_PERSIST_CASE(p)                                                                                     \
    case p:                                                                                                      \
        hipLaunchKernelGGL((stft8192_per_persist_kernel<p, WTAB>), dim3(g), dim3(64 * kPersistWaves), 0, s, A, \
                           (uint32_t)Fx, (uint32_t)U);                                                           \
        break
    switch (per) {
        DSPB_PERSIST_CASE(1);
        DSPB_PERSIST_CASE(2);
        DSPB_PERSIST_CASE(4);
        DSPB_PERSIST_CASE(8);
        DSPB_PERSIST_CASE(16);
    default: return DSP_ERR_INVALID;
    }
#undef DSPB_PERSIST_CASE
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
