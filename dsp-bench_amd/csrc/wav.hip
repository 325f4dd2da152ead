// wav.hip -- WAV payload decode / encode on the GPU (wav.h).
//
// Decode restates the reference's converters bit for bit (audio.h:66-110):
//   int16: value = d0 << 16 | d1 << 24, value / (float)(2^31 - 1); the
//          float divisor rounds to 2^31, so the result is s16 * 2^-15
//   int32: (float)value / 2^31 (int -> float rounds first: i32 max -> 1.0)
//   int24: value = d2 << 24 | d1 << 16 | d0 << 8, (float)((double)value /
//          (2^31 - 1)) -- a correctly rounded double division, then one
//          rounding to float
//   float: the payload bytes (format 3, wav_reader.h:186-189)
// followed by the planar split of deinterleave (audio.h:112-121).
//
// HBM-bound byte work: each thread converts 4 whole frames, reading their
// interleaved payload as dwords (4 frames x C x bytes is always a dword
// multiple) and writing one float4 per channel; mono / stereo are
// specialised (wav_decode_tile_kernel), other channel counts and unaligned
// starts use per-sample byte loads.
#include "kernels.hpp"

namespace dspb {

struct WavArgs {
    const uint8_t *payload;  // interleaved payload, byte 0 = frame 0
    uint64_t frame0;         // first frame converted
    uint64_t frames;         // frames converted
    uint32_t C;              // channels
    ChanOut pl;              // planar rows: out (decode) or in (encode)
};

template <int BITS, bool FLT>
__device__ __forceinline__ float pcm_to_float(uint32_t raw) {
    if constexpr (FLT) {
        return __uint_as_float(raw);
    } else if constexpr (BITS == 16) {
        return (float)(int16_t)(uint16_t)raw * 0x1p-15f;
    } else if constexpr (BITS == 32) {
        return (float)(int32_t)raw * 0x1p-31f;
    } else {
        const int32_t v = (int32_t)(raw << 8);
        return (float)((double)v / 2147483647.0);
    }
}

// one sample from bytes (any alignment)
template <int BITS>
__device__ __forceinline__ uint32_t load_raw(const uint8_t *p) {
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < BITS / 8; ++b) r |= (uint32_t)p[b] << (8 * b);
    return r;
}

// sample j (0-based, BITS wide) of a little-endian dword array
template <int BITS>
__device__ __forceinline__ uint32_t extract(const uint32_t *w, int j) {
    if constexpr (BITS == 32) return w[j];
    if constexpr (BITS == 16) return (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
    const int byte = 3 * j, q = byte >> 2, s = (byte & 3) * 8;
    const uint64_t pair = (uint64_t)w[q] | ((uint64_t)(s > 8 ? w[q + 1] : 0u) << 32);
    return (uint32_t)(pair >> s) & 0xffffffu;
}

template <int BITS, bool FLT, int CH>
__global__ __launch_bounds__(256) void wav_decode_kernel(WavArgs A) {
    constexpr int BPS = BITS / 8;
    const uint64_t groups = (A.frames + 3) / 4;
    const uint32_t C = CH ? (uint32_t)CH : A.C;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = 4 * g;  // local frame
        if (CH && f + 4 <= A.frames) {
            constexpr int W = (CH ? CH : 1) * BPS;  // dwords of 4 frames
            const uint32_t *src =
                reinterpret_cast<const uint32_t *>(A.payload + (A.frame0 + f) * (uint64_t)(CH * BPS));
            uint32_t w[W + 1];
#pragma unroll
            for (int i = 0; i < W; ++i) w[i] = src[i];
            w[W] = 0;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                float4 o;
                o.x = pcm_to_float<BITS, FLT>(extract<BITS>(w, 0 * CH + c));
                o.y = pcm_to_float<BITS, FLT>(extract<BITS>(w, 1 * CH + c));
                o.z = pcm_to_float<BITS, FLT>(extract<BITS>(w, 2 * CH + c));
                o.w = pcm_to_float<BITS, FLT>(extract<BITS>(w, 3 * CH + c));
                *reinterpret_cast<float4 *>(A.pl.p[c] + f) = o;
            }
        } else {
            const uint64_t fe = f + 4 < A.frames ? f + 4 : A.frames;
            for (uint64_t ff = f; ff < fe; ++ff)
                for (uint32_t c = 0; c < C; ++c)
                    A.pl.p[c][ff] = pcm_to_float<BITS, FLT>(
                        load_raw<BITS>(A.payload + ((A.frame0 + ff) * C + c) * (uint64_t)BPS));
        }
    }
}

// Mono / stereo fast path: one tile of 256 x kWavU groups of 4 frames per
// block (all of a thread's payload loads issue before its first store), 16- or
// 8-byte payload loads when the payload start allows (LDW dwords per load),
// non-temporal float4 stores (the planar output is written once).
constexpr int kWavU = 4;
typedef float f4w __attribute__((ext_vector_type(4)));
template <int BITS, bool FLT, int CH, int LDW>
__global__ __launch_bounds__(256) void wav_decode_tile_kernel(WavArgs A) {
    constexpr int BPS = BITS / 8;
    constexpr int W = CH * BPS;  // dwords of 4 frames
    static_assert(W % LDW == 0, "load width");
    const uint64_t g0 = blockIdx.x * (256ull * kWavU) + threadIdx.x;
    uint32_t w[kWavU][W + 1];
#pragma unroll
    for (int u = 0; u < kWavU; ++u) {
        const uint64_t f = 4 * (g0 + 256u * (uint32_t)u);
        w[u][W] = 0;
        if (f + 4 <= A.frames) {
            const uint8_t *src = A.payload + (A.frame0 + f) * (uint64_t)W;
#pragma unroll
            for (int i = 0; i < W; i += LDW) {
                if constexpr (LDW == 4) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(src + 4 * i);
                    w[u][i] = q.x, w[u][i + 1] = q.y, w[u][i + 2] = q.z, w[u][i + 3] = q.w;
                } else if constexpr (LDW == 2) {
                    const uint2 q = *reinterpret_cast<const uint2 *>(src + 4 * i);
                    w[u][i] = q.x, w[u][i + 1] = q.y;
                } else {
                    w[u][i] = *reinterpret_cast<const uint32_t *>(src + 4 * i);
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kWavU; ++u) {
        const uint64_t f = 4 * (g0 + 256u * (uint32_t)u);
        if (f + 4 <= A.frames) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const f4w o = f4w{pcm_to_float<BITS, FLT>(extract<BITS>(w[u], 0 * CH + c)),
                                  pcm_to_float<BITS, FLT>(extract<BITS>(w[u], 1 * CH + c)),
                                  pcm_to_float<BITS, FLT>(extract<BITS>(w[u], 2 * CH + c)),
                                  pcm_to_float<BITS, FLT>(extract<BITS>(w[u], 3 * CH + c))};
                __builtin_nontemporal_store(o, reinterpret_cast<f4w *>(A.pl.p[c] + f));
            }
        } else if (f < A.frames) {  // the last, partial group
            for (uint64_t ff = f; ff < A.frames; ++ff)
                for (uint32_t c = 0; c < (uint32_t)CH; ++c)
                    A.pl.p[c][ff] = pcm_to_float<BITS, FLT>(
                        load_raw<BITS>(A.payload + ((A.frame0 + ff) * CH + c) * (uint64_t)BPS));
        }
    }
}

template <int BITS, bool FLT>
__device__ __forceinline__ uint32_t float_to_pcm(float x) {
    if constexpr (FLT) {
        return __float_as_uint(x);
    } else if constexpr (BITS == 32) {
        double r = rint((double)x * 2147483648.0);
        r = fmin(fmax(r, -2147483648.0), 2147483647.0);
        return (uint32_t)(int32_t)r;
    } else {
        constexpr float S = BITS == 16 ? 32768.f : 8388608.f;
        float r = rintf(x * S);  // exact scaling, round half to even
        r = fminf(fmaxf(r, -S), S - 1.f);
        return (uint32_t)(int32_t)r & (BITS == 16 ? 0xffffu : 0xffffffu);
    }
}

template <int BITS, bool FLT>
__global__ __launch_bounds__(256) void wav_encode_kernel(WavArgs A) {
    constexpr int BPS = BITS / 8;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < A.frames * A.C;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = i / A.C;
        const uint32_t c = (uint32_t)(i - f * A.C);
        const uint32_t raw = float_to_pcm<BITS, FLT>(A.pl.p[c][f]);
        uint8_t *d = const_cast<uint8_t *>(A.payload) + i * BPS;
        if constexpr (BPS == 4) {
            *reinterpret_cast<uint32_t *>(d) = raw;
        } else if constexpr (BPS == 2) {
            *reinterpret_cast<uint16_t *>(d) = (uint16_t)raw;
        } else {
            d[0] = (uint8_t)raw;
            d[1] = (uint8_t)(raw >> 8);
            d[2] = (uint8_t)(raw >> 16);
        }
    }
}

// Mono / stereo encode, the decode tile run backwards: each thread reads one
// float4 per channel for each of kWavU groups of 4 frames (planar rows
// 16-byte aligned), packs the group's W = CH * BITS / 8 dwords of
// interleaved payload and stores them LDW dwords at a time (LDW from the
// payload's alignment); the last partial group byte by byte.
template <int BITS>
__device__ __forceinline__ void pack(uint32_t *w, int j, uint32_t raw) {
    if constexpr (BITS == 32) {
        w[j] = raw;
    } else if constexpr (BITS == 16) {
        w[j >> 1] |= raw << (16 * (j & 1));
    } else {
        const int byte = 3 * j, q = byte >> 2, sh = (byte & 3) * 8;
        w[q] |= raw << sh;
        if (sh > 8) w[q + 1] |= raw >> (32 - sh);
    }
}
template <int BITS, bool FLT, int CH, int LDW>
__global__ __launch_bounds__(256) void wav_encode_tile_kernel(WavArgs A) {
    constexpr int BPS = BITS / 8;
    constexpr int W = CH * BPS;  // dwords of 4 frames
    static_assert(W % LDW == 0, "store width");
    const uint64_t g0 = blockIdx.x * (256ull * kWavU) + threadIdx.x;
    float4 v[kWavU][CH];
#pragma unroll
    for (int u = 0; u < kWavU; ++u) {
        const uint64_t f = 4 * (g0 + 256u * (uint32_t)u);
        if (f + 4 <= A.frames) {
#pragma unroll
            for (int c = 0; c < CH; ++c) v[u][c] = *reinterpret_cast<const float4 *>(A.pl.p[c] + f);
        }
    }
#pragma unroll
    for (int u = 0; u < kWavU; ++u) {
        const uint64_t f = 4 * (g0 + 256u * (uint32_t)u);
        if (f + 4 <= A.frames) {
            uint32_t w[W];
#pragma unroll
            for (int i = 0; i < W; ++i) w[i] = 0;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                pack<BITS>(w, 0 * CH + c, float_to_pcm<BITS, FLT>(v[u][c].x));
                pack<BITS>(w, 1 * CH + c, float_to_pcm<BITS, FLT>(v[u][c].y));
                pack<BITS>(w, 2 * CH + c, float_to_pcm<BITS, FLT>(v[u][c].z));
                pack<BITS>(w, 3 * CH + c, float_to_pcm<BITS, FLT>(v[u][c].w));
            }
            uint8_t *dst = const_cast<uint8_t *>(A.payload) + f * (uint64_t)W;  // W bytes per frame
#pragma unroll
            for (int i = 0; i < W; i += LDW) {
                if constexpr (LDW == 4)
                    *reinterpret_cast<uint4 *>(dst + 4 * i) = make_uint4(w[i], w[i + 1], w[i + 2], w[i + 3]);
                else if constexpr (LDW == 2)
                    *reinterpret_cast<uint2 *>(dst + 4 * i) = make_uint2(w[i], w[i + 1]);
                else
                    *reinterpret_cast<uint32_t *>(dst + 4 * i) = w[i];
            }
        } else if (f < A.frames) {  // the last, partial group
            for (uint64_t ff = f; ff < A.frames; ++ff)
                for (int c = 0; c < CH; ++c) {
                    const uint32_t raw = float_to_pcm<BITS, FLT>(A.pl.p[c][ff]);
                    uint8_t *d = const_cast<uint8_t *>(A.payload) + (ff * CH + c) * (uint64_t)BPS;
#pragma unroll
                    for (int b = 0; b < BPS; ++b) d[b] = (uint8_t)(raw >> (8 * b));
                }
        }
    }
}

template <int BITS, bool FLT, int CH>
static void enc_tile(const WavArgs &A, dim3 grid, hipStream_t s) {
    constexpr int W = CH * BITS / 8;
    const uintptr_t start = reinterpret_cast<uintptr_t>(A.payload);
    if constexpr (W % 4 == 0) {
        if (start % 16 == 0) {
            hipLaunchKernelGGL((wav_encode_tile_kernel<BITS, FLT, CH, 4>), grid, dim3(256), 0, s, A);
            return;
        }
    }
    if constexpr (W % 2 == 0) {
        if (start % 8 == 0) {
            hipLaunchKernelGGL((wav_encode_tile_kernel<BITS, FLT, CH, 2>), grid, dim3(256), 0, s, A);
            return;
        }
    }
    hipLaunchKernelGGL((wav_encode_tile_kernel<BITS, FLT, CH, 1>), grid, dim3(256), 0, s, A);
}

template <int BITS, bool FLT>
static void enc(const WavArgs &A, bool vec, hipStream_t s);

static dim3 grid_for(uint64_t items) {
    uint64_t g = (items + 255) / 256;
    if (g > 4096) g = 4096;
    return dim3((uint32_t)(g ? g : 1));
}

template <int BITS, bool FLT, int CH>
static void dec_tile(const WavArgs &A, dim3 grid, hipStream_t s) {
    constexpr int W = CH * BITS / 8;
    const uintptr_t start = reinterpret_cast<uintptr_t>(A.payload) + A.frame0 * (uint64_t)W;
    // every group starts W dwords after the previous one
    if constexpr (W % 4 == 0) {
        if (start % 16 == 0) {
            hipLaunchKernelGGL((wav_decode_tile_kernel<BITS, FLT, CH, 4>), grid, dim3(256), 0, s, A);
            return;
        }
    }
    if constexpr (W % 2 == 0) {
        if (start % 8 == 0) {
            hipLaunchKernelGGL((wav_decode_tile_kernel<BITS, FLT, CH, 2>), grid, dim3(256), 0, s, A);
            return;
        }
    }
    hipLaunchKernelGGL((wav_decode_tile_kernel<BITS, FLT, CH, 1>), grid, dim3(256), 0, s, A);
}

template <int BITS, bool FLT>
static void dec(const WavArgs &A, bool vec, hipStream_t s) {
    if (vec && (A.C == 1 || A.C == 2)) {
        const uint64_t tiles = ((A.frames + 3) / 4 + 256u * kWavU - 1) / (256u * kWavU);
        const dim3 grid((uint32_t)(tiles ? tiles : 1));
        if (A.C == 1) dec_tile<BITS, FLT, 1>(A, grid, s);
        else dec_tile<BITS, FLT, 2>(A, grid, s);
        return;
    }
    hipLaunchKernelGGL((wav_decode_kernel<BITS, FLT, 0>), grid_for((A.frames + 3) / 4), dim3(256), 0, s, A);
}

int launch_wav_decode(const uint8_t *payload, uint32_t C, uint16_t bits, bool is_float, uint64_t frame0,
                      uint64_t frames, const ChanOut &out, bool out_aligned16, hipStream_t s) {
    if (frames == 0) return DSP_OK;
    WavArgs A{payload, frame0, frames, C, out};
    const uint64_t start = frame0 * (uint64_t)C * (bits / 8u);
    const bool vec = out_aligned16 && ((uintptr_t)payload % 4 == 0) && (start % 4 == 0);
    if (is_float) dec<32, true>(A, vec, s);
    else if (bits == 16) dec<16, false>(A, vec, s);
    else if (bits == 24) dec<24, false>(A, vec, s);
    else if (bits == 32) dec<32, false>(A, vec, s);
    else return DSP_ERR_UNSUPPORTED;
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

template <int BITS, bool FLT>
static void enc(const WavArgs &A, bool vec, hipStream_t s) {
    if (vec && (A.C == 1 || A.C == 2)) {
        const uint64_t tiles = ((A.frames + 3) / 4 + 256u * kWavU - 1) / (256u * kWavU);
        const dim3 grid((uint32_t)(tiles ? tiles : 1));
        if (A.C == 1) enc_tile<BITS, FLT, 1>(A, grid, s);
        else enc_tile<BITS, FLT, 2>(A, grid, s);
        return;
    }
    hipLaunchKernelGGL((wav_encode_kernel<BITS, FLT>), grid_for(A.frames * A.C), dim3(256), 0, s, A);
}

int launch_wav_encode(uint8_t *payload, uint32_t C, uint16_t bits, bool is_float, uint64_t frames,
                      const ChanOut &in, hipStream_t s) {
    if (frames == 0) return DSP_OK;
    WavArgs A{payload, 0, frames, C, in};
    bool vec = ((uintptr_t)payload % 4 == 0) && (C == 1 || C == 2);
    for (uint32_t c = 0; c < C && vec; ++c) vec = ((uintptr_t)in.p[c] % 16) == 0;
    if ((frames + 3) / 4 / (256u * kWavU) > 0x7fffffffull) vec = false;
    if (is_float) enc<32, true>(A, vec, s);
    else if (bits == 16) enc<16, false>(A, vec, s);
    else if (bits == 24) enc<24, false>(A, vec, s);
    else if (bits == 32) enc<32, false>(A, vec, s);
    else return DSP_ERR_UNSUPPORTED;
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
