// render.hip -- CDNA4 kernels for the offline block render.
//
// Replaces the per-block render loop of the reference: render_audio
// (audio.cpp:13-175) pumped in whole blocks of B samples
// (wasapi_audio.cpp:223-251) with the plugin's audio_callback applied in
// place (audio.cpp:160-165).
//
// The offline render of an L-sample file is nblocks = ceil(L/B) blocks; the
// block semantics collapse to a per-sample rule for every sample i of the
// padded render [0, nblocks*B):
//
//     base[c][i] = (c < file_channels && i < L) ? file[c][i] : 0.0f
//     out[c][i]  = callback(base)[c][i]
//
// For the stock plugins whose callback is a per-sample map that rule is one
// streaming kernel: 16-byte loads and non-temporal stores, four float4 per
// thread in flight, one tile per block (HBM-bound, no reuse to tile for).
//
// IR_test's callback is a sequential double recurrence that restarts at
// every block (build/IR_test.cpp:47-58), so its output is input-independent
// and B-periodic.  ramp_table_kernel runs that recurrence on the device,
// exactly as written (one lane, B dependent f64 subtractions), and the
// render broadcasts the B-entry table: 4 B/sample of HBM writes, no reads.
#include "kernels.hpp"

namespace dspb {

__global__ void ramp_table_kernel(float *table, uint32_t B, float gain, float step) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double g = (double)gain;         // double gain = param.gain;
    const double s = (double)step;   // gain -= param.step (float promoted)
#pragma unroll 16
    for (uint32_t i = 0; i < B; ++i) {
        table[i] = (float)g;         // out_buffer[channel][sample] = gain;
        g = g - s;
    }
}


// the launch's map as kernel K applies it to channel c of the launch (a
// gain table: that channel's row of C x B gains)
template <MapKind K>
__device__ __forceinline__ SampleMap map_for(const SampleMap &a, uint32_t c) {
    SampleMap m = a;
    m.kind = K;
    if constexpr (K == MapKind::GainTable) m.table += (uint64_t)c * m.B;
    return m;
}

template <MapKind K>
__device__ __forceinline__ float4 render4(const RenderArgs &A, const float *x, uint64_t i, uint32_t c) {
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (K != MapKind::Ramp && x != nullptr) {
        if (i + 4 <= A.L) {
            b = *reinterpret_cast<const float4 *>(x + i);
        } else {
            if (i + 0 < A.L) b.x = x[i + 0];
            if (i + 1 < A.L) b.y = x[i + 1];
            if (i + 2 < A.L) b.z = x[i + 2];
        }
    }
    if (K == MapKind::Noop) return b;
    const SampleMap m = map_for<K>(A.map, c);
    const uint64_t g = A.goff + i;
    return make_float4(apply_map(m, b.x, g), apply_map(m, b.y, g + 1),
                       apply_map(m, b.z, g + 2), apply_map(m, b.w, g + 3));
}

// Vector path: start % 4 == 0 and every pointer 16-byte aligned.  One tile
// of 256 x kVecU float4 per block (no grid-stride loop: the tile's loads all
// issue before its first store), non-temporal 16-byte stores (the render is
// written once and not read back by this call).  tools/copy_probe.hip: this
// shape streams y = g x at 5.6-5.8 TB/s where a grid-stride loop over a
// capped grid reached 4.6-4.8 (inputs rotated past the Infinity Cache).
constexpr int kVecU = 4;
typedef float f4nt __attribute__((ext_vector_type(4)));
template <MapKind K>
__global__ __launch_bounds__(256) void render_vec_kernel(RenderArgs A) {
    const uint32_t c = blockIdx.y;
    const float *x = (c < A.in_ch) ? A.in.p[c] : nullptr;
    float *o = A.out.p[c];
    const uint64_t n4 = (A.end - A.start) >> 2;
    const uint64_t q0 = (uint64_t)blockIdx.x * (256u * kVecU) + threadIdx.x;
    float4 r[kVecU];
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q < n4) r[u] = render4<K>(A, x, A.start + 4 * q, c);
    }
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q < n4)
            __builtin_nontemporal_store(f4nt{r[u].x, r[u].y, r[u].z, r[u].w},
                                        reinterpret_cast<f4nt *>(o + A.start + 4 * q));
    }
    // scalar tail (end - start not a multiple of 4)
    if (blockIdx.x == 0 && threadIdx.x < ((A.end - A.start) & 3)) {
        const uint64_t i = A.start + 4 * n4 + threadIdx.x;
        const float b = (K != MapKind::Ramp && x != nullptr && i < A.L) ? x[i] : 0.f;
        const SampleMap m = map_for<K>(A.map, c);
        o[i] = apply_map(m, b, A.goff + i);
    }
}

// Scalar path for unaligned pointers or odd starts.
template <MapKind K>
__global__ __launch_bounds__(256) void render_scalar_kernel(RenderArgs A) {
    const uint32_t c = blockIdx.y;
    const float *x = (c < A.in_ch) ? A.in.p[c] : nullptr;
    float *o = A.out.p[c];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const SampleMap m = map_for<K>(A.map, c);
    for (uint64_t i = A.start + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.end;
         i += stride) {
        const float b = (K != MapKind::Ramp && x != nullptr && i < A.L) ? x[i] : 0.f;
        o[i] = apply_map(m, b, A.goff + i);
    }
}

// Elementwise services (dsp.cpp:171-181, 166-168, 208-210).
__global__ __launch_bounds__(256) void gain_kernel(const float *in, float *out, float g,
                                                   uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i] * g;
}
__global__ __launch_bounds__(256) void set_kernel(float v, float *out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = v;
}
__global__ __launch_bounds__(256) void magnitude_kernel(const float *re, const float *im,
                                                        float *out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        // ippsMagnitude_32f (dsp.cpp:166-168) restated without contraction:
        // two rounded products, a rounded sum, a correctly rounded root
        out[i] = __builtin_sqrtf(__fadd_rn(__fmul_rn(re[i], re[i]), __fmul_rn(im[i], im[i])));
}

// Vector path of the elementwise services: every pointer 16-byte aligned,
// one tile of 256 x kVecU float4 per block (all loads before the first
// store, as render_vec_kernel), non-temporal stores, the n % 4 tail by block
// 0.  tools/bw_probe.py: the grid-stride scalar kernels below moved 4.9 TB/s
// (gain) and 6.0 TB/s (set) on 2.76 GB.
enum class Ew { Gain, Set, Mag, Copy };
template <Ew OP>
__device__ __forceinline__ float ew1(const float *a, const float *b, float v, uint64_t i) {
    if constexpr (OP == Ew::Gain) return a[i] * v;
    if constexpr (OP == Ew::Set) return v;
    if constexpr (OP == Ew::Copy) return a[i];
    // ippsMagnitude_32f restated without contraction (see magnitude_kernel)
    return __builtin_sqrtf(__fadd_rn(__fmul_rn(a[i], a[i]), __fmul_rn(b[i], b[i])));
}
template <Ew OP>
__global__ __launch_bounds__(256) void ew_vec_kernel(const float *a, const float *b, float *out, float v,
                                                     uint64_t n) {
    const uint64_t n4 = n >> 2;
    const uint64_t q0 = (uint64_t)blockIdx.x * (256u * kVecU) + threadIdx.x;
    float4 r[kVecU];
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q >= n4) continue;
        if constexpr (OP == Ew::Set) {
            r[u] = make_float4(v, v, v, v);
        } else {
            const float4 x = reinterpret_cast<const float4 *>(a)[q];
            if constexpr (OP == Ew::Gain) r[u] = make_float4(x.x * v, x.y * v, x.z * v, x.w * v);
            if constexpr (OP == Ew::Copy) r[u] = x;
            if constexpr (OP == Ew::Mag) {
                const float4 y = reinterpret_cast<const float4 *>(b)[q];
                r[u] = make_float4(__builtin_sqrtf(__fadd_rn(__fmul_rn(x.x, x.x), __fmul_rn(y.x, y.x))),
                                   __builtin_sqrtf(__fadd_rn(__fmul_rn(x.y, x.y), __fmul_rn(y.y, y.y))),
                                   __builtin_sqrtf(__fadd_rn(__fmul_rn(x.z, x.z), __fmul_rn(y.z, y.z))),
                                   __builtin_sqrtf(__fadd_rn(__fmul_rn(x.w, x.w), __fmul_rn(y.w, y.w))));
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q >= n4) continue;
        if constexpr (OP == Ew::Set)  // a pure write stream: plain stores
            reinterpret_cast<float4 *>(out)[q] = r[u];
        else
            __builtin_nontemporal_store(f4nt{r[u].x, r[u].y, r[u].z, r[u].w}, reinterpret_cast<f4nt *>(out) + q);
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const uint64_t i = 4 * n4 + threadIdx.x;
        out[i] = ew1<OP>(a, b, v, i);
    }
}
static bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
template <Ew OP>
static int launch_ew_vec(const float *a, const float *b, float *out, float v, uint64_t n, hipStream_t s) {
    const uint64_t tiles = ((n >> 2) + 256u * kVecU - 1) / (256u * kVecU);
    if (tiles > 0x7fffffffull) return DSP_ERR_INVALID;
    hipLaunchKernelGGL(ew_vec_kernel<OP>, dim3(tiles ? (uint32_t)tiles : 1u), dim3(256), 0, s, a, b, out, v, n);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

static uint32_t stream_grid(uint64_t work_items) {
    // 256 CUs x 8 blocks: enough to saturate HBM, grid-stride the rest.
    uint64_t g = (work_items + 255) / 256;
    if (g > 2048) g = 2048;
    return g ? (uint32_t)g : 1u;
}

// Loop mode (audio.cpp:100-132): the file wraps, so output sample i of the
// render reads file sample (cursor + i) mod L.  One float per lane and step,
// the index advanced incrementally (one 64-bit modulo per thread): lanes
// stay consecutive, so loads coalesce except at the wrap point.
template <MapKind K>
__global__ __launch_bounds__(256) void render_wrap_kernel(RenderArgs A, uint64_t cursor) {
    const uint32_t c = blockIdx.y;
    const float *x = (c < A.in_ch) ? A.in.p[c] : nullptr;
    float *o = A.out.p[c];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = A.start + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i0 >= A.end) return;
    const uint64_t L = A.L;
    uint64_t j = (K == MapKind::Ramp || x == nullptr) ? 0 : (cursor + i0) % L;
    const uint64_t dj = (K == MapKind::Ramp || x == nullptr) ? 0 : stride % L;
    const SampleMap m = map_for<K>(A.map, c);
    for (uint64_t i = i0; i < A.end; i += stride) {
        const float b = (K != MapKind::Ramp && x != nullptr) ? x[j] : 0.f;
        o[i] = apply_map(m, b, A.goff + i);
        j += dj;
        if (j >= L) j -= L;
    }
}

// Loop mode, vector path (output rows 16-byte aligned, start % 4 == 0): the
// tile of render_vec_kernel -- kVecU float4 outputs per thread, all loads
// before the first non-temporal store -- with the file index advanced per
// sample and wrapped by compare (one wave-uniform 64-bit modulo per block).
// tools/loop_probe.py: the scalar kernel rendered a stereo hour from a 10 s
// file in 0.359 ms (3.9 TB/s of writes).
template <MapKind K>
__global__ __launch_bounds__(256) void render_wrap_vec_kernel(RenderArgs A, uint64_t cursor) {
    const uint32_t c = blockIdx.y;
    const float *x = (c < A.in_ch) ? A.in.p[c] : nullptr;
    float *o = A.out.p[c];
    const uint64_t n4 = (A.end - A.start) >> 2;
    const uint64_t q0 = (uint64_t)blockIdx.x * (256u * kVecU) + threadIdx.x;
    const uint64_t L = A.L;
    const bool rd = K != MapKind::Ramp && x != nullptr;
    const SampleMap m = map_for<K>(A.map, c);
    // the block's first file index is wave-uniform (one scalar modulo per
    // wave); lanes add 4 t < 1024 and wrap by compare when L > 1024
    uint64_t j = 0;
    if (rd) {
        const uint64_t jb = (cursor + A.start + (uint64_t)blockIdx.x * (4u * 256u * kVecU)) % L;
        j = jb + 4u * threadIdx.x;
        if (L > 1024u) j = j >= L ? j - L : j;
        else j %= L;
    }
    float4 r[kVecU];
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q >= n4) continue;
        float b[4] = {0.f, 0.f, 0.f, 0.f};
        if (rd) {
            const uint32_t ra = (uint32_t)(j & 3);  // the same on every lane until a wrap
            if (ra == 0 && j + 4 <= L) {  // aligned, no wrap inside: one 16-byte load
                const float4 t = *reinterpret_cast<const float4 *>(x + j);
                b[0] = t.x, b[1] = t.y, b[2] = t.z, b[3] = t.w;
            } else if (j - ra + 8 <= L) {  // two aligned 16-byte loads, shifted by ra
                const float4 t0 = *reinterpret_cast<const float4 *>(x + (j - ra));
                const float4 t1 = *reinterpret_cast<const float4 *>(x + (j - ra) + 4);
                if (ra == 1) b[0] = t0.y, b[1] = t0.z, b[2] = t0.w, b[3] = t1.x;
                else if (ra == 2) b[0] = t0.z, b[1] = t0.w, b[2] = t1.x, b[3] = t1.y;
                else b[0] = t0.w, b[1] = t1.x, b[2] = t1.y, b[3] = t1.z;
            } else {
                uint64_t jj = j;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    b[k] = x[jj];
                    jj = jj + 1 == L ? 0 : jj + 1;
                }
            }
            j += 4u * 256u;  // the next float4 of this thread
            if (L > 1024u) j = j >= L ? j - L : j;
            else j %= L;
        }
        const uint64_t g = A.goff + A.start + 4 * q;
        r[u] = make_float4(apply_map(m, b[0], g), apply_map(m, b[1], g + 1), apply_map(m, b[2], g + 2),
                           apply_map(m, b[3], g + 3));
    }
#pragma unroll
    for (int u = 0; u < kVecU; ++u) {
        const uint64_t q = q0 + 256u * (uint32_t)u;
        if (q < n4)
            __builtin_nontemporal_store(f4nt{r[u].x, r[u].y, r[u].z, r[u].w},
                                        reinterpret_cast<f4nt *>(o + A.start + 4 * q));
    }
    if (blockIdx.x == 0 && threadIdx.x < ((A.end - A.start) & 3)) {
        const uint64_t i = A.start + 4 * n4 + threadIdx.x;
        const float b = rd ? x[(cursor + i) % L] : 0.f;
        o[i] = apply_map(m, b, A.goff + i);
    }
}

int launch_render_wrap(const RenderArgs &A, uint32_t C, uint64_t cursor, hipStream_t s) {
    if (A.end <= A.start || C == 0) return DSP_OK;
    if (A.in_ch && (A.L == 0 || cursor >= A.L)) return DSP_ERR_INVALID;
    bool vec = (A.start & 3) == 0;
    for (uint32_t c = 0; c < C && vec; ++c) vec = ((uintptr_t)A.out.p[c] & 15u) == 0;
    const uint64_t tiles = (((A.end - A.start) >> 2) + 256u * kVecU - 1) / (256u * kVecU);
    if (vec && tiles <= 0x7fffffffull) {
        const dim3 vgrid(tiles ? (uint32_t)tiles : 1u, C);
        switch (A.map.kind) {
        case MapKind::Noop: hipLaunchKernelGGL(render_wrap_vec_kernel<MapKind::Noop>, vgrid, dim3(256), 0, s, A, cursor); break;
        case MapKind::Gain: hipLaunchKernelGGL(render_wrap_vec_kernel<MapKind::Gain>, vgrid, dim3(256), 0, s, A, cursor); break;
        case MapKind::Ramp: hipLaunchKernelGGL(render_wrap_vec_kernel<MapKind::Ramp>, vgrid, dim3(256), 0, s, A, cursor); break;
        case MapKind::GainTable:
            hipLaunchKernelGGL(render_wrap_vec_kernel<MapKind::GainTable>, vgrid, dim3(256), 0, s, A, cursor);
            break;
        default: return DSP_ERR_INVALID;
        }
        DSPB_HIP(hipGetLastError());
        return DSP_OK;
    }
    uint32_t gx = stream_grid(A.end - A.start);
    gx = (gx + C - 1) / C;
    if (gx == 0) gx = 1;
    dim3 grid(gx, C), block(256);
    switch (A.map.kind) {
    case MapKind::Noop: hipLaunchKernelGGL(render_wrap_kernel<MapKind::Noop>, grid, block, 0, s, A, cursor); break;
    case MapKind::Gain: hipLaunchKernelGGL(render_wrap_kernel<MapKind::Gain>, grid, block, 0, s, A, cursor); break;
    case MapKind::Ramp: hipLaunchKernelGGL(render_wrap_kernel<MapKind::Ramp>, grid, block, 0, s, A, cursor); break;
    case MapKind::GainTable: hipLaunchKernelGGL(render_wrap_kernel<MapKind::GainTable>, grid, block, 0, s, A, cursor); break;
    default: return DSP_ERR_INVALID;
    }
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_ramp_table(float *table, uint32_t B, float gain, float step, hipStream_t s) {
    hipLaunchKernelGGL(ramp_table_kernel, dim3(1), dim3(64), 0, s, table, B, gain, step);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_render(const RenderArgs &A, uint32_t C, bool vec, hipStream_t s) {
    if (A.end <= A.start || C == 0) return DSP_OK;
    uint32_t gx;
    if (vec) {  // one block per 256 x kVecU float4 of every channel
        const uint64_t tiles = ((A.end - A.start) / 4 + 256u * kVecU - 1) / (256u * kVecU);
        if (tiles > 0x7fffffffull) return DSP_ERR_INVALID;
        gx = tiles ? (uint32_t)tiles : 1u;
    } else {
        gx = stream_grid(A.end - A.start);
        gx = (gx + C - 1) / C;  // keep ~2048 blocks in total across channels
        if (gx == 0) gx = 1;
    }
    dim3 grid(gx, C), block(256);
#define DSPB_RENDER_CASE(KIND)                                                            \
    case KIND:                                                                            \
        if (vec)                                                                          \
            hipLaunchKernelGGL(render_vec_kernel<KIND>, grid, block, 0, s, A);            \
        else                                                                              \
            hipLaunchKernelGGL(render_scalar_kernel<KIND>, grid, block, 0, s, A);         \
        break;
    switch (A.map.kind) {
        DSPB_RENDER_CASE(MapKind::Noop)
        DSPB_RENDER_CASE(MapKind::Gain)
        DSPB_RENDER_CASE(MapKind::Ramp)
        DSPB_RENDER_CASE(MapKind::GainTable)
    default:
        return DSP_ERR_INVALID;
    }
#undef DSPB_RENDER_CASE
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_gain(const float *in, float *out, float g, uint64_t n, hipStream_t s) {
    if (!n) return DSP_OK;
    if (al16(in) && al16(out)) return launch_ew_vec<Ew::Gain>(in, nullptr, out, g, n, s);
    hipLaunchKernelGGL(gain_kernel, dim3(stream_grid(n)), dim3(256), 0, s, in, out, g, n);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}
// dsp_copy: the vector kernel when both rows are 16-byte aligned (0 = not
// handled: the caller falls back to hipMemcpyAsync)
int launch_copy(const float *in, float *out, uint64_t n, hipStream_t s, bool *done) {
    *done = false;
    if (!n || !al16(in) || !al16(out)) return DSP_OK;
    *done = true;
    return launch_ew_vec<Ew::Copy>(in, nullptr, out, 0.f, n, s);
}
int launch_set(float v, float *out, uint64_t n, hipStream_t s) {
    if (!n) return DSP_OK;
    if (al16(out)) return launch_ew_vec<Ew::Set>(nullptr, nullptr, out, v, n, s);
    hipLaunchKernelGGL(set_kernel, dim3(stream_grid(n)), dim3(256), 0, s, v, out, n);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}
// compute_IR's impulse (plugin.cpp:27-34): buf[c][i] = (i == 0) for every
// channel, one launch (was a memset + a pageable 4-byte copy per channel)
__global__ void impulse_kernel(ChanOut buf, uint32_t C, uint32_t n) {
    const uint32_t c = blockIdx.y;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        buf.p[c][i] = i == 0 ? 1.f : 0.f;
}
int launch_impulse(const ChanOut &buf, uint32_t C, uint32_t n, hipStream_t s) {
    if (!n || !C) return DSP_OK;
    if (C > (uint32_t)kMaxChannels) return DSP_ERR_INVALID;
    const uint32_t g = (n + 255) / 256 < 32 ? (n + 255) / 256 : 32;
    hipLaunchKernelGGL(impulse_kernel, dim3(g, C), dim3(256), 0, s, buf, C, n);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

int launch_magnitude(const float *re, const float *im, float *out, uint64_t n,
                     hipStream_t s) {
    if (!n) return DSP_OK;
    if (al16(re) && al16(im) && al16(out)) return launch_ew_vec<Ew::Mag>(re, im, out, 0.f, n, s);
    hipLaunchKernelGGL(magnitude_kernel, dim3(stream_grid(n)), dim3(256), 0, s, re, im, out, n);
    DSPB_HIP(hipGetLastError());
    return DSP_OK;
}

}  // namespace dspb
