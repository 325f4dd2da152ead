// stft_pk.hpp -- 8192-point STFT, one wavefront per frame, PACKED fp32 math.
//
// On gfx950 a wave issues one VALU instruction per ~4 cycles whether it is
// v_add_f32 or v_pk_add_f32 (tools/valu_probe.hip: 4.1 vs 4.2 cycles), and
// the scalar SoA kernel (stft_soa.hip) is VALU-bound (PMC: 3979 VALU per
// frame, two waves saturate the SIMD).  This kernel runs the same 64 x 64
// four-step transform with two independent sub-problems in the two halves
// of every VGPR pair, so the butterflies cost half the instructions:
//
//   DFT64 over b as radix-2 DIT: Y[k] = E[k] + W64^k O[k],
//   Y[k+32] = E[k] - W64^k O[k], E/O = DFT32 of the even/odd b.  The
//   pair P[j] = (v[2j], v[2j+1]) (one cx2: re halves, im halves) carries the
//   even and the odd sequence, x2dft32 transforms both at once, one scalar
//   combine step writes (Y[k], Y[k+32]) into the halves of Q[k] -- the
//   two columns kb = k, k + 32 that share the stage twiddle's low digit.
//   Stage twiddles, the LDS transpose (two dwords per pair) and the second
//   DFT64 use the same pairing; the real split pairs (ka, ka + 16).
//
// Loads, render, window and stores are those of stft_soa.hip with options
// 14 (LDS ramp table, lane-major twiddles issued first, computed window).
//
// The kernel template lives in this header; its instantiations are split over
// three translation units, so that each code object is loaded (on the first
// launch of one of its kernels) only when its path is used: stft_pk.hip (the
// dispatcher and the fused IR_test "PER" kernels of the headline),
// stft_pk_paths.hip (the other fused maps and the memory-source STFT),
// stft_pk_ab.hip (A/B and ablation options).
#pragma once
#include "fft_pk.hpp"
#include "frame_load.hpp"

namespace dspb {

// OPT bits (A/B, dsp_stft_soa_options >> 4): 1 = no scheduling barriers in
// the DFT32s, 2 = none in the twiddle loop, 4 = none in the split loop
// 8 = cached render stores (default: non-temporal -- the render is written
// once and never read back; 2% faster at the headline shape), 16 =
// non-temporal magnitude stores (slower: 256-byte row pieces need the L2 to
// merge them), 32 = 4097-bin rows staged through LDS and stored as 16-byte
// segments (no gain; implies 64), 64 = the older scalar last combine and
// (ka, ka + 16) split (default: the packed combine + split_y2, 60 VALU
// fewer per frame, the same bits)
enum { kPkNoBarDft = 1, kPkNoBarTw = 2, kPkNoBarSplit = 4, kPkRenderCached = 8, kPkNtMag = 16, kPkMagLds = 32,
       kPkOldSplit = 64, kPkAbNoRender = 128, kPkAbNoMag = 256, kPkMagStage = 512, kPkOcc3 = 1024,
       kPkMemAos = 2048, kPkNoRemap = 4096, kPkAbNoXpose = 8192, kPkMemPf = 16384, kPkW1 = 65536,
       kPkMemHop = 131072 };
// 65536 = one wave per workgroup (64 threads, one 64 x 65 tile): a slot frees as its frame ends
// 131072 = memory frames on stft8192_mem_hop_kernel (a workgroup's 5 hops staged once in LDS)
// 16384 = memory frames on stft8192_mem_pf_kernel (persistent, LDS hop prefetch)
// 8192: ablation only (results discarded): no LDS transpose
// 4096 = frames in dispatch order (no XCD remap: all XCDs write one frontier)
// 2048 = memory frames (computed window) loaded as 64 pairs and regrouped
// after the window multiply (the older path; default: regrouped at the load)
// 1024 = 3 waves per SIMD (OCC template argument): fft4096_pk_y2_lo's
// 64 x 33 transpose tile and just-in-time stage twiddles
// 512 = split_y2 stages the row in LDS at the row's 16-byte phase and stores
// it as aligned 16-byte pieces (16 dwordx4 + <= 7 dwords instead of 65 dwords);
// with 16, those pieces are non-temporal stores (16 alone: split_y2's
// dword row stores non-temporal)
// 128 / 256: ablation only (A/B of what the stores cost): skip the render
// stores / the magnitude stores of split_y2 (results discarded)
// default: no scheduling barriers (round 2: 1.0-1.7% faster on the headline,
// 0.1-0.5% on the memory and gain STFTs, the same VGPRs and spills;
// profiles/r02_default_opt_ab.txt)
constexpr int kPkDefaultOpt = kPkNoBarDft | kPkNoBarTw | kPkNoBarSplit;
// the fused IR_test (PER) kernels of the headline add one wave per workgroup:
// 0.8-2.2% faster there, but 1-2% slower for the paths that read a signal
// (memory, gain), whose four-frame workgroups share their hops in L2
// (profiles/r02_w1_ab.txt)
constexpr int kPkPerOpt = kPkDefaultOpt | kPkW1;

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // a row is only dword-aligned
typedef float f4a __attribute__((ext_vector_type(4)));               // 16-byte aligned

template <bool NT, typename T>
__device__ __forceinline__ void st(T *p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__device__ __forceinline__ void st4u(float *p, f4u v) {  // p: dword-aligned
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4u *>(p));
    else *reinterpret_cast<f4u *>(p) = v;
}

template <int KM>
__device__ __forceinline__ void put_bin(float *mrow, uint32_t K, uint32_t k, float m) {
    if constexpr (KM == kKPartial) {
        if (k < K) mrow[k] = m;
    } else {
        mrow[k] = m;
        if constexpr (KM == kKMirror) mrow[(8192u - k) & 8191u] = m;  // k = 0: itself
    }
}

// Real split and |X| from the packed last combine (fft4096_pk_y2):
// Y2[q] = (Z[l + 64 q], Z[l + 64 (q + 32)]), q < 32, Z = the 4096-point FFT
// of z[m] = x[2m] + i x[2m+1] (window pre-scaled by 0.5/sqrt N).
//   X[k] = E + T, X[M - k] = conj(E - T), E = Z[k] + conj Z[M - k],
//   T = W8192^k (-i)(Z[k] - conj Z[M - k]), M = 4096.
// Iteration q < 16 takes k = l + 64 q and k + 2048 in the two halves; the
// twiddle of the upper half is -i times the lower one, so one complex
// W8192^(l + 64 q) serves both.  The partners Z[M - k], Z[M - k - 2048]
// are the two halves of Y2[31 - q], swapped, on lane 64 - l (lane 0: its
// own Y2[32 - q], or Y2[0] unswapped at q = 0, which pairs bin 0 with 4096
// and bin 2048 with itself).  Bins 1024 / 3072 (lane 0, Y2[16]) are left
// over and done at the end.  Bins per iteration: l + 64 q, 2048 + l + 64 q,
// 4096 - l - 64 q, 2048 - l - 64 q.
template <int KM, bool BAR, bool NOSTORE = false, bool STAGE = false, bool STAGE_NT = false>
__device__ __forceinline__ void split_y2(const cx2 (&Y2)[32], float *mrow, uint32_t K, const v2f *tw,
                                         uint32_t lane, float *lds) {
    static_assert(!STAGE || KM == kKHalf, "staged rows: 4097 bins");
    float acc = 0.f;  // NOSTORE: keeps the magnitudes live
    // STAGE: bin k goes to lds[k + a], a = the row's dword phase mod 4, so
    // LDS float4 j is the 16-byte-aligned global piece at bins [4j - a, 4j - a + 4)
    const uint32_t a = (uint32_t)(reinterpret_cast<uintptr_t>(mrow) >> 2) & 3u;
    float *sl = lds + a;
    const uint32_t src = ((64u - lane) & 63u) * 4u;
    const bool l0 = lane == 0;
    const v2f wl = tw[lane];  // W8192^l
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        if (BAR) __builtin_amdgcn_sched_barrier(0);
        const cx2 a = Y2[q == 0 ? 0 : 32 - q], b = Y2[31 - q];
        // what this lane sends to lane 64 - l (select on values: keeps Y2 in VGPRs)
        const float sxr = l0 ? (q == 0 ? a.r.x : a.r.y) : b.r.y;
        const float sxi = l0 ? (q == 0 ? a.i.x : a.i.y) : b.i.y;
        const float syr = l0 ? (q == 0 ? a.r.y : a.r.x) : b.r.x;
        const float syi = l0 ? (q == 0 ? a.i.y : a.i.x) : b.i.x;
        const cx2 Pp = cx2{v2f{bperm(src, sxr), bperm(src, syr)}, v2f{bperm(src, sxi), bperm(src, syi)}};
        const cx2 Z = Y2[q];
        const cx2 E = cx2{Z.r + Pp.r, Z.i - Pp.i};
        const cx2 D = cx2{Z.r - Pp.r, Z.i + Pp.i};
        // u = W8192^(l + 64 q); T = (-i D.x u, -i D.y (-i u)) with U1 = u, U2 = (u.i, -u.r)
        v2f u = wl;
        if (q) u = v2f{wl.x, wl.x} * v2f{kW128_re[q], kW128_im[q]} + v2f{wl.y, wl.y} * v2f{-kW128_im[q], kW128_re[q]};
        // a (.) U2 with U2 = (u.y, -u.x) as one v_pk_mul: the swap and the
        // negation ride on the operand's op_sel / neg_hi (the compiler builds
        // U2 with a v_xor + v_mov otherwise)
        v2f rU2, iU2;
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(rU2) : "v"(D.r), "v"(u));
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(iU2) : "v"(D.i), "v"(u));
        const cx2 T = cx2{D.i * u + rU2, iU2 - D.r * u};
        const cx2 X1 = E + T;  // 2 X[k], k = l + 64 q (+ 2048)
        const cx2 X2 = E - T;  // 2 conj X[M - k]
        const v2f q1 = X1.r * X1.r + X1.i * X1.i;
        const v2f q2 = X2.r * X2.r + X2.i * X2.i;
        const uint32_t k = lane + 64u * (uint32_t)q;
        if constexpr (NOSTORE) {
            acc += __builtin_amdgcn_sqrtf(q1.x) + __builtin_amdgcn_sqrtf(q1.y) + __builtin_amdgcn_sqrtf(q2.x) +
                   __builtin_amdgcn_sqrtf(q2.y);
        } else if constexpr (STAGE) {
            (sl + lane)[64 * q] = __builtin_amdgcn_sqrtf(q1.x);
            (sl + 2048u + lane)[64 * q] = __builtin_amdgcn_sqrtf(q1.y);
            (sl + 4096u - lane)[-64 * q] = __builtin_amdgcn_sqrtf(q2.x);
            (sl + 2048u - lane)[-64 * q] = __builtin_amdgcn_sqrtf(q2.y);
        } else if constexpr (KM == kKHalf) {  // four lane-based row pointers, constant offsets
            st<STAGE_NT>(&(mrow + lane)[64 * q], __builtin_amdgcn_sqrtf(q1.x));
            st<STAGE_NT>(&(mrow + 2048u + lane)[64 * q], __builtin_amdgcn_sqrtf(q1.y));
            st<STAGE_NT>(&(mrow + 4096u - lane)[-64 * q], __builtin_amdgcn_sqrtf(q2.x));
            st<STAGE_NT>(&(mrow + 2048u - lane)[-64 * q], __builtin_amdgcn_sqrtf(q2.y));
        } else {
            put_bin<KM>(mrow, K, k, __builtin_amdgcn_sqrtf(q1.x));
            put_bin<KM>(mrow, K, 2048u + k, __builtin_amdgcn_sqrtf(q1.y));
            put_bin<KM>(mrow, K, 4096u - k, __builtin_amdgcn_sqrtf(q2.x));
            put_bin<KM>(mrow, K, 2048u - k, __builtin_amdgcn_sqrtf(q2.y));
        }
    }
    if constexpr (NOSTORE) {
        if (acc == -1.f) mrow[lane] = acc;  // never true: |X| >= 0
        return;
    }
    if (l0) {  // bins 1024 and 3072: Z[1024] = Y2[16].x, Z[3072] = Y2[16].y
        const cx z1 = cx{Y2[16].r.x, Y2[16].i.x}, z2 = cx{Y2[16].r.y, Y2[16].i.y};
        const cx E = cx{z1.r + z2.r, z1.i - z2.i}, D = cx{z1.r - z2.r, z1.i + z2.i};
        const float c = 0x1.6a09e6p-1f;  // W8192^1024 = (c, -c)
        const cx T = cx{c * (D.i - D.r), -c * (D.i + D.r)};
        const cx X1 = E + T, X2 = E - T;
        const float m1 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X1.r, X1.r, X1.i * X1.i));
        const float m2 = __builtin_amdgcn_sqrtf(__builtin_fmaf(X2.r, X2.r, X2.i * X2.i));
        if constexpr (STAGE) {
            sl[1024] = m1;
            sl[3072] = m2;
        } else {
            put_bin<KM>(mrow, K, 1024u, m1);
            put_bin<KM>(mrow, K, 3072u, m2);
        }
    }
    if constexpr (STAGE) {
        lds_fence();
        // aligned pieces j in [j0, j1]: bins [4j - a, 4j - a + 4) inside [0, 4097)
        const uint32_t j0 = a ? 1u : 0u, j1 = (4093u + a) >> 2;
        float *gb = mrow - a;  // 16-byte aligned
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const uint32_t j = j0 + 64u * (uint32_t)it + lane;
            if (it < 15 || j <= j1)
            {
                const float4 q = reinterpret_cast<const float4 *>(lds)[j];
                st<STAGE_NT>(reinterpret_cast<f4a *>(gb + 4u * j), f4a{q.x, q.y, q.z, q.w});
            }
        }
        // head bins [0, 4 j0 - a) and tail bins [4 j1 + 4 - a, 4097): at most 3 + 4
        const uint32_t head = 4u * j0 - a, tail0 = 4u * j1 + 4u - a;
        if (lane < head) mrow[lane] = sl[lane];
        if (lane >= 8u && tail0 + (lane - 8u) < 4097u) mrow[tail0 + lane - 8u] = sl[tail0 + lane - 8u];
    }
}

// PER (Ramp, pow2 B <= 4096): the frame's sample pairs repeat every PER
// values of b (PER = max(1, B / 128)), so only v[0 .. PER) are fetched from
// the block table -- 4 gathers at B = 512 -- and v[b] = v[b mod PER] is a
// register alias.  PER = 0: generic path.
template <int OPT>
constexpr uint32_t pk_waves_per_block() { return (OPT & kPkW1) ? 1u : 4u; }
// waves per workgroup of the default and the PER kernels (the launches size
// their grids by them)
constexpr uint32_t kPkWpb = pk_waves_per_block<kPkDefaultOpt>();
constexpr uint32_t kPkPerWpb = pk_waves_per_block<kPkPerOpt>();

template <int SRC, int KM, MapKind MK, bool POW2, bool WINC, int PER = 0, int OPT = kPkDefaultOpt, int OCC = 2>
// (OCC waves per SIMD whatever the workgroup size: stated as waves per EU,
// which __launch_bounds__' workgroup count does not pin for one-wave groups)
__global__ __launch_bounds__(64 * pk_waves_per_block<OPT>()) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
void stft8192_pk_kernel(Stft8kArgs A) {
    constexpr uint32_t WPB = pk_waves_per_block<OPT>();
    __shared__ __attribute__((aligned(16))) float lds_all[WPB][OCC >= 3 ? 64 * 33 : 64 * 65];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ch = blockIdx.y;
    const uint64_t f = (uint64_t)((OPT & kPkNoRemap) ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x)) * WPB + wave;
    constexpr bool SOA = WINC && MK == MapKind::Ramp && PER > 0 && SRC == kSrcRender;
    // memory frames with the computed window: two dwordx2 loads per pair
    // (columns 2j, 2j+1) regrouped into even/odd halves
    constexpr bool MSOA = WINC && SRC == kSrcMemory && !(OPT & kPkMemAos);
    // periodic frames whose period in j divides 8: the window is fused into
    // the first DFT4s (x2dft4 over j0 + 8 m sees one x), on the default FFT
    constexpr bool W4 = SOA && (8 % (PER >= 2 ? PER / 2 : 1)) == 0 && OCC == 2 &&
                        !(OPT & (kPkOldSplit | kPkMagLds | kPkAbNoXpose));
    const uint64_t fs = f * (uint64_t)A.H;
    if (f >= A.F) {  // whole wave leaves; nothing below waits on other waves
        if constexpr (SOA) {
            // the render tail no frame owns, [F H, tail_end): H samples per wave
            if (fs < A.tail_end) {
                const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
                float *o = A.out.p[ch] + fs;
                const uint64_t n = A.tail_end - fs;
#pragma unroll 4
                for (uint32_t b = 0; 128u * b < A.H; ++b) {
                    const uint32_t e = 128u * b + 2u * lane;  // even: tail_end is a multiple of B >= 2
                    if (e < n) {
                        const uint32_t q = (p0 + 128u * b) & A.map.b_mask;
                        const v2f t = A.map.closed ? v2f{ramp_value(A.map, q), ramp_value(A.map, q + 1)}
                                                   : v2f{A.map.table[q], A.map.table[q + 1]};
                        reinterpret_cast<v2f *>(o + 128u * b)[lane] = t;
                    }
                }
            }
        }
        return;
    }
    float *lds = lds_all[wave];
    const float *x = (ch < A.in_ch) ? A.in.p[ch] : nullptr;

    // ---- 0. constants, issued before the frame -----------------------------
    // tlo[j] = W4096^(l j), thp[h] = (W4096^(8 l h), W4096^(8 l (h + 4)))
    // (capi.cpp get_tw: lane-major rows after T8192)
    static_assert(OCC == 2 || (SOA && !(OPT & (kPkOldSplit | kPkMagLds | kPkMagStage))),
                  "3 waves per SIMD: the PER path with split_y2");
    cx tlo[8];
    cx2 thp[4];
    if constexpr (OCC == 2) {  // (OCC 3 loads them inside fft4096_pk_y2_lo)
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            const v2f a = (A.tw + 8192u + 64u * (uint32_t)(j - 1))[lane];
            tlo[j] = cx{a.x, a.y};
        }
        const float4 *tp4 = reinterpret_cast<const float4 *>(A.tw + 8192u + 896u);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const float4 t = tp4[64u * (uint32_t)h + lane];
            thp[h] = cx2{v2f{t.x, t.y}, v2f{t.z, t.w}};
        }
    }
    float4 wbase = float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (WINC) wbase = A.wbase[lane];

    cx2 P[32];
    // SoA frame path (computed window, and a periodic ramp table or a full
    // frame in memory): the frame is loaded straight into even/odd pairs --
    // X[j] = ((x_e(2j), x_e(2j+1)), (x_o(2j), x_o(2j+1))), x_e(b) = sample
    // 2 lane + 128 b, x_o(b) the next one -- so the window is two v_pk_mul
    // per pair with no register shuffles.
    // (for a frame in memory the 128 dword loads this needs cost more than
    // the shuffles they save: 0.75 vs 0.65 ms per stereo hour, so memory
    // frames keep the dwordx2 path below)
    if constexpr (SOA || MSOA) {
        constexpr int NJ = PER >= 2 ? PER / 2 : 1;
        cx2 X[NJ];
        if constexpr (SOA) {
            const uint32_t p0 = (uint32_t)(A.goff + fs) + 2u * lane;
            const float *T = A.map.table;
            if (A.map.closed) {  // table values in closed form (common.hpp ramp_value)
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
            // the render output: sample pairs of column b repeat with period PER
            float *o = A.out.p[ch] + fs;
            v2f st[PER >= 2 ? PER : 1];
#pragma unroll
            for (int b = 0; b < (PER >= 2 ? PER : 1); ++b)
                st[b] = v2f{X[b / 2].r[b & 1], X[b / 2].i[b & 1]};
            constexpr bool NT = !(OPT & kPkRenderCached);
            if (OPT & kPkAbNoRender) {
            } else if (A.H == 4096u) {  // the headline hop: 32 columns, no per-store branch
#pragma unroll
                for (int b = 0; b < 32; ++b)
                    dspb::st<NT>(reinterpret_cast<v2f *>(o + 128u * (uint32_t)b) + lane, st[b % (PER >= 2 ? PER : 1)]);
            } else {
#pragma unroll
                for (int b = 0; b < 64; ++b)
                    if (128u * (uint32_t)b < A.H)
                        dspb::st<NT>(reinterpret_cast<v2f *>(o + 128u * (uint32_t)b) + lane,
                                     st[b % (PER >= 2 ? PER : 1)]);
            }
        }
        // w(n) = wa - wb cos(theta n) = wa - u C_b + v S_b per parity, with
        // u = wb cos(theta n0), v = wb sin(theta n0) of the lane's base angle
        const float ue = A.wb * wbase.x, ve = A.wb * wbase.y, uo = A.wb * wbase.z, vo = A.wb * wbase.w;
        if constexpr (SOA) {
            // the frame repeats with period NJ in j: x w = x wa - (x u) C + (x v) S
            // with x wa, x u, x v formed once per distinct x (XA holds 4 x wa
            // when the first DFT4s are fused: W4)
            cx2 XA[NJ], XU[NJ], XV[NJ];
            const float wa = W4 ? 4.f * A.wa : A.wa;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                XA[jj] = cx2{X[jj].r * v2f{wa, wa}, X[jj].i * v2f{wa, wa}};
                XU[jj] = cx2{X[jj].r * v2f{ue, ue}, X[jj].i * v2f{uo, uo}};
                XV[jj] = cx2{X[jj].r * v2f{ve, ve}, X[jj].i * v2f{vo, vo}};
            }
            auto fma2 = [](v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); };
            if constexpr (W4) {
                // the first DFT32's first DFT4s, over j = j0 + 8 m (m < 4), of
                // the windowed frame P[j] = XA + XV S_j - XU C_j: every input of
                // one DFT4 has the same x (8 is a multiple of NJ), so each output
                // is XA, XV and XU times sums of window constants -- 20 packed
                // instructions per DFT4 instead of 16 for the window and 16 for
                // the butterflies (x2dft8<true> continues from here)
                auto Sv = [](int j) { return v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]}; };
                auto Cv = [](int j) { return v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}; };
#pragma unroll
                for (int j0 = 0; j0 < 8; ++j0) {
                    const int jj = j0 % NJ;
                    const v2f s0 = Sv(j0), s1 = Sv(j0 + 8), s2 = Sv(j0 + 16), s3 = Sv(j0 + 24);
                    const v2f c0 = Cv(j0), c1 = Cv(j0 + 8), c2 = Cv(j0 + 16), c3 = Cv(j0 + 24);
                    const cx2 xa = XA[jj], xu = XU[jj], xv = XV[jj];
                    // X0 = 4 XA + XV (s0 + s1 + s2 + s3) - XU (c0 + ... + c3)
                    const v2f sA = (s0 + s1) + (s2 + s3), cA = (c0 + c1) + (c2 + c3);
                    P[j0] = cx2{fma2(-xu.r, cA, fma2(xv.r, sA, xa.r)), fma2(-xu.i, cA, fma2(xv.i, sA, xa.i))};
                    // X2 = XV (s0 - s1 + s2 - s3) - XU (...)
                    const v2f sC = (s0 - s1) + (s2 - s3), cC = (c0 - c1) + (c2 - c3);
                    P[j0 + 16] = cx2{fma2(-xu.r, cC, xv.r * sC), fma2(-xu.i, cC, xv.i * sC)};
                    // t1 = P[j0] - P[j0 + 16] terms, q = P[j0 + 8] - P[j0 + 24]:
                    // X1 = t1 - i q, X3 = t1 + i q
                    const v2f sT = s0 - s2, cT = c0 - c2, sQ = s1 - s3, cQ = c1 - c3;
                    const cx2 t1 = cx2{fma2(-xu.r, cT, xv.r * sT), fma2(-xu.i, cT, xv.i * sT)};
                    const cx2 q = cx2{fma2(-xu.r, cQ, xv.r * sQ), fma2(-xu.i, cQ, xv.i * sQ)};
                    P[j0 + 8] = cx2{t1.r + q.i, t1.i - q.r};
                    P[j0 + 24] = cx2{t1.r - q.i, t1.i + q.r};
                }
            } else {
#pragma unroll
                for (int j = 0; j < 32; ++j) {
                    const v2f C = v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}, S = v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]};
                    const int jj = j % NJ;
                    P[j] = cx2{fma2(-XU[jj].r, C, fma2(XV[jj].r, S, XA[jj].r)),
                               fma2(-XU[jj].i, C, fma2(XV[jj].i, S, XA[jj].i))};
                }
            }
        } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const v2f C = v2f{kWinB_c[2 * j], kWinB_c[2 * j + 1]}, S = v2f{kWinB_s[2 * j], kWinB_s[2 * j + 1]};
            const v2f we = (v2f{ve, ve} * S + v2f{A.wa, A.wa}) - v2f{ue, ue} * C;
            const v2f wo = (v2f{vo, vo} * S + v2f{A.wa, A.wa}) - v2f{uo, uo} * C;
            // (x[2l + 256 j], x[2l + 256 j + 1]) and 128 samples on
            const v2f a = reinterpret_cast<const v2f *>(x + fs + 256u * (uint32_t)j)[lane];
            const v2f b = reinterpret_cast<const v2f *>(x + fs + 256u * (uint32_t)j + 128u)[lane];
            const cx2 xj = cx2{v2f{a.x, b.x}, v2f{a.y, b.y}};
            P[j] = cx2{xj.r * we, xj.i * wo};
        }
        }
    } else {
    // ---- 1. frame (+ fused render) -----------------------------------------
    cx v[64];
    if constexpr (SRC == kSrcMemory) {
        if (A.valid >= 8192u) {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const v2f t = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
                v[b] = cx{t.x, t.y};
            }
        } else {
#pragma unroll
            for (int b = 0; b < 64; ++b) {
                const uint32_t s = 2u * lane + 128u * (uint32_t)b;
                v2f t = v2f{0.f, 0.f};
                if (s < A.valid) t = reinterpret_cast<const v2f *>(x + fs + 128u * (uint32_t)b)[lane];
                v[b] = cx{t.x, t.y};
            }
        }
    } else {
        if constexpr (MK == MapKind::Ramp && POW2) {
            if (A.map.B >= 4u && A.map.B <= 4096u) lds_table_frame(A, lds, fs, lane, v);
            else s_render_frame<MK, POW2>(A, x, fs, lane, v);
        } else if constexpr (MK == MapKind::GainTable && POW2) {
            if (A.map.B >= 4u && A.map.B <= 512u) reg_gain_table_frame(A, x, fs, lane, v, ch);
            else if (A.map.B >= 4u && A.map.B <= 4096u) lds_gain_table_frame(A, lds, x, fs, lane, v, ch);
            else s_render_frame<MK, POW2>(A, x, fs, lane, v, ch);
        } else {
            s_render_frame<MK, POW2>(A, x, fs, lane, v, ch);
        }
        float *o = A.out.p[ch] + fs;
        constexpr bool NT = !(OPT & kPkRenderCached);
        if (A.H == 4096u) {
#pragma unroll
            for (int b = 0; b < 32; ++b)
                st<NT>(reinterpret_cast<v2f *>(o + 128u * (uint32_t)b) + lane, v2f{v[b].r, v[b].i});
        } else {
#pragma unroll
            for (int b = 0; b < 64; ++b)
                if (128u * (uint32_t)b < A.H)
                    st<NT>(reinterpret_cast<v2f *>(o + 128u * (uint32_t)b) + lane, v2f{v[b].r, v[b].i});
        }
    }

    // ---- 2. window (pre-scaled by 0.5/sqrt N), packed into even/odd pairs ---
    {
        // w(n) = wa - wb cos(theta n) = wa - u C_b + v S_b, n = 2 lane + {0, 1} + 128 b
        const v2f uu = v2f{A.wb * wbase.x, A.wb * wbase.z}, vv = v2f{A.wb * wbase.y, A.wb * wbase.w};
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            v2f w[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int b = 2 * j + h;
                if constexpr (WINC) {
                    w[h] = (vv * kWinB_s[b] + v2f{A.wa, A.wa}) - uu * kWinB_c[b];
                } else {
                    w[h] = (A.win2 + 64u * (uint32_t)b)[lane];
                }
            }
            P[j] = cx2{v2f{v[2 * j].r * w[0].x, v[2 * j + 1].r * w[1].x},
                       v2f{v[2 * j].i * w[0].y, v[2 * j + 1].i * w[1].y}};
        }
    }
    }  // !SOA

    if constexpr (!(OPT & (kPkOldSplit | kPkMagLds))) {
        // ---- 3-5. 4096-point FFT with a packed last combine:
        // Y2[q] = (Z[l + 64 q], Z[l + 64 (q + 32)])
        cx2 Y2[32];
        if constexpr (OCC >= 3) fft4096_pk_y2_lo<!(OPT & kPkNoBarDft)>(P, lds, A.tw, lane, Y2);
        else fft4096_pk_y2<!(OPT & kPkNoBarDft), !(OPT & kPkNoBarTw), (OPT & kPkAbNoXpose) != 0, NoHook, W4>(
            P, lds, tlo, thp, lane, Y2);
        split_y2<KM, !(OPT & kPkNoBarSplit), (OPT & kPkAbNoMag) != 0, KM == kKHalf && (OPT & kPkMagStage) != 0,
                 (OPT & kPkNtMag) != 0>(Y2, A.mag.p[ch] + f * A.ld, A.K, A.tw, lane, lds);
        return;
    }

    // ---- 3-5. 4096-point complex FFT of the packed frame (fft_pk.hpp):
    // Z[l + 64 ka] = zp[ka] (ka < 32), zm[ka - 32]
    cx zp[32], zm[32];
    fft4096_pk<false, !(OPT & kPkNoBarDft), !(OPT & kPkNoBarTw)>(P, lds, tlo, thp, lane, zp, zm);

    // ---- 6. paired real split over (ka, ka + 16), ka < 16 ------------------
    // X[k] = E + T and X[M-k] = conj(E - T), k = l + 64 ka, partner
    // Z[M - k] = Z[63 - ka] of lane 64 - l (lane 0: its own Z[64 - ka]).
    float *mrow = A.mag.p[ch] + f * A.ld;
    const uint32_t src = ((64u - lane) & 63u) * 4u;
    const bool l0 = lane == 0;
    const v2f wl2 = A.tw[lane];  // W8192^l
    const cx wl = cx{wl2.x, wl2.y};
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) {
        if (!(OPT & kPkNoBarSplit)) __builtin_amdgcn_sched_barrier(0);
        // (select on values: a select of two array addresses would keep
        // zp/zm in scratch)
        const cx a0 = ka == 0 ? zp[0] : zm[32 - ka], b0 = zm[31 - ka];
        const cx a1 = zm[16 - ka], b1 = zm[15 - ka];
        const cx s0 = cx{l0 ? a0.r : b0.r, l0 ? a0.i : b0.i};
        const cx s1 = cx{l0 ? a1.r : b1.r, l0 ? a1.i : b1.i};
        const cx2 Pp = cx2{v2f{bperm(src, s0.r), bperm(src, s1.r)}, v2f{bperm(src, s0.i), bperm(src, s1.i)}};
        const cx2 Z = cx2{v2f{zp[ka].r, zp[ka + 16].r}, v2f{zp[ka].i, zp[ka + 16].i}};
        const cx2 E = cx2{Z.r + Pp.r, Z.i - Pp.i};  // 2 E   (partner conjugated)
        const cx2 D = cx2{Z.r - Pp.r, Z.i + Pp.i};  // 2 i O
        const cx2 tw = cmulb(wl, cx2{v2f{kW128_re[ka], kW128_re[ka + 16]},
                                     v2f{kW128_im[ka], kW128_im[ka + 16]}});  // W8192^k
        const cx2 T = cmul2(negi(D), tw);  // 2 W^k O
        const cx2 X1 = E + T;              // 2 X[k]
        const cx2 X2 = E - T;              // 2 conj X[M - k]
        const v2f q1 = X1.r * X1.r + X1.i * X1.i;
        const v2f q2 = X2.r * X2.r + X2.i * X2.i;
        const float m1[2] = {__builtin_amdgcn_sqrtf(q1.x), __builtin_amdgcn_sqrtf(q1.y)};
        const float m2[2] = {__builtin_amdgcn_sqrtf(q2.x), __builtin_amdgcn_sqrtf(q2.y)};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t kk = (uint32_t)(ka + 16 * h);
            const uint32_t k1 = lane + 64u * kk;  // < 2048
            const uint32_t k2 = 4096u - k1;        // > 2048 (4096 at k1 = 0)
            if constexpr (KM == kKHalf && (OPT & kPkMagLds)) {
                lds[64u * kk + lane] = m1[h];
                lds[4096u - 64u * kk - lane] = m2[h];
            } else if constexpr (KM == kKPartial) {
                if (k1 < A.K) mrow[k1] = m1[h];
                if (k2 < A.K) mrow[k2] = m2[h];
            } else {
                st<(OPT & kPkNtMag) != 0>(mrow + 64u * kk + lane, m1[h]);
                st<(OPT & kPkNtMag) != 0>(mrow + 4096u - 64u * kk - lane, m2[h]);
                if constexpr (KM == kKMirror) {
                    mrow[k1 == 0 ? 0u : 8192u - k1] = m1[h];
                    (mrow + 4096u + 64u * kk)[lane] = m2[h];
                }
            }
        }
    }
    if constexpr (KM == kKHalf && (OPT & kPkMagLds)) {
        if (l0) {
            const cx Z = zm[0];
            lds[2048] = 2.f * __builtin_amdgcn_sqrtf(__builtin_fmaf(Z.r, Z.r, Z.i * Z.i));
        }
        lds_fence();
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 q = reinterpret_cast<const float4 *>(lds)[64 * i + lane];
            st4u<(OPT & kPkNtMag) != 0>(mrow + 256u * (uint32_t)i + 4u * lane, f4u{q.x, q.y, q.z, q.w});
        }
        if (l0) mrow[4096] = lds[4096];
        return;
    }
    if (l0) {  // the self-paired bin k = 2048: |X| = 2 |Z[2048]| (scaled), Z[2048] = zm[0]
        const cx Z = zm[0];
        const float m = 2.f * __builtin_amdgcn_sqrtf(__builtin_fmaf(Z.r, Z.r, Z.i * Z.i));
        if (KM != kKPartial || 2048u < A.K) mrow[2048] = m;
        if (KM == kKMirror) mrow[6144] = m;
    }
}

// the launches of stft_pk_paths.hip / stft_pk_ab.hip (DSP_OK or a status)
int launch_pk_paths(const Stft8kArgs &A, bool fused, int km, bool pow2, bool winc, dim3 grid, hipStream_t s);
// the A/B and ablation variants (tools build, stft_pk_ab.hip): launches the
// variant `opt` selects and returns true, or false when it has none for A
bool stft_pk_ab_dispatch(const Stft8kArgs &A, uint32_t C, bool fused, int opt, dim3 grid, hipStream_t s, int *st);


}  // namespace dspb
