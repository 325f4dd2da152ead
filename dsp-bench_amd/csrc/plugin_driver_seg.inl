// plugin_driver_seg.inl -- the speculative-segment kernels of the plugin
// driver (a State-writing callback rendered in parallel with the serial
// chain's bits; DESIGN 4.6, module.cpp module_render_seg).  Appended to
// plugin_driver.inl in the module's translation unit.
// ---- a State the callback writes: speculative segments (module_render_seg)
// The file's blocks are cut into K segments of `seg` blocks.  Pass 1 runs
// every segment at once, one lane each, from the live State after `warm`
// blocks of warm-up on the blocks before it (their output discarded), and
// records the State it rendered each kept block from (st_blk, one per block
// of the file) and the State it ended with (st_end).  The callback is a
// function of (Parameters, State, block) -- the analysis proved it writes no
// other memory -- so a segment whose first block's State equals, bit for bit,
// the true State there rendered exactly what the serial chain renders;
// segment 0 starts from the live State itself, and by induction every segment
// k whose st_blk at its first block equals st_end[k - 1] is exact when
// segment k - 1 is.  A check lists the others (and hands each its
// predecessor's st_end), a rerun pass renders the listed segments again from
// those States, in parallel, each only until its State meets the one
// recorded at a block boundary (from there on the recorded blocks were
// rendered from the same bits); after the last check one workgroup walks the
// segments in order and reruns serially, with the same early stop, whatever
// still differs, so the result is the serial chain's whatever the plugin
// does.  Filters forget their State: their trajectories from different States
// meet bit for bit within a few hundred samples, and one pass suffices.
struct dspb_seg_args {
    dspb_render_args R;
    State *st_blk;          // [nblocks] the State each block was rendered from
    State *st_end;          // [K] the State each segment ended with
    unsigned *list;         // segments to rerun (check -> rerun)
    unsigned *count;        // how many
    unsigned *prev_count;   // a rerun's check: the rerun's count (0: nothing changed, skip)
    unsigned char *flags;   // the last check: 1 = differed
    unsigned *stats;        // [0, 4) segments that differed per warm-up level, [4] / [5] after
                            // rerun 1 / 2, [7] serial reruns of the walk, [8, 12) levels run,
                            // [12] the State chain took over from the levels (dspb_seg_chain),
                            // [13] segments whose first State (the chain's record) differed from
                            // the State the segment before ended with, [14] blocks whose State in
                            // the exact rerun differed from the chain's record
    unsigned long long seg; // blocks per segment
    unsigned K;             // segments
    unsigned warm;          // pass 1: warm-up blocks
    unsigned prev_warm;     // pass 1 at level > 0: the warm-up of the level before
    unsigned level;         // pass 1 / its check: the warm-up level (~0u: a rerun's check)
    unsigned mode;          // segments: 0 = pass 1 (every segment), 1 = rerun the listed ones;
                            // check: 1 = list the differing ones for a rerun (0: flag only)
    unsigned pass;          // the check's stats slot
    unsigned exact;         // a rerun of every segment from the States the chain kernel recorded
                            // (dspb_seg_chain): no list, no early stop (2: only if the chain ran);
                            // the check and the walk after it: every segment boundary
    unsigned long long perturb;  // test hook (dsp_module_debug): the chain kernel flips a bit of the
                                 // State it recorded for block perturb - 1 (0: none)
    State *st_ind;          // [4][K] a split State's block-independent words where pass 1 at each
                            // warm-up level starts segment k's warm-up (dspb_seg_chain_ind); the
                            // other words are not written
    unsigned split;         // pass 1 starts each segment's warm-up from st_ind's words
};
// a split State (dsp_callback_facts.state_split): the 4-byte words a store of
// a block-dependent value may hit (dsp_module_compile defines the list from
// the callback's facts; -1: none; -(T + 2): every word from T on)
#ifndef DSPB_STATE_DEP_WORDS
#define DSPB_STATE_DEP_WORDS -1
#endif
static constexpr int dspb_state_dep_words[] = {DSPB_STATE_DEP_WORDS};
__device__ static constexpr bool dspb_word_dep(unsigned w) {
    for (int d : dspb_state_dep_words)
        if (d == (int)w || (d <= -2 && (int)w >= -d - 2)) return true;  // (-(T + 2): every word from T on)
    return false;
}
constexpr bool kStateWords = sizeof(State) % 4 == 0 && alignof(State) >= 4;
__device__ static constexpr unsigned dspb_first_ind_word() {
    for (unsigned i = 0; i < sizeof(State) / 4; ++i)
        if (!dspb_word_dep(i)) return i;
    return ~0u;
}
// the State chain took over within this render: the reruns, their checks and
// the walk have nothing to do
__device__ static bool dspb_seg_chained(const dspb_seg_args &G) { return *(volatile unsigned *)&G.stats[12] != 0; }
// a rerun, check or walk launch with nothing to do: those after the State
// chain (G.exact: 1 always, 2 only when the chain ran in this render) and the
// speculative ones (only when it did not)
__device__ static bool dspb_seg_skip(const dspb_seg_args &G) {
    return G.exact ? (G.exact == 2 && !dspb_seg_chained(G)) : dspb_seg_chained(G);
}
// pass 1 at warm-up level L > 0 (and its check) runs only when level L - 1
// ran and more than 1/8 of the segments it guessed -- those whose warm-up
// began after block 0 -- started from a State that was not the true one: the
// trajectories had not met within its warm-up, so a 16x longer one is tried
__device__ static bool dspb_seg_level_runs(const dspb_seg_args &G) {
    if (G.level == 0) return true;
    const volatile unsigned *st = G.stats;
    const unsigned prev = G.level - 1;
    if (!st[8 + prev]) return false;
    const unsigned long long early = G.prev_warm / G.seg < G.K - 1 ? G.prev_warm / G.seg : G.K - 1;
    const unsigned long long guessed = G.K - 1 - early;
    return guessed && st[prev] * 8ull > guessed;
}
// a State's words: accesses that may alias the State's own fields (without
// may_alias, type-based alias analysis lets the compiler take a word copy of
// a State of doubles for unrelated memory -- and drop the callback's updates)
typedef unsigned __attribute__((may_alias)) dspb_word;
// a State copy as whole words, fully unrolled (a private State stays in
// registers; a memcpy this size would be lowered to a loop over it)
__device__ static inline void dspb_copy_state(void *dst, const void *src) {
    if constexpr (sizeof(State) % 4 == 0 && alignof(State) >= 4) {
#pragma unroll
        for (unsigned i = 0; i < sizeof(State) / 4; ++i) ((dspb_word *)dst)[i] = ((const dspb_word *)src)[i];
    } else {
#pragma unroll
        for (unsigned i = 0; i < sizeof(State); ++i) ((unsigned char *)dst)[i] = ((const unsigned char *)src)[i];
    }
}
// bit-for-bit equality; every word is loaded before any is compared (no
// short circuit: one memory round trip, not one per word)
__device__ static bool dspb_same_state(const State *a, const State *b) {
    unsigned d = 0;
    if constexpr (sizeof(State) % 4 == 0 && alignof(State) >= 4) {
        const dspb_word *x = (const dspb_word *)a, *y = (const dspb_word *)b;
#pragma unroll
        for (unsigned i = 0; i < sizeof(State) / 4; ++i) d |= x[i] ^ y[i];
    } else {
        const unsigned char *x = (const unsigned char *)a, *y = (const unsigned char *)b;
#pragma unroll
        for (unsigned i = 0; i < sizeof(State); ++i) d |= (unsigned)(x[i] ^ y[i]);
    }
    return d == 0;
}
// a split State's block-independent words from src into dst (the others stay)
__device__ static inline void dspb_copy_ind_words(void *dst, const void *src) {
    if constexpr (kStateWords) {
#pragma unroll
        for (unsigned i = 0; i < sizeof(State) / 4; ++i)
            if (!dspb_word_dep(i)) ((dspb_word *)dst)[i] = ((const dspb_word *)src)[i];
    }
}
// lane t's segment: its index (~0u: none), first block rendered (warm-up
// included), warm-up blocks, blocks rendered
__device__ static unsigned dspb_seg_lane(const dspb_seg_args &G, unsigned base, unsigned t, unsigned nseg,
                                         unsigned *s_first, unsigned *s_warm, unsigned *s_len) {
    const dspb_render_args &A = G.R;
    unsigned k = 0xffffffffu, f = 0, w = 0, len = 0;
    if (base + t < nseg) {
        k = (G.mode && !G.exact) ? G.list[base + t] : base + t;
        const unsigned long long b0 = (unsigned long long)k * G.seg;
        const unsigned long long b1 = b0 + G.seg < A.nblocks ? b0 + G.seg : A.nblocks;
        w = (G.mode || k == 0) ? 0u : (unsigned)(G.warm < b0 ? G.warm : b0);
        f = (unsigned)(b0 - w);
        len = w + (unsigned)(b1 - b0);
    }
    s_first[t] = f;
    s_warm[t] = w;
    s_len[t] = len;
    return k;
}
// a lane about to render block b in its round r (w: its warm-up blocks):
// pass 1 records the State a kept block is rendered from; a rerun stops
// (false) where its State meets the one recorded there
template <bool kRerun>
__device__ static bool dspb_seg_block(const dspb_seg_args &G, unsigned long long b, unsigned r, unsigned w,
                                      State &st) {
    if (r < w) return true;  // warm-up: nothing kept
    if (kRerun && G.exact) {
        // from the chain's record of the segment's first State: the record of
        // every later block is checked against the State the callback renders
        // it from, and takes that State (so the walk after the boundary check
        // stops only where it meets what was rendered here)
        if (r > 0 && !dspb_same_state(&st, &G.st_blk[b])) {
            atomicAdd(&G.stats[14], 1u);
            dspb_copy_state((void *)&G.st_blk[b], (const void *)&st);
        }
        return true;
    }
    if (kRerun && r > 0 && dspb_same_state(&st, &G.st_blk[b])) return false;
    dspb_copy_state((void *)&G.st_blk[b], (const void *)&st);
    return true;
}
// pass 1 / rerun, any shape: lane t of wave 0 runs segment k_t, rounds of one
// block per lane staged in LDS by all 256 threads (render_audio's copy: zeros
// past EOF and for the channels the file lacks), kept blocks copied out after
// the callbacks.  CC / BB constants as in the LDS-blocks path.
template <unsigned CC, unsigned BB>
__device__ static void dspb_segments(const dspb_seg_args &G) {
    extern __shared__ float dspb_lbuf[];
    __shared__ unsigned s_first[64], s_warm[64], s_len[64];
    const dspb_render_args &A = G.R;
    const unsigned C = CC ? CC : A.C, B = BB ? BB : A.B, CB = C * B, NB = A.lds_nb, SB = A.lds_stride;
    const unsigned t = threadIdx.x, nt = blockDim.x;
    const unsigned base = blockIdx.x * NB;
    if (!G.mode) {  // pass 1: at a warm-up level that runs; it restarts the listing
        if (!dspb_seg_level_runs(G)) return;
        if (G.level && blockIdx.x == 0 && t == 0) *G.count = 0;
    } else if (dspb_seg_skip(G)) {
        return;
    }
    const unsigned nseg = (G.mode && !G.exact) ? *(volatile unsigned *)G.count : G.K;
    if (base >= nseg) return;  // the same for the whole workgroup
    unsigned k = 0xffffffffu;
    if (t < NB) k = dspb_seg_lane(G, base, t, nseg, s_first, s_warm, s_len);
    __syncthreads();
    unsigned rounds = 0;
    for (unsigned i = 0; i < NB; ++i) rounds = s_len[i] > rounds ? s_len[i] : rounds;
    Parameters prm = dspb_from_global<Parameters>(A.P);
    State st;
    bool stopped = false;
    if (k != 0xffffffffu) {
        dspb_copy_state((void *)&st, (G.mode && (k || !G.exact)) ? (const void *)&G.st_blk[(unsigned long long)k * G.seg]
                                                                 : (const void *)A.S);
        // pass 1 of a split State: the warm-up starts from the independent
        // words the State chain recorded at its first block
        if (!G.mode && G.split && k) dspb_copy_ind_words((void *)&st, (const void *)&G.st_ind[G.level * G.K + k]);
    }
    // the channels' rows in LDS (an access by a lane-dependent channel reads
    // them there, not from the argument block in memory)
    __shared__ const float *s_in[16];
    __shared__ float *s_out[16];
    if (t < C) {
        s_in[t] = t < A.in_ch ? A.in[t] : nullptr;
        s_out[t] = A.out[t];
    }
    __syncthreads();
    const unsigned NE = NB * CB;
    for (unsigned r = 0; r < rounds; ++r) {
        // render_audio's copy in batches of 8 loads in flight per thread
        for (unsigned j0 = t; j0 < NE; j0 += 8 * nt) {
            float v[8];
            unsigned dst[8];
#pragma unroll
            for (unsigned u = 0; u < 8; ++u) {
                const unsigned j = j0 + u * nt;
                v[u] = 0.0f;
                dst[u] = 0xffffffffu;
                if (j < NE) {
                    const unsigned i = j / CB, e = j - i * CB, c = e / B, s = e - c * B;
                    if (r < s_len[i]) {
                        const unsigned long long gi = (unsigned long long)(s_first[i] + r) * B + s;
                        if (s_in[c] && gi < A.L) v[u] = ((const dspb_gfloat *)s_in[c])[gi];
                        dst[u] = i * SB + e;
                    }
                }
            }
#pragma unroll
            for (unsigned u = 0; u < 8; ++u)
                if (dst[u] != 0xffffffffu) dspb_lbuf[dst[u]] = v[u];
        }
        __syncthreads();
        if (k != 0xffffffffu && r < s_len[t]) {
            if (G.mode ? dspb_seg_block<true>(G, (unsigned long long)s_first[t] + r, r, s_warm[t], st)
                       : dspb_seg_block<false>(G, (unsigned long long)s_first[t] + r, r, s_warm[t], st)) {
                float *blk = dspb_lbuf + t * SB;
                float *ptrs[CC ? CC : 16];
                for (unsigned c = 0; c < C; ++c) ptrs[c] = blk + c * B;
                audio_callback(prm, st, ptrs, C, B, A.sr);
            } else {
                s_len[t] = r;  // met the recorded chain: the rest stands
                stopped = true;
            }
        }
        __syncthreads();
        for (unsigned j = t; j < NE; j += nt) {
            const unsigned i = j / CB, e = j - i * CB, c = e / B, s = e - c * B;
            if (r >= s_warm[i] && r < s_len[i])
                ((dspb_gfloat *)s_out[c])[(unsigned long long)(s_first[i] + r) * B + s] = dspb_lbuf[i * SB + e];
        }
        __syncthreads();
        rounds = 0;
        for (unsigned i = 0; i < NB; ++i) rounds = s_len[i] > rounds ? s_len[i] : rounds;
    }
    if (k != 0xffffffffu && !stopped) dspb_copy_state((void *)&G.st_end[k], (const void *)&st);
}
// the same for a constant channel count and 4 | B, software pipelined: round
// r + 1's blocks are in flight into registers (16-byte loads, all issued at
// once) while round r's callbacks run; blocks at a stride of C B + 2 floats
// (float2 LDS moves; the callback lanes on distinct banks), as
// dspb_stateless_lds_pf.  BB = 0: B from the arguments (the host checks
// 4 | B), the registers sized for the most float4 a round can hold.
template <unsigned CC, unsigned BB, bool kRerun>
__device__ static void dspb_segments_pf(const dspb_seg_args &G) {
    extern __shared__ float dspb_lbuf[];
    __shared__ unsigned s_first[64], s_warm[64], s_len[64];
    constexpr unsigned C = CC;
    const unsigned B = BB ? BB : G.R.B, CB = C * B, SB = CB + 2u, NB = BB ? dspb_seg_nb(CC * BB + 2u) : G.R.lds_nb;
    // per channel: NB rows of B / 4 float4, at most PV of them per thread
    // (a round holds fewer than DSPB_LDS_ROUND_BYTES / (16 C) float4 per channel)
    const unsigned R4 = B / 4u, T4 = NB * R4;
    constexpr unsigned PV = BB ? (dspb_seg_nb(CC * BB + 2u) * (BB / 4u) + 255u) / 256u
                               : (DSPB_LDS_ROUND_BYTES / (16u * CC) + 255u) / 256u;
    constexpr bool kFull = BB && (dspb_seg_nb(CC * BB + 2u) * (BB / 4u)) % 256u == 0;
    static_assert(!BB || (dspb_seg_nb(CC * BB + 2u) <= 64 && BB % 4 == 0), "one wave runs a round's callbacks");
    typedef __attribute__((address_space(1))) float4 gfloat4;
    const dspb_render_args &A = G.R;
    const unsigned t = threadIdx.x;
    const unsigned base = blockIdx.x * NB;
    if (!kRerun) {  // pass 1: at a warm-up level that runs; it restarts the listing
        if (!dspb_seg_level_runs(G)) return;
        if (G.level && blockIdx.x == 0 && t == 0) *G.count = 0;
    } else if (dspb_seg_skip(G)) {
        return;
    }
    const unsigned nseg = (kRerun && !G.exact) ? *(volatile unsigned *)G.count : G.K;
    if (base >= nseg) return;  // the same for the whole workgroup
    unsigned k = 0xffffffffu;
    if (t < NB) k = dspb_seg_lane(G, base, t, nseg, s_first, s_warm, s_len);
    __syncthreads();
    unsigned rounds = 0;
    for (unsigned i = 0; i < NB; ++i) rounds = s_len[i] > rounds ? s_len[i] : rounds;
    // the channels' rows as uniform values (the channel of every access below
    // is a constant, so none of them is an indexed load of the argument block)
    const dspb_gfloat *xin[C];
    dspb_gfloat *xout[C];
    bool aligned_in = true, aligned_out = true;
#pragma unroll
    for (unsigned c = 0; c < C; ++c) {
        xin[c] = (const dspb_gfloat *)A.in[c < A.in_ch ? c : 0];
        xout[c] = (dspb_gfloat *)A.out[c];
        if (c < A.in_ch) aligned_in = aligned_in && !(((unsigned long long)A.in[c]) & 15);
        aligned_out = aligned_out && !(((unsigned long long)A.out[c]) & 15);
    }
    Parameters prm = dspb_from_global<Parameters>(A.P);
    State st;
    bool stopped = false;
    if (k != 0xffffffffu) {
        dspb_copy_state((void *)&st, (kRerun && (k || !G.exact)) ? (const void *)&G.st_blk[(unsigned long long)k * G.seg]
                                                                  : (const void *)A.S);
        // pass 1 of a split State: the warm-up starts from the independent
        // words the State chain recorded at its first block
        if (!kRerun && G.split && k) dspb_copy_ind_words((void *)&st, (const void *)&G.st_ind[G.level * G.K + k]);
    }
    // a constant B prefetches a whole round (PB = PV) while the callbacks run;
    // a runtime B stages in batches of 4 float4 per channel at the round's
    // start (a whole round's registers would spill)
    constexpr unsigned PB = BB ? PV : 4u;
    float4 pf[C][PB];
    auto load = [&](unsigned r, unsigned v0) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c) {
#pragma unroll
            for (unsigned v = 0; v < PB; ++v) {
                const unsigned q = t + 256u * (v0 + v), i = q / R4, s = (q - i * R4) * 4u;
                float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
                if ((kFull || q < T4) && r < s_len[i] && c < A.in_ch) {
                    const unsigned long long gi = (unsigned long long)(s_first[i] + r) * B + s;
                    if (aligned_in && gi + 4 <= A.L) {
                        x = *(const gfloat4 *)(xin[c] + gi);
                    } else {
                        x.x = gi < A.L ? xin[c][gi] : 0.f;
                        x.y = gi + 1 < A.L ? xin[c][gi + 1] : 0.f;
                        x.z = gi + 2 < A.L ? xin[c][gi + 2] : 0.f;
                        x.w = gi + 3 < A.L ? xin[c][gi + 3] : 0.f;
                    }
                }
                pf[c][v] = x;
            }
        }
    };
    auto put = [&](unsigned r, unsigned v0) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c) {
#pragma unroll
            for (unsigned v = 0; v < PB; ++v) {
                const unsigned q = t + 256u * (v0 + v), i = q / R4, s = (q - i * R4) * 4u;
                if ((kFull || q < T4) && r < s_len[i]) {
                    float2 *d = (float2 *)(dspb_lbuf + i * SB + c * B + s);
                    d[0] = make_float2(pf[c][v].x, pf[c][v].y);
                    d[1] = make_float2(pf[c][v].z, pf[c][v].w);
                }
            }
        }
    };
#ifdef DSPB_SEG_TIMING
    // diagnostics (a module compiled with DSPB_SEG_TIMING set, module.cpp):
    // where wave 0's lane 0 spends pass 1's rounds, in shader clocks, summed
    // over the workgroups into stats[16, 24) (dsp_module_seg_timing)
    unsigned long long tm[5] = {0, 0, 0, 0, 0}, t0 = __builtin_amdgcn_s_memtime(), nr = 0;
#define DSPB_TMARK(i)                                                   \
    if (!kRerun && t == 0) {                                            \
        const unsigned long long tn = __builtin_amdgcn_s_memtime();     \
        tm[i] += tn - t0;                                               \
        t0 = tn;                                                        \
    }
#else
#define DSPB_TMARK(i)
#endif
    if (BB && rounds) load(0, 0);
    for (unsigned r = 0; r < rounds; ++r) {
        if constexpr (BB != 0) {
            put(r, 0);
        } else {
            for (unsigned v0 = 0; v0 < PV; v0 += PB) {
                load(r, v0);
                put(r, v0);
            }
        }
        __syncthreads();
        DSPB_TMARK(0)
        if (BB && r + 1 < rounds) load(r + 1, 0);  // in flight while the callbacks run
        DSPB_TMARK(1)
        if (k != 0xffffffffu && r < s_len[t]) {
            if (dspb_seg_block<kRerun>(G, (unsigned long long)s_first[t] + r, r, s_warm[t], st)) {
                float *blk = dspb_lbuf + t * SB;
                float *ptrs[C];
                for (unsigned c = 0; c < C; ++c) ptrs[c] = blk + c * B;
                audio_callback(prm, st, ptrs, C, B, A.sr);
            } else {
                s_len[t] = r;  // met the recorded chain: the rest stands
                stopped = true;
            }
        }
        DSPB_TMARK(2)
        __syncthreads();
        DSPB_TMARK(3)
#pragma unroll
        for (unsigned c = 0; c < C; ++c) {
#pragma unroll
            for (unsigned v = 0; v < PV; ++v) {
                const unsigned q = t + 256u * v, i = q / R4, s = (q - i * R4) * 4u;
                if ((kFull || q < T4) && r >= s_warm[i] && r < s_len[i]) {
                    const unsigned long long gi = (unsigned long long)(s_first[i] + r) * B + s;
                    const float2 *d = (const float2 *)(dspb_lbuf + i * SB + c * B + s);
                    const float2 lo = d[0], hi = d[1];
                    if (aligned_out) {
                        *(gfloat4 *)(xout[c] + gi) = make_float4(lo.x, lo.y, hi.x, hi.y);
                    } else {
                        xout[c][gi] = lo.x, xout[c][gi + 1] = lo.y, xout[c][gi + 2] = hi.x, xout[c][gi + 3] = hi.y;
                    }
                }
            }
        }
        __syncthreads();
        rounds = 0;
        for (unsigned i = 0; i < NB; ++i) rounds = s_len[i] > rounds ? s_len[i] : rounds;
        DSPB_TMARK(4)
#ifdef DSPB_SEG_TIMING
        ++nr;
#endif
    }
    if (k != 0xffffffffu && !stopped) dspb_copy_state((void *)&G.st_end[k], (const void *)&st);
#ifdef DSPB_SEG_TIMING
    if (!kRerun && t == 0) {
        // (phases: 0 staging + barrier, 1 next round's loads issued, 2 the
        // callbacks, 3 the barrier after them, 4 copy-out + barrier)
        for (int i = 0; i < 5; ++i) atomicAdd(&G.stats[16 + i], (unsigned)(tm[i] >> 4));
        atomicAdd(&G.stats[21], 1u);
        atomicAdd(&G.stats[22], (unsigned)nr);
    }
#endif
#undef DSPB_TMARK
}
// the same for a constant B, with the work split by role: wave 0 runs the
// callbacks and nothing else; waves 1-3 move the blocks.  A round's kept
// blocks go from LDS into registers and the next round's blocks from
// registers into the same slots (each thread the slots it read: no barrier
// between), then -- after the barrier that frees wave 0 for the next
// round's callbacks -- the kept blocks are stored and the round after next
// is loaded.  The stores and loads (a chip-wide burst of a round's blocks
// each way) drain while the callbacks run instead of holding up the
// callback wave's issue (dsp_module_seg_timing: a round of
// envelope_counter.cpp spent 29% of its clocks issuing the next loads
// behind the copy-out's stores and 14% in the copy-out).
template <unsigned CC, unsigned BB, bool kRerun>
__device__ __attribute__((always_inline, flatten)) static void dspb_segments_roles(const dspb_seg_args &G) {
    extern __shared__ float dspb_lbuf[];
    __shared__ unsigned s_first[64], s_warm[64], s_len[64];
    constexpr unsigned C = CC, B = BB, SB = C * B + 2u, NB = dspb_seg_nb(CC * BB + 2u);
    // the movers (waves 1-3) move float4 units: one 16-byte load / store per
    // unit in HBM, two 8-byte LDS accesses (rows are 8-byte aligned: C B + 2
    // floats apart, so that the callback lanes sit on distinct banks).
    // (float2 units -- 512 contiguous bytes per LDS instruction, no bank
    // conflicts -- measured slower: twice the slots' bookkeeping, 16.4k vs
    // 8.0k clocks per round for the swap; profiles/r06_seg_roles.txt)
    constexpr unsigned R4 = B / 4u, T4 = NB * R4, NW = 192u;
    constexpr unsigned PV = (T4 + NW - 1u) / NW;
    constexpr bool kFull = T4 % NW == 0;
    static_assert(NB <= 64 && BB % 4 == 0, "one wave runs a round's callbacks");
    const dspb_render_args &A = G.R;
    const unsigned t = threadIdx.x;
    const unsigned base = blockIdx.x * NB;
    if (!kRerun) {  // pass 1: at a warm-up level that runs; it restarts the listing
        if (!dspb_seg_level_runs(G)) return;
        if (G.level && blockIdx.x == 0 && t == 0) *G.count = 0;
    } else if (dspb_seg_skip(G)) {
        return;
    }
    const unsigned nseg = (kRerun && !G.exact) ? *(volatile unsigned *)G.count : G.K;
    if (base >= nseg) return;  // the same for the whole workgroup
    unsigned k = 0xffffffffu;
    if (t < NB) k = dspb_seg_lane(G, base, t, nseg, s_first, s_warm, s_len);
    __syncthreads();
    unsigned rounds = 0;
    for (unsigned i = 0; i < NB; ++i) rounds = s_len[i] > rounds ? s_len[i] : rounds;
    const dspb_gfloat *xin[C];
    dspb_gfloat *xout[C];
    bool aligned_in = true, aligned_out = true;
#pragma unroll
    for (unsigned c = 0; c < C; ++c) {
        xin[c] = (const dspb_gfloat *)A.in[c < A.in_ch ? c : 0];
        xout[c] = (dspb_gfloat *)A.out[c];
        if (c < A.in_ch) aligned_in = aligned_in && !(((unsigned long long)A.in[c]) & 15);
        aligned_out = aligned_out && !(((unsigned long long)A.out[c]) & 15);
    }
    const bool mover = t >= 64u;
    // (movers only; made opaque once per round, so that the slots' indices
    // are recomputed where used instead of 24 of them held in registers
    // across the loop)
    unsigned tm = t - 64u;
    // mover slot v: float4 s of block i's row.  A wave's 64 slots of one v
    // start at a multiple of 64 units and a row holds 128: i is the same for
    // the whole wave, so the block's first / warm-up / length come from the
    // lanes' copies (lane l: block l's, read once per round) by readlane,
    // not from LDS once per slot
    unsigned m_first = 0, m_warm = 0, m_len = 0;
    auto refresh = [&]() {
        const unsigned l = t & 63u;
        m_first = l < NB ? s_first[l] : 0u;
        m_warm = l < NB ? s_warm[l] : 0u;
        m_len = l < NB ? s_len[l] : 0u;
    };
    static_assert(R4 % 64u == 0 && NW % 64u == 0, "a wave's 64 units of one slot lie in one block row");
    auto slot = [&](unsigned v, unsigned &i, unsigned &s) -> bool {
        const unsigned q = tm + NW * v;
        i = __builtin_amdgcn_readfirstlane(q / R4);
        s = (q - i * R4) * 4u;
        return kFull || q < T4;
    };
    auto len_of = [&](unsigned i) { return (unsigned)__builtin_amdgcn_readlane((int)m_len, (int)i); };
    auto warm_of = [&](unsigned i) { return (unsigned)__builtin_amdgcn_readlane((int)m_warm, (int)i); };
    auto first_of = [&](unsigned i) { return (unsigned)__builtin_amdgcn_readlane((int)m_first, (int)i); };
    typedef __attribute__((address_space(1))) float4 gfloat4;
    float4 pf[C][PV], ob[C][PV];
    auto load = [&](unsigned r) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c)
#pragma unroll
            for (unsigned v = 0; v < PV; ++v) {
                unsigned i, s;
                float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
                if (slot(v, i, s) && r < len_of(i) && c < A.in_ch) {
                    const unsigned long long gi = (unsigned long long)(first_of(i) + r) * B + s;
                    if (aligned_in && gi + 4 <= A.L) {
                        x = *(const gfloat4 *)(xin[c] + gi);
                    } else {
                        x.x = gi < A.L ? xin[c][gi] : 0.f;
                        x.y = gi + 1 < A.L ? xin[c][gi + 1] : 0.f;
                        x.z = gi + 2 < A.L ? xin[c][gi + 2] : 0.f;
                        x.w = gi + 3 < A.L ? xin[c][gi + 3] : 0.f;
                    }
                }
                pf[c][v] = x;
            }
    };
    auto put = [&](unsigned r) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c)
#pragma unroll
            for (unsigned v = 0; v < PV; ++v) {
                unsigned i, s;
                if (slot(v, i, s) && r < len_of(i)) {
                    float2 *d = (float2 *)(dspb_lbuf + i * SB + c * B + s);
                    d[0] = make_float2(pf[c][v].x, pf[c][v].y);
                    d[1] = make_float2(pf[c][v].z, pf[c][v].w);
                }
            }
    };
    // round r's kept blocks out of their slots, round r + 1's in (put: r + 1
    // is rendered), slot by slot: a slot's outgoing unit takes the registers
    // its incoming one frees (one set of registers live, not two)
    auto swap = [&](unsigned r, bool put_next) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c)
#pragma unroll
            for (unsigned v = 0; v < PV; ++v) {
                unsigned i, s;
                const bool in = slot(v, i, s);
                float2 *d = (float2 *)(dspb_lbuf + i * SB + c * B + s);
                if (in && r >= warm_of(i) && r < len_of(i)) {
                    const float2 lo = d[0], hi = d[1];
                    ob[c][v] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
                if (in && put_next && r + 1 < len_of(i)) {
                    d[0] = make_float2(pf[c][v].x, pf[c][v].y);
                    d[1] = make_float2(pf[c][v].z, pf[c][v].w);
                }
            }
    };
    auto send = [&](unsigned r) {
#pragma unroll
        for (unsigned c = 0; c < C; ++c)
#pragma unroll
            for (unsigned v = 0; v < PV; ++v) {
                unsigned i, s;
                if (slot(v, i, s) && r >= warm_of(i) && r < len_of(i)) {
                    const unsigned long long gi = (unsigned long long)(first_of(i) + r) * B + s;
                    const float4 o = ob[c][v];
                    if (aligned_out) {
                        *(gfloat4 *)(xout[c] + gi) = o;
                    } else {
                        xout[c][gi] = o.x, xout[c][gi + 1] = o.y, xout[c][gi + 2] = o.z, xout[c][gi + 3] = o.w;
                    }
                }
            }
    };
    Parameters prm = dspb_from_global<Parameters>(A.P);
    State st;
    bool stopped = false;
    if (k != 0xffffffffu) {
        dspb_copy_state((void *)&st, (kRerun && (k || !G.exact)) ? (const void *)&G.st_blk[(unsigned long long)k * G.seg]
                                                                  : (const void *)A.S);
        if (!kRerun && G.split && k) dspb_copy_ind_words((void *)&st, (const void *)&G.st_ind[G.level * G.K + k]);
    }
#ifdef DSPB_SEG_TIMING
    unsigned long long tmk[5] = {0, 0, 0, 0, 0}, t0 = __builtin_amdgcn_s_memtime(), nr = 0;
#define DSPB_TMARK(i)                                                   \
    if (!kRerun && t == 0) {                                            \
        const unsigned long long tn = __builtin_amdgcn_s_memtime();     \
        tmk[i] += tn - t0;                                              \
        t0 = tn;                                                        \
    }
#else
#define DSPB_TMARK(i)
#endif
    if (mover && rounds) {
        refresh();
        load(0);
        put(0);
        if (rounds > 1) load(1);
    }
    __syncthreads();
    DSPB_TMARK(0)
    // two loops, one per role, behind a wave-uniform branch: each wave meets
    // the same barriers (two per round, the round count read from s_len by
    // all alike), and the movers' registers (a round's blocks in flight) are
    // not live across the callbacks' code, which has the registers to itself
    if (__builtin_amdgcn_readfirstlane(t >> 6) == 0) {
        for (unsigned r = 0; r < rounds;) {
            if (k != 0xffffffffu && r < s_len[t]) {
                if (dspb_seg_block<kRerun>(G, (unsigned long long)s_first[t] + r, r, s_warm[t], st)) {
                    float *blk = dspb_lbuf + t * SB;
                    float *ptrs[C];
                    for (unsigned c = 0; c < C; ++c) ptrs[c] = blk + c * B;
                    audio_callback(prm, st, ptrs, C, B, A.sr);
                } else {
                    s_len[t] = r;  // met the recorded chain: the rest stands
                    stopped = true;
                }
            }
            DSPB_TMARK(2)
            __syncthreads();  // (A) the callbacks of round r are done, s_len final for it
            DSPB_TMARK(3)
            unsigned next = 0;
            for (unsigned i = 0; i < NB; ++i) next = s_len[i] > next ? s_len[i] : next;
            __syncthreads();  // (B) round r + 1 staged by the movers
            DSPB_TMARK(4)
            rounds = next;
            ++r;
#ifdef DSPB_SEG_TIMING
            ++nr;
#endif
        }
    } else {
        for (unsigned r = 0; r < rounds;) {
            asm volatile("" : "+v"(tm));
            __syncthreads();  // (A)
            refresh();  // (s_len as the callbacks of round r left it)
            // the next round count from the lanes' copies (one LDS read per
            // lane, then scalar maxima) rather than NB reads in a row
            unsigned next = 0;
            for (unsigned i = 0; i < NB; ++i) {
                const unsigned l = (unsigned)__builtin_amdgcn_readlane((int)m_len, (int)i);
                next = l > next ? l : next;
            }
            swap(r, r + 1 < next);  // (each thread the slots it reads)
            __syncthreads();  // (B)
            asm volatile("" : "+v"(tm));
            send(r);
            if (r + 2 < next) load(r + 2);
            rounds = next;
            ++r;
        }
    }
    if (k != 0xffffffffu && !stopped) dspb_copy_state((void *)&G.st_end[k], (const void *)&st);
#ifdef DSPB_SEG_TIMING
    if (!kRerun && t == 0) {
        // (phases: 0 the first round staged, 2 the callbacks, 3 the barrier
        // after them, 4 take / put + barrier; 1 unused)
        for (int i = 0; i < 5; ++i) atomicAdd(&G.stats[16 + i], (unsigned)(tmk[i] >> 4));
        atomicAdd(&G.stats[21], 1u);
        atomicAdd(&G.stats[22], (unsigned)nr);
    }
#endif
#undef DSPB_TMARK
}
#define DSPB_SEG_KERNEL(name, CC, BB)                                                \
    extern "C" __global__ __launch_bounds__(256) void name(dspb_seg_args G) { dspb_segments<CC, BB>(G); }
// pass 1 and the reruns as kernels of their own: pass 1 carries no
// comparison (its registers are the callback's)
// pass 1 at two waves per SIMD: both workgroups of a CU resident (their LDS
// rounds are what the lanes are); a rerun renders few segments, each until
// its chain meets the recorded one, and may take the registers of one
#define DSPB_SEG_PF_KERNEL(name, CC, BB, RR)                                           \
    extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RR ? 1 : 2, 2))) void name(  \
        dspb_seg_args G) { dspb_segments_pf<CC, BB, RR>(G); }
// (dspb_segments_roles is flattened: the movers' unrolled code makes it
// large enough that the inliner would otherwise leave audio_callback a call
// -- its block pointers through scratch, its LDS accesses flat: 6x slower
// callbacks, measured)
#define DSPB_SEG_ROLES_KERNEL(name, CC, BB, RR)                                        \
    extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RR ? 1 : 2, 2))) void name(  \
        dspb_seg_args G) { dspb_segments_roles<CC, BB, RR>(G); }
DSPB_SEG_ROLES_KERNEL(dspb_seg_c2b512, 2, 512, false)
// (the reruns keep the single-role kernel: the roles' unrolled movers leave
// the rerun's State comparison no registers, and their arrays go to scratch)
DSPB_SEG_PF_KERNEL(dspb_seg_c2b512_rerun, 2, 512, true)
DSPB_SEG_PF_KERNEL(dspb_seg_c2, 2, 0, false)
DSPB_SEG_PF_KERNEL(dspb_seg_c2_rerun, 2, 0, true)
DSPB_SEG_PF_KERNEL(dspb_seg_c1, 1, 0, false)
DSPB_SEG_PF_KERNEL(dspb_seg_c1_rerun, 1, 0, true)
DSPB_SEG_PF_KERNEL(dspb_seg_c4, 4, 0, false)
DSPB_SEG_PF_KERNEL(dspb_seg_c4_rerun, 4, 0, true)
DSPB_SEG_KERNEL(dspb_seg, 0, 0)
// segment k (k >= 1) rendered its first block from st_blk[k seg]; the true
// State there is st_end[k - 1] if segment k - 1 is exact: flag the segments
// where the two differ and, when a rerun follows, list them and give each
// the State to start again from.  One wavefront per segment, its lanes over
// the State's words; a check after a pass that found nothing to rerun
// returns at once (nothing changed: the flags stand).
extern "C" __global__ void dspb_seg_check(dspb_seg_args G) {
    if (dspb_seg_skip(G)) return;
    if (G.exact) {
        // after the State chain's exact rerun: every boundary, the chain's
        // record of a segment's first State against the State the segment
        // before ended with (the chain is checked, not trusted)
    } else if (G.level != 0xffffffffu) {  // pass 1's check: where pass 1 ran
        if (!dspb_seg_level_runs(G)) return;
        if (blockIdx.x == 0 && threadIdx.x == 0) G.stats[8 + G.level] = 1;
    } else if (*(volatile unsigned *)G.prev_count == 0) {
        return;  // the rerun before rendered nothing: the flags stand
    }
    const unsigned lane = threadIdx.x & 63u;
    const unsigned k = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (k >= G.K) return;  // the same for the whole wavefront
    if (k == 0) {
        if (lane == 0) G.flags[0] = 0;
        return;
    }
    State *first = &G.st_blk[(unsigned long long)k * G.seg];
    const State *prev = &G.st_end[k - 1];
    bool diff = false;
    constexpr bool kWords = sizeof(State) % 4 == 0 && alignof(State) >= 4;
    constexpr unsigned n = kWords ? sizeof(State) / 4 : sizeof(State);
    if constexpr (kWords) {
        for (unsigned i = lane; i < n; i += 64) diff = diff || ((const dspb_word *)first)[i] != ((const dspb_word *)prev)[i];
    } else {
        for (unsigned i = lane; i < n; i += 64)
            diff = diff || ((const unsigned char *)first)[i] != ((const unsigned char *)prev)[i];
    }
    const bool any = __any(diff) != 0;
    if (lane == 0) G.flags[k] = any ? 1 : 0;
    if (!any) return;
    if (lane == 0) atomicAdd(&G.stats[G.pass], 1u);
    if (G.mode) {
        if constexpr (kWords) {
            for (unsigned i = lane; i < n; i += 64) ((dspb_word *)first)[i] = ((const dspb_word *)prev)[i];
        } else {
            for (unsigned i = lane; i < n; i += 64) ((unsigned char *)first)[i] = ((const unsigned char *)prev)[i];
        }
        if (lane == 0) G.list[atomicAdd(G.count, 1u)] = k;
    }
}
// the walk: one workgroup, segments in order; a segment is looked at when the
// last check flagged it or its predecessor's final State changed here; one
// whose first block's State differs is rendered serially from its
// predecessor's final State (thread 0 runs the callback on an LDS double
// buffer, the other waves stage blocks in and out, as dspb_stateful_lds)
// until its State meets the recorded one.  Then the live State = the last
// segment's final State.
template <unsigned CC, unsigned NB_>
__device__ static void dspb_seg_walk(const dspb_seg_args &G) {
    extern __shared__ float dspb_lbuf[];
    __shared__ unsigned s_next;
    __shared__ int s_bad, s_stop;
    __shared__ unsigned long long s_prev[(sizeof(State) + 7) / 8];  // the predecessor's final State
    const dspb_render_args &A = G.R;
    if (dspb_seg_skip(G)) return;  // the same for the whole workgroup
    const unsigned B = NB_ ? NB_ : A.B, C = CC ? CC : A.C, CB = C * B, t = threadIdx.x, nt = blockDim.x;
    float *buf0 = dspb_lbuf, *buf1 = dspb_lbuf + CB;
    Parameters prm = dspb_from_global<Parameters>(A.P);
    State local;
    bool prev_ended = false;  // s_prev holds a final State the walk rendered
    unsigned reruns = 0;
    for (unsigned k = 1; k < G.K; ++k) {
        if (!prev_ended) {  // the next flagged segment at or after k
            // every thread its stride of the flags with its loads in flight
            // together, one minimum (a scan of 256 flags per barrier round
            // trip took 16 us over a stereo hour's 9,122 segments)
            if (t == 0) s_next = G.K;
            __syncthreads();
            unsigned mine = G.K;
#pragma unroll 16
            for (unsigned c = k + t; c < G.K; c += nt)
                if (G.flags[c] && c < mine) mine = c;
            if (mine < G.K) atomicMin(&s_next, mine);
            __syncthreads();
            const unsigned found = s_next;
            __syncthreads();
            if (found >= G.K) break;
            k = found;
            for (unsigned i = t; i < sizeof(State); i += nt)
                ((unsigned char *)s_prev)[i] = ((const unsigned char *)&G.st_end[k - 1])[i];
        }
        const unsigned long long b0 = (unsigned long long)k * G.seg;
        const unsigned long long b1 = b0 + G.seg < A.nblocks ? b0 + G.seg : A.nblocks;
        if (t == 0) s_bad = 0;
        __syncthreads();
        for (unsigned i = t; i < sizeof(State); i += nt)
            if (((const unsigned char *)s_prev)[i] != ((const unsigned char *)&G.st_blk[b0])[i]) s_bad = 1;
        __syncthreads();
        prev_ended = false;
        if (s_bad) {
            ++reruns;
            dspb_copy_state((void *)&local, (const void *)s_prev);
            dspb_stage_in(A, b0, buf0, t, nt);
            __syncthreads();
            unsigned long long b = b0;
            bool ended = true;
            for (; b < b1; ++b) {
                float *cur = ((b - b0) & 1) ? buf1 : buf0, *oth = ((b - b0) & 1) ? buf0 : buf1;
                if (t == 0) {  // does the chain meet the recorded one here?
                    s_stop = (b > b0 && dspb_same_state(&local, &G.st_blk[b])) ? 1 : 0;
                    if (!s_stop) dspb_copy_state((void *)&G.st_blk[b], (const void *)&local);
                }
                __syncthreads();
                if (s_stop) {
                    ended = false;
                    break;
                }
                if (t == 0) {
                    float *ptrs[CC ? CC : 16];
                    for (unsigned c = 0; c < C; ++c) ptrs[c] = cur + c * B;
                    audio_callback(prm, local, ptrs, C, B, A.sr);
                } else if (t >= 64) {
                    if (b > b0) dspb_stage_out(A, b - 1, oth, t - 64, nt - 64);
                    if (b + 1 < b1) dspb_stage_in(A, b + 1, oth, t - 64, nt - 64);
                }
                __syncthreads();
            }
            // the last block rendered here
            dspb_stage_out(A, b - 1, ((b - 1 - b0) & 1) ? buf1 : buf0, t, nt);
            if (ended && t == 0) {
                dspb_copy_state((void *)s_prev, (const void *)&local);
                dspb_copy_state((void *)&G.st_end[k], (const void *)&local);
            }
            prev_ended = ended;
            __syncthreads();
        }
    }
    __syncthreads();
    if (t == 0) G.stats[7] = reruns;
    // the live State: the last segment's final State (s_prev when the walk
    // rendered it to its end, else st_end as pass 1 / a rerun left it)
    const unsigned char *last = prev_ended ? (const unsigned char *)s_prev
                                           : (const unsigned char *)&G.st_end[G.K - 1];
    for (unsigned i = t; i < sizeof(State); i += nt) ((unsigned char *)A.S)[i] = last[i];
}
#define DSPB_WALK_KERNEL(name, CC, BB)                                                 \
    extern "C" __global__ __launch_bounds__(256) void name(dspb_seg_args G) { dspb_seg_walk<CC, BB>(G); }
DSPB_WALK_KERNEL(dspb_seg_walk_c2b512, 2, 512)
DSPB_WALK_KERNEL(dspb_seg_walk_any, 0, 0)

// ---- a State that never forgets (module_render_seg, chain) -----------------
// An oscillator's phase never forgets where it started: no warm-up level
// meets the true State, and the module learns to render these Parameters
// without speculation.  The chain kernel then runs the callback on every
// block in order on one lane and records the State each block starts from
// (st_blk); the block it hands the callback is a private array filled from the
// input and read by nothing afterwards, so once the callback is inlined the
// compiler keeps only the arithmetic the State needs (a phase update, not its
// cosine).  The exact rerun (G.exact) then renders every segment from its
// recorded first State, in parallel -- the serial chain's bits.  The host
// takes a chain kernel only when its private memory is smaller than the block
// (module.cpp kChainShapes): a block the State depends on stays in scratch,
// and such a callback renders serially as before.  Within a speculative
// render (G.mode 2) the chain runs only when the last warm-up level tried
// failed (dspb_seg_level_runs on the level after it), and says so in
// stats[12]: the reruns and the walk then return at once, and the exact
// rerun (G.exact 2) renders the segments.  The chain is checked, not trusted:
// the exact rerun compares every block's record with the State it renders the
// block from, a check compares every segment's first State with the State the
// segment before ended with, and the walk renders serially from the true
// State whatever differs (stats[13], [14]: the host then stops taking the
// chain for these Parameters).
template <unsigned CC, unsigned BB>
__device__ static void dspb_seg_chain(const dspb_seg_args &G) {
    const dspb_render_args &A = G.R;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (G.mode == 2) {
        if (!dspb_seg_level_runs(G)) return;
        G.stats[12] = 1u;
    }
    constexpr unsigned BMAX = BB ? BB : 4096u;
    const unsigned B = BB ? BB : A.B;
    const Parameters prm = dspb_from_global<Parameters>(A.P);
    State st;
    dspb_copy_state((void *)&st, (const void *)A.S);
    for (unsigned long long b = 0; b < A.nblocks; ++b) {
        dspb_copy_state((void *)&G.st_blk[b], (const void *)&st);
        // (named, and filled with non-temporal stores, so that the module
        // compiler can tell the callback's stores to it apart in the IR:
        // module.cpp compile_chain_ir)
        float dspb_chain_blk[CC * BMAX];
        float *ptrs[CC];
#pragma unroll
        for (unsigned c = 0; c < CC; ++c) {
            ptrs[c] = dspb_chain_blk + c * B;
            const dspb_gfloat *x = (const dspb_gfloat *)A.in[c < A.in_ch ? c : 0];
            for (unsigned i = 0; i < B; ++i) {
                const unsigned long long gi = b * B + i;
                __builtin_nontemporal_store((c < A.in_ch && gi < A.L) ? x[gi] : 0.0f, &dspb_chain_blk[c * B + i]);
            }
        }
        audio_callback(prm, st, ptrs, CC, B, A.sr);
    }
    // (the live State is written by the walk after the check, from the States
    // the exact rerun rendered with, not from this chain's)
    if (G.perturb && G.perturb - 1 < A.nblocks) {  // test hook: a wrong record (high bit of the first word)
        constexpr unsigned kByte = (sizeof(State) < 8 ? sizeof(State) : 8) - 1;
        ((unsigned char *)&G.st_blk[G.perturb - 1])[kByte] ^= 0x40u;
    }
}
#define DSPB_CHAIN_KERNEL(name, CC, BB)                                                \
    extern "C" __global__ __launch_bounds__(64) void name(dspb_seg_args G) { dspb_seg_chain<CC, BB>(G); }
DSPB_CHAIN_KERNEL(dspb_seg_chain_c2b512, 2, 512)
DSPB_CHAIN_KERNEL(dspb_seg_chain_c2, 2, 0)
DSPB_CHAIN_KERNEL(dspb_seg_chain_c1, 1, 0)
DSPB_CHAIN_KERNEL(dspb_seg_chain_c4, 4, 0)

// ---- a split State: the chain of its block-independent words --------------
// The callback in file order, as dspb_seg_chain (over 64 lanes' ranges of
// segments, below), recording only the words no block-dependent store can hit (dspb_word_dep: compile-time, so
// the arithmetic that feeds only the other words -- an envelope, and with it
// the block -- is compiled away and the chain is the counter's alone).  Pass 1
// then starts each segment's warm-up from these words and the live State's
// others; the segments are checked bit for bit as always, so a wrong word here
// costs reruns, never output.
template <unsigned CC, unsigned BB>
__device__ static void dspb_seg_chain_ind(const dspb_seg_args &G) {
    const dspb_render_args &A = G.R;
    if (blockIdx.x != 0 || !kStateWords) return;
    if (!dspb_seg_level_runs(G)) return;  // launched before each warm-up level's pass 1
    constexpr unsigned BMAX = BB ? BB : 4096u;
    const unsigned B = BB ? BB : A.B;
    const Parameters prm = dspb_from_global<Parameters>(A.P);
    // (block indices fit 32 bits: the host renders no longer file this way)
    const unsigned nb = (unsigned)A.nblocks, seg = (unsigned)G.seg;
    // the segments 1 .. K - 1 in 64 contiguous ranges, one per lane: a lane
    // runs the chain from the file's start to its range's first record, then
    // on through its range.  Each stretch between records is the callback over
    // the blocks of the stretch, the block compiled away: a counter's or a
    // phase step's stretch the optimizer closes into a few instructions, so the
    // lanes' long first stretches cost what a short one does, and the 9,122
    // records of a stereo hour come from 64 lanes (one lane took 0.58 ms);
    // a stretch that stays a loop costs the longest lane's blocks, as the one
    // lane's chain over the whole file did.
    const unsigned n = G.K - 1, per = (n + 63u) / 64u, lane = threadIdx.x & 63u;
    const unsigned k0 = 1u + lane * per, k1 = k0 + per < G.K ? k0 + per : G.K;
    State st;
    dspb_copy_state((void *)&st, (const void *)A.S);
    unsigned b = 0;
    for (unsigned k = k0; k < k1; ++k) {
        // pass 1 at this level starts segment k's warm-up at block p: the
        // callback up to there, then the record
        const unsigned b0 = k * seg, p = b0 > G.warm ? b0 - G.warm : 0u, e = p < nb ? p : nb;
        for (; b < e; ++b) {
            float dspb_chain_blk[CC * BMAX];
            float *ptrs[CC];
#pragma unroll
            for (unsigned c = 0; c < CC; ++c) {
                ptrs[c] = dspb_chain_blk + c * B;
                const dspb_gfloat *x = (const dspb_gfloat *)A.in[c < A.in_ch ? c : 0];
                for (unsigned i = 0; i < B; ++i) {
                    const unsigned long long gi = (unsigned long long)b * B + i;
                    dspb_chain_blk[c * B + i] = (c < A.in_ch && gi < A.L) ? x[gi] : 0.0f;
                }
            }
            audio_callback(prm, st, ptrs, CC, B, A.sr);
        }
        State *rec = &G.st_ind[(unsigned long long)G.level * G.K + k];
        dspb_copy_ind_words((void *)rec, (const void *)&st);
        if constexpr (kStateWords) {
            // test hook: a wrong record (the low bit of the first independent
            // word) for segment perturb-1 at the first level
            constexpr unsigned kW = dspb_first_ind_word();
            if (kW < sizeof(State) / 4 && G.perturb && G.level == 0 && G.perturb - 1 == k)
                ((dspb_word *)rec)[kW] ^= 1u;
        }
    }
}
#define DSPB_CHAIN_IND_KERNEL(name, CC, BB)                                            \
    extern "C" __global__ __launch_bounds__(64) void name(dspb_seg_args G) { dspb_seg_chain_ind<CC, BB>(G); }
DSPB_CHAIN_IND_KERNEL(dspb_seg_chain_ind_c2b512, 2, 512)
DSPB_CHAIN_IND_KERNEL(dspb_seg_chain_ind_c2, 2, 0)
DSPB_CHAIN_IND_KERNEL(dspb_seg_chain_ind_c1, 1, 0)
DSPB_CHAIN_IND_KERNEL(dspb_seg_chain_ind_c4, 4, 0)
