// shard.cpp -- multi-GPU sharding of the render + STFT path (shard.h,
// SURVEY 8(e)): the shard / chunk planners, an RCCL communicator, the gather
// and the pipelined per-rank driver.
//
// RCCL is loaded on first use (dlopen "librccl.so.1", the NCCL API of
// /opt/rocm/include/rccl/rccl.h), so the library, its planners and its CPU
// tests do not depend on it.  When torch has already loaded its own copy the
// same object is reused (dlopen by soname).
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dspbench/shard.h"

namespace dspb {
void set_last_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
}  // namespace dspb
using dspb::set_last_error;

#define SH_HIP(x)                                                  \
    do {                                                           \
        hipError_t e_ = (x);                                       \
        if (e_ != hipSuccess) return dspb::hip_fail(e_, #x);       \
    } while (0)

namespace {

int invalid(const char *fmt, ...) {
    char buf[400];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    set_last_error("%s", buf);
    return DSP_ERR_INVALID;
}

uint64_t gcd64(uint64_t a, uint64_t b) {
    while (b) {
        const uint64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

uint64_t frames_of(uint64_t L, uint32_t N, uint32_t H) { return (N == 0 || H == 0 || L < N) ? 0 : (L - N) / H + 1; }

// the time share [lo, hi) of an L-sample file (units of lcm(B, H)): halo and
// owned frames, as dspbench/shard.py plan()
void time_range(uint64_t L, uint64_t lo, uint64_t hi, uint32_t B, uint32_t N, uint32_t H, int render,
                dsp_shard *s) {
    s->start = lo;
    s->owned = hi - lo;
    const bool last = hi >= L;
    s->halo = last ? 0 : std::min<uint64_t>(N - H, L - hi);
    const uint64_t Lf = render ? (L + B - 1) / B * B : L;
    const uint64_t F = frames_of(Lf, N, H);
    const uint64_t f0 = std::min<uint64_t>(lo / H, F);
    const uint64_t f1 = last ? F : std::min<uint64_t>((hi + H - 1) / H, F);
    s->frame0 = f0;
    s->frames = f1 > f0 ? f1 - f0 : 0;
}

// ---- RCCL, loaded on first use -------------------------------------------
typedef int ncclResult_t;
typedef void *ncclComm_t;
struct ncclUniqueId {
    char internal[DSP_COMM_ID_BYTES];
};
constexpr int kNcclFloat32 = 7;

struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*Send)(const void *, size_t, int, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void *, size_t, int, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    const char *(*GetErrorString)(ncclResult_t);
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            r.err = std::string("cannot load librccl: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](const char *n) {
            void *p = dlsym(h, n);
            if (!p) all = false;
            return p;
        };
        r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
        r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
        r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
        r.Send = (decltype(r.Send))sym("ncclSend");
        r.Recv = (decltype(r.Recv))sym("ncclRecv");
        r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
        r.ok = all;
        if (!all) r.err = "librccl lacks an NCCL entry point";
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char *what) {
    set_last_error("%s: RCCL error %d (%s)", what, e, rccl().GetErrorString ? rccl().GetErrorString(e) : "?");
    return DSP_ERR_HIP;
}

#define NCCL_CK(x)                                   \
    do {                                             \
        ncclResult_t e_ = (x);                       \
        if (e_ != 0) return nccl_fail(e_, #x);       \
    } while (0)

}  // namespace

struct dsp_comm {
    ncclComm_t comm = nullptr;
    uint32_t world = 0, rank = 0;
    int device = -1;
    hipStream_t stream = nullptr;  // the pipeline's gather stream
};

extern "C" {

int dsp_shard_plan(uint64_t L, uint32_t C, uint32_t world, uint32_t rank, uint32_t B, uint32_t N, uint32_t H,
                   uint32_t mode, int render, dsp_shard *out) {
    if (!out) return invalid("dsp_shard_plan: out is NULL");
    if (world == 0 || rank >= world || B == 0 || H == 0 || N < H)
        return invalid("dsp_shard_plan: bad world %u / rank %u / B %u / N %u / H %u", world, rank, B, N, H);
    std::memset(out, 0, sizeof *out);
    out->rank = rank;
    out->world = world;
    out->mode = mode;
    if (mode == DSP_SHARD_CHANNELS) {
        const uint32_t c0 = (uint32_t)((uint64_t)rank * C / world), c1 = (uint32_t)((uint64_t)(rank + 1) * C / world);
        out->chan0 = c0;
        out->channels = c1 - c0;
        time_range(L, 0, L, B, N, H, render, out);
        if (out->channels == 0) out->frames = 0, out->owned = 0;
        return DSP_OK;
    }
    if (mode != DSP_SHARD_TIME) return invalid("dsp_shard_plan: unknown mode %u", mode);
    out->chan0 = 0;
    out->channels = C;
    const uint64_t unit = (uint64_t)B / gcd64(B, H) * H;
    const uint64_t units = (L + unit - 1) / unit;
    const uint64_t u0 = units * rank / world, u1 = units * (rank + 1) / world;
    time_range(L, std::min(u0 * unit, L), std::min(u1 * unit, L), B, N, H, render, out);
    return DSP_OK;
}

int64_t dsp_shard_chunks(const dsp_shard *s, uint64_t L, uint32_t B, uint32_t N, uint32_t H, int render,
                         uint64_t chunk, dsp_shard *out, uint64_t cap) {
    if (!s || B == 0 || H == 0 || N < H) return invalid("dsp_shard_chunks: bad arguments");
    const uint64_t unit = (uint64_t)B / gcd64(B, H) * H;
    const uint64_t step = chunk == 0 ? (s->owned ? s->owned : 1) : (chunk + unit - 1) / unit * unit;
    const uint64_t end = s->start + s->owned;
    int64_t n = 0;
    if (s->owned == 0) return 0;
    for (uint64_t lo = s->start; lo < end; lo += step, ++n) {
        if (out && (uint64_t)n < cap) {
            dsp_shard c = *s;
            time_range(L, lo, std::min(lo + step, end), B, N, H, render, &c);
            out[n] = c;
        }
    }
    return n;
}

int dsp_comm_unique_id(void *id) {
    if (!id) return invalid("dsp_comm_unique_id: NULL");
    Rccl &r = rccl();
    if (!r.ok) return invalid("%s", r.err.c_str());
    ncclUniqueId u;
    NCCL_CK(r.GetUniqueId(&u));
    std::memcpy(id, u.internal, DSP_COMM_ID_BYTES);
    return DSP_OK;
}

int dsp_comm_init(const void *id, uint32_t world, uint32_t rank, int32_t device, dsp_comm **out) {
    if (!id || !out || world == 0 || rank >= world) return invalid("dsp_comm_init: bad arguments");
    *out = nullptr;
    Rccl &r = rccl();
    if (!r.ok) return invalid("%s", r.err.c_str());
    int prev = -1;
    SH_HIP(hipGetDevice(&prev));
    if (device >= 0 && device != prev) SH_HIP(hipSetDevice(device));
    dsp_comm *c = new dsp_comm();
    (void)hipGetDevice(&c->device);
    c->world = world;
    c->rank = rank;
    ncclUniqueId u;
    std::memcpy(u.internal, id, DSP_COMM_ID_BYTES);
    ncclResult_t e = r.CommInitRank(&c->comm, (int)world, u, (int)rank);
    hipError_t he = e == 0 ? hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) : hipSuccess;
    if (prev >= 0 && prev != c->device) (void)hipSetDevice(prev);
    if (e != 0) {
        delete c;
        return nccl_fail(e, "ncclCommInitRank");
    }
    if (he != hipSuccess) {
        (void)r.CommDestroy(c->comm);
        delete c;
        return dspb::hip_fail(he, "hipStreamCreate");
    }
    *out = c;
    return DSP_OK;
}

void dsp_comm_destroy(dsp_comm *c) {
    if (!c) return;
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->comm) (void)rccl().CommDestroy(c->comm);
    delete c;
}

}  // extern "C"

namespace {

// one gather step: rank `src` sends `count` floats to the root's `dst`
struct Piece {
    uint32_t src;
    const float *send;  // on src
    float *dst;         // on the root
    uint64_t count;
};

int run_pieces(dsp_comm *c, uint32_t root, const std::vector<Piece> &pieces, hipStream_t s) {
    Rccl &r = rccl();
    bool any_p2p = false;
    for (const Piece &p : pieces) any_p2p = any_p2p || (p.src != root && p.count);
    if (any_p2p) NCCL_CK(r.GroupStart());
    for (const Piece &p : pieces) {
        if (!p.count) continue;
        if (p.src == root) {
            if (c->rank == root && p.dst != p.send)
                SH_HIP(hipMemcpyAsync(p.dst, p.send, p.count * sizeof(float), hipMemcpyDeviceToDevice, s));
        } else if (c->rank == root) {
            NCCL_CK(r.Recv(p.dst, p.count, kNcclFloat32, (int)p.src, c->comm, s));
        } else if (c->rank == p.src) {
            NCCL_CK(r.Send(p.send, p.count, kNcclFloat32, (int)root, c->comm, s));
        }
    }
    if (any_p2p) NCCL_CK(r.GroupEnd());
    return DSP_OK;
}

}  // namespace

extern "C" {

int dsp_comm_gather(dsp_comm *c, const float *send, uint64_t count, float *const *recv, uint32_t root,
                    void *stream) {
    if (!c || root >= c->world) return invalid("dsp_comm_gather: bad communicator / root");
    if (count && !send) return invalid("dsp_comm_gather: send is NULL");
    if (c->rank == root && count && !recv) return invalid("dsp_comm_gather: recv is NULL on the root");
    std::vector<Piece> pieces;
    for (uint32_t r = 0; r < c->world; ++r) {
        float *dst = (c->rank == root) ? recv[r] : nullptr;
        if (c->rank == root && count && !dst) return invalid("dsp_comm_gather: recv[%u] is NULL", r);
        pieces.push_back(Piece{r, r == c->rank ? send : nullptr, dst, count});
    }
    return run_pieces(c, root, pieces, (hipStream_t)stream);
}

int dsp_render_stft_sharded(const float *const *in, uint32_t in_channels, uint64_t L, float *const *out,
                            float *const *mag, uint64_t ld, uint32_t C, uint32_t B, float sr,
                            const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window, uint32_t K,
                            const dsp_shard *sh, uint64_t chunk, dsp_comm *comm, uint32_t root,
                            float *const *all_out, float *const *all_mag, const dsp_exec *ex) {
    if (!sh || B == 0 || H == 0 || N < H) return invalid("dsp_render_stft_sharded: bad arguments");
    if (ex && (ex->flags & DSP_EXEC_HOST_BUFFERS)) return invalid("dsp_render_stft_sharded: device buffers only");
    if (in_channels > sh->channels) return invalid("in_channels %u > the shard's %u channels", in_channels, sh->channels);
    const uint32_t world = comm ? comm->world : sh->world, rank = comm ? comm->rank : sh->rank;
    if (comm && (sh->world != world || sh->rank != rank))
        return invalid("shard (rank %u of %u) is not this communicator's", sh->rank, sh->world);
    if (root >= world) return invalid("root %u >= world %u", root, world);
    // with a communicator every rank takes part in the gather; without one
    // there is no collective (world 1 with all_out: device copies)
    const bool gather = comm ? true : (world == 1 && (all_out || all_mag));
    if (gather && rank == root && !(all_out && all_mag)) return invalid("the root needs both all_out and all_mag");
    const uint64_t goff0 = ex ? ex->sample_offset : 0;
    if (sh->mode == DSP_SHARD_TIME && plugin && plugin->kind == DSP_PLUGIN_GENERIC && plugin->state_size)
        return invalid("time sharding needs a state-free plugin");

    int prev = -1;
    SH_HIP(hipGetDevice(&prev));
    const int dev = (ex && ex->device >= 0) ? ex->device : prev;
    if (comm && comm->device != dev) return invalid("communicator on device %d, call on device %d", comm->device, dev);
    if (dev != prev) SH_HIP(hipSetDevice(dev));
    struct Restore {
        int p, d;
        ~Restore() { if (p >= 0 && p != d) (void)hipSetDevice(p); }
    } restore{prev, dev};
    hipStream_t s = ex ? (hipStream_t)ex->stream : nullptr;

    // a chunk's render, padded to whole blocks, must end before the first
    // frame of the next chunk: ceil((N - H) / B) B < N, else a chunk would
    // also compute (from a cut halo) a frame it does not own
    const bool halo_fits = (uint64_t)(N - H + B - 1) / B * B < N;
    if (!halo_fits && sh->mode == DSP_SHARD_TIME && sh->world > 1)
        return invalid("time sharding needs ceil((N - H) / B) B < N (B = %u, N = %u, H = %u)", B, N, H);
    // this rank's chunks (a GENERIC plugin is rendered as one call: its
    // State, if any, carries through the whole channel)
    const bool one_chunk = (plugin && plugin->kind == DSP_PLUGIN_GENERIC) || !halo_fits;
    const int64_t nch = dsp_shard_chunks(sh, L, B, N, H, 1, one_chunk ? 0 : chunk, nullptr, 0);
    if (nch < 0) return (int)nch;
    std::vector<dsp_shard> chunks((size_t)nch);
    dsp_shard_chunks(sh, L, B, N, H, 1, one_chunk ? 0 : chunk, chunks.data(), chunks.size());
    // the root's view of every rank's plan and chunks
    std::vector<dsp_shard> plans(world);
    std::vector<std::vector<dsp_shard>> rchunks(world);
    int64_t steps = nch;
    if (gather && comm) {
        for (uint32_t r = 0; r < world; ++r) {
            int st = dsp_shard_plan(L, C, world, r, B, N, H, sh->mode, 1, &plans[r]);
            if (st) return st;
        }
        if (plans[rank].chan0 != sh->chan0 || plans[rank].channels != sh->channels || plans[rank].start != sh->start ||
            plans[rank].owned != sh->owned)
            return invalid("the shard does not match dsp_shard_plan(L, C = %u, world %u, rank %u)", C, world, rank);
        for (uint32_t r = 0; r < world; ++r) {
            const int64_t n = dsp_shard_chunks(&plans[r], L, B, N, H, 1, one_chunk ? 0 : chunk, nullptr, 0);
            rchunks[r].resize((size_t)std::max<int64_t>(n, 0));
            dsp_shard_chunks(&plans[r], L, B, N, H, 1, one_chunk ? 0 : chunk, rchunks[r].data(), rchunks[r].size());
            steps = std::max<int64_t>(steps, n);
        }
    }
    const uint64_t Lpad = (L + B - 1) / B * B;
    const uint32_t nrow = sh->channels;
    hipEvent_t ev_done = nullptr;
    std::vector<hipEvent_t> evs;
    struct Events {
        std::vector<hipEvent_t> *v;
        hipEvent_t *e;
        ~Events() {
            for (hipEvent_t x : *v) (void)hipEventDestroy(x);
            if (*e) (void)hipEventDestroy(*e);
        }
    } evg{&evs, &ev_done};
    for (int64_t t = 0; t < steps; ++t) {
        // compute chunk t on the caller's stream
        if (t < nch && nrow) {
            const dsp_shard &c = chunks[(size_t)t];
            const uint64_t o = c.start - sh->start;
            const uint64_t avail = L > c.start ? L - c.start : 0;
            const uint64_t Lc = std::min<uint64_t>(avail, c.owned + c.halo);
            std::vector<const float *> cin(in_channels);
            std::vector<float *> cout(nrow), cmag(nrow);
            for (uint32_t j = 0; j < in_channels; ++j) cin[j] = in[j] + o;
            for (uint32_t j = 0; j < nrow; ++j) {
                cout[j] = out[j] + o;
                cmag[j] = mag[j] + (c.frame0 - sh->frame0) * ld;
            }
            dsp_exec e{};
            e.device = dev;
            e.flags = 0;
            e.stream = s;
            e.sample_offset = goff0 + c.start;
            const uint64_t Fc = frames_of((Lc + B - 1) / B * B, N, H);
            if (Fc > c.frames && c.frames) return invalid("chunk plan: %llu frames computed, %llu owned",
                                                          (unsigned long long)Fc, (unsigned long long)c.frames);
            int st = dsp_render_stft(cin.data(), in_channels, Lc, cout.data(), nrow, B, sr, plugin, N, H, window, K,
                                     cmag.data(), ld, &e);
            if (st) return st;
        }
        if (!gather) continue;
        // gather chunk t to the root on the comm stream, behind its compute
        hipEvent_t ev;
        SH_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        evs.push_back(ev);
        SH_HIP(hipEventRecord(ev, s));
        hipStream_t gs = comm ? comm->stream : s;
        if (comm) SH_HIP(hipStreamWaitEvent(gs, ev, 0));
        std::vector<Piece> pieces;
        for (uint32_t r = 0; r < world; ++r) {
            const dsp_shard &pr = comm ? plans[r] : *sh;
            const std::vector<dsp_shard> &rc = comm ? rchunks[r] : chunks;
            if (t >= (int64_t)rc.size()) continue;
            const dsp_shard &c = rc[(size_t)t];
            // the render rows a chunk contributes: its owned samples, and the
            // block padding past EOF for the chunk that reaches it
            const uint64_t rlen = (c.start + c.owned >= L) ? Lpad - c.start : c.owned;
            for (uint32_t j = 0; j < pr.channels; ++j) {
                const uint32_t gc = pr.chan0 + j;
                const bool mine = r == rank;
                const uint64_t o = c.start - pr.start;
                pieces.push_back(Piece{r, mine ? out[j] + o : nullptr, rank == root ? all_out[gc] + c.start : nullptr, rlen});
                pieces.push_back(Piece{r, mine ? mag[j] + (c.frame0 - pr.frame0) * ld : nullptr,
                                       rank == root ? all_mag[gc] + c.frame0 * ld : nullptr, c.frames * ld});
            }
        }
        if (comm) {
            int st = run_pieces(comm, root, pieces, gs);
            if (st) return st;
        } else {  // world 1 without a communicator: device copies
            for (const Piece &p : pieces)
                if (p.count && p.dst != p.send)
                    SH_HIP(hipMemcpyAsync(p.dst, p.send, p.count * sizeof(float), hipMemcpyDeviceToDevice, s));
        }
    }
    if (gather && comm) {  // the caller's stream sees the gathered rows
        SH_HIP(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
        SH_HIP(hipEventRecord(ev_done, comm->stream));
        SH_HIP(hipStreamWaitEvent(s, ev_done, 0));
    }
    if (ex && (ex->flags & DSP_EXEC_SYNC)) SH_HIP(hipStreamSynchronize(s));
    return DSP_OK;
}

}  // extern "C"
