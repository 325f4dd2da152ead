// shard.cpp -- multi-GPU sharding of the render + STFT path (shard.h,
// SURVEY 8(e)): the shard / chunk planners, the gather schedule, the
// communicators (a transport table: RCCL, an in-process loopback, or the
// caller's) and the pipelined per-rank driver.
//
// RCCL is loaded on first use (dlopen "librccl.so.1"; the types come from
// /opt/rocm/include/rccl/rccl.h), so the library, its planners and its CPU
// tests do not depend on it.  When torch has already loaded its own copy the
// same object is reused (dlopen by soname).
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "dspbench/module.h"
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
// (types from rccl.h; the entry points resolved by dlsym)
static_assert(NCCL_UNIQUE_ID_BYTES == DSP_COMM_ID_BYTES, "communicator id size");

struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) GetUniqueId;
    decltype(&ncclCommInitRank) CommInitRank;
    decltype(&ncclCommDestroy) CommDestroy;
    decltype(&ncclSend) Send;
    decltype(&ncclRecv) Recv;
    decltype(&ncclGroupStart) GroupStart;
    decltype(&ncclGroupEnd) GroupEnd;
    decltype(&ncclGetErrorString) GetErrorString;
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
    set_last_error("%s: RCCL error %d (%s)", what, (int)e, rccl().GetErrorString ? rccl().GetErrorString(e) : "?");
    return DSP_ERR_HIP;
}

#define NCCL_CK(x)                                   \
    do {                                             \
        ncclResult_t e_ = (x);                       \
        if (e_ != ncclSuccess) return nccl_fail(e_, #x); \
    } while (0)

// the RCCL transport: user = the ncclComm_t
int rccl_group_start(void *) {
    NCCL_CK(rccl().GroupStart());
    return DSP_OK;
}
int rccl_group_end(void *) {
    NCCL_CK(rccl().GroupEnd());
    return DSP_OK;
}
int rccl_send(void *u, const float *buf, uint64_t count, uint32_t peer, void *stream) {
    NCCL_CK(rccl().Send(buf, count, ncclFloat32, (int)peer, (ncclComm_t)u, (hipStream_t)stream));
    return DSP_OK;
}
int rccl_recv(void *u, float *buf, uint64_t count, uint32_t peer, void *stream) {
    NCCL_CK(rccl().Recv(buf, count, ncclFloat32, (int)peer, (ncclComm_t)u, (hipStream_t)stream));
    return DSP_OK;
}
void rccl_destroy(void *u) {
    if (u) (void)rccl().CommDestroy((ncclComm_t)u);
}
const dsp_comm_transport kRcclTransport = {rccl_group_start, rccl_group_end, rccl_send, rccl_recv, rccl_destroy};

// ---- the in-process loopback transport -------------------------------------
// Ranks are host threads of one process on one device.  A send posts
// (pointer, count, an event recorded on the sender's stream) to the
// (src, dst) mailbox; the matching recv makes its stream wait for that event,
// copies device to device, records `done` and hands it back; the sender's
// stream waits for `done`.  Inside a group, recvs and the sends' completion
// are deferred to group_end (sends post at once), so a group never blocks on
// its peers' issue order.  A wait that times out fails the hub: every rank's
// later call returns an error at once (no recv can pair with a stale message
// of the failed step), and the failing rank takes its own unreceived
// messages back out of the mailboxes.
constexpr int kLoopWaitSeconds = 120;

struct LoopMsg {
    const float *ptr = nullptr;
    uint64_t count = 0;
    hipEvent_t ready = nullptr, done = nullptr;
    bool taken = false;   // a recv has it
    bool copied = false;  // the copy and `done` are enqueued (or failed)
    int status = DSP_OK;
};

struct LoopHub {
    std::mutex mu;
    std::condition_variable cv;
    uint32_t world = 0;
    bool failed = false;  // a rank timed out: every later call fails
    std::vector<std::deque<std::shared_ptr<LoopMsg>>> box;  // [src * world + dst]
};

struct LoopRank {
    std::shared_ptr<LoopHub> hub;
    uint32_t rank = 0;
    int depth = 0;
    struct Sent {
        std::shared_ptr<LoopMsg> m;
        hipStream_t s;
    };
    struct Recv {
        float *buf;
        uint64_t count;
        uint32_t peer;
        hipStream_t s;
    };
    std::vector<Sent> sent;
    std::vector<Recv> recvs;
};

int loop_flush(LoopRank *lr);

// after a failure: this rank's pending recvs are dropped, and its sends that
// no recv has taken leave their mailboxes (their events destroyed); a send a
// recv has taken but not finished keeps its events (the copy may use them)
void loop_abandon(LoopRank *lr) {
    LoopHub &h = *lr->hub;
    lr->recvs.clear();
    std::vector<LoopRank::Sent> sent;
    sent.swap(lr->sent);
    std::lock_guard<std::mutex> g(h.mu);
    for (const LoopRank::Sent &s : sent) {
        if (s.m->taken) continue;
        for (auto &q : h.box) {
            for (auto it = q.begin(); it != q.end(); ++it)
                if (*it == s.m) {
                    q.erase(it);
                    break;
                }
        }
        (void)hipEventDestroy(s.m->ready);
        (void)hipEventDestroy(s.m->done);
    }
}

int loop_group_start(void *u) {
    ++((LoopRank *)u)->depth;
    return DSP_OK;
}

int loop_group_end(void *u) {
    LoopRank *lr = (LoopRank *)u;
    if (lr->depth <= 0) return invalid("loopback: group_end without group_start");
    return --lr->depth == 0 ? loop_flush(lr) : DSP_OK;
}

int hub_failed(LoopHub &h, uint32_t rank) {
    std::lock_guard<std::mutex> g(h.mu);
    return h.failed ? invalid("loopback: rank %u: the communicators failed in an earlier call (a timeout)", rank)
                    : DSP_OK;
}

int loop_send(void *u, const float *buf, uint64_t count, uint32_t peer, void *stream) {
    LoopRank *lr = (LoopRank *)u;
    LoopHub &h = *lr->hub;
    if (peer >= h.world || peer == lr->rank) return invalid("loopback: bad peer %u (rank %u)", peer, lr->rank);
    if (int st = hub_failed(h, lr->rank)) return st;
    auto m = std::make_shared<LoopMsg>();
    m->ptr = buf;
    m->count = count;
    SH_HIP(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    SH_HIP(hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
    SH_HIP(hipEventRecord(m->ready, (hipStream_t)stream));
    {
        std::lock_guard<std::mutex> g(h.mu);
        h.box[(size_t)lr->rank * h.world + peer].push_back(m);
    }
    h.cv.notify_all();
    lr->sent.push_back({m, (hipStream_t)stream});
    return lr->depth ? DSP_OK : loop_flush(lr);
}

int loop_recv(void *u, float *buf, uint64_t count, uint32_t peer, void *stream) {
    LoopRank *lr = (LoopRank *)u;
    if (peer >= lr->hub->world || peer == lr->rank) return invalid("loopback: bad peer %u (rank %u)", peer, lr->rank);
    if (int st = hub_failed(*lr->hub, lr->rank)) return st;
    lr->recvs.push_back({buf, count, peer, (hipStream_t)stream});
    return lr->depth ? DSP_OK : loop_flush(lr);
}

int loop_flush(LoopRank *lr) {
    LoopHub &h = *lr->hub;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(kLoopWaitSeconds);
    int st = DSP_OK;
    std::vector<LoopRank::Recv> recvs;
    recvs.swap(lr->recvs);
    for (const LoopRank::Recv &r : recvs) {
        std::shared_ptr<LoopMsg> m;
        {
            std::unique_lock<std::mutex> g(h.mu);
            auto &q = h.box[(size_t)r.peer * h.world + lr->rank];
            if (!h.cv.wait_until(g, deadline, [&] { return h.failed || !q.empty(); }) || h.failed) {
                const bool mine = !h.failed;
                h.failed = true;
                g.unlock();
                h.cv.notify_all();
                loop_abandon(lr);
                return mine ? invalid("loopback: rank %u waited %d s for a send from rank %u", lr->rank,
                                      kLoopWaitSeconds, r.peer)
                            : invalid("loopback: rank %u: another rank timed out", lr->rank);
            }
            m = q.front();
            q.pop_front();
            m->taken = true;
        }
        int ms = DSP_OK;
        if (m->count != r.count)
            ms = invalid("loopback: rank %u receives %llu floats, rank %u sent %llu", lr->rank,
                         (unsigned long long)r.count, r.peer, (unsigned long long)m->count);
        hipError_t e = hipSuccess;
        if (ms == DSP_OK) e = hipStreamWaitEvent(r.s, m->ready, 0);
        if (ms == DSP_OK && e == hipSuccess && r.count)
            e = hipMemcpyAsync(r.buf, m->ptr, r.count * sizeof(float), hipMemcpyDeviceToDevice, r.s);
        if (ms == DSP_OK && e == hipSuccess) e = hipEventRecord(m->done, r.s);
        if (ms == DSP_OK && e != hipSuccess) ms = dspb::hip_fail(e, "loopback copy");
        {
            std::lock_guard<std::mutex> g(h.mu);
            m->status = ms;
            m->copied = true;
        }
        h.cv.notify_all();
        if (ms && !st) st = ms;
    }
    std::vector<LoopRank::Sent> sent;
    sent.swap(lr->sent);
    for (const LoopRank::Sent &s : sent) {
        {
            std::unique_lock<std::mutex> g(h.mu);
            if (!h.cv.wait_until(g, deadline, [&] { return s.m->copied || h.failed; }) || !s.m->copied) {
                h.failed = true;
                g.unlock();
                h.cv.notify_all();
                lr->sent.push_back(s);  // (and the rest: loop_abandon takes them back)
                if (!st) st = invalid("loopback: rank %u: its send was not received in %d s", lr->rank,
                                      kLoopWaitSeconds);
                continue;
            }
        }
        if (s.m->status == DSP_OK) {
            const hipError_t e = hipStreamWaitEvent(s.s, s.m->done, 0);
            if (e != hipSuccess && !st) st = dspb::hip_fail(e, "loopback: wait for the copy");
        } else if (!st) {
            st = s.m->status;
        }
        // a recorded event may be destroyed while pending: the waits above
        // hold what they need
        (void)hipEventDestroy(s.m->ready);
        (void)hipEventDestroy(s.m->done);
    }
    if (!lr->sent.empty()) loop_abandon(lr);  // the sends no recv took after a timeout
    return st;
}

void loop_destroy(void *u) { delete (LoopRank *)u; }

const dsp_comm_transport kLoopTransport = {loop_group_start, loop_group_end, loop_send, loop_recv, loop_destroy};

}  // namespace

struct dsp_comm {
    dsp_comm_transport t{};
    void *user = nullptr;
    uint32_t world = 0, rank = 0;
    int device = -1;
    hipStream_t stream = nullptr;  // the pipeline's gather stream
};

namespace {

// a communicator on `device` with its gather stream; takes `user` (released
// through t.destroy when this fails)
int make_comm(const dsp_comm_transport &t, void *user, uint32_t world, uint32_t rank, int32_t device,
              dsp_comm **out) {
    int prev = -1;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && device >= 0 && device != prev) e = hipSetDevice(device);
    dsp_comm *c = new dsp_comm();
    c->t = t;
    c->user = user;
    c->world = world;
    c->rank = rank;
    if (e == hipSuccess) e = hipGetDevice(&c->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (prev >= 0 && prev != c->device) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        if (t.destroy) t.destroy(user);
        delete c;
        return dspb::hip_fail(e, "dsp_comm: device / stream");
    }
    *out = c;
    return DSP_OK;
}

}  // namespace

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

}  // extern "C"

namespace {

// every rank's plan and chunks, and the pieces of the gather in schedule order
struct GatherPlan {
    std::vector<dsp_shard> plans;
    std::vector<std::vector<dsp_shard>> chunks;
    std::vector<dsp_gather_piece> pieces;
    uint64_t steps = 0;
};

int gather_plan(uint64_t L, uint32_t C, uint32_t world, uint32_t B, uint32_t N, uint32_t H, uint32_t mode,
                uint64_t chunk, uint64_t ld, GatherPlan *g) {
    if (world == 0) return invalid("gather plan: world 0");
    g->plans.assign(world, dsp_shard{});
    g->chunks.assign(world, {});
    g->pieces.clear();
    g->steps = 0;
    for (uint32_t r = 0; r < world; ++r) {
        int st = dsp_shard_plan(L, C, world, r, B, N, H, mode, 1, &g->plans[r]);
        if (st) return st;
        const int64_t n = dsp_shard_chunks(&g->plans[r], L, B, N, H, 1, chunk, nullptr, 0);
        if (n < 0) return (int)n;
        g->chunks[r].resize((size_t)n);
        dsp_shard_chunks(&g->plans[r], L, B, N, H, 1, chunk, g->chunks[r].data(), g->chunks[r].size());
        g->steps = std::max<uint64_t>(g->steps, (uint64_t)n);
    }
    const uint64_t Lpad = (L + B - 1) / B * B;
    for (uint64_t t = 0; t < g->steps; ++t)
        for (uint32_t r = 0; r < world; ++r) {
            const dsp_shard &p = g->plans[r];
            if (t >= g->chunks[r].size()) continue;
            const dsp_shard &c = g->chunks[r][t];
            // the render samples a chunk contributes: its owned samples, and
            // the block padding past EOF for the chunk that reaches it
            const uint64_t rlen = (c.start + c.owned >= L) ? Lpad - c.start : c.owned;
            for (uint32_t j = 0; j < p.channels; ++j) {
                const uint32_t gc = p.chan0 + j;
                if (rlen) g->pieces.push_back({(uint32_t)t, r, gc, DSP_PIECE_RENDER, c.start - p.start, c.start, rlen});
                if (c.frames)
                    g->pieces.push_back({(uint32_t)t, r, gc, DSP_PIECE_MAG, (c.frame0 - p.frame0) * ld, c.frame0 * ld,
                                         c.frames * ld});
            }
        }
    return DSP_OK;
}

// one gather step through the communicator's transport: rank src's pieces
// into the root's rows (the root's own pieces are device copies)
struct Move {
    uint32_t src;
    const float *send;  // on src
    float *dst;         // on the root
    uint64_t count;
};

int run_moves(dsp_comm *c, uint32_t root, const std::vector<Move> &moves, hipStream_t s) {
    bool any_p2p = false;
    for (const Move &m : moves) any_p2p = any_p2p || (m.src != root && m.count && (c->rank == root || c->rank == m.src));
    int st = DSP_OK;
    if (any_p2p && (st = c->t.group_start(c->user))) return st;
    for (const Move &m : moves) {
        if (!m.count || st) continue;
        if (m.src == root) {
            if (c->rank == root && m.dst != m.send) {
                const hipError_t e = hipMemcpyAsync(m.dst, m.send, m.count * sizeof(float), hipMemcpyDeviceToDevice, s);
                if (e != hipSuccess) st = dspb::hip_fail(e, "gather: root copy");
            }
        } else if (c->rank == root) {
            st = c->t.recv(c->user, m.dst, m.count, m.src, s);
        } else if (c->rank == m.src) {
            st = c->t.send(c->user, m.send, m.count, root, s);
        }
    }
    if (any_p2p) {  // close the group even after a failed call
        const int ge = c->t.group_end(c->user);
        if (!st) st = ge;
    }
    return st;
}

}  // namespace

extern "C" {

int64_t dsp_shard_gather_plan(uint64_t L, uint32_t C, uint32_t world, uint32_t B, uint32_t N, uint32_t H,
                              uint32_t mode, uint64_t chunk, uint64_t ld, dsp_gather_piece *out, uint64_t cap,
                              uint64_t *steps) {
    if (B == 0 || H == 0 || N < H) return invalid("dsp_shard_gather_plan: bad B / N / H");
    GatherPlan g;
    int st = gather_plan(L, C, world, B, N, H, mode, chunk, ld, &g);
    if (st) return st;
    if (out)
        for (size_t i = 0; i < g.pieces.size() && i < cap; ++i) out[i] = g.pieces[i];
    if (steps) *steps = g.steps;
    return (int64_t)g.pieces.size();
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
    ncclUniqueId u;
    std::memcpy(u.internal, id, DSP_COMM_ID_BYTES);
    ncclComm_t nc = nullptr;
    const ncclResult_t e = r.CommInitRank(&nc, (int)world, u, (int)rank);
    if (prev >= 0 && device >= 0 && device != prev) (void)hipSetDevice(prev);
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitRank");
    return make_comm(kRcclTransport, nc, world, rank, device, out);
}

int dsp_comm_init_transport(const dsp_comm_transport *t, void *user, uint32_t world, uint32_t rank,
                            int32_t device, dsp_comm **out) {
    if (!t || !out || world == 0 || rank >= world || !t->group_start || !t->group_end || !t->send || !t->recv)
        return invalid("dsp_comm_init_transport: bad arguments");
    *out = nullptr;
    return make_comm(*t, user, world, rank, device, out);
}

int dsp_comm_init_loopback(uint32_t world, int32_t device, dsp_comm **out) {
    if (!out || world == 0) return invalid("dsp_comm_init_loopback: bad arguments");
    auto hub = std::make_shared<LoopHub>();
    hub->world = world;
    hub->box.resize((size_t)world * world);
    for (uint32_t r = 0; r < world; ++r) out[r] = nullptr;
    for (uint32_t r = 0; r < world; ++r) {
        LoopRank *lr = new LoopRank();
        lr->hub = hub;
        lr->rank = r;
        int st = make_comm(kLoopTransport, lr, world, r, device, &out[r]);
        if (st) {
            for (uint32_t q = 0; q < r; ++q) dsp_comm_destroy(out[q]), out[q] = nullptr;
            return st;
        }
    }
    return DSP_OK;
}

void dsp_comm_destroy(dsp_comm *c) {
    if (!c) return;
    if (c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    if (c->t.destroy) c->t.destroy(c->user);
    delete c;
}

int dsp_comm_info(const dsp_comm *c, uint32_t *rank, uint32_t *world) {
    if (!c) return invalid("dsp_comm_info: NULL");
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    return DSP_OK;
}

int dsp_comm_gather(dsp_comm *c, const float *send, uint64_t count, float *const *recv, uint32_t root,
                    void *stream) {
    if (!c || root >= c->world) return invalid("dsp_comm_gather: bad communicator / root");
    if (count && !send) return invalid("dsp_comm_gather: send is NULL");
    if (c->rank == root && count && !recv) return invalid("dsp_comm_gather: recv is NULL on the root");
    std::vector<Move> moves;
    for (uint32_t r = 0; r < c->world; ++r) {
        float *dst = (c->rank == root) ? recv[r] : nullptr;
        if (c->rank == root && count && !dst) return invalid("dsp_comm_gather: recv[%u] is NULL", r);
        moves.push_back(Move{r, r == c->rank ? send : nullptr, dst, count});
    }
    return run_moves(c, root, moves, (hipStream_t)stream);
}

int dsp_render_stft_sharded(const float *const *in, uint32_t in_channels, uint64_t L, float *const *out,
                            float *const *mag, uint64_t ld, uint32_t C, uint32_t B, float sr,
                            const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window, uint32_t K,
                            const dsp_shard *sh, uint64_t chunk, dsp_comm *comm, uint32_t root,
                            float *const *all_out, float *const *all_mag, const dsp_exec *ex) {
    if (ex && ex->result) *ex->result = 0;  // the chunks' DSP_RESULT_* bits are OR-ed in
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
    // a GENERIC plugin's State lives in its module (plugin->state_size is 0):
    // ask the module whether it has one
    int stateless = 1;
    if (plugin && plugin->kind == DSP_PLUGIN_GENERIC) {
        if (!plugin->module) return invalid("GENERIC plugin needs a loaded dsp_module");
        if (int st = dsp_module_sizes((const dsp_module *)plugin->module, nullptr, nullptr, &stateless)) return st;
    }
    const bool stateful_generic = plugin && plugin->kind == DSP_PLUGIN_GENERIC && !stateless;
    // a State carried from block to block (audio.cpp:160-165) cannot start
    // mid-file: time shards need blocks that render independently
    if (sh->mode == DSP_SHARD_TIME && sh->world > 1 && stateful_generic)
        return invalid("time sharding needs blocks that render independently: this plugin's callback writes its "
                       "State, which the reference carries from block to block (audio.cpp:160-165); shard it by "
                       "channel (DSP_SHARD_CHANNELS)");
    if (sh->mode == DSP_SHARD_TIME && sh->world > 1 && plugin &&
        (plugin->kind == DSP_PLUGIN_FIR || plugin->kind == DSP_PLUGIN_BIQUAD))
        return invalid("time sharding needs blocks that render independently: a %s filter's state runs through "
                       "the whole file; shard it by channel (DSP_SHARD_CHANNELS)",
                       plugin->kind == DSP_PLUGIN_FIR ? "FIR" : "BIQUAD");

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
    // this rank's chunks (a GENERIC plugin with a State is rendered as one
    // call: the State carries through the whole channel)
    const bool one_chunk = stateful_generic || !halo_fits;
    const uint64_t eff_chunk = one_chunk ? 0 : chunk;
    const int64_t nch = dsp_shard_chunks(sh, L, B, N, H, 1, eff_chunk, nullptr, 0);
    if (nch < 0) return (int)nch;
    std::vector<dsp_shard> chunks((size_t)nch);
    dsp_shard_chunks(sh, L, B, N, H, 1, eff_chunk, chunks.data(), chunks.size());
    // the gather schedule: every rank's plan, chunks and pieces
    GatherPlan gp;
    if (gather) {
        int st = gather_plan(L, C, world, B, N, H, sh->mode, eff_chunk, ld, &gp);
        if (st) return st;
        const dsp_shard &p = gp.plans[rank];
        if (p.chan0 != sh->chan0 || p.channels != sh->channels || p.start != sh->start || p.owned != sh->owned)
            return invalid("the shard does not match dsp_shard_plan(L, C = %u, world %u, rank %u)", C, world, rank);
    }
    const int64_t steps = gather ? std::max<int64_t>(nch, (int64_t)gp.steps) : nch;
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
    size_t pi = 0;  // the next gather piece
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
            e.flags = ex ? (ex->flags & DSP_EXEC_METHOD_FLAGS) : 0;
            e.stream = s;
            e.sample_offset = goff0 + c.start;
            uint32_t chunk_res = 0;  // DSP_RESULT_* of this chunk, OR-ed into the caller's
            e.result = &chunk_res;
            const uint64_t Fc = frames_of((Lc + B - 1) / B * B, N, H);
            if (Fc > c.frames && c.frames) return invalid("chunk plan: %llu frames computed, %llu owned",
                                                          (unsigned long long)Fc, (unsigned long long)c.frames);
            int st = dsp_render_stft(cin.data(), in_channels, Lc, cout.data(), nrow, B, sr, plugin, N, H, window, K,
                                     cmag.data(), ld, &e);
            if (st) return st;
            if (ex && ex->result) *ex->result |= chunk_res;
        }
        if (!gather) continue;
        // gather step t to the root on the comm stream, behind its compute
        std::vector<Move> moves;
        for (; pi < gp.pieces.size() && gp.pieces[pi].step == (uint32_t)t; ++pi) {
            const dsp_gather_piece &p = gp.pieces[pi];
            const dsp_shard &pr = gp.plans[p.src];
            const uint32_t j = p.channel - pr.chan0;
            const float *send = nullptr;
            float *dst = nullptr;
            if (p.src == rank) send = (p.what == DSP_PIECE_RENDER ? out[j] : mag[j]) + p.src_off;
            if (rank == root) dst = (p.what == DSP_PIECE_RENDER ? all_out[p.channel] : all_mag[p.channel]) + p.dst_off;
            moves.push_back(Move{p.src, send, dst, p.count});
        }
        if (moves.empty()) continue;
        hipStream_t gs = s;
        if (comm) {
            hipEvent_t ev;
            SH_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            evs.push_back(ev);
            SH_HIP(hipEventRecord(ev, s));
            gs = comm->stream;
            SH_HIP(hipStreamWaitEvent(gs, ev, 0));
            int st = run_moves(comm, root, moves, gs);
            if (st) return st;
        } else {  // world 1 without a communicator: device copies
            for (const Move &m : moves)
                if (m.count && m.dst != m.send)
                    SH_HIP(hipMemcpyAsync(m.dst, m.send, m.count * sizeof(float), hipMemcpyDeviceToDevice, s));
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
