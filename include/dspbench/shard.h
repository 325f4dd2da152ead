/*
 * shard.h -- multi-GPU sharding of the render + STFT path.
 *
 * One process per GPU.  A long or multichannel render is split into
 * independent units with one exchange step at the end, a gather to a root
 * rank over RCCL (xGMI):
 *
 *   DSP_SHARD_CHANNELS  channel -> GPU (BASELINE configs[4]: 8 channels of
 *                       96 kHz, one per GPU).  Valid for channel-separable
 *                       plugins: the map plugins (gain_test, static_gain,
 *                       IR_test, no_op; IR_test writes the same ramp to every
 *                       channel, build/IR_test.cpp:48-58) and GENERIC plugins
 *                       the caller declares separable.  The reference's
 *                       multichannel rule is kept per channel: device
 *                       channels past the file's are rendered from zeros
 *                       (audio.cpp:65-81, 138-141).
 *   DSP_SHARD_TIME      time chunk -> GPU for state-free plugins: chunk
 *                       boundaries aligned to lcm(B, H), each rank re-renders
 *                       the N - H sample halo of the next chunk so every frame
 *                       starting in its chunk is local (no halo exchange).
 *
 * Within a rank the owned range is processed in chunks (dsp_shard_chunks)
 * and each chunk's render rows and magnitude rows are gathered to the root
 * on a separate HIP stream while the next chunk computes, following
 * dsp_shard_gather_plan, over a communicator's transport: RCCL between
 * processes (the product), or an in-process loopback (ranks as threads on
 * one GPU) that runs the same driver at world > 1 without a second GPU.
 *
 * The reference has no multi-GPU path (single audio thread, audio.cpp:13-175);
 * everything here is new, built around its single-GPU semantics.
 */
#ifndef DSPBENCH_SHARD_H
#define DSPBENCH_SHARD_H

#include <stddef.h>
#include <stdint.h>

#include "dspbench.h"

#ifdef __cplusplus
extern "C" {
#endif

enum dsp_shard_mode { DSP_SHARD_TIME = 0, DSP_SHARD_CHANNELS = 1 };

typedef struct dsp_shard {
    uint32_t rank, world;
    uint32_t mode;            /* dsp_shard_mode */
    uint32_t chan0, channels; /* device channels this rank renders: [chan0, chan0 + channels) */
    uint64_t start;           /* first owned sample (global), a multiple of lcm(B, H) */
    uint64_t owned;           /* owned samples per channel */
    uint64_t halo;            /* samples read past the owned range (<= N - H; 0 at EOF) */
    uint64_t frame0, frames;  /* owned STFT frames (global index, count) */
} dsp_shard;

/* The share of a C-channel, L-sample render + STFT (N, H, block B) that
 * `rank` of `world` owns.  render != 0: frames over the block-padded render
 * (ceil(L / B) B samples, as dsp_render_stft); 0: over the raw signal
 * (dsp_stft_magnitude).  Channel mode: channels split into contiguous runs
 * (rank r: [r C / world, (r + 1) C / world)), every rank owns the whole
 * time axis.  Time mode: every rank owns all C channels of its chunk. */
int dsp_shard_plan(uint64_t L, uint32_t C, uint32_t world, uint32_t rank, uint32_t B, uint32_t N,
                   uint32_t H, uint32_t mode, int render, dsp_shard *out);

/* The pipeline's chunks of a shard: sub-ranges of [start, start + owned) of
 * about `chunk` samples (rounded up to lcm(B, H); 0 = one chunk), each with
 * its halo and owned frames, in order.  Writes min(n, cap) entries to out
 * (out may be NULL), returns n (or a negative status). */
int64_t dsp_shard_chunks(const dsp_shard *s, uint64_t L, uint32_t B, uint32_t N, uint32_t H, int render,
                         uint64_t chunk, dsp_shard *out, uint64_t cap);

/* ---- the gather schedule ---------------------------------------------------
 * Every rank's chunk t is gathered to the root as one step: for each of the
 * rank's channels, its owned render samples (plus the block padding past EOF
 * for the chunk that reaches it) and its owned magnitude rows.  One entry per
 * non-empty move, ordered by (step, src, channel, what). */
enum dsp_piece_what { DSP_PIECE_RENDER = 0, DSP_PIECE_MAG = 1 };

typedef struct dsp_gather_piece {
    uint32_t step;     /* pipeline step (the sender's chunk index) */
    uint32_t src;      /* sending rank */
    uint32_t channel;  /* global device channel; the sender's row is channel - its chan0 */
    uint32_t what;     /* dsp_piece_what */
    uint64_t src_off;  /* floats into the sender's local row (out[j] / mag[j]) */
    uint64_t dst_off;  /* floats into the root's whole-file row (all_out[channel] / all_mag[channel]) */
    uint64_t count;    /* floats */
} dsp_gather_piece;

/* The gather schedule of a `world`-rank sharded render + STFT (the plans of
 * dsp_shard_plan(..., render = 1), chunks of dsp_shard_chunks(..., chunk);
 * chunk 0 = one chunk per rank), magnitude rows of stride ld.  Writes
 * min(n, cap) pieces to out (may be NULL), returns n (or a negative status);
 * *steps (may be NULL) receives the number of pipeline steps.
 * dsp_render_stft_sharded moves exactly these pieces. */
int64_t dsp_shard_gather_plan(uint64_t L, uint32_t C, uint32_t world, uint32_t B, uint32_t N, uint32_t H,
                              uint32_t mode, uint64_t chunk, uint64_t ld, dsp_gather_piece *out, uint64_t cap,
                              uint64_t *steps);

/* ---- communicators (one per rank) -------------------------------------------
 * A communicator moves floats between ranks through a transport with NCCL
 * point-to-point semantics.  The product transport is RCCL over xGMI
 * (dsp_comm_init); others plug in through dsp_comm_init_transport. */
#define DSP_COMM_ID_BYTES 128
typedef struct dsp_comm dsp_comm;

/* A transport: every call is enqueued on a HIP stream and returns 0 or a
 * negative dsp_status.  A send and its matching recv carry the same count;
 * between group_start and group_end (which nest) the sends and recvs of one
 * gather step are issued in schedule order by every rank and must complete
 * without deadlock whatever the peers' order; a send's buffer may be reused
 * once `stream` has passed the send. */
typedef struct dsp_comm_transport {
    int (*group_start)(void *user);
    int (*group_end)(void *user);
    int (*send)(void *user, const float *buf, uint64_t count, uint32_t peer, void *stream);
    int (*recv)(void *user, float *buf, uint64_t count, uint32_t peer, void *stream);
    void (*destroy)(void *user); /* NULL: nothing to release */
} dsp_comm_transport;

/* A fresh RCCL communicator id (ncclGetUniqueId), made on one rank and
 * handed to the others out of band (torch.distributed, a file, a socket). */
int dsp_comm_unique_id(void *id);
/* Join the RCCL communicator of `world` ranks on `device` (-1: current). */
int dsp_comm_init(const void *id, uint32_t world, uint32_t rank, int32_t device, dsp_comm **out);
/* Rank `rank` of `world` over a caller's transport (copied; `user` is passed
 * to every call and to destroy when the communicator goes). */
int dsp_comm_init_transport(const dsp_comm_transport *t, void *user, uint32_t world, uint32_t rank,
                            int32_t device, dsp_comm **out);
/* In-process loopback: `world` communicators (out[0 .. world)) whose ranks
 * are host threads of this process sharing `device` (-1: current), one
 * thread per rank.  A send records an event on the sender's stream; the
 * matching recv makes the receiver's stream wait for it and copies device to
 * device; the sender's stream then waits for that copy.  A peer that never
 * posts its side fails the wait after 120 s (DSP_ERR_INVALID).  Each
 * communicator is destroyed on its own. */
int dsp_comm_init_loopback(uint32_t world, int32_t device, dsp_comm **out);
void dsp_comm_destroy(dsp_comm *c);
/* The rank and world of a communicator (either may be NULL). */
int dsp_comm_info(const dsp_comm *c, uint32_t *rank, uint32_t *world);

/* Gather: every rank sends `count` floats from `send` (device memory); the
 * root receives rank r's into recv[r] (device memory, world entries; its own
 * entry is copied device to device).  recv is ignored on other ranks.
 * Enqueued on `stream` (NULL: the legacy default stream). */
int dsp_comm_gather(dsp_comm *c, const float *send, uint64_t count, float *const *recv, uint32_t root,
                    void *stream);

/* The sharded render + STFT of this rank (device buffers, all local to the
 * shard: index 0 is global sample `start`, frame `frame0`):
 *   in[c]       this rank's file rows, c < in_channels (global channel
 *               chan0 + c), holding min(L - start, owned + halo) samples
 *   out[c] /    this rank's render rows (ceil((owned + halo) / B) B floats)
 *   mag[c]      and magnitude rows (`frames` rows of stride ld)
 *   all_out /   the root's C render rows (ceil(L / B) B floats) / C magnitude
 *   all_mag     rows (F rows of stride ld) of the whole file (ignored on
 *               other ranks)
 * L is the whole file's length, C its device channel count (the plan's).
 * Chunks (dsp_shard_chunks, about `chunk` samples) are computed on
 * ex->stream.  With a communicator every chunk's rows are gathered to `root`
 * on the communicator's stream behind them (every rank takes part) and the
 * caller's stream then waits for the gather.  comm NULL: no collective --
 * each rank computes its share only; at world 1 with all_out / all_mag the
 * rows are copied there.  Per channel and chunk the result is
 * dsp_render_stft's with sample_offset = the chunk's global start. */
int dsp_render_stft_sharded(const float *const *in, uint32_t in_channels, uint64_t L, float *const *out,
                            float *const *mag, uint64_t ld, uint32_t C, uint32_t B, float sr,
                            const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window, uint32_t K,
                            const dsp_shard *shard, uint64_t chunk, dsp_comm *comm, uint32_t root,
                            float *const *all_out, float *const *all_mag, const dsp_exec *ex);

#ifdef __cplusplus
}
#endif
#endif
