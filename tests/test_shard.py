"""Time-chunk sharding (dspbench/shard.py) on CPU.

The plan is checked two ways: exhaustively as arithmetic (chunks tile the
file, frames tile the whole-file frame range, every owned frame's samples
lie inside owned + halo), and end to end with world_size-2 and -4 gloo processes
that each render + STFT their chunk with the oracle and gather to rank 0,
which must reproduce the whole-file oracle result exactly.
"""
import numpy as np
import pytest

import dspbench.shard as sh
import rankrun


@pytest.mark.parametrize("B", [1, 64, 384, 512, 4096, 8192])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("render", [True, False])
def test_plan_tiles_file_and_frames(B, world, render):
    N, H = 8192, 4096
    for L in [0, 1, 8191, 8192, 8193, 50_000, 3 * 49152 + 17, 1_000_000]:
        shards = [sh.plan(L, world, r, B, N, H, render) for r in range(world)]
        Lf = (-(-L // B) * B) if render else L
        F = sh.stft_frames(Lf, N, H)
        pos, f = 0, 0
        for s in shards:
            assert s.start == pos and s.owned >= 0
            assert s.start % B == 0 and s.start % H == 0
            assert s.frame0 == f or s.frames == 0
            pos, f = s.end, s.frame0 + s.frames if s.frames else f
            last = s.end >= L
            # every owned frame starts in the chunk and its samples are read
            for g in (s.frame0, s.frame0 + s.frames - 1) if s.frames else ():
                assert s.start <= g * H < max(s.end, s.start + 1) or last
                if not last:  # (a halo cut at EOF reads up to the padded end)
                    assert g * H + N <= (Lf if s.end + s.halo >= L else s.end + s.halo)
        assert pos == L and f == F


def _worker(rank, world, L, B):
    import torch
    import torch.distributed as dist
    import oracle as o
    rng = np.random.default_rng(11)
    x = (rng.random((2, L), dtype=np.float32) * 2 - 1).astype(np.float32)
    s = sh.plan(L, world, rank, B)
    chunk = x[:, s.start:s.start + s.read_len]
    out = o.render_offline([chunk[0], chunk[1]], 2, B, 48000.0, o.restated_plugin("IR_test"),
                           L=s.read_len)
    mags = [o.np_stft_mag(out[c], 8192, 4096, o.WIN_HANN, 4097)[: s.frames] for c in range(2)]
    own = torch.from_numpy(np.ascontiguousarray(out[:, : s.owned]))
    mag = torch.from_numpy(np.ascontiguousarray(np.stack(mags)))
    parts = [None] * world
    dist.all_gather_object(parts, (own, mag))
    if rank == 0:
        ren = np.concatenate([p[0].numpy() for p in parts], axis=1)
        mg = np.concatenate([p[1].numpy() for p in parts], axis=1)
        ref = o.render_offline([x[0], x[1]], 2, B, 48000.0, o.restated_plugin("IR_test"))
        ok_r = ren.shape == (2, L) and np.array_equal(ren, ref[:, :L])
        mref = np.stack([o.np_stft_mag(ref[c], 8192, 4096, o.WIN_HANN, 4097) for c in range(2)])
        ok_m = mg.shape == mref.shape and np.array_equal(mg, mref)
        return ok_r, ok_m, mg.shape, mref.shape


@pytest.mark.parametrize("B,world", [(512, 2), (384, 2), (512, 4)])
def test_gloo_ranks_match_whole_file(B, world, tmp_path):
    L = 5 * 49152 + 1234
    ok_r, ok_m, shape, rshape = rankrun.run(_worker, world, tmp_path, args=(L, B), timeout=240)
    assert ok_r, "sharded render differs from the whole-file render"
    assert ok_m, f"sharded STFT differs from the whole-file STFT {shape} vs {rshape}"


# ---- the product's gather schedule, executed over gloo ----------------------

def _sharded_worker(rank, world, mode, C_total, C_file, L, B, chunk):
    """The product's plan (dsp_shard_plan), chunk schedule (dsp_shard_chunks)
    and gather schedule (dsp_shard_gather_plan, the pieces
    dsp_render_stft_sharded moves) executed over gloo, with the oracle
    standing in for the GPU render of each chunk."""
    import torch
    import torch.distributed as dist
    import oracle as o
    N, H, K = 8192, 4096, 4097
    rng = np.random.default_rng(21)
    x = (rng.random((C_file, L), dtype=np.float32) * 2 - 1).astype(np.float32)
    s = sh.plan(L, world, rank, B, N, H, True, C_total, mode)
    nb = -(-s.read_len // B)
    out = np.zeros((s.channels, nb * B), np.float32)
    mag = np.zeros((s.channels, max(s.frames, 1), K), np.float32)
    plug = o.restated_plugin("IR_test", [0.7, 0.003])
    for c in sh.chunks(s, L, B, N, H, True, chunk):  # this rank's compute, chunk by chunk
        o_ = c.start - s.start
        Lc = min(max(L - c.start, 0), c.owned + c.halo)
        rows = [x[g, c.start:c.start + Lc] for g in range(s.chan0, s.chan0 + s.channels) if g < C_file]
        ren = o.render_offline(rows, s.channels, B, 48000.0, plug, L=Lc)
        out[:, o_:o_ + ren.shape[1]] = ren
        for j in range(s.channels):
            m = o.np_stft_mag(ren[j], N, H, o.WIN_HANN, K)[: c.frames]
            mag[j, c.frame0 - s.frame0:c.frame0 - s.frame0 + m.shape[0]] = m
    pieces, steps = sh.gather_plan(L, C_total, world, B, N, H, mode, chunk, K)
    Lpad = -(-L // B) * B
    F = sh.stft_frames(Lpad, N, H)
    all_out = np.zeros((C_total, Lpad), np.float32)
    all_mag = np.zeros((C_total, F * K), np.float32)
    for p in pieces:  # in schedule order, as the driver moves them
        if p.src == rank:
            j = p.channel - s.chan0
            row = out[j] if p.what == sh.PIECE_RENDER else mag[j].reshape(-1)
            buf = torch.from_numpy(np.ascontiguousarray(row[p.src_off:p.src_off + p.count]))
        dst = (all_out if p.what == sh.PIECE_RENDER else all_mag)[p.channel]
        if p.src == 0 and rank == 0:
            dst[p.dst_off:p.dst_off + p.count] = buf.numpy()
        elif rank == 0:
            t = torch.empty(p.count)
            dist.recv(t, src=p.src)
            dst[p.dst_off:p.dst_off + p.count] = t.numpy()
        elif p.src == rank:
            dist.send(buf, dst=0)
    if rank == 0:
        ref = o.render_offline([x[c] for c in range(C_file)], C_total, B, 48000.0, plug)
        ok_r = np.array_equal(all_out, ref)
        mref = np.stack([o.np_stft_mag(ref[c], N, H, o.WIN_HANN, K) for c in range(C_total)]).astype(np.float32)
        ok_m = np.array_equal(all_mag.reshape(C_total, F, K), mref)
        return ok_r, ok_m, steps


@pytest.mark.parametrize("mode,C_total,C_file,B,world,chunk", [
    (sh.CHANNELS, 4, 3, 512, 2, 49152),   # cfg5's shape in small: a channel run per rank, chunked
    (sh.CHANNELS, 3, 3, 384, 4, 0),       # more ranks than channels: rank 3 idles
    (sh.TIME, 2, 2, 512, 2, 36864),       # time chunks with halos, chunked inside each rank
])
def test_gloo_sharded_driver_reassembles_the_whole_file(mode, C_total, C_file, B, world, chunk, tmp_path):
    L = 4 * 49152 + 777
    ok_r, ok_m, steps = rankrun.run(_sharded_worker, world, tmp_path,
                                    args=(mode, C_total, C_file, L, B, chunk), timeout=300)
    assert ok_r, "gathered render differs from the whole-file render"
    assert ok_m, "gathered STFT differs from the whole-file STFT"


@pytest.mark.parametrize("mode,C_total,world,B,chunk", [
    (sh.CHANNELS, 8, 8, 512, 1 << 16), (sh.CHANNELS, 8, 3, 512, 0), (sh.CHANNELS, 3, 4, 384, 49152),
    (sh.TIME, 2, 4, 512, 36864), (sh.TIME, 2, 3, 384, 0), (sh.TIME, 1, 2, 1, 12288), (sh.TIME, 2, 1, 512, 20000),
])
def test_gather_plan_covers_every_row_once(mode, C_total, world, B, chunk):
    """dsp_shard_gather_plan: the pieces cover every render sample of the
    block-padded file and every magnitude row of every channel exactly once,
    read inside each sender's local rows, in (step, src) order."""
    N, H, K = 8192, 4096, 4097
    for L in [0, 8191, 8192 * 3 + 5, 4 * 49152 + 777, 300_000]:
        pieces, steps = sh.gather_plan(L, C_total, world, B, N, H, mode, chunk, K)
        Lpad = -(-L // B) * B
        F = sh.stft_frames(Lpad, N, H)
        ren = np.zeros((C_total, Lpad), np.int32)
        mg = np.zeros((C_total, F * K), np.int32)
        plans = [sh.plan(L, world, r, B, N, H, True, C_total, mode) for r in range(world)]
        assert [(p.step, p.src) for p in pieces] == sorted((p.step, p.src) for p in pieces)
        for p in pieces:
            assert p.step < steps and p.count > 0
            s = plans[p.src]
            assert s.chan0 <= p.channel < s.chan0 + s.channels
            if p.what == sh.PIECE_RENDER:
                assert p.src_off + p.count <= -(-s.read_len // B) * B
                ren[p.channel, p.dst_off:p.dst_off + p.count] += 1
            else:
                assert p.src_off + p.count <= s.frames * K and p.count % K == 0
                mg[p.channel, p.dst_off:p.dst_off + p.count] += 1
        assert (ren == 1).all() and (mg == 1).all(), (L, ren.min(), ren.max(), mg.min() if mg.size else None)


def test_channel_plan_and_chunks():
    """Channel runs tile the channels; chunks tile each shard's owned range
    with lcm(B, H)-aligned boundaries and owned frames that tile the shard's."""
    for C_total, world in [(8, 8), (8, 3), (2, 4), (1, 1)]:
        runs = [sh.plan(10 ** 6, world, r, 512, 8192, 4096, True, C_total, sh.CHANNELS) for r in range(world)]
        assert sum(r.channels for r in runs) == C_total
        assert [r.chan0 for r in runs] == sorted(r.chan0 for r in runs)
    for L in [8192, 10 ** 6 + 3, 3 * 36864]:
        s = sh.plan(L, 1, 0, 512, 8192, 4096, True, 2, sh.TIME)
        for chunk in (0, 1, 36864, 100_000):
            cs = sh.chunks(s, L, 512, 8192, 4096, True, chunk)
            assert cs[0].start == s.start and cs[-1].end == s.end
            assert all(a.end == b.start and a.start % 4096 == 0 for a, b in zip(cs, cs[1:]))
            assert sum(c.frames for c in cs) == s.frames


# ---- the rank harness itself (tests/rankrun.py) -----------------------------

def _rank1_fails(rank, world):
    import torch.distributed as dist
    if rank == 1:
        raise ValueError("rank 1 fails after the rendezvous")
    dist.barrier()  # rank 0 would wait here until its collective timeout


def _rank1_hangs(rank, world):
    import time
    if rank == 1:
        time.sleep(600)
    return "rank 0 done"


def _pre_init_failure(rank, world):
    if rank == 1:
        raise OSError("rank 1 fails before its rendezvous")


def _rank_id(rank, world):
    return rank


def test_rank_failure_before_rendezvous_fails_fast(tmp_path):
    """A rank that raises -- after the rendezvous while its peer waits in a
    collective, or before its rendezvous while its peer waits in
    init_process_group -- fails the call in well under 100 s with that rank's
    traceback, and no child outlives the call."""
    import multiprocessing
    import time
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="rank 1 failed"):
        rankrun.run(_rank1_fails, 2, tmp_path, init_timeout=30, timeout=90)
    assert time.monotonic() - t0 < 60
    assert not multiprocessing.active_children()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="rank 1 failed"):
        rankrun.run(_rank_id, 2, tmp_path, before=_pre_init_failure, init_timeout=30, timeout=90)
    assert time.monotonic() - t0 < 60
    assert not multiprocessing.active_children()


def test_rank_hang_times_out_and_is_reaped(tmp_path):
    import multiprocessing
    import time
    t0 = time.monotonic()
    with pytest.raises(TimeoutError):
        rankrun.run(_rank1_hangs, 2, tmp_path, timeout=8)
    assert time.monotonic() - t0 < 40
    assert not multiprocessing.active_children()
