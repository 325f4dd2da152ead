"""Time-chunk sharding (dspbench/shard.py) on CPU.

The plan is checked two ways: exhaustively as arithmetic (chunks tile the
file, frames tile the whole-file frame range, every owned frame's samples
lie inside owned + halo), and end to end with world_size-2 and -4 gloo processes
that each render + STFT their chunk with the oracle and gather to rank 0,
which must reproduce the whole-file oracle result exactly.
"""
import os
import socket

import numpy as np
import pytest

import dspbench.shard as sh


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


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, world, port, L, B, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
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
            q.put((ok_r, ok_m, mg.shape, mref.shape))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B,world", [(512, 2), (384, 2), (512, 4)])
def test_gloo_ranks_match_whole_file(B, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    L = 5 * 49152 + 1234
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, L, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ok_r, ok_m, shape, rshape = res
    assert ok_r, "sharded render differs from the whole-file render"
    assert ok_m, f"sharded STFT differs from the whole-file STFT {shape} vs {rshape}"


# ---- the product's sharded driver with a torch.distributed transport -------

def _sharded_worker(rank, world, port, mode, C_total, C_file, L, B, chunk, q):
    """dspbench.shard.render_stft_sharded over gloo (TorchComm): the product's
    plan (dsp_shard_plan), chunk schedule (dsp_shard_chunks) and gather
    pieces, with the oracle standing in for the GPU render of each chunk."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as o
        N, H, K = 8192, 4096, 4097
        rng = np.random.default_rng(21)
        x = (rng.random((C_file, L), dtype=np.float32) * 2 - 1).astype(np.float32)
        s = sh.plan(L, world, rank, B, N, H, True, C_total, mode)
        # this rank's file rows, local to the shard
        rows = [c for c in range(s.chan0, s.chan0 + s.channels) if c < C_file]
        xl = torch.from_numpy(np.ascontiguousarray(x[rows, s.start:s.start + s.read_len]))
        nb = -(-s.read_len // B)
        out = torch.zeros((s.channels, nb * B))
        mag = torch.zeros((s.channels, max(s.frames, 1), K))
        plug = o.restated_plugin("IR_test", [0.7, 0.003])

        def compute(c, xo, oo, mo, goff):
            fc = [xo[j].numpy() for j in range(xo.shape[0])] if xo is not None else []
            Lc = oo.shape[1] if xo is None else xo.shape[1]
            ren = o.render_offline(fc, s.channels, B, 48000.0, plug, L=Lc)
            oo.copy_(torch.from_numpy(ren[:, :oo.shape[1]]))
            for j in range(s.channels):
                m = o.np_stft_mag(ren[j], N, H, o.WIN_HANN, K)
                mo[j].copy_(torch.from_numpy(m[: mo.shape[1]].astype(np.float32)))

        Lpad = -(-L // B) * B
        F = sh.stft_frames(Lpad, N, H)
        all_out = torch.zeros((C_total, Lpad)) if rank == 0 else None
        all_mag = torch.zeros((C_total, F, K)) if rank == 0 else None
        sh.render_stft_sharded(xl if rows else None, L, C_total, B, 48000.0, None, s, out, mag,
                               comm=sh.TorchComm(), root=0, all_out=all_out, all_mag=all_mag, chunk=chunk,
                               compute=compute)
        if rank == 0:
            ref = o.render_offline([x[c] for c in range(C_file)], C_total, B, 48000.0, plug)
            ok_r = np.array_equal(all_out.numpy(), ref)
            mref = np.stack([o.np_stft_mag(ref[c], N, H, o.WIN_HANN, K) for c in range(C_total)]).astype(np.float32)
            ok_m = np.array_equal(all_mag.numpy(), mref)
            q.put((ok_r, ok_m))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,C_total,C_file,B,world,chunk", [
    (sh.CHANNELS, 4, 3, 512, 2, 49152),   # cfg5's shape in small: a channel run per rank, chunked
    (sh.CHANNELS, 3, 3, 384, 4, 0),       # more ranks than channels: rank 3 idles
    (sh.TIME, 2, 2, 512, 2, 36864),       # time chunks with halos, chunked inside each rank
])
def test_gloo_sharded_driver_reassembles_the_whole_file(mode, C_total, C_file, B, world, chunk):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    L = 4 * 49152 + 777
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, mode, C_total, C_file, L, B, chunk, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ok_r, ok_m = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok_r, "gathered render differs from the whole-file render"
    assert ok_m, "gathered STFT differs from the whole-file STFT"


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
