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
