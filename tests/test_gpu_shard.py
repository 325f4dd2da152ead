"""cfg 5 (BASELINE configs[4]: 8-channel 96 kHz render through IR_test + 8192-pt
FFT, one channel per GPU, RCCL gather) through the product's shard path on
one GPU: the per-GPU unit (C = 1, 96 kHz, IR_test + fused STFT) against the
oracle, the pipelined C++ driver (dsp_render_stft_sharded) with an RCCL
communicator of one rank, and a two-rank rehearsal of the N > 1 path (both
ranks on cuda:0, gloo as the transport) that must reassemble the whole-file
result.  The 8-GPU run itself is the driver's (unmeasured on hardware here).
"""
import os
import socket

import numpy as np
import pytest

import dspbench as d
import dspbench.shard as sh

pytestmark = pytest.mark.gpu

PEAK_REL_TOL = 1e-6


def peak_rel_err(m, ref):
    m = np.asarray(m, np.float64)
    ref = np.asarray(ref, np.float64)
    peak = np.maximum(ref.max(axis=-1), 1e-30)
    return float(np.max(np.abs(m - ref).max(axis=-1) / peak))


def test_cfg5_per_gpu_unit_vs_oracle(torch_cuda, oracle):
    """One 96 kHz channel through IR_test (B = 512) + the fused Hann STFT, as
    one rank of cfg 5 renders it (C = 1)."""
    torch = torch_cuda
    L, B = 8192 * 9 + 1111, 512
    x = np.random.default_rng(31).uniform(-1, 1, (1, L)).astype(np.float32)
    out, mag = d.render_stft(torch.from_numpy(x).cuda(), 1, B, 96000.0, d.Plugin.ir_test(0.9, 0.002),
                             window=d.DSP_WIN_HANN)
    ref = oracle.render_offline([x[0]], 1, B, 96000.0, oracle.restated_plugin("IR_test"))
    assert np.array_equal(out.cpu().numpy(), ref)
    mref = oracle.np_stft_mag(ref[0], 8192, 4096, d.DSP_WIN_HANN, 4097)
    assert peak_rel_err(mag.cpu().numpy()[0], mref) <= PEAK_REL_TOL


def test_cfg5_per_gpu_unit_full_size_1h_96k(torch_cuda, oracle):
    """The per-GPU unit at full size: 1 h of one 96 kHz channel (345.6 M
    samples).  Properties: the render is the B-periodic ramp; every frame of
    a B-periodic signal with B | H is the same spectrum, matching float64."""
    torch = torch_cuda
    L, B = 96_000 * 3600, 512
    x = torch.zeros((1, L), device="cuda")
    out, mag = d.render_stft(x, 1, B, 96000.0, d.Plugin.ir_test(), window=d.DSP_WIN_HANN)
    ramp = torch.from_numpy(oracle.ir_ramp_reference(0.9, 0.002, B)).cuda()
    assert torch.equal(out.view(1, -1, B), ramp.expand(1, L // B, B))
    F = mag.shape[1]
    assert F == (L - 8192) // 4096 + 1
    ref0 = oracle.np_stft_mag(np.tile(ramp.cpu().numpy(), 16), 8192, 4096, d.DSP_WIN_HANN, 4097)[0]
    for f in [0, 1, F // 3, F - 1]:
        assert peak_rel_err(mag[0, f].cpu().numpy(), ref0) <= PEAK_REL_TOL
    assert (mag[0] - mag[0, :1]).abs().max().item() <= 1e-6 * float(ref0.max())


def _whole(torch, x, C_total, B, plugin, L):
    out, mag = d.render_stft(x, C_total, B, 96000.0, plugin, window=d.DSP_WIN_HANN, L_file=L)
    torch.cuda.synchronize()
    return out, mag


@pytest.mark.parametrize("use_comm", [False, True])
@pytest.mark.parametrize("mode,C_total,C_file,chunk", [(sh.CHANNELS, 8, 8, 1 << 16), (sh.CHANNELS, 8, 6, 0),
                                                       (sh.TIME, 2, 2, 3 * 4096)])
def test_sharded_driver_world1_equals_whole_file(torch_cuda, mode, C_total, C_file, chunk, use_comm):
    """dsp_render_stft_sharded (chunked compute, gather on the communicator's
    stream) at world 1, with and without an RCCL communicator: the root's
    rows equal dsp_render_stft of the whole file bit for bit."""
    torch = torch_cuda
    L, B = 8192 * 20 + 3333, 512
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.rand((C_file, L), device="cuda", generator=g) * 2 - 1
    plugin = d.Plugin.ir_test(0.8, 0.001) if mode == sh.CHANNELS else d.Plugin.gain_test(0.3)
    ref_out, ref_mag = _whole(torch, x, C_total, B, plugin, L)
    s = sh.plan(L, 1, 0, B, 8192, 4096, True, C_total, mode)
    nb = -(-L // B)
    out = torch.empty((C_total, nb * B), device="cuda")
    mag = torch.empty((C_total, s.frames, 4097), device="cuda")
    all_out = torch.full((C_total, nb * B), -7.0, device="cuda")
    all_mag = torch.full((C_total, s.frames, 4097), -7.0, device="cuda")
    comm = sh.RcclComm(sh.RcclComm.unique_id(), 1, 0, torch.cuda.current_device()) if use_comm else None
    sh.render_stft_sharded(x, L, C_total, B, 96000.0, plugin, s, out, mag, comm=comm, root=0,
                           all_out=all_out, all_mag=all_mag, chunk=chunk)
    torch.cuda.synchronize()
    assert torch.equal(all_out, ref_out)
    assert torch.equal(all_mag, ref_mag)


def test_rccl_gather_one_rank(torch_cuda):
    torch = torch_cuda
    comm = sh.RcclComm(sh.RcclComm.unique_id(), 1, 0, torch.cuda.current_device())
    src = torch.arange(10_000, dtype=torch.float32, device="cuda")
    dst = torch.zeros_like(src)
    comm.gather(src, [dst], root=0, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rehearsal_worker(rank, world, port, q):
    """One rank of the N > 1 cfg 5 path on cuda:0: the product's plan, its GPU
    render + fused STFT per chunk, the gather over gloo."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        C_total, L, B = 4, 8192 * 12 + 999, 512
        g = torch.Generator(device="cuda").manual_seed(11)
        x = torch.rand((C_total, L), device="cuda", generator=g) * 2 - 1
        plugin = d.Plugin.ir_test(0.9, 0.002)
        s = sh.plan(L, world, rank, B, 8192, 4096, True, C_total, sh.CHANNELS)
        nb = -(-L // B)
        xl = x[s.chan0:s.chan0 + s.channels].contiguous()
        out = torch.empty((s.channels, nb * B), device="cuda")
        mag = torch.empty((s.channels, s.frames, 4097), device="cuda")
        all_out = torch.zeros((C_total, nb * B), device="cuda") if rank == 0 else None
        all_mag = torch.zeros((C_total, s.frames, 4097), device="cuda") if rank == 0 else None
        sh.render_stft_sharded(xl, L, C_total, B, 96000.0, plugin, s, out, mag, comm=sh.TorchComm(), root=0,
                               all_out=all_out, all_mag=all_mag, chunk=1 << 15)
        if rank == 0:
            torch.cuda.synchronize()
            ref_out, ref_mag = d.render_stft(x, C_total, B, 96000.0, plugin, window=d.DSP_WIN_HANN)
            torch.cuda.synchronize()
            q.put((bool(torch.equal(all_out, ref_out)), bool(torch.equal(all_mag, ref_mag))))
    finally:
        dist.destroy_process_group()


def test_two_rank_rehearsal_on_one_gpu(torch_cuda):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rehearsal_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok_r, ok_m = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok_r and ok_m
