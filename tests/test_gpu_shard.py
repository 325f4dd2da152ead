"""cfg 5 (BASELINE configs[4]: 8-channel 96 kHz render through IR_test + 8192-pt
FFT, one channel per GPU, RCCL gather) through the product's shard path on
one GPU: the per-GPU unit (C = 1, 96 kHz, IR_test + fused STFT) against the
oracle, the pipelined C++ driver (dsp_render_stft_sharded) with an RCCL
communicator of one rank, the same driver at world 2 and 4 with the ranks as
threads on one GPU (the in-process loopback transport: the C++ chunk and
gather schedule, every rank's pieces), and a two-process rehearsal with gloo
as the transport; each must reassemble the whole-file result bit for bit.
The 8-GPU run itself is the driver's.
"""
import threading

import numpy as np
import pytest

import dspbench as d
import dspbench.shard as sh
import rankrun

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


def _run_ranks(torch, world, fn):
    """fn(rank) on `world` host threads at once; re-raise the first failure."""
    errs = [None] * world

    def body(r):
        try:
            torch.cuda.set_device(0)
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
    # daemon threads: a rank stuck in a GPU call cannot hold the interpreter
    # at exit after the assertion below has failed the test
    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
        assert not t.is_alive(), "a rank thread hung"
    for e in errs:
        if e is not None:
            raise e


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode,C_total,C_file,chunk,root", [
    (sh.CHANNELS, 8, 6, 1 << 16, 0),   # cfg 5 in small: 8 device channels, a 6-channel file
    (sh.CHANNELS, 8, 8, 0, 1),         # one chunk per rank, root 1
    (sh.TIME, 2, 2, 3 * 4096, 0),      # time shards with halos, chunked inside each rank
])
def test_loopback_sharded_driver_equals_whole_file(torch_cuda, world, mode, C_total, C_file, chunk, root):
    """dsp_render_stft_sharded at world 2 / 4 over the loopback transport:
    every rank a host thread with its own stream, its own file rows and
    render / magnitude rows; the root's gathered rows equal dsp_render_stft
    of the whole file bit for bit (the reference's per-channel rule for the
    channels the file lacks, audio.cpp:65-81,138-141)."""
    torch = torch_cuda
    L, B, K = 8192 * 14 + 2345, 512, 4097
    g = torch.Generator(device="cuda").manual_seed(5 + world)
    # rows 8-byte aligned (an even row stride), so the whole-file call and
    # every rank take the fused kernel: the two-pass path (render, then the
    # memory STFT) that misaligned rows take agrees with it to ~1e-8 of the
    # peak, not bit for bit
    x = (torch.rand((C_file, L + 1), device="cuda", generator=g) * 2 - 1)[:, :L]
    plugin = d.Plugin.ir_test(0.8, 0.001) if mode == sh.CHANNELS else d.Plugin.gain_test(0.3)
    ref_out, ref_mag = _whole(torch, x, C_total, B, plugin, L)
    nb = -(-L // B)
    F = ref_mag.shape[1]
    all_out = torch.full((C_total, nb * B), -7.0, device="cuda")
    all_mag = torch.full((C_total, F, K), -7.0, device="cuda")
    comms = sh.loopback(world, 0)
    assert [c.rank for c in comms] == list(range(world)) and all(c.world == world for c in comms)

    def rank_fn(r):
        s = sh.plan(L, world, r, B, 8192, 4096, True, C_total, mode)
        nf = max(0, min(s.chan0 + s.channels, C_file) - s.chan0)  # the file rows this rank reads
        xl = x[s.chan0:s.chan0 + nf, s.start:s.start + s.read_len] if nf else None  # views: no copy
        out = torch.empty((max(s.channels, 1), -(-s.read_len // B) * B), device="cuda")
        mag = torch.empty((max(s.channels, 1), max(s.frames, 1), K), device="cuda")
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            sh.render_stft_sharded(xl, L, C_total, B, 96000.0, plugin, s, out, mag, comm=comms[r], root=root,
                                   all_out=all_out if r == root else None, all_mag=all_mag if r == root else None,
                                   chunk=chunk, stream=st.cuda_stream)
        st.synchronize()
    _run_ranks(torch, world, rank_fn)
    torch.cuda.synchronize()
    for c in comms:
        c.close()
    assert torch.equal(all_out, ref_out), _where(torch, all_out, ref_out)
    assert torch.equal(all_mag, ref_mag), _where(torch, all_mag, ref_mag)


def _where(torch, got, ref):
    """Which channels / rows differ, by how much, and whether unwritten (-7)."""
    bad = (got != ref).reshape(got.shape[0], got.shape[1], -1).any(dim=-1)
    lines = []
    for c in range(got.shape[0]):
        rows = torch.nonzero(bad[c]).flatten().tolist()
        if rows:
            d = (got[c] - ref[c]).abs().max().item()
            unwritten = bool((got[c][rows[0]] == -7.0).any().item())
            lines.append(f"ch {c}: {len(rows)} rows differ, first {rows[:6]}, max |diff| {d:.3g}, "
                         f"unwritten {unwritten}")
    return "; ".join(lines)


@pytest.mark.parametrize("spec", [True, False])
def test_time_shards_of_a_stateless_source_plugin(torch_cuda, spec):
    """IR_test.cpp compiled from source, time-sharded over two loopback ranks
    with chunks inside each rank (its block class, or its callback on every
    block): the root's rows equal the whole-file call bit for bit.  A plugin
    with a State (sine_test.cpp) is refused for time shards at world > 1."""
    import os
    torch = torch_cuda
    mods = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_IR_test.co")):
        pytest.skip("modules not built")
    mod = d.module.Module(open(os.path.join(mods, "mod_IR_test.co"), "rb").read())
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    plugin = mod.plugin(params, "IR_test", specialize=spec)
    L, B, K, world = 8192 * 12 + 999, 512, 4097, 2
    x = (torch.rand((2, L + 1), device="cuda") * 2 - 1)[:, :L]
    ref_out, ref_mag = _whole(torch, x, 2, B, plugin, L)
    all_out = torch.full_like(ref_out, -7.0)
    all_mag = torch.full_like(ref_mag, -7.0)
    comms = sh.loopback(world, 0)

    def rank_fn(r):
        s = sh.plan(L, world, r, B, 8192, 4096, True, 2, sh.TIME)
        out = torch.empty((2, -(-s.read_len // B) * B), device="cuda")
        mag = torch.empty((2, max(s.frames, 1), K), device="cuda")
        st = torch.cuda.Stream()
        sh.render_stft_sharded(x[:, s.start:s.start + s.read_len], L, 2, B, 96000.0, plugin, s, out, mag,
                               comm=comms[r], root=0, all_out=all_out if r == 0 else None,
                               all_mag=all_mag if r == 0 else None, chunk=3 * 4096, stream=st.cuda_stream)
        st.synchronize()
    _run_ranks(torch, world, rank_fn)
    for c in comms:
        c.close()
    assert torch.equal(all_out, ref_out), _where(torch, all_out, ref_out)
    assert torch.equal(all_mag, ref_mag), _where(torch, all_mag, ref_mag)
    smod = d.module.Module(open(os.path.join(mods, "mod_sine_test.co"), "rb").read())
    sp = smod.default_parameters()
    smod.initialize_state(sp, 2, 48000.0)
    s0 = sh.plan(L, world, 0, B, 8192, 4096, True, 2, sh.TIME)
    with pytest.raises(d.DspError, match="writes its State.*shard it by channel"):
        sh.render_stft_sharded(x[:, :s0.read_len], L, 2, B, 96000.0, smod.plugin(sp, "sine_test"), s0,
                               torch.empty((2, -(-s0.read_len // B) * B), device="cuda"),
                               torch.empty((2, s0.frames, K), device="cuda"), comm=None, gather=False)


@pytest.mark.parametrize("kind", ["biquad_src", "biquad", "fir"])
def test_time_shards_refuse_a_state_through_the_file(torch_cuda, kind):
    """A plugin whose state runs through the whole file -- plugins/biquad.cpp
    compiled unchanged (its callback writes its State), DSP_PLUGIN_BIQUAD,
    DSP_PLUGIN_FIR -- asked for time shards at world > 1: refused with an
    error that names the reason and the channel shards; the same plugin
    channel-sharded renders."""
    import os
    torch = torch_cuda
    L, B, K, world = 8192 * 6 + 5, 512, 4097, 2
    x = (torch.rand((2, L + 1), device="cuda") * 2 - 1)[:, :L]
    if kind == "biquad_src":
        src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dsp-bench_amd", "plugins",
                           "biquad.cpp")
        mod = d.module.Module(d.module.compile_source(open(src).read(), "biquad.cpp"))
        p = mod.default_parameters()
        mod.initialize_state(p, 2, 48000.0)
        plugin = mod.plugin(p, "biquad")
    elif kind == "biquad":
        plugin = d.Plugin.biquad(np.array([d.Plugin.biquad_lowpass_coefficients(1000.0, 0.7071, 48000.0)],
                                          np.float32))
    else:
        plugin = d.Plugin.fir(np.hanning(64).astype(np.float32))
    s0 = sh.plan(L, world, 0, B, 8192, 4096, True, 2, sh.TIME)
    with pytest.raises(d.DspError, match="shard it by channel"):
        sh.render_stft_sharded(x[:, :s0.read_len], L, 2, B, 96000.0, plugin, s0,
                               torch.empty((2, -(-s0.read_len // B) * B), device="cuda"),
                               torch.empty((2, s0.frames, K), device="cuda"), comm=None, gather=False)
    reset = (lambda: mod.initialize_state(p, 2, 48000.0)) if kind == "biquad_src" else (lambda: None)
    c0 = sh.plan(L, world, 0, B, 8192, 4096, True, 2, sh.CHANNELS)
    reset()
    out = torch.empty((c0.channels, -(-c0.read_len // B) * B), device="cuda")
    mag = torch.empty((c0.channels, c0.frames, K), device="cuda")
    sh.render_stft_sharded(x[c0.chan0:c0.chan0 + c0.channels], L, 2, B, 96000.0, plugin, c0, out, mag,
                           comm=None, gather=False)
    torch.cuda.synchronize()
    reset()  # (a State-writing module: the reference render starts from the same State)
    ref_out, ref_mag = _whole(torch, x[c0.chan0:c0.chan0 + c0.channels].contiguous(), c0.channels, B, plugin, L)
    assert torch.equal(out, ref_out)


@pytest.mark.parametrize("world,root,L", [(4, 3, 8192 * 10 + 4321), (8, 0, 96000 * 60 + 123)])
def test_channel_shards_of_the_source_headline_plugin(torch_cuda, world, root, L):
    """cfg 5's shape with the bench's headline plugin (IR_test.cpp compiled
    unchanged, its block in the verified closed form): 8 device channels from
    a 6-channel file, channel-sharded over 4 loopback ranks gathered to root
    3, and over cfg 5's own 8 ranks (one channel each, a minute of 96 kHz per
    rank) gathered to root 0 -- equal bit for bit to the whole-file call, and
    to the enum's."""
    import os
    torch = torch_cuda
    mods = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_IR_test.co")):
        pytest.skip("modules not built")
    mod = d.module.Module(open(os.path.join(mods, "mod_IR_test.co"), "rb").read())
    params = mod.default_parameters()
    mod.initialize_state(params, 8, 96000.0)
    plugin = mod.plugin(params, "IR_test")
    B, K = 512, 4097
    x = (torch.rand((6, L + 1), device="cuda") * 2 - 1)[:, :L]
    ref_out, ref_mag = _whole(torch, x, 8, B, plugin, L)
    e_out, e_mag = _whole(torch, x, 8, B, d.Plugin.ir_test(0.9, 0.002), L)
    assert torch.equal(ref_out, e_out) and torch.equal(ref_mag, e_mag)
    all_out = torch.full_like(ref_out, -7.0)
    all_mag = torch.full_like(ref_mag, -7.0)
    comms = sh.loopback(world, 0)

    def rank_fn(r):
        s = sh.plan(L, world, r, B, 8192, 4096, True, 8, sh.CHANNELS)
        nf = max(0, min(s.chan0 + s.channels, 6) - s.chan0)
        xl = x[s.chan0:s.chan0 + nf, s.start:s.start + s.read_len] if nf else None
        out = torch.empty((max(s.channels, 1), -(-s.read_len // B) * B), device="cuda")
        mag = torch.empty((max(s.channels, 1), max(s.frames, 1), K), device="cuda")
        st = torch.cuda.Stream()
        sh.render_stft_sharded(xl, L, 8, B, 96000.0, plugin, s, out, mag, comm=comms[r], root=root,
                               all_out=all_out if r == root else None, all_mag=all_mag if r == root else None,
                               chunk=1 << 15, stream=st.cuda_stream)
        st.synchronize()
    _run_ranks(torch, world, rank_fn)
    torch.cuda.synchronize()
    for c in comms:
        c.close()
    assert torch.equal(all_out, ref_out), _where(torch, all_out, ref_out)
    assert torch.equal(all_mag, ref_mag), _where(torch, all_mag, ref_mag)


def test_loopback_gather_and_errors(torch_cuda):
    """dsp_comm_gather over the loopback (3 ranks, root 2); a count mismatch
    between a send and its recv fails both sides instead of copying."""
    torch = torch_cuda
    world, n = 3, 50_001
    comms = sh.loopback(world, 0)
    srcs = [torch.arange(n, dtype=torch.float32, device="cuda") + 1000 * r for r in range(world)]
    dst = [torch.zeros(n, device="cuda") for _ in range(world)]

    def rank_fn(r):
        st = torch.cuda.Stream()
        comms[r].gather(srcs[r], dst if r == 2 else None, root=2, stream=st.cuda_stream)
        st.synchronize()
    _run_ranks(torch, world, rank_fn)
    for r in range(world):
        assert torch.equal(dst[r], srcs[r])

    def bad_fn(r):
        st = torch.cuda.Stream()
        src = srcs[r][: n - (1 if r == 1 else 0)]
        comms[r].gather(src, dst if r == 2 else None, root=2, stream=st.cuda_stream)
    errs = []

    def wrapped(r):
        try:
            bad_fn(r)
        except d.DspError as e:
            errs.append((r, str(e)))
    _run_ranks(torch, world, wrapped)
    assert sorted(r for r, _ in errs) == [1, 2], errs
    for c in comms:
        c.close()


def _rehearsal_worker(rank, world):
    """One rank of the N > 1 cfg 5 path on cuda:0, one process per rank: the
    C++ sharded driver (plan, chunks, GPU render + fused STFT, gather
    schedule) with gloo as its transport (dsp_comm_init_transport)."""
    import torch
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
    comm = sh.TorchComm(device=0)  # gloo as the transport of the C++ driver
    sh.render_stft_sharded(xl, L, C_total, B, 96000.0, plugin, s, out, mag, comm=comm, root=0,
                           all_out=all_out, all_mag=all_mag, chunk=1 << 15)
    torch.cuda.synchronize()
    comm.close()
    if rank == 0:
        ref_out, ref_mag = d.render_stft(x, C_total, B, 96000.0, plugin, window=d.DSP_WIN_HANN)
        torch.cuda.synchronize()
        return bool(torch.equal(all_out, ref_out)), bool(torch.equal(all_mag, ref_mag))
    return None


def test_two_rank_rehearsal_on_one_gpu(torch_cuda, tmp_path):
    """Two processes on cuda:0 (FileStore rendezvous, bounded waits, daemon
    ranks reaped on any failure: tests/rankrun.py)."""
    ok_r, ok_m = rankrun.run(_rehearsal_worker, 2, tmp_path, timeout=100, init_timeout=60)
    assert ok_r and ok_m
