"""GPU parity: libdspbench (HIP, gfx950) against the CPU oracle.

Bars:
  * render (gain / static gain / IR_test / no_op, copy, padding): bit-exact
  * FFT magnitudes: per frame max|m - m_ref| <= 1e-6 * max(m_ref)  
    against the float64 restatement (oracle.np_stft_mag / oracle.c).
"""
import numpy as np
import pytest

import dspbench as d

pytestmark = pytest.mark.gpu

PEAK_REL_TOL = 1e-6  # peak-relative, per frame


def peak_rel_err(m, ref):
    m = np.asarray(m, np.float64)
    ref = np.asarray(ref, np.float64)
    assert m.shape == ref.shape, (m.shape, ref.shape)
    if ref.ndim == 1:
        ref, m = ref[None], m[None]
    peak = np.maximum(ref.max(axis=-1), 1e-30)
    return float(np.max(np.abs(m - ref).max(axis=-1) / peak))


def rnd(shape, seed):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, size=shape).astype(np.float32)


def to_dev(torch, x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


PLUGINS = {
    "gain_test": (lambda: d.Plugin.gain_test(0.2), "gain_test"),
    "static_gain_plugin": (lambda: d.Plugin.static_gain(0.1), "static_gain_plugin"),
    "IR_test": (lambda: d.Plugin.ir_test(0.9, 0.002), "IR_test"),
    "no_op": (lambda: d.Plugin.no_op(), "no_op"),
}

RENDER_SHAPES = [
    # (file channels, device channels, L, B)
    (2, 2, 50_000, 512),
    (1, 2, 48_000, 256),   # cfg1 shape: mono file, stereo device (ch1 zeroed)
    (2, 1, 10_007, 512),
    (2, 2, 12_345, 100),   # non power-of-two block, ragged tail
    (2, 2, 100, 512),      # shorter than one block
    (3, 2, 4096, 4096),    # exact multiple
    (0, 2, 1000, 128),     # no file: silence through the plugin
    (2, 2, 1_000_003, 512),  # ~245 tiles of the vector kernel, ragged last tile
]


def oracle_plugin(oracle, name):
    return oracle.restated_plugin(name)


@pytest.mark.parametrize("pname", list(PLUGINS))
@pytest.mark.parametrize("shape", RENDER_SHAPES)
def test_render_bit_exact(torch_cuda, oracle, pname, shape):
    cin, cout, L, B = shape
    x = rnd((max(cin, 1), L), 11)[:cin]
    ref = oracle.render_offline([x[c] for c in range(cin)], cout, B, 48000.0,
                                oracle_plugin(oracle, pname), L=L)
    file = to_dev(torch_cuda, x) if cin else None
    out = d.render_offline(file, cout, B, 48000.0, PLUGINS[pname][0](), L_file=L,
                           out=torch_cuda.empty((cout, d.num_blocks(L, B) * B), device="cuda"))
    got = out.cpu().numpy()
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
        f"max abs diff {np.max(np.abs(got - ref))}"


def test_render_unaligned_scalar_path(torch_cuda, oracle):
    L, B = 9_999, 256
    base = to_dev(torch_cuda, rnd((2, L + 1), 3))
    file = base[:, 1:]  # 4-byte offset: not 16-byte aligned -> scalar kernel
    assert file.data_ptr() % 16 != 0
    out = torch_cuda.empty((2, d.num_blocks(L, B) * B + 1), device="cuda")[:, 1:]
    got = d.render_offline(file, 2, B, 48000.0, d.Plugin.gain_test(0.7), out=out).cpu().numpy()
    x = base.cpu().numpy()[:, 1:]
    ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.restated_plugin("gain_test", params=[0.7]))
    assert np.array_equal(got, ref)


def test_render_matches_reference_plugin_so(torch_cuda, oracle):
    """Against the stock plugins compiled from the reference sources."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    for name, mk in [("gain_test", lambda: d.Plugin.gain_test(0.2)),
                     ("IR_test", lambda: d.Plugin.ir_test(0.9, 0.002)),
                     ("static_gain_plugin", lambda: d.Plugin.static_gain(0.1))]:
        L, B = 20_000, 512
        x = rnd((2, L), 5)
        ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.RefPlugin(name, 2, 48000.0).as_oracle())
        got = d.render_offline(to_dev(torch_cuda, x), 2, B, 48000.0, mk()).cpu().numpy()
        assert np.array_equal(got, ref), name


@pytest.mark.parametrize("window", [d.DSP_WIN_HANN, d.DSP_WIN_HAMMING])
@pytest.mark.parametrize("K", [4097, 8192, 1000])
@pytest.mark.parametrize("H", [4096, 2048, 8192, 1000])
def test_stft_8192_vs_f64(torch_cuda, oracle, window, K, H):
    L = 8192 * 3 + 1234
    x = rnd((2, L), 21)
    mag = d.stft_magnitude(to_dev(torch_cuda, x), N=8192, H=H, window=window, K=K).cpu().numpy()
    for c in range(2):
        ref = oracle.np_stft_mag(x[c], 8192, H, window, K if K <= 4097 else 8192)
        err = peak_rel_err(mag[c], ref)
        assert err <= PEAK_REL_TOL, err


@pytest.mark.parametrize("N", [16, 256, 1024, 4096])
def test_stft_generic_sizes(torch_cuda, oracle, N):
    L = N * 5 + 17
    x = rnd((1, L), 22)
    H = N // 2
    mag = d.stft_magnitude(to_dev(torch_cuda, x), N=N, H=H, window=d.DSP_WIN_HANN, K=N // 2 + 1).cpu().numpy()
    ref = oracle.np_stft_mag(x[0], N, H, d.DSP_WIN_HANN, N // 2 + 1)
    assert peak_rel_err(mag[0], ref) <= PEAK_REL_TOL


def test_stft_sine_tone_peak(torch_cuda, oracle):
    """A pure tone: peak bin, and sidelobes relative to the peak."""
    n = np.arange(8192 * 4)
    x = (0.5 * np.sin(2 * np.pi * 1000.25 / 48000 * n)).astype(np.float32)[None]
    mag = d.stft_magnitude(to_dev(torch_cuda, x), window=d.DSP_WIN_HANN).cpu().numpy()[0]
    ref = oracle.np_stft_mag(x[0], 8192, 4096, d.DSP_WIN_HANN, 4097)
    assert peak_rel_err(mag, ref) <= PEAK_REL_TOL
    assert int(np.argmax(mag[0])) == int(np.argmax(ref[0]))


@pytest.mark.parametrize("pname", ["IR_test", "gain_test", "static_gain_plugin", "no_op"])
@pytest.mark.parametrize("B", [512, 384, 1, 4096])
def test_render_stft_fused(torch_cuda, oracle, pname, B):
    L = 8192 * 6 + 777
    x = rnd((2, L), 31)
    out, mag = d.render_stft(to_dev(torch_cuda, x), 2, B, 48000.0, PLUGINS[pname][0](),
                             window=d.DSP_WIN_HANN)
    out = out.cpu().numpy()
    mag = mag.cpu().numpy()
    ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle_plugin(oracle, pname))
    assert np.array_equal(out, ref)
    for c in range(2):
        mref = oracle.np_stft_mag(ref[c], 8192, 4096, d.DSP_WIN_HANN, 4097)
        assert mag.shape[1] == mref.shape[0]
        assert peak_rel_err(mag[c], mref) <= PEAK_REL_TOL


def test_render_stft_shards_match_whole(torch_cuda):
    """Time-chunk sharding with a halo: each shard's frames and
    render equal the corresponding slice of the unsharded result."""
    torch = torch_cuda
    B, N, H = 512, 8192, 4096
    L = 4096 * 40
    x = to_dev(torch, rnd((2, L), 41))
    out_all, mag_all = d.render_stft(x, 2, B, 48000.0, d.Plugin.ir_test(), N=N, H=H)
    chunk = 4096 * 10
    for s0 in range(0, L - chunk + 1, chunk):
        Lc = min(chunk + (N - H), L - s0)
        xs = x[:, s0:s0 + Lc]
        out_s, mag_s = d.render_stft(xs.contiguous(), 2, B, 48000.0, d.Plugin.ir_test(), N=N, H=H,
                                     sample_offset=s0)
        f0 = s0 // H
        nf = mag_s.shape[1]
        assert torch.equal(out_s[:, :chunk], out_all[:, s0:s0 + chunk])
        assert torch.equal(mag_s, mag_all[:, f0:f0 + nf])


def test_ir_analysis_gain_flat(torch_cuda, oracle):
    """K4: IR of gain_test(0.2) = 0.2 delta; w[0] = 0.08 -> flat 0.2*0.08/sqrt(8192)."""
    ir, mag = d.ir_analysis(d.Plugin.gain_test(0.2), 2, 48000.0)
    expect = np.zeros((2, 2048), np.float32)
    expect[:, 0] = np.float32(1.0) * np.float32(0.2)
    assert np.array_equal(ir, expect)
    flat = 0.2 * 0.08 / np.sqrt(8192)
    assert abs(flat - 1.7677669529663688e-4) < 1e-15
    assert np.max(np.abs(mag - flat)) <= 1e-6 * flat * 8


def test_ir_analysis_ir_test_kat(torch_cuda, oracle):
    """K5: IR_test(0.9, 0.002) magnitudes at bins 0, 1, 2, 4096, 8191."""
    ir, mag = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), 1, 48000.0)
    ramp = oracle.ir_ramp_reference(0.9, 0.002, 2048)
    assert np.array_equal(ir[0], ramp)
    ref = oracle.np_ir_magnitude(ramp)
    assert peak_rel_err(mag, ref) <= PEAK_REL_TOL
    kat = {0: 14.009141585190642, 1: 13.668769897308243, 2: 12.634933902307377,
           4096: 0.0018101951313910219, 8191: 13.668769897308243}
    for k, v in kat.items():
        assert abs(mag[k] - v) <= 1e-6 * 14.009141585190642, (k, mag[k], v)


@pytest.mark.parametrize("ir_len", [16, 512, 1024])
def test_ir_analysis_other_lengths(torch_cuda, oracle, ir_len):
    ir, mag = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), 1, 48000.0, ir_len=ir_len)
    ref = oracle.np_ir_magnitude(ir[0], ir_len)
    assert peak_rel_err(mag, ref) <= PEAK_REL_TOL


@pytest.mark.parametrize("n", [2, 8, 128, 2048, 8192])
def test_fft_services(torch_cuda, oracle, n):
    x = rnd((n,), 51)
    re, im = d.fft_forward(x)
    ref = np.fft.fft(x.astype(np.float64)) / np.sqrt(n)
    peak = np.max(np.abs(ref))
    assert np.max(np.abs(re - ref.real)) <= 1e-6 * peak * 4
    assert np.max(np.abs(im - ref.imag)) <= 1e-6 * peak * 4
    back = d.fft_reverse(re, im)  # both directions scale 1/sqrt(n): identity
    assert np.max(np.abs(back - x)) <= 1e-6 * 8


def test_fft_service_rejects_non_pow2(torch_cuda):
    with pytest.raises(d.DspError):
        d.fft_forward(np.zeros(1000, np.float32))


# ---------------------------------------------------------------- full sizes
def test_full_size_gain_render_10min(torch_cuda):
    """BASELINE cfg 2 at full size: gain_test on 10 min stereo 48 kHz, B=512.
    out = x * 0.2f exactly (the callback is one fp32 multiply per sample)."""
    torch = torch_cuda
    L, B = 28_800_000, 512
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.rand((2, L), device="cuda", generator=g) * 2 - 1
    out = d.render_offline(x, 2, B, 48000.0, d.Plugin.gain_test(0.2))
    assert torch.equal(out, x * torch.tensor(0.2, dtype=torch.float32, device="cuda"))


def test_full_size_ir_test_stft_1h(torch_cuda, oracle):
    """Headline workload at full size: 1 h stereo 48 kHz through IR_test +
    8192-pt Hann STFT (hop 4096).  Properties: the render is the B-periodic
    ramp everywhere; every frame of a B-periodic signal with B | H is the same
    spectrum, which matches the float64 oracle."""
    torch = torch_cuda
    L, B = 48_000 * 3600, 512
    x = torch.zeros((2, L), device="cuda")
    out, mag = d.render_stft(x, 2, B, 48000.0, d.Plugin.ir_test(), window=d.DSP_WIN_HANN)
    ramp = torch.from_numpy(oracle.ir_ramp_reference(0.9, 0.002, B)).cuda()
    assert torch.equal(out.view(2, -1, B), ramp.expand(2, L // B, B))
    F = mag.shape[1]
    assert F == (L - 8192) // 4096 + 1
    ref0 = oracle.np_stft_mag(np.tile(ramp.cpu().numpy(), 16), 8192, 4096, d.DSP_WIN_HANN, 4097)[0]
    for c in range(2):
        for f in [0, 1, F // 2, F - 1]:
            assert peak_rel_err(mag[c, f].cpu().numpy(), ref0) <= PEAK_REL_TOL
        spread = (mag[c] - mag[c, :1]).abs().max().item()
        assert spread <= 1e-6 * float(ref0.max())


@pytest.mark.parametrize("B", [2, 64, 128, 256, 1024, 2048, 4096, 8192])
def test_pk_ramp_table_periods(torch_cuda, oracle, B):
    """Packed kernel: the IR_test block table is fetched once per period of
    B / 128 columns and aliased (stft_pk.hip PER)."""
    n = 8192 * 4 + 777
    x = rnd((2, n), 62)
    out, mag = d.render_stft(to_dev(torch_cuda, x), 2, B, 48000.0, d.Plugin.ir_test(0.7, 0.001),
                             window=d.DSP_WIN_HANN, sample_offset=B * 3)
    ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.restated_plugin("IR_test", [0.7, 0.001]))
    assert np.array_equal(out.cpu().numpy(), ref)
    mref = oracle.np_stft_mag(ref[1], 8192, 4096, d.DSP_WIN_HANN, 4097)
    assert peak_rel_err(mag.cpu().numpy()[1], mref) <= PEAK_REL_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("gain,step,B", [(0.9, 0.002, 512),    # recurrence exact: closed form
                                         (0.9, 1e-10, 512),    # not exact: block table kernel
                                         (0.9, 1e-10, 4),      # exact for 4 steps
                                         (0.5, 1 / 3, 2048),
                                         (-0.25, 3e-9, 256),   # not exact
                                         (0.9, 0.002, 384)])   # non-pow2 B: table path
def test_ir_ramp_closed_form_and_table(torch_cuda, oracle, gain, step, B):
    """capi.cpp ramp_closed_form: IR_test's block table is evaluated in
    closed form only when the sequential f64 recurrence is exact; either
    way the render is bit-identical to the reference callback."""
    n = 8192 * 3 + 1000
    x = rnd((2, n), 64)
    plug = d.Plugin.ir_test(gain, step)
    ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.restated_plugin("IR_test", [gain, step]))
    out, mag = d.render_stft(to_dev(torch_cuda, x), 2, B, 48000.0, plug, window=d.DSP_WIN_HANN)
    assert np.array_equal(out.cpu().numpy(), ref)
    mref = oracle.np_stft_mag(ref[1], 8192, 4096, d.DSP_WIN_HANN, 4097)
    assert peak_rel_err(mag.cpu().numpy()[1], mref) <= PEAK_REL_TOL
    out2 = d.render_offline(to_dev(torch_cuda, x), 2, B, 48000.0, plug)
    assert np.array_equal(out2.cpu().numpy(), ref)


# ---- device elementwise services (dsp.cpp:166-181, 208-210) ---------------

def test_elementwise_services_bit_exact(torch_cuda):
    """dsp_gain / dsp_copy / dsp_set / dsp_magnitude through the C ABI, bit for
    bit against float32 numpy (gain_32_array = MulC, copy_array, set_array,
    pythagore_array = sqrt(re^2 + im^2) with rounded products and sum)."""
    import ctypes as C
    torch = torch_cuda
    L = d.lib()
    n = 1_000_003
    rng = np.random.default_rng(41)
    a = rng.uniform(-3, 3, n).astype(np.float32)
    b = rng.uniform(-3, 3, n).astype(np.float32)
    ga, gb = to_dev(torch, a), to_dev(torch, b)
    out = torch.empty(n, device="cuda")
    ex = d._lib.dsp_exec(torch.cuda.current_device(), d._lib.DSP_EXEC_SYNC,
                         C.c_void_p(torch.cuda.current_stream().cuda_stream), 0)
    fp = lambda t: C.cast(C.c_void_p(t.data_ptr()), d._lib.FP)  # noqa: E731
    assert L.dsp_gain(fp(ga), fp(out), 0.37, n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), a * np.float32(0.37))
    assert L.dsp_copy(fp(gb), fp(out), n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), b)
    assert L.dsp_set(-2.5, fp(out), n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), np.full(n, -2.5, np.float32))
    assert L.dsp_magnitude(fp(ga), fp(gb), fp(out), n, C.byref(ex)) == 0
    want = np.sqrt((a * a) + (b * b)).astype(np.float32)
    assert np.array_equal(out.cpu().numpy(), want)
    # in place (gain_ip_32_array) and n = 0
    assert L.dsp_gain(fp(ga), fp(ga), 2.0, n, C.byref(ex)) == 0
    assert np.array_equal(ga.cpu().numpy(), a * np.float32(2.0))
    assert L.dsp_set(1.0, fp(out), 0, C.byref(ex)) == 0


@pytest.mark.parametrize("n", [1, 3, 4, 5, 4095, 4096, 4097, 70_001])
@pytest.mark.parametrize("off", [0, 1])
def test_elementwise_services_shapes(torch_cuda, n, off):
    """The services' vector path (16-byte aligned rows, one float4 tile per
    block, the n % 4 tail) and scalar path (a row offset by one float), bit
    for bit against float32 numpy."""
    import ctypes as C
    torch = torch_cuda
    L = d.lib()
    rng = np.random.default_rng(n + off)
    a = rng.uniform(-3, 3, n).astype(np.float32)
    b = rng.uniform(-3, 3, n).astype(np.float32)
    ga = torch.zeros(n + 1, device="cuda")[off:off + n]
    gb = torch.zeros(n + 1, device="cuda")[off:off + n]
    ga.copy_(torch.from_numpy(a))
    gb.copy_(torch.from_numpy(b))
    base = torch.full((n + 2,), 7.0, device="cuda")
    out = base[off:off + n]
    ex = d._lib.dsp_exec(torch.cuda.current_device(), d._lib.DSP_EXEC_SYNC,
                         C.c_void_p(torch.cuda.current_stream().cuda_stream), 0)
    fp = lambda t: C.cast(C.c_void_p(t.data_ptr()), d._lib.FP)  # noqa: E731
    assert L.dsp_gain(fp(ga), fp(out), 0.37, n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), a * np.float32(0.37))
    assert L.dsp_copy(fp(gb), fp(out), n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), b)
    assert L.dsp_set(-2.5, fp(out), n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), np.full(n, -2.5, np.float32))
    assert L.dsp_magnitude(fp(ga), fp(gb), fp(out), n, C.byref(ex)) == 0
    assert np.array_equal(out.cpu().numpy(), np.sqrt((a * a) + (b * b)).astype(np.float32))
    assert float(base[off + n]) == 7.0  # nothing written past the row


def test_full_size_cfg4_stft_1h_96k_from_hbm(torch_cuda, oracle):
    """BASELINE cfg 4 at full size: the Hann 8192 / 4096 STFT of 1 h of 96 kHz
    stereo (2 x 345.6 M samples) from HBM.  Frame count, and sampled frames
    (first, last, and 12 seeded ones per channel) against float64."""
    torch = torch_cuda
    L_ = 96_000 * 3600
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand((2, L_), device="cuda", generator=g) * 0.2 - 0.1
    mag = d.stft_magnitude(x, N=8192, H=4096, window=d.DSP_WIN_HANN, K=4097)
    F = mag.shape[1]
    assert F == (L_ - 8192) // 4096 + 1 == 84_374
    rng = np.random.default_rng(5)
    for c in range(2):
        for f in [0, F - 1] + list(rng.integers(0, F, 12)):
            seg = x[c, f * 4096:f * 4096 + 8192].cpu().numpy()
            ref = oracle.np_stft_mag(seg, 8192, 4096, d.DSP_WIN_HANN, 4097)[0]
            assert peak_rel_err(mag[c, f].cpu().numpy(), ref) <= PEAK_REL_TOL, (c, f)


# ---- loop mode (audio.cpp:100-132) ------------------------------------------

@pytest.mark.parametrize("pname", list(PLUGINS))
@pytest.mark.parametrize("cin,cout,L,B,nblocks,cursor", [
    (2, 2, 10_007, 512, 60, 0),      # several wraps, ragged file
    (1, 2, 300, 512, 9, 123),        # file shorter than a block: wraps inside every block
    (2, 1, 4096, 4096, 5, 4095),     # cursor at the last sample
    (3, 2, 50_000, 384, 200, 49_000),
])
def test_render_loop_bit_exact(torch_cuda, oracle, pname, cin, cout, L, B, nblocks, cursor):
    x = rnd((cin, L), 71)
    ref, ref_cur = oracle.render_loop([x[c] for c in range(cin)], cout, B, nblocks, 48000.0,
                                      oracle_plugin(oracle, pname), cursor=cursor)
    got, cur = d.render_loop(to_dev(torch_cuda, x), cout, B, nblocks, 48000.0, PLUGINS[pname][0](), cursor=cursor)
    assert cur == ref_cur == (cursor + nblocks * B) % L
    assert np.array_equal(got.cpu().numpy(), ref)


def test_render_loop_generic_and_fir(torch_cuda, oracle):
    """Non-map plugins loop over the materialised wrapped stream: the
    reference's gain_test compiled by the module compiler (bit-exact) and the
    cfg 3b FIR (the whole wrapped stream convolved, 2e-6 of the peak)."""
    import os
    torch = torch_cuda
    L, B, nb, cursor = 7_777, 512, 40, 5_000
    x = rnd((2, L), 72)
    co = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dsp-bench_amd", "modules",
                      "mod_gain_test.co")
    if os.path.exists(co):
        mod = d.module.Module(open(co, "rb").read())
        mod.initialize_state(mod.default_parameters(), 2, 48000.0)
        ref, _ = oracle.render_loop([x[0], x[1]], 2, B, nb, 48000.0, oracle.restated_plugin("gain_test", [0.45]),
                                    cursor=cursor)
        for spec in (True, False):  # its block class (the gain map in the wrap kernel), and the callback
            p = mod.plugin_from_values({"gain": 0.45})
            if not spec:
                p.exec_flags = d._lib.DSP_EXEC_NO_SPECIALIZE
            got, _ = d.render_loop(to_dev(torch, x), 2, B, nb, 48000.0, p, cursor=cursor)
            assert np.array_equal(got.cpu().numpy(), ref), spec
    taps = rnd((1, 300), 73)[0] * 0.05
    got, _ = d.render_loop(to_dev(torch, x), 2, B, nb, 48000.0, d.Plugin.fir(taps), cursor=cursor)
    idx = (cursor + np.arange(nb * B)) % L
    for c in range(2):
        want = oracle.fir_f64(x[c][idx], taps)
        g = got[c].cpu().numpy().astype(np.float64)
        assert np.max(np.abs(g - want[: nb * B])) <= 2e-6 * np.max(np.abs(want))
