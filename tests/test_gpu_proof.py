"""GENERIC plugins whose fast path the callback's IR decides (module.h
dsp_callback_facts, csrc/ir_proof.cpp), rendered on the GPU and compared bit
for bit with the plugin's semantics computed here in numpy (each test plugin
is a few lines: tests/plugins/).  The reference calls the callback on every
block, in order (audio.cpp:160-165), so whatever path the library takes --
a block class, parallel blocks, or the blocks in order on one lane -- the
render must equal that.

The plugins are the cases round 3's probes could not tell from a gain or a
table: a clip beyond the probes' range, an exact-value branch, a branch on a
sample, a function-local static counter; plus a per-position gain, per-channel
gains, a gain applied twice, a State that is only read, a constant level.
"""
import os
import struct

import numpy as np
import pytest

import dspbench as d

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PLUG = os.path.join(HERE, "plugins")
PEAK_REL_TOL = 1e-6
F = np.float32


def load(name):
    with open(os.path.join(PLUG, name + ".cpp")) as f:
        src = f.read()
    return d.module.Module(d.module.compile_source(src, name + ".cpp"))


def blocks(x, C, B):
    """render_audio's input to each callback: the file in blocks of B, zero
    past EOF and for the channels the file lacks (audio.cpp:13-175)."""
    cin, L = x.shape
    nb = -(-L // B)
    buf = np.zeros((C, nb * B), F)
    buf[:min(cin, C), :L] = x[:C]
    return buf.reshape(C, nb, B)


def semantics(name, xb, params, state=None, call0=0):
    """The plugin's callback applied to every block, in numpy float32 (the
    operations in the order the source writes them)."""
    g = F(struct.unpack("<f", params[:4])[0])
    C, nb, B = xb.shape
    y = xb.copy()
    if name == "clip_beyond_2000":
        y = np.where(np.abs(xb) > F(2000), F(0), xb * g).astype(F)
    elif name == "exact_value_branch":
        y = np.where(xb == F(0.25), F(7), xb * g).astype(F)
    elif name == "gain_until_loud":
        for c in range(C):
            for k in range(nb):
                row = xb[c, k]
                loud = np.nonzero(row > F(5000))[0]
                stop = loud[0] if loud.size else B
                y[c, k, :stop] = row[:stop] * g
    elif name == "static_counter":
        for k in range(nb):
            calls = call0 + k + 1
            gk = F(g * (F(1) if calls % 2 else F(0.5)))
            y[:, k] = xb[:, k] * gk
    elif name == "fade_in":
        s = np.arange(B, dtype=F)
        gs = (g * s).astype(F) / F(B)
        y = (xb * gs.astype(F)).astype(F)
    elif name == "balance":
        left, right = struct.unpack("<ff", params[:8])
        y[0] = xb[0] * F(left)
        if C > 1:
            y[1] = xb[1] * F(right)
    elif name == "gain_twice":
        y = ((xb * g).astype(F) * g).astype(F)
    elif name == "half_block":
        y[:, :, : B // 2] = (xb[:, :, : B // 2] * g).astype(F)
    elif name == "state_shaper":
        a, b = F(-g / F(3)), F(F(1) + g)
        t = ((a * xb).astype(F) * xb).astype(F) * xb
        y = (t.astype(F) + (b * xb).astype(F)).astype(F)
    elif name == "dc_level":
        y[:] = g
    return y.reshape(C, -1)


# name -> (block class at the defaults, blocks in parallel)
EXPECT = {
    "clip_beyond_2000": ("callback", True),
    "exact_value_branch": ("callback", True),
    "gain_until_loud": ("callback", True),
    "static_counter": ("callback", False),
    "fade_in": ("gain_table", True),      # x * G[position] (round 5: the gain-table class)
    "balance": ("gain_table", True),      # x * G[channel]
    "gain_twice": ("callback", True),
    "half_block": ("gain_table", True),   # x * g on half the block, x elsewhere
    "state_shaper": ("callback", True),
    "dc_level": ("table", True),
}


def make_input(L, C=2, seed=0):
    """Noise over +-3000 with exact 0.25 values and samples above 5000."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-3000, 3000, (C, L)).astype(F)
    x[:, ::97] = F(0.25)
    x[:, 5::1013] = F(6000)
    x[:, 7::211] = F(-2500)
    return x


@pytest.mark.parametrize("name", sorted(EXPECT))
@pytest.mark.parametrize("C,B,L", [(2, 512, 512 * 37 + 101), (1, 480, 480 * 20), (3, 256, 9_999)])
def test_render_equals_the_callback_on_every_block(torch_cuda, name, C, B, L):
    torch = torch_cuda
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, C, 48000.0)
    cls, _ = mod.block_class(params, C, B, 48000.0)
    want_cls, want_par = EXPECT[name]
    assert cls == want_cls, (name, cls, mod.facts)
    assert mod.stateless == want_par, mod.facts
    x = make_input(L, min(C, 2), seed=B)
    want = semantics(name, blocks(x, C, B), params)
    got = d.render_offline(torch.from_numpy(x).cuda(), C, B, 48000.0, mod.plugin(params, name)).cpu().numpy()
    assert np.array_equal(got, want), name


def test_static_counter_runs_in_order_across_calls(torch_cuda):
    """The counter lives outside State: blocks run in order, and a second
    render continues the count where the first stopped (the JIT's static
    persists in the reference too)."""
    torch = torch_cuda
    mod = load("static_counter")
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    assert not mod.stateless and not mod.facts["analyzed"]
    B, L = 512, 512 * 11
    x = make_input(L)
    xg = torch.from_numpy(x).cuda()
    nb = L // B
    a = d.render_offline(xg, 2, B, 48000.0, mod.plugin(params, "static_counter")).cpu().numpy()
    b = d.render_offline(xg, 2, B, 48000.0, mod.plugin(params, "static_counter")).cpu().numpy()
    assert np.array_equal(a, semantics("static_counter", blocks(x, 2, B), params, call0=0))
    assert np.array_equal(b, semantics("static_counter", blocks(x, 2, B), params, call0=nb))


@pytest.mark.parametrize("name", ["clip_beyond_2000", "state_shaper", "dc_level", "gain_until_loud", "balance",
                                  "fade_in", "half_block"])
def test_render_stft_of_proof_plugins(torch_cuda, oracle, name):
    """render + STFT through the same dispatch: the render bit for bit, the
    spectra within 1e-6 of the peak of float64."""
    torch = torch_cuda
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    B, L = 512, 8192 * 6 + 333
    x = make_input(L, seed=3)
    want = semantics(name, blocks(x, 2, B), params)
    out, mag = d.render_stft(torch.from_numpy(x).cuda(), 2, B, 48000.0, mod.plugin(params, name),
                             window=d.DSP_WIN_HANN)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    m64 = oracle.np_stft_mag(want[0], 8192, 4096, d.DSP_WIN_HANN, 4097)
    mm = mag[0].cpu().numpy().astype(np.float64)
    peak = np.maximum(m64.max(axis=1), 1e-30)
    assert float(np.max(np.abs(mm - m64).max(axis=1) / peak)) <= PEAK_REL_TOL


def test_gain_twice_is_a_gain_only_when_g_squared_is_g(torch_cuda):
    """Every store of gain_twice.cpp is x * g at x's address (the IR's gain
    form); the probe of ones sees g^2: the class is refused for g = 0.5 and
    taken for g = 1 and g = 0, where x g g = x g for every x."""
    torch = torch_cuda
    mod = load("gain_twice")
    mod.initialize_state(mod.default_parameters(), 2, 48000.0)
    assert mod.facts["gain_form"]
    x = torch.from_numpy(make_input(512 * 9)).cuda()
    for g, cls in ((0.5, "callback"), (1.0, "gain"), (0.0, "gain")):
        params = struct.pack("<f", g)
        assert mod.block_class(params, 2, 512, 48000.0)[0] == cls, g
        got = d.render_offline(x, 2, 512, 48000.0, mod.plugin(params, "gain_twice")).cpu().numpy()
        assert np.array_equal(got, semantics("gain_twice", blocks(x.cpu().numpy(), 2, 512), params))


def test_half_block_gain_is_refused_unless_it_is_the_identity(torch_cuda):
    """half_block.cpp stores x * g (the IR's gain form) on the first half of
    each block only: the probe of ones sees 1 in the second half, so the gain
    class is refused for g = 0.5 and g = 0 and taken for g = 1, where the
    callback is the identity.  Each element is stored at most once (the IR's
    loops), so g = 0.5 and 0 take the gain-table class: G = g on the first
    half, 1 on the second (round 5) -- the same rows either way."""
    torch = torch_cuda
    mod = load("half_block")
    mod.initialize_state(mod.default_parameters(), 2, 48000.0)
    assert mod.facts["gain_form"]
    x = torch.from_numpy(make_input(512 * 9 + 5)).cuda()
    for g, cls in ((0.5, "gain_table"), (0.0, "gain_table"), (1.0, "gain")):
        params = struct.pack("<f", g)
        assert mod.block_class(params, 2, 512, 48000.0)[0] == cls, g
        got = d.render_offline(x, 2, 512, 48000.0, mod.plugin(params, "half_block")).cpu().numpy()
        assert np.array_equal(got, semantics("half_block", blocks(x.cpu().numpy(), 2, 512), params)), g


def test_subnormals_are_kept_as_on_the_audio_thread(torch_cuda):
    """The reference's audio thread computes with IEEE subnormals: FTZ/DAZ are
    set by ipp_initialize on the thread that calls it, the main thread
    (dsp.cpp:141-142, main.cpp:235,247), not on the WASAPI thread that runs the
    callback.  Every GPU kernel keeps f32 subnormals (.amdhsa_float_denorm_mode_32
    3), so gain_test.cpp as its gain class and with its callback on every block
    render the same bits, the exact products: subnormal x = k 2^-149 (k even)
    times 0.5 is (k/2) 2^-149, times 2^20 is the normal k 2^-129."""
    mods = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_gain_test.co")):
        pytest.skip("modules not built")
    torch = torch_cuda
    with open(os.path.join(mods, "mod_gain_test.co"), "rb") as f:
        mod = d.module.Module(f.read())
    mod.initialize_state(mod.default_parameters(), 2, 48000.0)
    rng = np.random.default_rng(11)
    n = 512 * 8
    # (k >= 16: the x 2^20 products are normal, so building the expected
    # values on the host needs no subnormal arithmetic)
    k = (rng.integers(8, 1 << 22, (2, n), dtype=np.uint32) * 2).astype(np.uint32)
    sign = (rng.integers(0, 2, (2, n), dtype=np.uint32) << 31).astype(np.uint32)
    xg = torch.from_numpy((k | sign).view(np.float32).copy()).cuda()
    for g in (0.5, 2.0 ** 20):
        params = struct.pack("<f", g)
        assert mod.block_class(params, 2, 512, 48000.0)[0] == "gain"
        a = d.render_offline(xg, 2, 512, 48000.0, mod.plugin(params, "gain_test")).cpu().numpy()
        b = d.render_offline(xg, 2, 512, 48000.0, mod.plugin(params, "gain_test", specialize=False)).cpu().numpy()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), g
        if g == 0.5:  # (k / 2) 2^-149, sign kept: exact
            assert np.array_equal(a.view(np.uint32), (k >> 1) | sign)
        else:  # k 2^-129
            want = (np.ldexp(k.astype(np.float64), -129) * np.where(sign != 0, -1.0, 1.0)).astype(np.float32)
            assert np.array_equal(a.view(np.uint32), want.view(np.uint32))


def test_static_gain_plugin_is_a_proven_gain(torch_cuda, oracle):
    """test/static_gain_plugin.cpp (State {gain} set by initialize_state, only
    read by the callback): parallel blocks, the gain class with g = state.gain
    = 0.1f, bit-exact against the reference plugin compiled for the CPU; a new
    initialize_state forgets the class it found."""
    mods = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_static_gain_plugin.co")):
        pytest.skip("modules not built")
    torch = torch_cuda
    with open(os.path.join(mods, "mod_static_gain_plugin.co"), "rb") as f:
        mod = d.module.Module(f.read())
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    assert mod.stateless and mod.facts["gain_form"] and not mod.facts["writes_state"]
    cls, g = mod.block_class(params, 2, 512, 48000.0)
    assert cls == "gain" and g == F(0.1)
    x = np.random.default_rng(4).uniform(-1, 1, (2, 512 * 50 + 7)).astype(F)
    got = d.render_offline(torch.from_numpy(x).cuda(), 2, 512, 48000.0, mod.plugin(params, "static_gain")).cpu()
    ref = oracle.RefPlugin("static_gain_plugin", 2, 48000.0)
    want = oracle.render_offline([x[0], x[1]], 2, 512, 48000.0, ref.as_oracle())
    assert np.array_equal(got.numpy(), want)


def test_evicted_table_outlives_a_captured_graph(torch_cuda):
    """A table-class render captured into a graph keeps its table: four more
    Parameters sets push its entry out of the module's class cache, and the
    replay still renders the first level (module.cpp: evicted tables are
    freed only by dsp_module_destroy)."""
    torch = torch_cuda
    mod = load("dc_level")
    p0 = struct.pack("<f", 0.125)
    mod.initialize_state(p0, 2, 48000.0)
    assert mod.block_class(p0, 2, 512, 48000.0)[0] == "table"
    x = torch.zeros((2, 512 * 8), device="cuda")
    plug = mod.plugin(p0, "dc_level")
    out = torch.empty((2, 512 * 8), device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        d.render_offline(x, 2, 512, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        d.render_offline(x, 2, 512, 48000.0, plug, out=out)
    for v in (0.25, 0.5, -0.75, 0.875, 0.0625):
        p = struct.pack("<f", v)
        assert mod.block_class(p, 2, 512, 48000.0)[0] == "table"
        y = d.render_offline(x, 2, 512, 48000.0, mod.plugin(p, "dc_level"))
        assert bool((y == v).all())
    out.fill_(-1.0)
    g.replay()
    torch.cuda.synchronize()
    assert bool((out == 0.125).all())


def test_evicted_tables_are_freed_after_their_last_use(torch_cuda):
    """A Parameters sweep over a TABLE-class plugin, ten times more sets than
    the class cache keeps: every evicted table is freed once the calls that
    read it have passed (an event per call and stream), so the module's
    device memory stays flat; only a table a captured graph used is kept
    (test_evicted_table_outlives_a_captured_graph)."""
    torch = torch_cuda
    mod = load("dc_level")
    p0 = struct.pack("<f", 0.5)
    mod.initialize_state(p0, 2, 48000.0)
    x = torch.zeros((2, 512 * 4), device="cuda")
    most = 0
    for i in range(40):
        v = 0.01 * (i + 1)
        p = struct.pack("<f", v)
        y = d.render_offline(x, 2, 512, 48000.0, mod.plugin(p, "dc_level"))
        assert bool((y == torch.tensor(v, dtype=torch.float32)).all())
        most = max(most, mod.retired_tables())
    torch.cuda.synchronize()
    assert mod.retired_tables() == 0
    assert most <= 8, most


def test_verify_class_reports_and_catches_a_wrong_class(torch_cuda):
    """DSP_EXEC_VERIFY_CLASS, the second line of defence: a proven class is
    checked against the callback on four blocks of the call's own input
    (VERIFIED); a class taken on tampered facts -- gain_until_loud.cpp's code
    object edited to claim the gain form -- renders wrong rows, the check sees
    them, and the call is rendered again with the callback (RERENDERED): the
    result equals the plugin's semantics either way."""
    torch = torch_cuda
    import dspbench._lib as L
    from dspbench.api import last_result
    mods = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_gain_test.co")):
        pytest.skip("modules not built")
    with open(os.path.join(mods, "mod_gain_test.co"), "rb") as f:
        gmod = d.module.Module(f.read())
    gp = gmod.default_parameters()
    gmod.initialize_state(gp, 2, 48000.0)
    x = torch.rand((2, 512 * 40 + 7), device="cuda") * 2 - 1
    d.render_offline(x, 2, 512, 48000.0, gmod.plugin(gp, "gain_test", verify=True))
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_VERIFIED
    d.render_stft(x, 2, 512, 48000.0, gmod.plugin(gp, "gain_test", verify=True), window=d.DSP_WIN_HANN)
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_VERIFIED
    d.render_offline(x, 2, 512, 48000.0, gmod.plugin(gp, "gain_test"))
    assert last_result() == L.DSP_RESULT_CLASS  # not checked without the flag
    # in place (out = the input rows): the check would need the input after
    # the render, so a verified call runs the callback on every block
    xi = torch.rand((2, 512 * 12), device="cuda") * 2 - 1
    want_i = (xi * torch.tensor(struct.unpack("<f", gp[:4])[0], dtype=torch.float32)).cpu().numpy()
    d.render_offline(xi, 2, 512, 48000.0, gmod.plugin(gp, "gain_test", verify=True), out=xi)
    assert last_result() == 0
    assert np.array_equal(xi.cpu().numpy(), want_i)

    src = open(os.path.join(PLUG, "gain_until_loud.cpp")).read()
    code = d.module.compile_source(src, "gain_until_loud.cpp")
    assert b"gain_form=0" in code and b"input_control=1" in code and b"gain_src=P" in code
    bad = code.replace(b"gain_form=0", b"gain_form=1").replace(b"input_control=1", b"input_control=0")
    mod = d.module.Module(bad)
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    assert mod.block_class(params, 2, 512, 48000.0)[0] == "gain"  # the probes stay below 5000
    B, L_ = 512, 512 * 30
    xs = make_input(L_, seed=8)
    xs[:, ::300] = F(9000)  # every block has a sample above 5000
    want = semantics("gain_until_loud", blocks(xs, 2, B), params)
    xg = torch.from_numpy(xs).cuda()
    wrong = d.render_offline(xg, 2, B, 48000.0, mod.plugin(params, "gul")).cpu().numpy()
    assert not np.array_equal(wrong, want)  # the tampered class renders wrong rows
    got = d.render_offline(xg, 2, B, 48000.0, mod.plugin(params, "gul", verify=True)).cpu().numpy()
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_RERENDERED
    assert np.array_equal(got, want)
    out, mag = d.render_stft(xg, 2, B, 48000.0, mod.plugin(params, "gul", verify=True), window=d.DSP_WIN_HANN)
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_RERENDERED
    assert np.array_equal(out.cpu().numpy(), want)


def test_verify_class_result_through_every_driver(torch_cuda):
    """DSP_EXEC_VERIFY_CLASS reported by the chunked driver (the
    chunks' bits OR-ed into the caller's result) and by loop mode (which then
    runs the callback on every block: result 0, the plugin's rows)."""
    torch = torch_cuda
    import dspbench._lib as L
    from dspbench.api import last_result
    mods = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
    if not os.path.exists(os.path.join(mods, "mod_gain_test.co")):
        pytest.skip("modules not built")
    with open(os.path.join(mods, "mod_gain_test.co"), "rb") as f:
        gmod = d.module.Module(f.read())
    gp = gmod.default_parameters()
    gmod.initialize_state(gp, 2, 48000.0)
    g = np.float32(struct.unpack("<f", gp[:4])[0])
    xh = np.random.default_rng(4).uniform(-1, 1, (2, 512 * 300 + 11)).astype(np.float32)
    out, _ = d.render_stft_host(xh, 2, 512, 48000.0, gmod.plugin(gp, "gain_test", verify=True), stft=True,
                                chunk=1 << 16)
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_VERIFIED
    assert np.array_equal(out[:, :xh.shape[1]], xh * g)
    x = torch.from_numpy(xh[:, :5000]).cuda()
    y, _ = d.render_loop(x, 2, 512, 30, 48000.0, gmod.plugin(gp, "gain_test", verify=True), cursor=100)
    assert last_result() == 0
    y2, _ = d.render_loop(x, 2, 512, 30, 48000.0, gmod.plugin(gp, "gain_test"), cursor=100)
    assert last_result() == L.DSP_RESULT_CLASS
    assert torch.equal(y, y2)


@pytest.mark.parametrize("name", ["balance", "fade_in", "half_block"])
@pytest.mark.parametrize("B", [512, 384, 2048, 128])
def test_gain_table_class_in_every_path(torch_cuda, oracle, name, B):
    """The gain-table class (round 5): per-(channel, position) gains proven
    from the IR (each element stored at most once, x G at x's address, G free
    of samples) and pinned by the probe of ones.  The fused render + STFT,
    the two-pass path (an odd sample offset), loop mode and VERIFY_CLASS all
    render the callback's rows bit for bit; the spectra are within 1e-6 of
    the peak of float64."""
    torch = torch_cuda
    import dspbench._lib as L
    from dspbench.api import last_result
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    assert mod.facts["gain_table_form"], mod.facts
    L_ = 8192 * 9 + 700
    x = make_input(L_, seed=21)
    want = semantics(name, blocks(x, 2, B), params)
    xg = torch.from_numpy(x).cuda()
    out, mag = d.render_stft(xg, 2, B, 48000.0, mod.plugin(params, name, verify=True), window=d.DSP_WIN_HANN)
    assert last_result() == L.DSP_RESULT_CLASS | L.DSP_RESULT_VERIFIED
    assert np.array_equal(out.cpu().numpy(), want)
    for c in range(2):
        m64 = oracle.np_stft_mag(want[c], 8192, 4096, d.DSP_WIN_HANN, 4097)
        mm = mag[c].cpu().numpy().astype(np.float64)
        peak = np.maximum(m64.max(axis=1), 1e-30)
        assert float(np.max(np.abs(mm - m64).max(axis=1) / peak)) <= PEAK_REL_TOL
    # a channel the file lacks, three channels (balance: C > 1 scales channel 1 only)
    x1 = make_input(L_, C=1, seed=22)
    got3 = d.render_offline(torch.from_numpy(x1).cuda(), 3, B, 48000.0, mod.plugin(params, name)).cpu().numpy()
    assert np.array_equal(got3, semantics(name, blocks(x1, 3, B), params))
    # loop mode: the wrap kernels with the same gains
    y, _ = d.render_loop(xg, 2, B, 40, 48000.0, mod.plugin(params, name), cursor=333)
    assert last_result() == L.DSP_RESULT_CLASS
    y2, _ = d.render_loop(xg, 2, B, 40, 48000.0, mod.plugin(params, name, specialize=False), cursor=333)
    assert torch.equal(y, y2)
