"""Block classes (module.h dsp_module_block_class): a plugin compiled
unchanged from its source whose callback provably ignores its input
(IR_test.cpp, handmade_test.cpp) or scales it (gain_test.cpp,
static_gain_plugin.cpp, no_op.cpp) -- facts from its own IR, values pinned by
probes -- runs as its own callback's block tiled / as that gain, in the fused
kernels.

Bars: the render bit-exact against the reference plugin compiled for the CPU
with the JIT flags (oracle/_ref, through the oracle's render_audio loop,
audio.cpp:13-175) and against the same plugin with the callback on every
block (DSP_EXEC_NO_SPECIALIZE); IR_test's spectra bit-exact against the stock
fused IR_test kernel with the same parameters, within 1e-6 of the peak
against float64.  Plugins whose IR shows input dependence, and
input-independent plugins whose channels differ, keep the callback
(tests/test_gpu_proof.py: the cases probes alone could not see).
"""
import os
import struct

import numpy as np
import pytest

import dspbench as d

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(os.path.dirname(HERE), "oracle", "_ref")
MODS = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
PEAK_REL_TOL = 1e-6

# the class each stock plugin's default Parameters must get (stateful plugins
# keep the callback: their blocks depend on the State)
# (static_gain_plugin and plugin_with_parameters have a State the callback
# never writes -- the IR shows it -- so their blocks are independent too)
EXPECTED = {"IR_test": "table", "handmade_test": "table", "gain_test": "gain", "no_op": "gain",
            "template_plugin": "gain", "static_gain_plugin": "gain", "sine_test": "callback",
            "buffer_test": "callback", "plugin_with_parameters": "gain"}


def have(name):
    return os.path.exists(os.path.join(MODS, f"mod_{name}.co")) and os.path.exists(
        os.path.join(REF, f"libref_{name}.so"))


def load(name):
    with open(os.path.join(MODS, f"mod_{name}.co"), "rb") as f:
        return d.module.Module(f.read())


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_stock_plugin_block_classes(torch_cuda, name):
    if not have(name):
        pytest.skip("modules / oracle/_ref not built")
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    cls, g = mod.block_class(params, 2, 512, 48000.0)
    assert cls == EXPECTED[name], (name, cls, g)
    if name == "gain_test":
        assert g == struct.unpack("<f", params[:4])[0]
    if name in ("no_op", "template_plugin", "plugin_with_parameters"):
        assert g == 1.0
    if name == "static_gain_plugin":
        assert g == np.float32(0.1)


@pytest.mark.parametrize("name", ["IR_test", "handmade_test", "gain_test", "no_op", "static_gain_plugin"])
@pytest.mark.parametrize("cin,C,B,L", [(2, 2, 512, 20_000 + 37), (1, 2, 384, 50_001), (2, 2, 100, 9_999),
                                       (2, 3, 1024, 70_000)])
def test_specialized_render_is_the_plugins_own(torch_cuda, oracle, name, cin, C, B, L):
    """Specialised render == the callback on every block == the reference
    plugin compiled for the CPU, bit for bit (ragged tails, a mono file into
    stereo, a third channel the file lacks)."""
    if not have(name):
        pytest.skip("modules / oracle/_ref not built")
    torch = torch_cuda
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, C, 48000.0)
    ref = oracle.RefPlugin(name, C, 48000.0)
    x = np.random.default_rng(B).uniform(-1, 1, (cin, L)).astype(np.float32)
    want = oracle.render_offline([x[c] for c in range(cin)], C, B, 48000.0, ref.as_oracle())
    xg = torch.from_numpy(x).cuda()
    got = d.render_offline(xg, C, B, 48000.0, mod.plugin(params, name)).cpu().numpy()
    every = d.render_offline(xg, C, B, 48000.0, mod.plugin(params, name, specialize=False)).cpu().numpy()
    assert np.array_equal(every, want)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("B", [512, 256, 384])
def test_ir_test_source_render_stft_fused(torch_cuda, oracle, B):
    """IR_test.cpp compiled unchanged, render + STFT: the render bit-exact
    against the reference plugin (CPU), the spectra bit-exact against the
    stock fused IR_test kernel (DSP_PLUGIN_IR_RAMP) of the same parameters and
    within 1e-6 of the peak of float64; with the callback on every block the
    spectra (render, then the memory STFT) agree within the same bar."""
    if not have("IR_test"):
        pytest.skip("modules / oracle/_ref not built")
    torch = torch_cuda
    mod = load("IR_test")
    params = mod.default_parameters()
    gain, step = struct.unpack("<ff", params[:8])
    mod.initialize_state(params, 2, 48000.0)
    L = 8192 * 9 + 777
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, (2, L)).astype(np.float32)).cuda()
    out, mag = d.render_stft(x, 2, B, 48000.0, mod.plugin(params, "IR_test"), window=d.DSP_WIN_HANN)
    s_out, s_mag = d.render_stft(x, 2, B, 48000.0, d.Plugin.ir_test(gain, step), window=d.DSP_WIN_HANN)
    e_out, e_mag = d.render_stft(x, 2, B, 48000.0, mod.plugin(params, "IR_test", specialize=False),
                                 window=d.DSP_WIN_HANN)
    torch.cuda.synchronize()
    ref = oracle.RefPlugin("IR_test", 2, 48000.0)
    want = oracle.render_offline([x[0].cpu().numpy(), x[1].cpu().numpy()], 2, B, 48000.0, ref.as_oracle())
    assert np.array_equal(out.cpu().numpy(), want)
    assert torch.equal(out, s_out) and torch.equal(out, e_out)
    assert torch.equal(mag, s_mag)
    m64 = oracle.np_stft_mag(want[0], 8192, 4096, d.DSP_WIN_HANN, 4097)
    for m in (mag, e_mag):
        mm = m[0].cpu().numpy().astype(np.float64)
        assert float(np.max(np.abs(mm - m64).max(axis=1) / m64.max(axis=1))) <= PEAK_REL_TOL


@pytest.mark.parametrize("soff,C", [(0, 2), (4096 * 37, 2), (512 * 3 + 4096, 2), (512 * 7, 2), (0, 1), (4096 * 5, 8)])
def test_ir_test_source_is_the_headline(torch_cuda, soff, C):
    """The bench's headline call (bench.py --ir-plugin source, the default):
    IR_test.cpp compiled unchanged, 4097-bin Hann 8192 / 4096 STFT at a rank's
    sample offset, gives the render and spectra of the stock fused IR_test
    kernel (DSP_PLUGIN_IR_RAMP, closed-form ramp) bit for bit: the same
    instantiation (PER path), its block read from the callback's table."""
    if not have("IR_test"):
        pytest.skip("modules / oracle/_ref not built")
    torch = torch_cuda
    mod = load("IR_test")
    params = mod.default_parameters()
    gain, step = struct.unpack("<ff", params[:8])
    mod.initialize_state(params, C, 48000.0)
    assert mod.block_class(params, C, 512, 48000.0)[0] == "table"
    L = 4096 * 64 + 4096
    x = torch.zeros((min(C, 2), L), device="cuda")  # C = 8: six channels the file lacks
    out, mag = d.render_stft(x, C, 512, 48000.0, mod.plugin(params, "IR_test"), window=d.DSP_WIN_HANN,
                             sample_offset=soff)
    s_out, s_mag = d.render_stft(x, C, 512, 48000.0, d.Plugin.ir_test(gain, step), window=d.DSP_WIN_HANN,
                                 sample_offset=soff)
    torch.cuda.synchronize()
    assert torch.equal(out, s_out)
    assert torch.equal(mag, s_mag)
    with pytest.raises(d.DspError):  # a shard starts on a block boundary (the library's contract)
        d.render_stft(x, C, 512, 48000.0, mod.plugin(params, "IR_test"), window=d.DSP_WIN_HANN, sample_offset=777)


@pytest.mark.parametrize("seed", range(8))
def test_ir_test_source_random_parameters(torch_cuda, oracle, seed):
    """IR_test.cpp compiled unchanged with random Parameters and block sizes
    (seed 7: a step 2^-30 of the gain, whose f64 recurrence rounds): the
    render bit-exact against the reference plugin compiled for the CPU with
    the same Parameters, the spectra bit-exact against DSP_PLUGIN_IR_RAMP --
    whether the block went to the closed form (module.cpp affine_ramp) or
    stayed a table."""
    if not have("IR_test"):
        pytest.skip("modules / oracle/_ref not built")
    torch = torch_cuda
    rng = np.random.default_rng(100 + seed)
    g = float(np.float32(rng.uniform(0.0, 1.0)))
    st = float(np.float32(rng.uniform(0.001, 0.1) if seed < 7 else g * 2.0 ** -30))
    B = int(rng.choice([512, 256, 1024, 2048, 480, 128]))
    params = struct.pack("<ff", g, st)
    mod = load("IR_test")
    mod.initialize_state(params, 2, 48000.0)
    assert mod.block_class(params, 2, B, 48000.0)[0] == "table"
    L = 8192 * 5 + 1234
    x = torch.zeros((2, L), device="cuda")
    out, mag = d.render_stft(x, 2, B, 48000.0, mod.plugin(params, "IR_test"), window=d.DSP_WIN_HANN)
    s_out, s_mag = d.render_stft(x, 2, B, 48000.0, d.Plugin.ir_test(g, st), window=d.DSP_WIN_HANN)
    torch.cuda.synchronize()
    ref = oracle.RefPlugin("IR_test", 2, 48000.0)
    ref.params[:8] = np.frombuffer(params, np.uint8)
    want = oracle.render_offline([np.zeros(L, np.float32)] * 2, 2, B, 48000.0, ref.as_oracle())
    assert np.array_equal(out.cpu().numpy(), want)
    assert torch.equal(out, s_out)
    assert torch.equal(mag, s_mag)


CLIP_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) out[c][s] = out[c][s] > 5.0f ? 0.0f : out[c][s] * p.g;
}
'''

PER_CHANNEL_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };
struct State {};
Parameters default_parameters() { Parameters p = {0.25f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) out[c][s] = p.g * (float)(c + 1) - 0.001f * (float)s;
}
'''

TONE_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(20.0f, 2000.0f) f; };
struct State {};
Parameters default_parameters() { Parameters p = {375.0f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        const float v = (float)sin(2.0 * 3.14159265358979 * (double)p.f * (double)s / (double)sr);
        for (u32 c = 0; c < C; ++c) out[c][s] = v;
    }
}
'''


@pytest.mark.parametrize("src,name,cls", [(CLIP_SRC, "clip", "callback"), (PER_CHANNEL_SRC, "per_channel", "callback"),
                                          (TONE_SRC, "tone", "table")])
def test_probes_keep_the_callback_where_needed(torch_cuda, src, name, cls):
    """A gain that clips above 5 (the IR stores a select on the sample) and an
    input-independent plugin whose channels differ keep the callback; a tone
    whose block depends on the sample rate is a table.  Whatever the class,
    the render equals the callback on every block bit for bit."""
    torch = torch_cuda
    mod = d.module.Module(d.module.compile_source(src, f"{name}.cpp"))
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 44100.0)
    got_cls, _ = mod.block_class(params, 2, 480, 44100.0)
    assert got_cls == cls
    x = torch.from_numpy(np.random.default_rng(2).uniform(-8, 8, (2, 48_000 + 11)).astype(np.float32)).cuda()
    a = d.render_offline(x, 2, 480, 44100.0, mod.plugin(params, name))
    b = d.render_offline(x, 2, 480, 44100.0, mod.plugin(params, name, specialize=False))
    assert torch.equal(a, b)


RAMP_F32_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; FLOAT_PARAM(0.0f, 0.1f) st; };
struct State {};
Parameters default_parameters() { Parameters p = {0.7f, 0.0013f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    float g = p.g;
    for (u32 s = 0; s < B; ++s) {
        for (u32 c = 0; c < C; ++c) out[c][s] = g;
        g -= p.st;
    }
}
'''

RAMP_F64_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(-1.0f, 1.0f) g; FLOAT_PARAM(-0.1f, 0.1f) st; };
struct State {};
Parameters default_parameters() { Parameters p = {-0.3f, -0.00071f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s)
        for (u32 c = 0; c < C; ++c) out[c][s] = (float)((double)p.g - (double)s * (double)p.st);
}
'''


@pytest.mark.parametrize("src,name", [(RAMP_F32_SRC, "ramp_f32"), (RAMP_F64_SRC, "ramp_f64")])
@pytest.mark.parametrize("B", [512, 256, 480])
def test_ramp_blocks_in_closed_form_or_table(torch_cuda, oracle, src, name, B):
    """Table-class blocks that are ramps: a float recurrence (its rounding
    drifts from any f64 affine form) and an f64 affine ramp with negative
    values (module.cpp affine_ramp finds its closed form).  Whichever the
    fused kernel evaluates -- the closed form, checked against every table
    value, or the table -- the render equals the callback on every block bit
    for bit, and the spectra are within 1e-6 of the peak of float64."""
    torch = torch_cuda
    mod = d.module.Module(d.module.compile_source(src, f"{name}.cpp"))
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    assert mod.block_class(params, 2, B, 48000.0)[0] == "table"
    L = 4096 * 20 + 8192
    x = torch.zeros((2, L), device="cuda")
    out, mag = d.render_stft(x, 2, B, 48000.0, mod.plugin(params, name), window=d.DSP_WIN_HANN, sample_offset=B * 3)
    want = d.render_offline(x, 2, B, 48000.0, mod.plugin(params, name, specialize=False))
    torch.cuda.synchronize()
    nb = d.num_blocks(L, B)
    # sample_offset shifts only the block phase: B * 3 keeps it at 0
    assert torch.equal(out[:, :nb * B], want[:, :nb * B])
    m64 = oracle.np_stft_mag(want[0].cpu().numpy(), 8192, 4096, d.DSP_WIN_HANN, 4097)
    mm = mag[0].cpu().numpy().astype(np.float64)
    assert float(np.max(np.abs(mm - m64).max(axis=1) / m64.max(axis=1))) <= PEAK_REL_TOL


def test_new_parameters_are_probed_again(torch_cuda):
    """gain_test.cpp with other Parameters: the class follows the blob (a
    different g), and the render matches the stock gain map bit for bit."""
    if not have("gain_test"):
        pytest.skip("modules / oracle/_ref not built")
    torch = torch_cuda
    mod = load("gain_test")
    mod.initialize_state(mod.default_parameters(), 2, 48000.0)
    x = torch.rand((2, 30_000), device="cuda") * 2 - 1
    for g in (0.75, -0.125, 0.0):
        params = struct.pack("<f", g) + mod.default_parameters()[4:]
        cls, gg = mod.block_class(params, 2, 512, 48000.0)
        assert cls == "gain" and gg == np.float32(g)
        got = d.render_offline(x, 2, 512, 48000.0, mod.plugin(params, "gain_test"))
        want = d.render_offline(x, 2, 512, 48000.0, d.Plugin.gain_test(g))
        assert torch.equal(got, want)


@pytest.mark.parametrize("name", sorted(k for k, v in EXPECTED.items() if v != "callback"))
def test_shipped_object_confirms_the_class(torch_cuda, name):
    """The classes come from the callback's -O2 analysis IR; the module that
    runs is the -O3 object.  Both compile the same source with
    the same IEEE options, and the shipped object's own callback confirms the
    class on the call's input: DSP_EXEC_VERIFY_CLASS runs it on four blocks of
    each render and compares bit for bit (VERIFIED, never RERENDERED) --
    through render_offline, render_stft and the chunked host driver."""
    if not have(name):
        pytest.skip("modules / oracle/_ref not built")
    import dspbench._lib as L
    from dspbench.api import last_result
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    ok = L.DSP_RESULT_CLASS | L.DSP_RESULT_VERIFIED
    x = np.random.default_rng(31).uniform(-1, 1, (2, 512 * 200 + 77)).astype(np.float32)
    xg = torch_cuda.from_numpy(x).cuda()
    d.render_offline(xg, 2, 512, 48000.0, mod.plugin(params, name, verify=True))
    assert last_result() == ok
    d.render_stft(xg, 2, 512, 48000.0, mod.plugin(params, name, verify=True))
    assert last_result() == ok
    d.render_stft_host(x, 2, 512, 48000.0, mod.plugin(params, name, verify=True), chunk=1 << 15)
    assert last_result() == ok
