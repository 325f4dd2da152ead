"""A State-writing callback rendered in speculative segments (module.h
dsp_state_spec_info, csrc/module.cpp module_render_seg) against the serial
chain (DSP_EXEC_SERIAL_STATE: one lane, blocks in order, as the reference's
audio thread calls them, audio.cpp:160-165).  The bar is bit for bit: every
output sample and the State left behind, over consecutive renders (the State
carries), whatever the plugin -- filters that forget their State (one pass),
slow filters (reruns), oscillators and counters that never forget (the
in-order walk renders nearly everything again)."""
import os

import numpy as np
import pytest

import dspbench as d

HERE = os.path.dirname(os.path.abspath(__file__))
MODS = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")
PLUGIN_DIR = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "plugins")

# a one-pole smoother per channel (forgets its State within a few hundred samples)
ONE_POLE_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) a; };
struct State { float z[16]; };
Parameters default_parameters() { Parameters p = {0.05f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s; for (int c = 0; c < 16; ++c) s.z[c] = 0.0f; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            const float d = out[c][s] - st.z[c];
            st.z[c] = st.z[c] + p.a * d;
            out[c][s] = st.z[c];
        }
}
'''

# an envelope follower with a block counter: the counter never forgets, so
# no segment's speculative State is ever the true one
COUNTER_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) rel; };
struct State { float env; unsigned blocks; };
Parameters default_parameters() { Parameters p = {0.01f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s = {0.0f, 0u}; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        const float x = out[0][s] < 0.0f ? -out[0][s] : out[0][s];
        st.env = x > st.env ? x : st.env + p.rel * (x - st.env);
        for (u32 c = 0; c < C; ++c) out[c][s] = out[c][s] * st.env + (float)(st.blocks & 7u) * 1e-3f;
    }
    st.blocks += 1u;
}
'''

# a running sum of the input: never forgets and depends on every block (no
# warm-up level meets it, no State chain can follow it without the block)
RUNNING_SUM_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };
struct State { float sum; };
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s = {0.0f}; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        st.sum += out[0][s] * 1e-3f;
        for (u32 c = 0; c < C; ++c) out[c][s] = out[c][s] * p.g + st.sum;
    }
}
'''

# an oscillator bank: a phase per channel in State (never forgets), the
# block written and never read -- the State chain drops the block's arithmetic
OSC_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(20.0f, 2000.0f) freq; FLOAT_PARAM(0.0f, 1.0f) gain; };
struct State { double phase[4]; };
Parameters default_parameters() { Parameters p = {440.0f, 0.25f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s = {{0.0, 0.0, 0.0, 0.0}}; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c) {
        const double step = two_pi * (double)p.freq * (1.0 + 0.01 * (double)(c & 3u)) / (double)sr;
        double ph = st.phase[c & 3u];
        for (u32 s = 0; s < B; ++s) {
            out[c][s] = (float)(sin_64(ph) * (double)p.gain);
            ph += step;
            if (ph > two_pi) ph -= two_pi;
        }
        st.phase[c & 3u] = ph;
    }
}
'''

# a tremolo: a phase in State (never forgets) that does not depend on the
# block, which the callback reads and scales: the block stays in the chain
# kernel's private memory, so it renders serially
TREMOLO_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.1f, 20.0f) rate; FLOAT_PARAM(0.0f, 1.0f) depth; };
struct State { double phase; };
Parameters default_parameters() { Parameters p = {5.0f, 0.5f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s = {0.0}; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    const double step = two_pi * (double)p.rate / (double)sr;
    for (u32 s = 0; s < B; ++s) {
        const float g = (float)(1.0 - (double)p.depth * (0.5 + 0.5 * cos_64(st.phase)));
        for (u32 c = 0; c < C; ++c) out[c][s] = out[c][s] * g;
        st.phase += step;
        if (st.phase > two_pi) st.phase -= two_pi;
    }
}
'''

# a State of 2 KB: more than a lane copies (serial chain)
BIG_STATE_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) a; };
struct State { float z[512]; };
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s; for (int i = 0; i < 512; ++i) s.z[i] = 0.0f; return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            st.z[c] = st.z[c] + p.a * (out[c][s] - st.z[c]);
            out[c][s] = st.z[c];
        }
}
'''

_cache = {}


def module_of(src, name):
    if name not in _cache:
        _cache[name] = d.module.Module(d.module.compile_source(src, f"{name}.cpp"))
    return _cache[name]


def biquad_module(cutoff=None, q=None):
    mod = module_of(open(os.path.join(PLUGIN_DIR, "biquad.cpp")).read(), "biquad")
    params = mod.default_parameters()
    if cutoff is not None:
        params = np.frombuffer(params, np.float32).copy()
        params[0], params[1] = cutoff, q
        params = params.tobytes()
    return mod, params


def both(torch, mod, params, x, C, B, calls=2, sr=48000.0, stft=False):
    """The same renders with speculative segments and with the serial chain,
    each from a fresh initialize_state: [(output, State) per call], info."""
    res = {}
    info = []
    for serial in (False, True):
        mod.initialize_state(params, C, sr)
        plug = mod.plugin(params, serial_state=serial)
        xg = torch.from_numpy(x).cuda()
        outs = []
        for _ in range(calls):
            if stft:
                y, m = d.render_stft(xg, C, B, sr, plug)
                outs.append((y.cpu().numpy(), m.cpu().numpy(), mod.read_state()))
            else:
                y = d.render_offline(xg, C, B, sr, plug)
                outs.append((y.cpu().numpy(), mod.read_state()))
            if not serial:
                info.append(mod.state_spec())
        res[serial] = outs
    return res[False], res[True], info


def assert_same(a, b):
    for ra, rb in zip(a, b):
        for va, vb in zip(ra, rb):
            if isinstance(va, bytes):
                assert va == vb
            else:
                assert va.shape == vb.shape
                assert np.array_equal(va.view(np.uint32), vb.view(np.uint32))


def noise(C, L, seed):
    return np.random.default_rng(seed).uniform(-1, 1, (C, L)).astype(np.float32)


@pytest.mark.gpu
def test_biquad_source_one_minute_bit_exact(torch_cuda):
    """plugins/biquad.cpp compiled unchanged, 1 min of stereo noise: the
    segments reproduce the serial chain bit for bit, and the 1 kHz low-pass
    forgets its State within the warm-up (almost no segment differs)."""
    mod, params = biquad_module()
    assert mod.facts["analyzed"] and mod.facts["writes_state"]
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 48000 * 60, 1), 2, 512)
    assert_same(spec, ser)
    assert info[0]["used"] and info[0]["segments"] > 1000 and info[0]["levels"] == 1
    assert info[0]["differed"][0] * 50 < info[0]["segments"]
    assert info[0]["differed"][2] <= 2 and info[0]["serial_reruns"] <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("cutoff,q", [(100.0, 0.7071), (30.0, 5.0), (5000.0, 2.0)])
def test_biquad_slow_and_fast_filters(torch_cuda, cutoff, q):
    """Low cutoffs forget slowly: segments differ after pass 1, reruns and the
    walk make the render exact anyway."""
    mod, params = biquad_module(cutoff, q)
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 400_000 + 123, 2), 2, 512, calls=3)
    assert_same(spec, ser)
    assert all(i["used"] or i["disabled"] for i in info)


@pytest.mark.gpu
def test_longer_warm_up_within_one_render(torch_cuda):
    """A 300 Hz low-pass forgets within ~4,600 samples on average (26,000 at
    worst over 200 trials, tools/diag/biquad_state_sync.c): the first warm-up
    (4 blocks) leaves most segments wrong, so the same render tries 64 blocks,
    which stands; the next render starts there.  Bit-exact throughout."""
    mod, params = biquad_module(300.0, 0.7071)
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 1_500_000, 9), 2, 512)
    assert_same(spec, ser)
    assert info[0]["used"] and info[0]["levels"] == 2 and info[0]["warmup_blocks"] == 64
    guessed = info[0]["segments"] - 1 - 64 // info[0]["blocks_per_segment"]
    assert info[0]["differed"][0] * 8 <= guessed
    assert info[1]["used"] and info[1]["levels"] == 1 and info[1]["warmup_blocks"] == 64


@pytest.mark.gpu
@pytest.mark.parametrize("C,cin,B,L", [(1, 1, 512, 100_000), (2, 1, 256, 60_001), (3, 3, 512, 80_000),
                                       (2, 2, 100, 50_000), (4, 2, 64, 30_000), (2, 2, 1024, 200_000)])
def test_one_pole_shapes(torch_cuda, C, cin, B, L):
    """The kernel instantiations (stereo B = 512, mono, stereo any B, any
    C), missing channels (zeros), ragged tails, B not a multiple of 4."""
    mod = module_of(ONE_POLE_SRC, "one_pole_spec")
    params = mod.default_parameters()
    x = noise(cin, L, 3)
    spec, ser, info = both(torch_cuda, mod, params, x, C, B)
    assert_same(spec, ser)
    assert info[0]["used"]


@pytest.mark.gpu
def test_never_forgetting_state_is_exact_and_learned(torch_cuda):
    """A running sum of the input in the State: every speculative segment
    starts wrong at every warm-up level the render tries (4, then 64 blocks:
    a 1,024-block one would be more than half the file), the walk renders them
    again in order (exact), and the module renders these Parameters serially
    from the next call on (no State chain can follow a sum of the block)."""
    mod = module_of(RUNNING_SUM_SRC, "running_sum_spec")
    assert not mod.facts["state_split"]
    params = mod.default_parameters()
    x = noise(2, 150_000, 4)
    spec, ser, info = both(torch_cuda, mod, params, x, 2, 512, calls=3)
    assert_same(spec, ser)
    seg = info[0]["blocks_per_segment"]
    # (segments whose warm-up starts at block 0 start from the true State)
    assert info[0]["used"] and info[0]["levels"] == 2 and info[0]["warmup_blocks"] == 64
    assert info[0]["differed"][0] == info[0]["segments"] - 1 - 64 // seg
    assert info[0]["serial_reruns"] > 0
    assert info[1]["disabled"] and not info[1]["used"] and not info[1]["chain"]
    assert info[2]["disabled"] and not info[2]["used"]
    # new Parameters: learnt again
    p2 = np.frombuffer(params, np.float32).copy()
    p2[0] = 0.25
    spec, ser, info = both(torch_cuda, mod, p2.tobytes(), x, 2, 512, calls=1)
    assert_same(spec, ser)
    assert info[0]["used"]


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["counter", "envelope_counter"])
@pytest.mark.parametrize("C,cin,B,L", [(2, 2, 512, 300_000), (1, 1, 256, 120_000), (2, 1, 100, 80_001),
                                       (4, 2, 64, 40_000), (3, 3, 512, 60_000)])
def test_split_state_counter_beside_an_envelope(torch_cuda, src, C, cin, B, L):
    """An envelope follower (forgets) beside a block counter (never forgets,
    never reads the block): the analysis splits the State by 4-byte word
    (dsp_callback_facts.state_split), a State chain of the counter alone runs
    on one lane (the envelope and the block compiled away), and pass 1 starts
    each segment's warm-up from the counter it recorded there and the live
    State's envelope -- so the segments meet the true State after the warm-up
    and the render is speculative, not serial.  Bit for bit against the
    serial chain, State included, over three consecutive renders; three
    channels have no chain kernel shape and fall back as before."""
    if src == "counter":
        mod = module_of(COUNTER_SRC, "counter_spec")
    else:
        mod = module_of(open(os.path.join(PLUGIN_DIR, "envelope_counter.cpp")).read(), "envelope_counter")
    assert mod.facts["state_split"] and mod.facts["state_reads_block"]
    params = mod.default_parameters()
    spec, ser, info = both(torch_cuda, mod, params, noise(cin, L, 31), C, B, calls=3)
    assert_same(spec, ser)
    if C != 3:
        for i in info:
            assert i["used"] and i["split"] and not i["disabled"], info
        assert info[0]["differed"][0] * 8 <= info[0]["segments"], info


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["counter", "envelope_counter"])
@pytest.mark.parametrize("B,L", [(512, 300_000), (64, 40_000)])
def test_split_state_record_is_checked_not_trusted(torch_cuda, src, B, L):
    """A wrong record of the split State's independent words
    (DSP_MODULE_DEBUG_PERTURB_CHAIN in a split render flips the low bit of
    the block counter recorded for segment 7, as a wrong split would): that
    segment's warm-up ends in a State unlike the one segment 6 ends with, the
    boundary check fails and the segment is rendered again from the true
    State -- output and State equal to the serial chain bit for bit, the
    miss counted in pass 1's differed, the next calls unaffected."""
    torch = torch_cuda
    C = 2
    # (an instance of its own: nothing learnt by the other tests' renders)
    if src == "counter":
        mod = module_of(COUNTER_SRC, f"counter_spec_{B}")
    else:
        mod = module_of(open(os.path.join(PLUGIN_DIR, "envelope_counter.cpp")).read(), f"envelope_counter_{B}")
    params = mod.default_parameters()
    x = torch.from_numpy(noise(C, L, 41)).cuda()
    mod.initialize_state(params, C, 48000.0)
    ser = mod.plugin(params, serial_state=True)
    ref = [(d.render_offline(x, C, B, 48000.0, ser).cpu().numpy(), mod.read_state()) for _ in range(3)]
    # a clean speculative render first: what pass 1 misses without the hook
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params)
    clean = d.render_offline(x, C, B, 48000.0, plug)
    base = mod.state_spec()
    assert base["used"] and base["split"] and base["segments"] > 8, base
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params)
    outs, infos = [], []
    for call in range(3):
        if call == 0:
            mod.debug_perturb_chain(7)
        y = d.render_offline(x, C, B, 48000.0, plug)
        outs.append((y.cpu().numpy(), mod.read_state()))
        infos.append(mod.state_spec())
    assert_same(outs, ref)
    assert np.array_equal(clean.cpu().numpy().view(np.uint32), ref[0][0].view(np.uint32))
    hit = infos[0]
    assert hit["used"] and hit["split"] and not hit["chain"], infos
    assert hit["differed"][0] >= 1, (base, infos)
    for i in infos[1:]:
        assert i["used"] and i["split"] and i["differed"][0] * 8 <= i["segments"], (base, infos)


@pytest.mark.gpu
def test_reference_oscillator_sine_test(torch_cuda):
    """The reference's sine_test.cpp (a phase accumulator in State): on the
    first call every warm-up level fails and the State chain (the phase
    alone, in order, on one lane) takes over within the call, the walk
    skipped; the next calls run the chain from the start (learnt) and every
    segment from its recorded State -- exact, no speculation."""
    path = os.path.join(MODS, "mod_sine_test.co")
    if not os.path.exists(path):
        pytest.skip("reference modules not built")
    with open(path, "rb") as f:
        mod = d.module.Module(f.read())
    params = mod.default_parameters()
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 40_000, 5), 2, 512, calls=3)
    assert_same(spec, ser)
    assert info[0]["used"] and info[0]["chain"] and info[0]["levels"] >= 1 and info[0]["serial_reruns"] == 0
    for i in info[1:]:
        assert i["disabled"] and i["used"] and i["chain"] and i["segments"] > 1
    # a long render through the chain: 2 min of stereo, three calls
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 48000 * 120 + 77, 8), 2, 512, calls=3)
    assert_same(spec, ser)
    assert all(i["chain"] for i in info) and info[2]["segments"] > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("C,cin,B,L,chain", [(2, 2, 512, 300_000, True), (1, 1, 256, 100_000, True),
                                             (2, 2, 100, 80_001, True), (4, 2, 64, 40_000, True),
                                             (3, 3, 512, 60_000, False)])
def test_state_chain_of_an_oscillator_bank(torch_cuda, C, cin, B, L, chain):
    """An oscillator per channel (phases in State never forget; the block
    only written): after the first call the State chain kernel of the shape
    runs (stereo B = 512, any B for 1, 2 or 4 channels) with the sines
    dropped, and the segments render from its States; three channels have no
    chain kernel and render serially.  Bit for bit against the serial chain,
    State included."""
    mod = module_of(OSC_SRC, "osc_spec")
    params = mod.default_parameters()
    spec, ser, info = both(torch_cuda, mod, params, noise(cin, L, 11), C, B, calls=3)
    assert_same(spec, ser)
    assert info[2]["disabled"]
    assert bool(info[2]["chain"]) == chain and bool(info[2]["used"]) == chain
    assert bool(info[0]["chain"]) == chain  # the first call: the chain took over from the levels


# a wavetable oscillator: a 1 KB State (the table plus a phase), the table
# written once by initialize_state, the phase never forgetting
WAVETABLE_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(20.0f, 2000.0f) freq; };
struct State { float table[252]; double phase; double pad; };
Parameters default_parameters() { Parameters p = {330.0f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s;
    for (int i = 0; i < 252; ++i) s.table[i] = (float)sin_64(two_pi * (double)i / 250.0);
    s.phase = 0.0; s.pad = 0.0;
    return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    const double step = 250.0 * (double)p.freq / (double)sr;
    for (u32 s = 0; s < B; ++s) {
        const int i = (int)st.phase;
        const float v = st.table[i];
        for (u32 c = 0; c < C; ++c) out[c][s] = v * (c == 0 ? 1.0f : 0.5f);
        st.phase += step;
        if (st.phase >= 250.0) st.phase -= 250.0;
    }
}
'''


@pytest.mark.gpu
def test_state_chain_with_a_1kb_state(torch_cuda):
    """A wavetable oscillator whose State is 1,024 bytes (a table the callback
    only reads, a phase that never forgets): the State chain and the segments
    copy the whole State per block, bit for bit against the serial chain."""
    mod = module_of(WAVETABLE_SRC, "wavetable_spec")
    assert mod.state_size == 1024, mod.state_size
    params = mod.default_parameters()
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 250_000, 13), 2, 512, calls=3)
    assert_same(spec, ser)
    assert all(i["chain"] for i in info), info


@pytest.mark.gpu
def test_tremolo_reading_its_block_takes_the_ir_chain(torch_cuda):
    """A tremolo reads its block, but its phase never depends on it
    (facts.state_reads_block = 0): the module compiler builds its chain
    kernels from IR with the callback's block stores deleted
    (module.cpp, ir_proof.cpp strip_chain_block_stores), so the chain is the
    phase update alone and the segments render from its States -- bit for
    bit against the serial chain, State included."""
    mod = module_of(TREMOLO_SRC, "tremolo_spec")
    assert mod.facts["writes_state"] and not mod.facts["state_reads_block"]
    params = mod.default_parameters()
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 200_000, 12), 2, 512, calls=3)
    assert_same(spec, ser)
    assert info[0]["chain"] and info[2]["disabled"] and info[2]["chain"] and info[2]["used"]


@pytest.mark.gpu
def test_render_stft_through_segments(torch_cuda):
    """dsp_render_stft with a State-writing plugin: the render through the
    segments, then the STFT of it -- both equal the serial chain's."""
    mod, params = biquad_module()
    spec, ser, info = both(torch_cuda, mod, params, noise(2, 300_000, 6), 2, 512, stft=True)
    assert_same(spec, ser)
    assert info[0]["used"]


@pytest.mark.gpu
def test_in_place_and_large_state_take_the_serial_chain(torch_cuda):
    """Rows that overlap (in place) and a State beyond 1024 bytes are
    rendered by the serial chain."""
    torch = torch_cuda
    mod, params = biquad_module()
    x = noise(2, 50_000, 7)
    mod.initialize_state(params, 2, 48000.0)
    want = d.render_offline(torch.from_numpy(x).cuda(), 2, 512, 48000.0, mod.plugin(params, serial_state=True))
    mod.initialize_state(params, 2, 48000.0)
    buf = torch.zeros((2, want.shape[1]), device="cuda")
    buf[:, :x.shape[1]] = torch.from_numpy(x).cuda()
    d.render_offline(buf, 2, 512, 48000.0, mod.plugin(params), out=buf, L_file=x.shape[1])
    assert torch.equal(buf, want)
    assert not mod.state_spec()["used"]
    big = module_of(BIG_STATE_SRC, "big_state_spec")
    bp = big.default_parameters()
    spec, ser, info = both(torch, big, bp, x, 2, 512, calls=1)
    assert_same(spec, ser)
    assert not info[0]["used"]


@pytest.mark.gpu
def test_chunked_host_driver_carries_the_state(torch_cuda):
    """dsp_render_stft_host (host rows in and out): a State-writing plugin
    is one chunk, rendered through the segments."""
    torch = torch_cuda
    mod, params = biquad_module(300.0, 0.7071)
    x = noise(2, 3_000_000, 8)
    res = []
    for serial in (False, True):
        mod.initialize_state(params, 2, 48000.0)
        out, mag = d.render_stft_host(x, 2, 512, 48000.0, mod.plugin(params, serial_state=serial), chunk=1 << 20)
        res.append((np.asarray(out), np.asarray(mag), mod.read_state()))
    assert_same([res[0]], [res[1]])


# ---- generated State-writing plugins: whatever the callback does with its
# State (smoothers, envelopes with input-dependent branches, saturation, a
# counter, a padded State rewritten as a whole, a read-only arena table), the
# segments render the serial chain's bits
GEN_HEAD = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) a; FLOAT_PARAM(0.0f, 1.0f) b; };
Parameters default_parameters() { Parameters p = {0.03f, 0.3f}; return p; }
'''
GEN_BODIES = {
    # two cascaded one-poles with a saturation between them, per channel
    "sat_chain": r'''
struct State { float z1[16], z2[16]; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            st.z1[c] += p.a * (out[c][s] - st.z1[c]);
            const float u = 3.0f * st.z1[c];
            const float v = u / (1.0f + (u < 0.0f ? -u : u));
            st.z2[c] += p.b * (v - st.z2[c]);
            out[c][s] = st.z2[c];
        }
}''',
    # attack / release envelope (a branch on the sample) driving a gain
    "env_gate": r'''
struct State { float env; float g; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {0.0f, 1.0f}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        float m = 0.0f;
        for (u32 c = 0; c < C; ++c) { const float x = out[c][s] < 0.0f ? -out[c][s] : out[c][s]; m = x > m ? x : m; }
        if (m > st.env) st.env += p.b * (m - st.env); else st.env += p.a * (m - st.env);
        const float target = st.env > 0.5f ? 0.25f : 1.0f;
        st.g += 0.01f * (target - st.g);
        for (u32 c = 0; c < C; ++c) out[c][s] *= st.g;
    }
}''',
    # a padded State (char beside floats) assigned as a whole every block
    "padded_whole": r'''
struct State { char on; float y; double acc; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {1, 0.0f, 0.0}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    State n = st;
    for (u32 s = 0; s < B; ++s) {
        n.y += p.a * (out[0][s] - n.y);
        n.acc = 0.999 * n.acc + (double)n.y;
        for (u32 c = 0; c < C; ++c) out[c][s] = n.on ? n.y + 1e-4f * (float)n.acc : out[c][s];
    }
    n.on = n.acc > -1e30 ? 1 : 0;
    st = n;
}''',
    # a wavetable in the arena, only read; a phase that wraps (never forgets)
    "arena_table": r'''
struct State { float* tab; unsigned pos; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) {
    State s; s.tab = (float*)allocate_bytes(sizeof(float) * 64, ctx); s.pos = 0;
    for (int i = 0; i < 64; ++i) s.tab[i] = (float)i / 64.0f;
    return s;
}
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        const float t = st.tab[st.pos & 63u];
        for (u32 c = 0; c < C; ++c) out[c][s] = out[c][s] * p.b + t;
        st.pos += 3u;
    }
}''',
    # the plugin services on the block (copy_array, gain_ip_32_array): the
    # block's last 64 samples held in the State and played at the start of the
    # next block (forgets after one block)
    "service_copy": r'''
struct State { float prev[2][64]; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C && c < 2; ++c) {
        float t[64];
        copy_array(out[c] + (B - 64), t, 64);
        gain_ip_32_array(out[c] + 64, p.b, B - 64);
        copy_array(st.prev[c], out[c], 64);
        copy_array(t, st.prev[c], 64);
    }
}''',
    # a one-pole whose coefficient is read from a mutable-looking State field
    # the callback also rewrites (the same value every block)
    "self_coef": r'''
struct State { float k; float z[16]; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; s.k = p.a; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    st.k = p.a;
    for (u32 c = 0; c < C && c < 16; ++c)
        for (u32 s = 0; s < B; ++s) { st.z[c] = st.z[c] + st.k * (out[c][s] - st.z[c]); out[c][s] = st.z[c] - out[c][s]; }
}''',
    # a split State: a wrapping f64 phase (words 0-1, never forgets, never
    # reads the block) before per-channel envelopes (forget)
    "split_phase_env": r'''
struct State { double phase; float env[2]; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    const float g = (float)st.phase;
    for (u32 c = 0; c < C && c < 2; ++c)
        for (u32 s = 0; s < B; ++s) {
            const float x = out[c][s] < 0.0f ? -out[c][s] : out[c][s];
            st.env[c] += p.a * (x - st.env[c]);
            out[c][s] = out[c][s] * g + st.env[c];
        }
    st.phase += (double)p.b * 0.01;
    if (st.phase >= 1.0) st.phase -= 1.0;
}''',
    # a split State: one-poles before a u64 sample counter (words 2-3)
    "split_counter_tail": r'''
struct State { float z[2]; unsigned long long n; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    const float k = (float)(st.n & 15ull) * 0.0625f;
    for (u32 c = 0; c < C && c < 2; ++c)
        for (u32 s = 0; s < B; ++s) { st.z[c] += p.a * (out[c][s] - st.z[c]); out[c][s] = st.z[c] + k * out[c][s]; }
    st.n += B;
}''',
    # no split: a 16-bit counter shares its word with a block-dependent flag
    # (the counter never forgets: the State chain renders it)
    "shared_word": r'''
struct State { unsigned short cnt; unsigned short hot; float y; };
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) st.y += p.a * (out[0][s] - st.y);
    st.hot = st.y > 0.1f ? 1 : 0;
    st.cnt += 1;
    const float g = 1.0f + 0.001f * (float)(st.cnt & 7u), o = st.hot ? 0.01f : 0.0f;
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) out[c][s] = out[c][s] * g + o;
}''',
}
# the generated plugins whose State splits by word (and those that must not)
GEN_SPLIT = {"split_phase_env": True, "split_counter_tail": True, "shared_word": False}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GEN_BODIES))
def test_generated_plugins_match_the_serial_chain(torch_cuda, name):
    mod = module_of(GEN_HEAD + GEN_BODIES[name], f"gen_{name}")
    f = mod.facts
    params = mod.default_parameters()
    x = noise(2, 250_000 + 77, 11) * np.float32(0.8)
    spec, ser, info = both(torch_cuda, mod, params, x, 2, 512, calls=2)
    assert_same(spec, ser)
    if f["analyzed"] and f["writes_state"] and mod.state_size <= 1024:
        assert info[0]["used"] or info[0]["disabled"]
    if name in GEN_SPLIT:
        assert f["state_split"] == GEN_SPLIT[name], str(f)
        if GEN_SPLIT[name]:
            # the independent words' chain: every call speculative
            assert all(i["used"] and i["split"] and not i["chain"] for i in info), info


@pytest.mark.gpu
@pytest.mark.parametrize("plugin", ["biquad", "osc"])
def test_loop_mode_through_segments(torch_cuda, plugin):
    """dsp_render_loop (audio.cpp:100-132: the file wraps from the cursor)
    with a State-writing plugin: the wrapped block stream through the
    segments (biquad.cpp) or the State chain (the oscillator bank) equals the
    serial chain's, cursor and State included."""
    torch = torch_cuda
    if plugin == "biquad":
        mod, params = biquad_module(700.0, 0.9)
    else:
        mod = module_of(OSC_SRC, "osc_spec")
        params = mod.default_parameters()
    x = torch.from_numpy(noise(2, 33_333, 12)).cuda()
    res = []
    for serial in (False, True):
        mod.initialize_state(params, 2, 48000.0)
        plug = mod.plugin(params, serial_state=serial)
        y1, cur = d.render_loop(x, 2, 512, 700, 48000.0, plug, cursor=1234)
        y2, cur2 = d.render_loop(x, 2, 512, 300, 48000.0, plug, cursor=cur)
        res.append((y1.cpu().numpy(), y2.cpu().numpy(), cur, cur2, mod.read_state()))
        if not serial and plugin == "osc":
            assert mod.state_spec()["chain"]
    a, b = res
    assert a[2:4] == b[2:4] and a[4] == b[4]
    for i in (0, 1):
        assert np.array_equal(a[i].view(np.uint32), b[i].view(np.uint32))


@pytest.mark.gpu
def test_biquad_source_full_hour_bit_exact(torch_cuda):
    """The bench's full size: 1 h of 48 kHz stereo through plugins/biquad.cpp
    compiled unchanged, segments against the serial chain (≈10 s on one lane),
    compared on the device bit for bit, final State included."""
    torch = torch_cuda
    mod, params = biquad_module()
    L = 48000 * 3600
    g = torch.Generator(device="cuda").manual_seed(13)
    x = torch.rand((2, L), device="cuda", generator=g) * 2 - 1
    outs = []
    for serial in (False, True):
        mod.initialize_state(params, 2, 48000.0)
        y = d.render_offline(x, 2, 512, 48000.0, mod.plugin(params, serial_state=serial))
        torch.cuda.synchronize()
        outs.append((y, mod.read_state()))
        if not serial:
            info = mod.state_spec()
    assert info["used"] and info["segments"] > 8000
    assert outs[0][1] == outs[1][1]
    assert torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32))


@pytest.mark.gpu
def test_state_spec_names_the_last_render(torch_cuda):
    """Renders made back to back without reading the counters in between:
    dsp_module_state_spec describes the last one (the counters of the two
    newest renders are read oldest first; the newest was once skipped when
    the older sat in the second slot)."""
    torch = torch_cuda
    mod, params = biquad_module()
    mod.initialize_state(params, 2, 48000.0)
    plug = mod.plugin(params)
    xa = torch.from_numpy(noise(2, 200_000, 14)).cuda()
    xb = torch.from_numpy(noise(2, 900_000, 15)).cuda()
    for x in (xa, xa, xb):
        d.render_offline(x, 2, 512, 48000.0, plug)
    info = mod.state_spec()
    nb = (900_000 + 511) // 512
    assert info["used"] and info["segments"] == (nb + info["blocks_per_segment"] - 1) // info["blocks_per_segment"]
    for x in (xb, xa):
        d.render_offline(x, 2, 512, 48000.0, plug)
    info = mod.state_spec()
    nb = (200_000 + 511) // 512
    assert info["segments"] == (nb + info["blocks_per_segment"] - 1) // info["blocks_per_segment"]


def _chain_module(which, probe=False):
    if which == "sine_test":
        path = os.path.join(MODS, "mod_sine_test.co")
        if not os.path.exists(path):
            pytest.skip("reference modules not built")
        key = ("sine_test", probe)
        if key not in _cache:
            with open(path, "rb") as f:
                _cache[key] = d.module.Module(f.read())
        return _cache[key]
    return module_of({"osc": OSC_SRC, "tremolo": TREMOLO_SRC}[which], f"{which}_spec" + ("_probe" if probe else ""))


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["sine_test", "osc", "tremolo"])
@pytest.mark.parametrize("when,where", [("learnt", "segment_start"), ("learnt", "mid_segment"),
                                        ("first_call", "segment_start")])
def test_state_chain_is_checked_not_trusted(torch_cuda, which, when, where):
    """A wrong record in the State chain (dsp_module_debug
    DSP_MODULE_DEBUG_PERTURB_CHAIN flips a high bit of the State the chain
    recorded for one block, as a miscompiled chain would): the exact rerun
    compares every record with the State it renders from, a check compares
    every segment boundary, and the walk renders serially from the true State
    whatever differs -- the render equals the serial chain bit for bit, State
    included, the mismatch is reported (chain_mismatch,
    chain_records_differed), and the module renders these Parameters serially
    from the next call on.  When the chain runs within the first call (after
    its warm-up levels failed) and when it runs learnt, from the start."""
    torch = torch_cuda
    C, B, L = 2, 512, 300_000
    x = torch.from_numpy(noise(C, L, 21)).cuda()
    # the segment layout of this shape, from another instance of the module
    probe = _chain_module(which, probe=True)
    pp = probe.default_parameters()
    probe.initialize_state(pp, C, 48000.0)
    d.render_offline(x, C, B, 48000.0, probe.plugin(pp))
    seg = probe.state_spec()["blocks_per_segment"]
    assert seg >= 1
    mod = _chain_module(which)
    params = mod.default_parameters()
    # forget what earlier renders taught the module: other Parameters once
    other = bytearray(params)
    other[0] ^= 1
    mod.initialize_state(bytes(other), C, 48000.0)
    d.render_offline(x[:, :B].contiguous(), C, B, 48000.0, mod.plugin(bytes(other)))
    mod.initialize_state(params, C, 48000.0)
    ser = mod.plugin(params, serial_state=True)
    ref = [(d.render_offline(x, C, B, 48000.0, ser).cpu().numpy(), mod.read_state()) for _ in range(3)]
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params)
    perturbed = 0 if when == "first_call" else 1
    outs, infos = [], []
    for call in range(3):
        if call == perturbed:
            mod.debug_perturb_chain(7 * seg + (seg // 2 if where == "mid_segment" else 0))
        y = d.render_offline(x, C, B, 48000.0, plug)
        outs.append((y.cpu().numpy(), mod.read_state()))
        infos.append(mod.state_spec())
    assert_same(outs, ref)
    hit = infos[perturbed]
    assert hit["chain"] and hit["chain_records_differed"] >= 1, infos
    if where == "segment_start":
        # the perturbed segment and (the phase never forgets) the one after it
        assert hit["chain_mismatch"] >= 1, infos
    else:
        assert hit["chain_mismatch"] == 0, infos
    # learnt: the serial chain from then on
    for i in infos[perturbed + 1:]:
        assert i["disabled"] and not i["used"], infos
    # a render before it reports nothing
    for i in infos[:perturbed]:
        assert i["chain_mismatch"] == 0 and i["chain_records_differed"] == 0, infos


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["biquad", "envelope_counter"])
def test_segments_pinned_to_the_host_build(torch_cuda, oracle, name):
    """The speculative segments (and the split State's chain for
    envelope_counter.cpp) against the plugin built for the host the way the
    reference's JIT builds a plugin (oracle/_ref/libplug_<name>.so: the
    reference's own wrapper and flags, ref compiler.cpp:507-515) -- not a
    GPU self-comparison.  That build's flags let the compiler reassociate
    and contract, so it is not IEEE-per-operation like the module's: the
    bound is a tolerance (the GPU segments equal the GPU serial chain bit for
    bit, the other tests).  20 s of stereo, B = 512, two consecutive renders
    (the State carries), the default Parameters on both sides."""
    ref_so = os.path.join(os.path.dirname(HERE), "oracle", "_ref", f"libplug_{name}.so")
    path = os.path.join(MODS, f"mod_{name}.co")
    if not (os.path.exists(ref_so) and os.path.exists(path)):
        pytest.skip("oracle/_ref or the modules not built")
    torch = torch_cuda
    with open(path, "rb") as f:
        mod = d.module.Module(f.read())
    params = mod.default_parameters()
    ref = oracle.RefPlugin(name, 2, 48000.0, prefix="libplug_")
    assert bytes(ref.params[:mod.params_size]) == params
    C, B = 2, 512
    x = noise(C, 48000 * 20 + 77, 61) * np.float32(0.8)
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params, name)
    xg = torch.from_numpy(x).cuda()
    worst = 0.0
    for call in range(2):
        got = d.render_offline(xg, C, B, 48000.0, plug).cpu().numpy()
        info = mod.state_spec()
        want = oracle.render_offline([x[0], x[1]], C, B, 48000.0, ref.as_oracle())
        assert got.shape == want.shape
        assert np.all(np.isfinite(got))
        err = float(np.max(np.abs(got.astype(np.float64) - want)))
        worst = max(worst, err)
        assert info["used"] and not info["chain"], info
        if name == "envelope_counter":
            assert info["split"], info
    print(f"{name}: max |GPU segments - host build| = {worst:.3e}")
    assert worst <= 1e-4, worst


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["one_pole", "counter"])
def test_role_split_pass_edges(torch_cuda, src):
    """The role-split pass 1 of stereo B = 512 (dspb_seg_c2b512: wave 0 the
    callbacks, waves 1-3 the blocks) on its edge paths: one input channel for
    two output channels (the movers load zeros for the missing one), input
    and output rows 4 bytes off 16-byte alignment (the movers' dword path),
    a ragged tail -- against the serial chain bit for bit, State included,
    over two consecutive renders."""
    torch = torch_cuda
    mod = module_of(ONE_POLE_SRC if src == "one_pole" else COUNTER_SRC, f"{src}_roles_edges")
    params = mod.default_parameters()
    C, B, L = 2, 512, 300_001
    nb = (L + B - 1) // B
    base = torch.from_numpy(noise(1, L + 1, 71)).cuda()
    x = base[:, 1:]  # 4 bytes past a 16-byte boundary
    assert x.data_ptr() % 16 == 4
    res = {}
    for serial in (False, True):
        mod.initialize_state(params, C, 48000.0)
        plug = mod.plugin(params, serial_state=serial)
        outs = []
        for _ in range(2):
            big = torch.empty((C, nb * B + 1), device="cuda")
            out = big[:, 1:]
            y = d.render_offline(x, C, B, 48000.0, plug, out=out)
            outs.append((y.cpu().numpy(), mod.read_state()))
            if not serial:
                info = mod.state_spec()
                assert info["used"] and info["segments"] > 1, info
        res[serial] = outs
    assert_same(res[False], res[True])


# a peak follower with a slow release: two trajectories meet at the first
# sample louder than both, so how soon a segment's warm-up meets the true
# State depends on the input, not only on the Parameters
PEAK_SRC = r'''
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) rel; };
struct State { float env[2]; };
Parameters default_parameters() { Parameters p = {0.99999f}; return p; }
State initialize_state(const Parameters& p, const unsigned C, const float sr, void* ctx) { State s = {}; return s; }
void audio_callback(const Parameters& p, State& st, float** out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C && c < 2; ++c)
        for (u32 s = 0; s < B; ++s) {
            const float x = out[c][s] < 0.0f ? -out[c][s] : out[c][s];
            st.env[c] = x > st.env[c] ? x : st.env[c] * p.rel;
            out[c][s] = out[c][s] * (1.0f - 0.5f * st.env[c]);
        }
}
'''


@pytest.mark.gpu
def test_one_level_learning_unlearns_when_the_input_stops_forgetting(torch_cuda):
    """Once a render's first warm-up level met the State the module launches
    the first two levels alone; a later render whose input keeps the first
    from meeting the State (a peak follower fed a quiet signal after a loud
    one) takes the second and comes out exact, and the module goes back to
    every level.  Each render against the serial chain, bit for bit, State
    included."""
    torch = torch_cuda
    mod = module_of(PEAK_SRC, "peak_follower")
    params = mod.default_parameters()
    C, B, L = 2, 512, 48000 * 20
    loud = noise(C, L, 81)
    quiet = (noise(C, L, 82) * np.float32(1e-3)).astype(np.float32)
    inputs = [loud, loud, loud, quiet, quiet, quiet]
    res = {}
    infos = []
    for serial in (False, True):
        mod.initialize_state(params, C, 48000.0)
        plug = mod.plugin(params, serial_state=serial)
        outs = []
        for x in inputs:
            y = d.render_offline(torch.from_numpy(x).cuda(), C, B, 48000.0, plug)
            outs.append((y.cpu().numpy(), mod.read_state()))
            if not serial:
                infos.append(mod.state_spec())
        res[serial] = outs
    assert_same(res[False], res[True])
    for i in infos:
        print({k: i[k] for k in ("levels", "warmup_blocks", "differed", "serial_reruns", "chain", "disabled")})
    # the loud renders: the first level met the State; a quiet render
    # learnt that way needed the second level (launched for this) and came
    # out exact
    assert infos[0]["used"] and infos[2]["levels"] == 1, infos
    assert any(i["levels"] > 1 for i in infos[3:]), infos
