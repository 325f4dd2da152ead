"""The oracle pinned against the reference (CPU only).

  * golden vectors (tests/golden/make_golden.py): the reference's own unit
    test expectations K1-K3/K6, the IR-analysis KATs K4/K5, one-shot render
    hashes through the reference plugins, a float64 STFT;
  * the C restatement (oracle.c) against those vectors and against the
    reference plugins compiled from their sources (oracle/_ref), when present.
"""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden_v1.npz"))
META = json.load(open(os.path.join(HERE, "golden", "golden_v1.json")))
PEAK_REL_TOL = 1e-6


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def peak_rel(m, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(np.asarray(m, np.float64) - ref)) / np.max(ref))


def uniform(seed, shape):
    return (np.random.default_rng(seed).random(shape) * 2.0 - 1.0).astype(np.float32)


needs_ref = pytest.mark.skipif(not __import__("oracle").ref_available(),
                               reason="oracle/_ref not built (needs /root/reference at build time)")


# ---- the reference's own unit tests (test/tests.cpp) -------------------------

def test_k1_static_gain(oracle):
    x = np.arange(512, dtype=np.float32)[None, :]
    out = oracle.callback_once(oracle.restated_plugin("static_gain_plugin"), x.copy())[0]
    assert np.array_equal(out, G["k1_out"])
    assert np.allclose(out, np.arange(512) * 0.1, atol=1e-3 * 512)  # the reference's float_cmp
    assert np.array_equal(out, np.arange(512, dtype=np.float32) * np.float32(0.1))


def test_k2_no_op(oracle):
    x = np.arange(512, dtype=np.float32)[None, :]
    out = oracle.callback_once(oracle.restated_plugin("no_op"), x.copy())[0]
    assert np.array_equal(out, G["k2_out"]) and np.array_equal(out, x[0])


def test_k3_plugin_with_parameters_defaults():
    p, s = G["k3_params"], G["k3_state"]
    assert np.frombuffer(p[:4].tobytes(), "<i4")[0] == 0
    assert abs(np.frombuffer(p[4:8].tobytes(), "<f4")[0] - 0.9) < 1e-3
    assert np.frombuffer(p[8:12].tobytes(), "<i4")[0] == 0
    assert abs(np.frombuffer(s[:4].tobytes(), "<f4")[0] - 0.1) < 1e-3


def test_k6_normalisation(oracle):
    L = oracle.lib()
    nv = L.oracle_normalize_int(4, 8, 6.0)
    assert nv == 0.5 and L.oracle_denormalize_int(4, 8, nv) == 6
    nf = L.oracle_normalize_float(4.0, 8.0, 0, 6.0)
    assert nf == 0.5 and L.oracle_denormalize_float(4.0, 8.0, 0, nf) == 6.0
    # enum {0, 1, 256}: value 256 -> index 2 -> normalised -> index 2 -> 256
    ni = L.oracle_normalize_enum_index(3, 2)
    assert L.oracle_denormalize_enum_index(3, ni) == 2


# ---- IR analysis KATs ----------------------------------------------------

def test_k4_gain_test_ir_magnitude_is_flat(oracle):
    assert np.allclose(G["k4_mag"], META["k4_flat"], rtol=1e-12)
    m = oracle.c_ir_magnitude(G["ir_gain_test"][0])
    assert peak_rel(m, G["k4_mag"]) <= 1e-12


def test_k5_ir_test_ir_magnitude(oracle):
    ir = G["ir_IR_test"][0]
    assert np.array_equal(ir, oracle.ir_ramp_reference(0.9, 0.002, 2048))
    m = oracle.c_ir_magnitude(ir)
    assert peak_rel(m, G["k5_mag"]) <= 1e-12
    for k, v in META["k5_bins"].items():
        assert abs(m[int(k)] - v) <= 1e-9 * abs(v) + 1e-15
    assert m[8191] == pytest.approx(m[1], rel=1e-12)
    # the published KAT values
    assert m[0] == pytest.approx(14.009141585190642, rel=1e-12)
    assert m[4096] == pytest.approx(0.0018101951313910219, rel=1e-9)


# ---- render: restated callbacks vs reference vectors ----------------------

@pytest.mark.parametrize("key", ["r1", "r2", "r3"])
def test_render_offline_matches_reference_hash(oracle, key):
    r = META["renders"][key]
    sig = uniform(r["seed"], (r["in_channels"], r["L"]))
    out = oracle.render_offline([sig[c] for c in range(r["in_channels"])], r["out_channels"], r["B"],
                                48000.0, oracle.restated_plugin(r["plugin"]))
    assert list(out.shape) == r["shape"]
    assert np.array_equal(out[:, :256], G[f"{key}_head"])
    assert np.array_equal(out[:, -256:], G[f"{key}_tail"])
    assert sha(out) == r["sha256"]


def test_ir_test_callback_matches_reference_ir(oracle):
    imp = np.zeros((2, 2048), np.float32)
    imp[:, 0] = 1
    out = oracle.callback_once(oracle.restated_plugin("IR_test"), imp, 48000.0)
    assert np.array_equal(out, G["ir_IR_test"])
    imp = np.zeros((2, 2048), np.float32)
    imp[:, 0] = 1
    out = oracle.callback_once(oracle.restated_plugin("gain_test"), imp, 48000.0)
    assert np.array_equal(out, G["ir_gain_test"])


def test_render_edge_cases(oracle):
    """one-shot semantics (ref audio.cpp:13-175): zero past EOF, zero extra
    channels, empty file, B = 1, file with more channels than the device."""
    x = uniform(5, (3, 1001))
    plug = oracle.restated_plugin("gain_test")
    out = oracle.render_offline([x[0], x[1], x[2]], 2, 64, 48000.0, plug)   # C_file > C
    assert out.shape == (2, 1024)
    assert np.array_equal(out[:, :1001], x[:2] * np.float32(0.2))
    assert not out[:, 1001:].any()
    out = oracle.render_offline([x[0]], 3, 1, 48000.0, plug)                  # extra channels, B = 1
    assert np.array_equal(out[0], x[0] * np.float32(0.2)) and not out[1:].any()
    out = oracle.render_offline([np.zeros(0, np.float32)], 2, 512, 48000.0, plug, L=0)  # empty
    assert out.shape[1] == 0
    ir = oracle.render_offline([x[0]], 1, 100, 48000.0, oracle.restated_plugin("IR_test"))
    ramp = oracle.ir_ramp_reference(0.9, 0.002, 100)
    assert all(np.array_equal(ir[0, b * 100:(b + 1) * 100], ramp) for b in range(11))


def test_render_loop_wraps(oracle):
    x = uniform(6, (2, 1000))
    out, cur = oracle.render_loop([x[0], x[1]], 2, 256, 8, 48000.0, oracle.restated_plugin("no_op"))
    want = np.concatenate([x, x, x], axis=1)[:, :2048]
    assert np.array_equal(out, want) and cur == 2048 % 1000


@needs_ref
@pytest.mark.parametrize("name", ["gain_test", "IR_test", "static_gain_plugin", "no_op"])
@pytest.mark.parametrize("B", [1, 64, 512, 2048])
def test_restated_callbacks_equal_reference_plugins(oracle, name, B):
    x = uniform(7, (2, 3000))
    ref = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.RefPlugin(name, 2).as_oracle())
    got = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.restated_plugin(name))
    assert np.array_equal(ref, got)


@needs_ref
def test_stateful_reference_plugin_vector(oracle):
    sp = oracle.RefPlugin("sine_test", 2, 48000.0)
    blocks = [oracle.callback_once(sp.as_oracle(), np.zeros((2, 512), np.float32), 48000.0) for _ in range(4)]
    assert np.array_equal(np.concatenate(blocks, axis=1), G["p1_sine_test"])


# ---- spectral restatement ---------------------------------------------------

def test_windows(oracle):
    for kind in (oracle.WIN_HAMMING, oracle.WIN_HANN, oracle.WIN_RECT):
        for n in (2, 3, 2048, 8192):
            w = oracle.c_window_f32(kind, n)
            assert np.max(np.abs(w - oracle.np_window(kind, n))) <= 6e-8
    w = oracle.np_window(oracle.WIN_HAMMING, 2048)
    assert w[0] == pytest.approx(0.08) and w[-1] == pytest.approx(0.08)


def test_stft_restatements_match_golden(oracle):
    x = G["s1_signal"]
    ref = G["s1_mag"].astype(np.float64)
    assert peak_rel(oracle.np_stft_mag(x, 8192, 4096, oracle.WIN_HANN, 4097), ref) <= 1e-7
    assert peak_rel(oracle.c_stft_mag_f64(x, 8192, 4096, oracle.WIN_HANN, 4097), ref) <= 1e-7
    assert peak_rel(oracle.c_stft_mag_f32(x, 8192, 4096, oracle.WIN_HANN, 4097, 2), ref) <= PEAK_REL_TOL
    full = oracle.c_stft_mag_f64(x[:8192], 8192, 4096, oracle.WIN_HAMMING, 8192)
    assert peak_rel(full, G["s1_mag_hamming_full"]) <= 1e-7


def test_fft_roundtrip_and_scaling(oracle):
    rng = np.random.default_rng(9)
    for n in (2, 8, 1024, 8192):
        x = rng.standard_normal(n)
        re, im = oracle.c_fft_f64(x, np.zeros(n), -1)
        ref = np.fft.fft(x) / np.sqrt(n)                     # IPP_FFT_DIV_BY_SQRTN
        assert np.allclose(re + 1j * im, ref, atol=1e-12 * np.sqrt(n))
        br, bi = oracle.c_fft_f64(re, im, +1)
        assert np.allclose(br, x, atol=1e-12) and np.allclose(bi, 0, atol=1e-12)


@pytest.mark.parametrize("L,N,H", [(0, 8192, 4096), (8191, 8192, 4096), (8192, 8192, 4096),
                                   (8192 + 4095, 8192, 4096), (8192 + 4096, 8192, 4096), (100, 16, 7)])
def test_frame_count(oracle, L, N, H):
    assert oracle.stft_frames(L, N, H) == oracle.lib().oracle_stft_frames(L, N, H)
    assert oracle.stft_frames(L, N, H) == (0 if L < N else (L - N) // H + 1)


@needs_ref
@pytest.mark.parametrize("name", ["gain_test", "IR_test", "sine_test", "buffer_test", "handmade_test",
                                  "template_plugin", "static_gain_plugin", "no_op", "plugin_with_parameters"])
def test_reference_plugins_load_beside_the_product(oracle, name):
    """The reference plugins bind their services to oracle/ref_services.c
    even with libdspbench.so (same symbol names) loaded globally first."""
    import dspbench
    dspbench.lib()
    r = oracle.RefPlugin(name, 2, 48000.0)
    out = oracle.callback_once(r.as_oracle(), np.zeros((2, 64), np.float32), 48000.0)
    assert np.all(np.isfinite(out))
