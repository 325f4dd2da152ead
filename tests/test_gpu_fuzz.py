"""Seeded random cases of the fused render + STFT (dsp_render_stft) against
the oracle: the parametrized parity tests pin chosen shapes, these draw the
shape, the plugin and its parameters, the block size, the window, the hop and
the stored bins at random, so combinations nobody listed are covered too.

Bars as in test_gpu_parity.py: the render bit-exact against the oracle's
block loop (audio.cpp:13-175 restated, oracle/oracle.c), the magnitudes within
1e-6 of each frame's peak against the float64 STFT of the oracle's render.
"""
import numpy as np
import pytest

import dspbench as d

pytestmark = pytest.mark.gpu

PEAK_REL_TOL = 1e-6
N_CASES = 40


def peak_rel_err(m, ref):
    m = np.asarray(m, np.float64)
    ref = np.asarray(ref, np.float64)
    assert m.shape == ref.shape, (m.shape, ref.shape)
    peak = np.maximum(ref.max(axis=-1), 1e-30)
    return float(np.max(np.abs(m - ref).max(axis=-1) / peak))


def draw(seed):
    """One case: (plugin name, params, C_out, C_in, L, B, window, H, K)."""
    r = np.random.default_rng(seed)
    name = ["IR_test", "gain_test", "static_gain_plugin", "no_op"][int(r.integers(4))]
    if name == "IR_test":
        params = [float(np.float32(r.uniform(-1.0, 1.0))), float(np.float32(r.uniform(-0.01, 0.01)))]
    elif name == "gain_test":
        params = [float(np.float32(r.uniform(0.0, 2.0)))]
    elif name == "static_gain_plugin":
        params = [float(np.float32(r.uniform(0.0, 1.0)))]
    else:
        params = []
    C_out = int(r.integers(1, 4))
    C_in = int(r.integers(0, C_out + 2))
    B = int(r.choice([1, 3, 64, 100, 128, 256, 384, 512, 640, 1000, 1024, 2048, 4096]))
    L = int(r.integers(1, 60_000))
    window = int(r.choice([d.DSP_WIN_HANN, d.DSP_WIN_HAMMING, d.DSP_WIN_RECT]))
    H = int(r.choice([4096, 4096, 2048, 1000, 8192]))
    K = int(r.choice([4097, 4097, 8192, int(r.integers(1, 4097))]))
    return name, params, C_out, C_in, L, B, window, H, K


def device_plugin(name, params):
    if name == "IR_test":
        return d.Plugin.ir_test(*params)
    if name == "gain_test":
        return d.Plugin.gain_test(*params)
    if name == "static_gain_plugin":
        return d.Plugin.static_gain(*params)
    return d.Plugin.no_op()


def oracle_plugin(oracle, name, params):
    if name == "static_gain_plugin":
        return oracle.restated_plugin(name, state=params)
    return oracle.restated_plugin(name, params=params if params else None)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_render_stft_random_case(torch_cuda, oracle, seed):
    torch = torch_cuda
    name, params, C_out, C_in, L, B, window, H, K = draw(1000 + seed)
    x = np.random.default_rng(seed).uniform(-1.0, 1.0, (max(C_in, 1), L)).astype(np.float32)[:C_in]
    ref = oracle.render_offline([x[c] for c in range(C_in)], C_out, B, 48000.0,
                                oracle_plugin(oracle, name, params), L=L)
    file = torch.from_numpy(np.ascontiguousarray(x)).cuda() if C_in else None
    out, mag = d.render_stft(file, C_out, B, 48000.0, device_plugin(name, params), N=8192, H=H,
                             window=window, K=K, L_file=L, ref=torch.empty(1, device="cuda"))
    out = out.cpu().numpy()
    mag = mag.cpu().numpy()
    case = (name, params, C_out, C_in, L, B, window, H, K)
    assert out.shape == ref.shape, case
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), case
    Kref = K if K <= 4097 else 8192
    for c in range(C_out):
        mref = oracle.np_stft_mag(ref[c], 8192, H, window, Kref)
        if mref.shape[0] == 0:
            assert mag.shape[1] <= 1, case  # no whole frame: nothing (or a placeholder row) stored
            continue
        assert mag.shape[1] == mref.shape[0], case
        assert peak_rel_err(mag[c], mref) <= PEAK_REL_TOL, case


# ---- plugins compiled from the reference sources (DSP_PLUGIN_GENERIC) ------
# The same draw for the generic driver: a stock plugin compiled unchanged by
# the product's plugin compiler (dsp-bench_amd/modules/mod_*.co) against the
# same source compiled for the CPU with the JIT flags (oracle/_ref), whose
# default parameters and state both sides start from.
from test_gpu_module import EXACT, TOL, have, load  # noqa: E402

GENERIC = EXACT + sorted(TOL)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_generic_render_stft_random_case(torch_cuda, oracle, seed):
    torch = torch_cuda
    _, _, C_out, C_in, L, B, window, H, K = draw(2000 + seed)
    name = GENERIC[seed % len(GENERIC)]
    if not have(name):
        pytest.skip("modules / oracle/_ref not built")
    mod = load(name)
    params = mod.default_parameters()
    mod.initialize_state(params, C_out, 48000.0)
    refp = oracle.RefPlugin(name, C_out, 48000.0)
    x = np.random.default_rng(seed).uniform(-1.0, 1.0, (max(C_in, 1), L)).astype(np.float32)[:C_in]
    want = oracle.render_offline([x[c] for c in range(C_in)], C_out, B, 48000.0, refp.as_oracle(), L=L)
    file = torch.from_numpy(np.ascontiguousarray(x)).cuda() if C_in else None
    out, mag = d.render_stft(file, C_out, B, 48000.0, mod.plugin(params, name), N=8192, H=H,
                             window=window, K=K, L_file=L, ref=torch.empty(1, device="cuda"))
    got = out.cpu().numpy()
    mag = mag.cpu().numpy()
    case = (name, C_out, C_in, L, B, window, H, K)
    assert got.shape == want.shape, case
    if name in TOL:
        assert np.max(np.abs(got - want)) <= TOL[name], case
    else:
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), case
    Kref = K if K <= 4097 else 8192
    for c in range(C_out):
        # the spectra of the GPU's own render (for the TOL plugins the render
        # itself differs from the CPU's in the last ulp)
        mref = oracle.np_stft_mag(got[c], 8192, H, window, Kref)
        if mref.shape[0] == 0:
            assert mag.shape[1] <= 1, case
            continue
        assert mag.shape[1] == mref.shape[0], case
        assert peak_rel_err(mag[c], mref) <= PEAK_REL_TOL, case


# ---- the memory-source STFT and loop mode ----------------------------------
@pytest.mark.parametrize("seed", range(24))
def test_stft_magnitude_random_case(torch_cuda, oracle, seed):
    """dsp_stft_magnitude (fft_perform_and_get_magnitude per frame,
    dsp.cpp:208-271 restated): a random power-of-two size (the 8192-point
    kernel and the generic one), hop, window and stored bins."""
    torch = torch_cuda
    r = np.random.default_rng(3000 + seed)
    N = int(2 ** r.integers(4, 14))
    H = int(r.choice([N // 2, N, max(1, N // 4), int(r.integers(1, 2 * N))]))
    window = int(r.choice([d.DSP_WIN_HANN, d.DSP_WIN_HAMMING, d.DSP_WIN_RECT]))
    K = int(r.choice([N // 2 + 1, int(r.integers(1, N // 2 + 2))]))
    C = int(r.integers(1, 4))
    L = int(r.integers(N, N * 6 + 1))
    x = np.random.default_rng(seed).uniform(-1.0, 1.0, (C, L)).astype(np.float32)
    mag = d.stft_magnitude(torch.from_numpy(x).cuda(), N=N, H=H, window=window, K=K).cpu().numpy()
    case = (N, H, window, K, C, L)
    for c in range(C):
        mref = oracle.np_stft_mag(x[c], N, H, window, K)
        assert mag.shape[1] == mref.shape[0], case
        assert peak_rel_err(mag[c], mref) <= PEAK_REL_TOL, case


@pytest.mark.parametrize("seed", range(24))
def test_render_loop_random_case(torch_cuda, oracle, seed):
    """Loop mode (audio.cpp:100-132): the file wraps from a random cursor;
    bit-exact against oracle_render_loop, and the next cursor agrees."""
    torch = torch_cuda
    name, params, C_out, C_in, L, B, _, _, _ = draw(4000 + seed)
    C_in = max(C_in, 1)  # loop mode wraps a file: at least one channel
    nblocks = int(np.random.default_rng(seed).integers(1, 200))
    cursor = int(np.random.default_rng(seed + 1).integers(0, L))
    x = np.random.default_rng(seed).uniform(-1.0, 1.0, (C_in, L)).astype(np.float32)
    want, wcur = oracle.render_loop([x[c] for c in range(C_in)], C_out, B, nblocks, 48000.0,
                                    oracle_plugin(oracle, name, params), cursor=cursor)
    got, gcur = d.render_loop(torch.from_numpy(x).cuda(), C_out, B, nblocks, 48000.0, device_plugin(name, params),
                              cursor=cursor)
    case = (name, params, C_out, C_in, L, B, nblocks, cursor)
    assert gcur == wcur, case
    got = got.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), np.asarray(want, np.float32).view(np.uint32)), case


# ---- the FIR (DSP_PLUGIN_FIR, build-defined cfg 3b) -------------------------
# Random taps count (both kernels: overlap-save for T <= 1025, the direct form
# above and when asked), channel counts (overlap-save pairs channels as one
# complex signal, an odd last one runs alone), file channels, lengths and
# block sizes, against the float64 convolution.  Bars as test_gpu_fir.py: the
# direct form within its rigorous bound, overlap-save within OLS_TOL of the
# pair's peak.
from test_gpu_fir import OLS_TOL, U  # noqa: E402


@pytest.mark.parametrize("seed", range(24))
def test_fir_random_case(torch_cuda, oracle, seed):
    r = np.random.default_rng(5000 + seed)
    T = int(r.choice([1, 2, 15, 16, 17, 255, 1023, 1024, 1025, 1026, 2048, int(r.integers(1, 2049))]))
    direct = bool(r.integers(2)) if T <= 1025 else True
    C_out = int(r.integers(1, 7))
    C_in = int(r.integers(0, C_out + 2))
    L = int(r.integers(1, 40_000))
    B = int(r.choice([1, 7, 64, 512, 1000, 4096]))
    taps = (r.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    x = r.uniform(-1, 1, (max(C_in, 1), L)).astype(np.float32)[:C_in]
    file = torch_cuda.from_numpy(np.ascontiguousarray(x)).cuda() if C_in else None
    Ly = -(-L // B) * B
    dst = torch_cuda.empty((C_out, Ly), device="cuda")
    out = d.render_offline(file, C_out, B, 48000.0, d.Plugin.fir(taps, direct=direct), out=dst,
                           L_file=L).cpu().numpy()
    case = (T, direct, C_out, C_in, L, B)
    assert out.shape == (C_out, Ly), case
    y64 = [oracle.fir_f64(x[c] if c < C_in else None, taps, Ly) for c in range(C_out)]
    for c in range(C_out):
        if c >= C_in:
            assert not out[c].any(), case  # a channel the file lacks: exact zeros
            continue
        err = np.abs(out[c].astype(np.float64) - y64[c])
        if direct:
            bound = oracle.fir_f64(np.abs(x[c]), np.abs(taps), Ly) * (T + 1) * U
            assert np.all(err <= bound + 1e-30), case
        else:
            pair = [p for p in (c - c % 2, c - c % 2 + 1) if p < C_out and p < C_in]
            peak = max(float(np.max(np.abs(y64[p]))) for p in pair)
            assert float(np.max(err)) <= OLS_TOL * max(peak, 1e-30), case
