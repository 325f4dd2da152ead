"""DSP_PLUGIN_BIQUAD on the CPU: the oracle's cascade restatement and its
error bound, the kind's plan (dsp_biquad_plan, host only), and our biquad
plugin built for the CPU the way the reference's JIT builds a plugin
(oracle/_ref/libplug_biquad.so, -Ofast) against the float64 cascade.
The GPU side is tests/test_gpu_biquad.py."""
import ctypes as C
import math

import numpy as np
import pytest

import dspbench as d


def rbj_lp(fc, q, sr=48000.0):
    return d.Plugin.biquad_lowpass_coefficients(fc, q, sr)[0]


def plan(coef):
    c = np.ascontiguousarray(np.asarray(coef, np.float32).reshape(-1, 5))
    w = C.c_uint32()
    st = d.lib().dsp_biquad_plan(c.ctypes.data_as(C.c_void_p), c.shape[0], C.byref(w))
    return st, w.value


@pytest.mark.parametrize("S", [1, 2, 4])
def test_serial_fp32_chain_is_within_the_bound(oracle, S):
    """The bound the GPU kind is held to also holds for the serial fp32
    chain evaluated as plugins/biquad.cpp writes it."""
    rng = np.random.default_rng(S)
    coef = np.array([rbj_lp(float(rng.uniform(60, 12000)), float(rng.uniform(0.5, 3))) for _ in range(S)],
                    np.float32)
    x = rng.uniform(-1, 1, 20_000).astype(np.float32)
    y64, lmax = oracle.biquad_f64(x, coef, 20_480)
    y32 = oracle.biquad_f32(x, coef, 20_480)
    bound = oracle.biquad_error_bound(coef, lmax)
    err = float(np.max(np.abs(y32.astype(np.float64) - y64)))
    assert 0 < err <= bound, (err, bound)


def test_oracle_f64_is_the_difference_equation(oracle):
    """One section by hand: y = b0 x + b1 x1 + b2 x2 - a1 y1 - a2 y2."""
    coef = np.array([0.5, 0.25, -0.125, -0.3, 0.2], np.float32)
    x = np.array([1, 2, -1, 0.5, 0, 0, 3], np.float32)
    y, _ = oracle.biquad_f64(x, coef, 9)
    want, x1, x2, y1, y2 = [], 0.0, 0.0, 0.0, 0.0
    b0, b1, b2, a1, a2 = (float(v) for v in coef)
    for v in list(map(float, x)) + [0.0, 0.0]:
        yy = b0 * v + b1 * x1 + b2 * x2 - a1 * y1 - a2 * y2
        x2, x1, y2, y1 = x1, v, y1, yy
        want.append(yy)
    assert np.allclose(y, want, rtol=0, atol=1e-15)


def test_plan_windows():
    assert plan([rbj_lp(1000.0, 0.7071)]) == (0, 1)        # decays inside one 2048-sample tile
    st, w = plan([rbj_lp(20.0, 10.0)])
    assert st == 0 and 64 < w <= 192                        # three windows of 64 lanes
    th = 2 * math.pi * 440 / 48000
    assert plan([[1, 0, 0, -2 * math.cos(th), 0.9999999]]) == (0, 0)   # no decay: chained look-back
    assert plan([[1, 0, 0, 0.5, 2.0]]) == (0, 0)           # unstable: chained look-back
    assert plan([rbj_lp(1000.0, 0.7071)] * 4)[0] == 0
    assert plan([rbj_lp(1000.0, 0.7071)] * 5)[0] == d._lib.DSP_ERR_INVALID
    assert plan([[float("nan"), 0, 0, 0, 0]])[0] == d._lib.DSP_ERR_INVALID


def test_cpu_built_plugin_within_the_bound(oracle):
    """plugins/biquad.cpp built with the reference JIT's flags (-Ofast
    -ffast-math: the compiler may contract and reassociate the difference
    equation) and pumped block by block by the oracle's render loop: within
    the float64 bound -- the CPU baseline of the biquad bench lines."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    ref = oracle.RefPlugin("biquad", 2, 48000.0, prefix="libplug_")
    coef = np.frombuffer(ref.state.tobytes()[:20], np.float32).reshape(1, 5)
    assert np.allclose(coef, d.Plugin.biquad_lowpass_coefficients(1000.0, 0.7071, 48000.0), rtol=1e-6)
    x = np.random.default_rng(9).uniform(-1, 1, (2, 30_000)).astype(np.float32)
    got = oracle.render_offline([x[0], x[1]], 2, 512, 48000.0, ref.as_oracle())
    for c in range(2):
        y64, lmax = oracle.biquad_f64(x[c], coef, got.shape[1])
        assert float(np.max(np.abs(got[c] - y64))) <= oracle.biquad_error_bound(coef, lmax)
