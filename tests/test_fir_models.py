"""The numpy models of the overlap-save FIR index math (tools/): the
product's one-wave 8192-point kernel (olsave_model.py) and the next one,
an 8192-point channel-pair frame over two waves (ols2w_model.py),
against np.convolve in float64 (CPU)."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_two_wave_pair_frame_model():
    m = _load("ols2w_model")
    rng = np.random.default_rng(3)
    for L, T in [(7168 * 2 + 999, 1024), (333, 1025), (20_000, 5)]:
        taps = rng.standard_normal(T) / np.sqrt(T)
        x0, x1 = rng.uniform(-1, 1, L), rng.uniform(-1, 1, L)
        y = m.render(x0, x1, taps)
        assert np.abs(y.real - np.convolve(x0, taps)[:L]).max() < 1e-9
        assert np.abs(y.imag - np.convolve(x1, taps)[:L]).max() < 1e-9


def test_dif_two_wave_frame_model():
    """The algebra and H table layout of round 4's two-wave FIR attempt
    (fir_dif2_kernel, removed: 62% slower; tools/olsdif_model.py):
    decimation in frequency over the two waves, one exchange of outputs."""
    m = _load("olsdif_model")
    rng = np.random.default_rng(5)
    for L, T in [(7168 * 2 + 4321, 1024), (777, 1025), (15_000, 3)]:
        taps = rng.standard_normal(T) / np.sqrt(T)
        x0, x1 = rng.uniform(-1, 1, L), rng.uniform(-1, 1, L)
        y = m.render(x0, x1, taps)
        assert np.abs(y.real - np.convolve(x0, taps)[:L]).max() < 1e-9
        assert np.abs(y.imag - np.convolve(x1, taps)[:L]).max() < 1e-9
