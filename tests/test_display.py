"""Display reductions: the oracle restates the
reference's IR-view decimation (opengl.h:877-890) including its initial
values; the GPU reductions match the oracle exactly (max / min are exact)."""
import numpy as np
import pytest

import dspbench as d


def test_oracle_minmax_quirks(oracle):
    # pixels start at {max = -1, min = +1}: an all-positive pixel keeps min = 1
    x = np.array([0.5, 0.25, 2.0, 3.0], np.float32)
    vmax, vmin = oracle.minmax_decimate(x, 2)
    assert list(vmax) == [0.5, 3.0] and list(vmin) == [0.25, 1.0]
    vmax, vmin = oracle.minmax_decimate(np.array([-5.0], np.float32), 3)   # empty pixels
    assert list(vmax) == [-1.0, -1.0, -1.0] and list(vmin) == [-5.0, 1.0, 1.0]


def test_oracle_minmax_matches_literal_loop(oracle):
    rng = np.random.default_rng(2)
    x = (rng.standard_normal(1001) * 2).astype(np.float32)
    P = 37
    mx, mn = np.full(P, -1.0, np.float32), np.full(P, 1.0, np.float32)
    for s, v in enumerate(x):          # opengl.h:881-889
        p = s * P // len(x)
        mx[p], mn[p] = max(mx[p], v), min(mn[p], v)
    vmax, vmin = oracle.minmax_decimate(x, P)
    assert np.array_equal(vmax, mx) and np.array_equal(vmin, mn)


def test_oracle_spectrogram(oracle):
    rng = np.random.default_rng(3)
    m = rng.random((50, 7), dtype=np.float32)
    out = oracle.spectrogram_decimate(m, 8)
    for p in range(8):
        rows = [f for f in range(50) if f * 8 // 50 == p]
        assert np.array_equal(out[p], m[rows].max(axis=0))


@pytest.mark.gpu
@pytest.mark.parametrize("n,P", [(1, 1), (10, 37), (1000, 1000), (999_983, 1920), (48_000 * 60 + 3, 4096)])
def test_gpu_minmax(torch_cuda, oracle, n, P):
    x = (np.random.default_rng(n).standard_normal(n) * 1.5).astype(np.float32)
    vmax, vmin = d.minmax_decimate(torch_cuda.from_numpy(x).cuda(), P)
    rmax, rmin = oracle.minmax_decimate(x, P)
    assert np.array_equal(vmax.cpu().numpy(), rmax) and np.array_equal(vmin.cpu().numpy(), rmin)
    hmax, hmin = d.minmax_decimate(x, P)    # host buffers
    assert np.array_equal(hmax, rmax) and np.array_equal(hmin, rmin)


@pytest.mark.gpu
@pytest.mark.parametrize("F,K,P", [(5, 4097, 3), (1000, 4097, 640), (37, 100, 37), (10, 8, 64)])
def test_gpu_spectrogram(torch_cuda, oracle, F, K, P):
    m = np.random.default_rng(F).random((F, K), dtype=np.float32)
    got = d.spectrogram_decimate(torch_cuda.from_numpy(m).cuda(), P).cpu().numpy()
    assert np.array_equal(got, oracle.spectrogram_decimate(m, P))


@pytest.mark.gpu
def test_gpu_overview_of_a_long_stft(torch_cuda, oracle):
    """STFT of 10 min stereo -> 1920-column overview, vs the oracle on the
    same magnitudes."""
    torch = torch_cuda
    x = (torch.rand((1, 48_000 * 600), device="cuda") * 2 - 1)
    mag = d.stft_magnitude(x)[0]
    got = d.spectrogram_decimate(mag, 1920).cpu().numpy()
    assert np.array_equal(got, oracle.spectrogram_decimate(mag.cpu().numpy(), 1920))
