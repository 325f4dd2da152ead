"""FIR render (build-defined cfg 3b, BASELINE configs[2]): a 1024-tap FIR
whose taps are compute_IR(IR_test)[0:1024], over 48 kHz stereo in 512-sample
blocks.  The reference ships no FIR plugin; the oracle is the float64
convolution (oracle_fir_f64, pinned to numpy.convolve on CPU).

Tolerance (floating point): the GPU sums the T products of each output in
order k = 0..T-1 in fp32 with FMAs, so |y - y64| <= (T + 1) u sum_k
|h_k x_{n-k}| with u = 2^-24 -- checked per sample against that bound.
"""
import os

import numpy as np
import pytest

import dspbench as d

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden_v1.npz"))
U = 2.0 ** -24


def cfg3b_taps():
    return G["ir_IR_test"][0][:1024].copy()   # compute_IR(IR_test) of the reference plugin


# overlap-save: max |y - y64| <= OLS_TOL * max |y64| (fp32 FFT round trip); the
# channels of a pair (fir_pair_kernel) share one complex transform, so for them
# the max is the pair's (test_gpu_fir_pair_shares_its_rounding)
OLS_TOL = 2e-6


@pytest.fixture(params=[1, 2], ids=["direct", "ols"])
def fir_method(request):
    """Both FIR kernels: 1 = direct form (DSP_EXEC_FIR_DIRECT), 2 = FFT
    overlap-save (the default for T <= 1025)."""
    return request.param


def fplug(taps, method):
    return d.Plugin.fir(taps, direct=(method == 1))


def check_fir(oracle, y, x, taps, Ly, method=1):
    y64 = oracle.fir_f64(x, taps, Ly)
    err = np.abs(y.astype(np.float64) - y64)
    if method == 2 and len(taps) <= 1025:
        assert float(np.max(err)) <= OLS_TOL * max(float(np.max(np.abs(y64))), 1e-30), float(np.max(err))
        return
    bound = oracle.fir_f64(np.abs(x) if x is not None else None, np.abs(taps), Ly) * (len(taps) + 1) * U
    assert np.all(err <= bound + 1e-30), float(np.max(err - bound))


def test_oracle_fir_is_numpy_convolve(oracle):
    rng = np.random.default_rng(0)
    x, h = rng.standard_normal(3000).astype(np.float32), rng.standard_normal(77).astype(np.float32)
    ref = np.convolve(x.astype(np.float64), h.astype(np.float64))[:3072]
    want = np.zeros(3072)
    want[:ref.size] = ref
    assert np.max(np.abs(oracle.fir_f64(x, h, 3072) - want)) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 7, 8, 16, 17, 64, 1024, 1031, 2048])
@pytest.mark.parametrize("L,B", [(100, 512), (5000, 100), (70_001, 512)])
def test_gpu_fir_render(torch_cuda, oracle, fir_method, T, L, B):
    rng = np.random.default_rng(T * 7 + L)
    x = rng.uniform(-1, 1, (2, L)).astype(np.float32)
    taps = (rng.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    out = d.render_offline(torch_cuda.from_numpy(x).cuda(), 2, B, 48000.0, fplug(taps, fir_method)).cpu().numpy()
    Ly = -(-L // B) * B
    assert out.shape == (2, Ly)
    for c in range(2):
        check_fir(oracle, out[c], x[c], taps, Ly, fir_method)
    host = d.render_offline(x, 2, B, 48000.0, fplug(taps, fir_method))          # host buffers
    assert np.array_equal(host, out)


@pytest.mark.gpu
def test_gpu_fir_channels_and_missing_input(torch_cuda, oracle, fir_method):
    x = np.random.default_rng(5).uniform(-1, 1, (1, 9000)).astype(np.float32)
    taps = cfg3b_taps()
    out = d.render_offline(torch_cuda.from_numpy(x).cuda(), 3, 512, 48000.0, fplug(taps, fir_method)).cpu().numpy()
    check_fir(oracle, out[0], x[0], taps, out.shape[1], fir_method)
    assert not out[1:].any()   # extra channels: zero input through the FIR


@pytest.mark.gpu
@pytest.mark.parametrize("C,in_ch", [(1, 1), (3, 3), (4, 4), (5, 4), (4, 3), (17, 17)])
@pytest.mark.parametrize("L,B", [(3073, 64), (6144, 512), (12_289, 1)])
def test_gpu_fir_channel_counts(torch_cuda, oracle, fir_method, C, in_ch, L, B):
    """Overlap-save runs channel pairs as one complex signal (fir_pair_kernel)
    and an odd last channel on its own (fir_fft_kernel): odd and even counts,
    a pair with its second channel missing, more than one launch's 16
    channels, lengths at and beside the pair kernel's 3072-sample hop."""
    rng = np.random.default_rng(C * 1000 + L)
    x = rng.uniform(-1, 1, (in_ch, L)).astype(np.float32)
    taps = (rng.standard_normal(1024) / 32).astype(np.float32)
    out = d.render_offline(torch_cuda.from_numpy(x).cuda(), C, B, 48000.0, fplug(taps, fir_method)).cpu().numpy()
    Ly = -(-L // B) * B
    assert out.shape == (C, Ly)
    for c in range(C):
        if c < in_ch:
            check_fir(oracle, out[c], x[c], taps, Ly, fir_method)
        else:
            assert not out[c].any()


@pytest.mark.gpu
def test_gpu_fir_pair_shares_its_rounding(torch_cuda, oracle):
    """Overlap-save transforms a channel pair as one complex signal, so a
    channel's rounding error is bounded by the PAIR's peak: a quiet channel
    beside a loud one (60 dB down), and a silent one, stay within OLS_TOL of
    the pair's peak; a channel the file lacks is exact zeros."""
    rng = np.random.default_rng(12)
    L = 50_000
    loud = rng.uniform(-1, 1, L).astype(np.float32)
    x = np.stack([loud, (rng.uniform(-1, 1, L) * 1e-3).astype(np.float32), np.zeros(L, np.float32)])
    taps = cfg3b_taps()
    out = d.render_offline(torch_cuda.from_numpy(x).cuda(), 4, 512, 48000.0, fplug(taps, 2)).cpu().numpy()
    y64 = [oracle.fir_f64(x[c], taps, out.shape[1]) for c in range(3)]
    peak01 = max(np.max(np.abs(y64[0])), np.max(np.abs(y64[1])))
    for c in (0, 1):
        assert np.max(np.abs(out[c] - y64[c])) <= OLS_TOL * peak01
    # channels 2 (silent) and 3 (missing) form the second pair: both exact zeros
    assert not out[2].any() and not out[3].any()


@pytest.mark.gpu
def test_gpu_fir_cfg3b_full_size(torch_cuda, oracle, fir_method):
    """cfg 3b at full size: 10 min of 48 kHz stereo, B = 512, the 1024 IR_test
    taps; 4000 sampled outputs + both ends against float64."""
    torch = torch_cuda
    L = 28_800_000
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.rand((2, L), device="cuda", generator=g) * 2 - 1
    taps = cfg3b_taps()
    out = d.render_offline(x, 2, 512, 48000.0, fplug(taps, fir_method))
    rng = np.random.default_rng(1)
    idx = np.concatenate([np.arange(2048), np.arange(L - 2048, L), rng.integers(0, L, 4000)])
    peak = float(np.sum(np.abs(taps)))  # |y| <= sum |h| for |x| <= 1
    for c in range(2):
        xc = x[c].cpu().numpy()
        y = out[c].cpu().numpy()
        for n in idx[::7]:
            lo = max(0, n - 1023)
            seg = xc[lo:n + 1][::-1].astype(np.float64)
            ref = float(np.dot(taps[:seg.size].astype(np.float64), seg))
            bnd = 1025 * U * float(np.dot(np.abs(taps[:seg.size]).astype(np.float64), np.abs(seg)))
            if fir_method == 2:
                bnd = OLS_TOL * peak
            assert abs(float(y[n]) - ref) <= bnd + 1e-30


@pytest.mark.gpu
def test_gpu_fir_stft_and_ir(torch_cuda, oracle, fir_method):
    torch = torch_cuda
    taps = cfg3b_taps()
    x = np.random.default_rng(8).uniform(-1, 1, (2, 8192 * 3)).astype(np.float32)
    out, mag = d.render_stft(torch.from_numpy(x).cuda(), 2, 512, 48000.0, fplug(taps, fir_method))
    o = out.cpu().numpy()
    check_fir(oracle, o[1], x[1], taps, o.shape[1], fir_method)
    mref = oracle.np_stft_mag(o[1], 8192, 4096, d.DSP_WIN_HANN, 4097)
    m = mag.cpu().numpy()[1]
    assert np.max(np.abs(m - mref)) <= 1e-6 * np.max(mref)
    ir, imag = d.ir_analysis(fplug(taps, fir_method), C_out=2, device="cuda")    # IR of a FIR = its taps
    irn = ir.cpu().numpy()[0]
    want = np.concatenate([taps, np.zeros(1024, np.float32)])
    if fir_method == 1:
        assert np.array_equal(irn, want)
    else:  # an impulse through the FFT path: within the overlap-save tolerance
        assert np.max(np.abs(irn - want)) <= OLS_TOL * np.max(np.abs(taps))
    ref = oracle.np_ir_magnitude(np.concatenate([taps, np.zeros(1024, np.float32)]), 2048)
    assert np.max(np.abs(imag.cpu().numpy() - ref)) <= 1e-6 * np.max(ref)


@pytest.mark.gpu
def test_gpu_fir_rejects_too_many_taps(torch_cuda):
    x = torch_cuda.zeros((1, 4096), device="cuda")
    with pytest.raises(d.DspError):
        d.render_offline(x, 1, 512, 48000.0, d.Plugin.fir(np.ones(2049, np.float32)))


@pytest.mark.gpu
def test_fir_method_is_per_call(torch_cuda):
    """The FIR method travels with each call (dsp_exec flags): interleaved
    direct-form and overlap-save renders each reproduce their own result."""
    torch = torch_cuda
    rng = np.random.default_rng(77)
    taps = rng.uniform(-0.2, 0.2, 300).astype(np.float32)
    x = torch.from_numpy(rng.uniform(-1, 1, (2, 48_000)).astype(np.float32)).cuda()
    pd, po = d.Plugin.fir(taps, direct=True), d.Plugin.fir(taps)
    ref_d = d.render_offline(x, 2, 512, 48000.0, pd).clone()
    ref_o = d.render_offline(x, 2, 512, 48000.0, po).clone()
    assert not torch.equal(ref_d, ref_o)  # two different kernels (rounding differs)
    for _ in range(3):
        assert torch.equal(d.render_offline(x, 2, 512, 48000.0, po), ref_o)
        assert torch.equal(d.render_offline(x, 2, 512, 48000.0, pd), ref_d)
