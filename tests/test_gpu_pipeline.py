"""The end-to-end host path (dsp_render_stft_host, dsp_render_stft_wav):
host memory -> chunked H2D -> (decode) -> render + STFT -> D2H, three HIP
streams, two slots.  Bars: bit-identical to the device-buffer calls on the
same data (chunks are lcm(B, H)-aligned with an N - H halo), and the render
bit-exact against the oracle."""
import numpy as np
import pytest

import dspbench as d
from wavutil import wav_image

pytestmark = pytest.mark.gpu


def rnd(shape, seed):
    return np.random.default_rng(seed).uniform(-1, 1, shape).astype(np.float32)


@pytest.mark.parametrize("pin", [False, True])
@pytest.mark.parametrize("plugin,B,chunk", [
    (lambda: d.Plugin.ir_test(0.9, 0.002), 512, 3 * 4096),
    (lambda: d.Plugin.gain_test(0.3), 512, 5 * 4096),
    (lambda: d.Plugin.no_op(), 384, 0),
    (lambda: d.Plugin.fir(np.linspace(0.1, -0.05, 200).astype(np.float32)), 512, 4096),  # one chunk
])
def test_host_pipeline_equals_device_call(torch_cuda, plugin, B, chunk, pin):
    torch = torch_cuda
    L = 8192 * 9 + 333
    x = rnd((2, L), 81)
    # the reference call on 16-byte aligned rows, so that it takes the fused
    # kernel as every chunk does (an odd row stride would send it down the
    # unfused path, whose window is the table's: last-bit differences)
    xp = torch.zeros((2, L + 3), device="cuda")
    xp[:, :L] = torch.from_numpy(x).cuda()
    want_out, want_mag = d.render_stft(xp[:, :L], 2, B, 48000.0, plugin(), window=d.DSP_WIN_HANN, L_file=L)
    Lp = d.num_blocks(L, B) * B
    F = d.stft_frames(Lp, 8192, 4096)
    if pin:
        xs = torch.from_numpy(x).pin_memory()
        out = torch.empty((2, Lp), pin_memory=True)
        mag = torch.empty((2, F, 4097), pin_memory=True)
    else:
        xs, out, mag = x, None, None
    got_out, got_mag = d.render_stft_host(xs, 2, B, 48000.0, plugin(), chunk=chunk, out=out, mag=mag)
    got_out = np.asarray(got_out)
    got_mag = np.asarray(got_mag)
    assert np.array_equal(got_out, want_out.cpu().numpy())
    assert np.array_equal(got_mag, want_mag.cpu().numpy())


def test_host_pipeline_render_only(torch_cuda, oracle):
    L, B = 200_001, 384
    x = rnd((1, L), 82)
    out, mag = d.render_stft_host(x, 2, B, 48000.0, d.Plugin.gain_test(0.7), stft=False, chunk=10_000)
    assert mag is None
    want = oracle.render_offline([x[0]], 2, B, 48000.0, oracle.restated_plugin("gain_test", [0.7]))
    assert np.array_equal(out, want)


@pytest.mark.parametrize("Cf,C_out,bits", [(2, 2, 16), (3, 2, 24), (1, 2, 16)])
def test_wav_pipeline_matches_decode_and_oracle(torch_cuda, oracle, Cf, C_out, bits):
    """dsp_render_stft_wav: payload bytes to host spectra; the render equals
    the oracle's render of the reference converters' output bit for bit."""
    torch = torch_cuda
    L = 8192 * 7 + 55
    rng = np.random.default_rng(83)
    raw = rng.integers(0, 256, size=Cf * L * bits // 8, dtype=np.uint8)
    img = wav_image(raw.tobytes(), fmt=1, channels=Cf, bits=bits)
    info = d.wav.parse(img)
    pay = d.wav.payload(img, info)
    out, mag = d.wav.render_stft_wav(pay, info, C_out, 512, 48000.0, d.Plugin.gain_test(0.2), chunk=2 * 4096)
    x = oracle.deinterleave(oracle.pcm_to_float(raw, bits), Cf)
    want = oracle.render_offline([x[c] for c in range(Cf)][:C_out], C_out, 512, 48000.0,
                                 oracle.restated_plugin("gain_test", [0.2]))
    assert np.array_equal(out, want)
    nin = min(Cf, C_out)
    xd = torch.zeros((nin, L + 1), device="cuda")  # 8-byte aligned rows: the fused kernel, as the pipeline's chunks
    xd[:, :L] = torch.from_numpy(np.ascontiguousarray(x[:nin])).cuda()
    _, dmag = d.render_stft(xd[:, :L], C_out, 512, 48000.0, d.Plugin.gain_test(0.2), L_file=L)
    assert np.array_equal(mag, dmag.cpu().numpy())


@pytest.mark.parametrize("name,spec", [("IR_test", True), ("IR_test", False), ("gain_test", True),
                                       ("gain_test", False), ("sine_test", True)])
def test_host_pipeline_generic_plugin(torch_cuda, name, spec):
    """A plugin compiled from source through the host pipeline: a stateless
    one chunks like the stock maps (its block class, or its callback on every
    block); one with a State (sine_test) runs as one chunk.  Bit-identical to
    the device call."""
    import os
    torch = torch_cuda
    mods = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dsp-bench_amd", "modules")
    co = os.path.join(mods, f"mod_{name}.co")
    if not os.path.exists(co):
        pytest.skip("modules not built")
    mod = d.module.Module(open(co, "rb").read())
    params = mod.default_parameters()
    L, B = 8192 * 11 + 77, 512
    x = rnd((2, L), 84)
    xp = torch.zeros((2, L + 3), device="cuda")
    xp[:, :L] = torch.from_numpy(x).cuda()
    mod.initialize_state(params, 2, 48000.0)
    want_out, want_mag = d.render_stft(xp[:, :L], 2, B, 48000.0, mod.plugin(params, name, specialize=spec),
                                       window=d.DSP_WIN_HANN, L_file=L)
    torch.cuda.synchronize()
    mod.initialize_state(params, 2, 48000.0)  # (a State restarts from initialize_state, as on the device call)
    got_out, got_mag = d.render_stft_host(x, 2, B, 48000.0, mod.plugin(params, name, specialize=spec),
                                          chunk=3 * 4096)
    assert np.array_equal(np.asarray(got_out), want_out.cpu().numpy())
    assert np.array_equal(np.asarray(got_mag), want_mag.cpu().numpy())
