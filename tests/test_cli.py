"""The offline-render command line (dsp-bench_amd/cli/dspbench_render.cpp): a
C++ host driving the GPU path through the C ABI only -- WAV parse, GPU
decode, render (+ STFT), GPU encode, WAV write.

CPU: argument errors and unreadable files fail with a message (no GPU is
touched).  GPU: the written file equals the oracle's render of the decoded
input (the reference's converters, restated callbacks and render loop) bit
for bit; the spectra equal the Python face's fused render + STFT of the same
render; a plugin given as source (our biquad) renders as the Python face's
module path does.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import dspbench as d
from wavutil import wav_image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "dsp-bench_amd", "dspbench_render")
BIQUAD = os.path.join(ROOT, "dsp-bench_amd", "plugins", "biquad.cpp")

needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="dspbench_render not built")


def run(*args, env=None):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300, env=env)


@needs_cli
def test_usage_and_unreadable_input(tmp_path):
    r = run()
    assert r.returncode == 2 and "usage" in r.stderr
    r = run("a.wav", "b.wav", "--block")
    assert r.returncode == 2
    r = run(str(tmp_path / "missing.wav"), str(tmp_path / "o.wav"))
    assert r.returncode == 1 and "cannot read" in r.stderr


@needs_cli
def test_not_a_wav_fails_in_parse(tmp_path):
    p = tmp_path / "x.wav"
    p.write_bytes(b"RIFF\x04\x00\x00\x00WAVX")
    r = run(str(p), str(tmp_path / "o.wav"))
    assert r.returncode == 1 and "dsp_wav_parse" in r.stderr


def _pcm16_stereo(tmp_path, L=48_000 * 3 + 77, seed=11):
    raw = np.random.default_rng(seed).integers(-32768, 32768, size=2 * L, dtype=np.int64).astype("<i2")
    p = tmp_path / "in.wav"
    p.write_bytes(wav_image(raw.tobytes(), fmt=1, channels=2, bits=16))
    return p, raw, L


def _read_float_wav(path):
    x, info = d.wav.load(str(path))
    assert info.format == 3 and info.bits_per_sample == 32
    return np.asarray(x)


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("plugin,B", [("gain_test", 512), ("IR_test", 512), ("no_op", 384), ("static_gain", 100)])
def test_render_file_matches_oracle(torch_cuda, oracle, tmp_path, plugin, B):
    src, raw, L = _pcm16_stereo(tmp_path)
    out = tmp_path / "out.wav"
    r = run(str(src), str(out), "--plugin", plugin, "--block", str(B), "--bits", "float")
    assert r.returncode == 0, r.stderr
    got = _read_float_wav(out)
    x = oracle.deinterleave(oracle.pcm_to_float(raw.view(np.uint8), 16), 2)
    names = {"gain_test": ("gain_test", [0.2], None), "IR_test": ("IR_test", [0.9, 0.002], None),
             "no_op": ("no_op", None, None), "static_gain": ("static_gain_plugin", None, [0.1])}
    n, prm, sta = names[plugin]
    want = oracle.render_offline([x[0], x[1]], 2, B, 48000.0, oracle.restated_plugin(n, prm, sta))
    assert got.shape == want.shape
    assert np.array_equal(got, want)


@needs_cli
@pytest.mark.gpu
def test_render_stft_file(torch_cuda, oracle, tmp_path):
    src, raw, L = _pcm16_stereo(tmp_path, L=48_000 * 2)
    out, mag = tmp_path / "out.wav", tmp_path / "mag.f32"
    r = run(str(src), str(out), "--plugin", "IR_test", "--stft", str(mag), "--bits", "float")
    assert r.returncode == 0, r.stderr
    blob = mag.read_bytes()
    assert blob[:8] == b"DSPMAG1\0"
    C_, K = struct.unpack("<II", blob[8:16])
    F = struct.unpack("<Q", blob[16:24])[0]
    m = np.frombuffer(blob[24:], np.float32).reshape(C_, F, K)
    x = torch_cuda.from_numpy(_read_float_wav_pcm(src)).cuda()
    ref_out, ref_mag = d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test())
    assert (C_, F, K) == tuple(ref_mag.shape)
    assert np.array_equal(m, ref_mag.cpu().numpy())
    assert np.array_equal(_read_float_wav(out), ref_out.cpu().numpy())
    # and against the oracle: the render bit for bit, the spectra within the
    # STFT bar (1e-6 of each frame's peak, float64)
    want = oracle.render_offline([], 2, 512, 48000.0,
                                 oracle.restated_plugin("IR_test"), L=L)
    assert np.array_equal(_read_float_wav(out), want)
    for c in range(2):
        mref = oracle.np_stft_mag(want[c], 8192, 4096, d.DSP_WIN_HANN, 4097)
        err = np.max(np.abs(m[c] - mref).max(axis=1) / mref.max(axis=1))
        assert err <= 1e-6


def _read_float_wav_pcm(path):
    x, _ = d.wav.load(str(path))
    return np.ascontiguousarray(np.asarray(x))


@needs_cli
@pytest.mark.gpu
def test_plugin_source_file(torch_cuda, tmp_path):
    src, raw, L = _pcm16_stereo(tmp_path, L=20_000)
    out = tmp_path / "out.wav"
    r = run(str(src), str(out), "--plugin", BIQUAD, "--block", "256", "--bits", "float")
    assert r.returncode == 0, r.stderr
    got = _read_float_wav(out)
    mod = d.module.Module(d.module.compile_source(open(BIQUAD).read(), "biquad.cpp"))
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    x = torch_cuda.from_numpy(_read_float_wav_pcm(src)).cuda()
    want = d.render_offline(x, 2, 256, 48000.0, mod.plugin(params)).cpu().numpy()
    assert np.array_equal(got, want)


@needs_cli
def test_multi_rank_needs_stft(tmp_path):
    src, _, _ = _pcm16_stereo(tmp_path, L=1000)
    r = run(str(src), str(tmp_path / "o.wav"), "--comm-id", str(tmp_path / "id"), "--world", "2", "--rank", "0")
    assert r.returncode == 2 and "--comm-id needs --stft" in r.stderr


def _pcm16(tmp_path, C, L, sr, seed, name="in.wav"):
    raw = np.random.default_rng(seed).integers(-32768, 32768, size=C * L, dtype=np.int64).astype("<i2")
    p = tmp_path / name
    p.write_bytes(wav_image(raw.tobytes(), fmt=1, channels=C, bits=16, sr=sr))
    return p, raw


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("Cf,Cd", [(1, 2), (3, 2)])
def test_device_format_mode(torch_cuda, oracle, tmp_path, Cf, Cd):
    """the reference renders at the device's format -- 2
    channels, the device rate -- whatever the file's (wav_reader.h:7-14,
    wasapi_audio.cpp:432-447): extra file channels are dropped, missing ones
    render from zeros, the callback sees the device rate."""
    L = 30_011
    src, raw = _pcm16(tmp_path, Cf, L, 44100, 12)
    out = tmp_path / "out.wav"
    r = run(str(src), str(out), "--plugin", "gain_test", "--device-channels", str(Cd), "--device-rate", "48000",
            "--bits", "float")
    assert r.returncode == 0, r.stderr
    got, info = d.wav.load(str(out))
    assert info.sample_rate == 48000 and info.channels == Cd
    x = oracle.deinterleave(oracle.pcm_to_float(raw.view(np.uint8), 16), Cf)
    want = oracle.render_offline([x[c] for c in range(Cf)], Cd, 512, 48000.0, oracle.restated_plugin("gain_test", [0.2]))
    assert np.array_equal(np.asarray(got), want)


@needs_cli
@pytest.mark.gpu
def test_loop_mode_file(torch_cuda, oracle, tmp_path):
    """--loop: render_audio with the file looping (audio.cpp:100-132)."""
    src, raw, L = _pcm16_stereo(tmp_path, L=5_000)
    out = tmp_path / "out.wav"
    r = run(str(src), str(out), "--plugin", "gain_test", "--loop", "33", "--block", "512", "--bits", "float")
    assert r.returncode == 0, r.stderr
    x = oracle.deinterleave(oracle.pcm_to_float(raw.view(np.uint8), 16), 2)
    want, _ = oracle.render_loop([x[0], x[1]], 2, 512, 33, 48000.0, oracle.restated_plugin("gain_test", [0.2]))
    assert np.array_equal(_read_float_wav(out), want)


@needs_cli
@pytest.mark.gpu
def test_multi_rank_cli_one_rank(torch_cuda, oracle, tmp_path):
    """The CLI's multi-GPU mode (cfg 5 shape: 96 kHz, one channel run per rank,
    RCCL gather to rank 0) with one rank: the RCCL rendezvous file, the
    sharded pipelined driver and the root's output equal the single-process
    render + STFT."""
    L = 8192 * 10 + 321
    src, raw = _pcm16(tmp_path, 4, L, 96000, 13)
    a, am = tmp_path / "a.wav", tmp_path / "a.f32"
    b, bm = tmp_path / "b.wav", tmp_path / "b.f32"
    r = run(str(src), str(a), "--plugin", "IR_test", "--stft", str(am), "--bits", "float")
    assert r.returncode == 0, r.stderr
    r = run(str(src), str(b), "--plugin", "IR_test", "--stft", str(bm), "--bits", "float",
            "--comm-id", str(tmp_path / "rccl.id"), "--world", "1", "--rank", "0", "--chunk", "30000")
    assert r.returncode == 0, r.stderr
    assert a.read_bytes() == b.read_bytes()
    assert am.read_bytes() == bm.read_bytes()
    assert not (tmp_path / "rccl.id").exists(), "rank 0 leaves the spent id file behind"


@needs_cli
@pytest.mark.gpu
def test_multi_rank_cli_ignores_a_stale_id_file(torch_cuda, tmp_path):
    """A rank other than 0 never reads an id file another launch left: one
    written before it started (no run id), or one carrying another run id.
    With nothing fresh to read it gives up (DSPB_COMM_WAIT_S = 2) instead of
    joining a dead communicator."""
    import os
    import time
    src, raw = _pcm16(tmp_path, 2, 8192 * 3, 96000, 14)
    idf = tmp_path / "rccl.id"
    idf.write_bytes(bytes(128))                      # a previous launch's file, no run id
    old = time.time() - 60
    os.utime(idf, (old, old))
    env = dict(os.environ, DSPB_COMM_WAIT_S="2")
    env.pop("DSPB_RUN_ID", None)
    env.pop("TORCHELASTIC_RUN_ID", None)
    args = [str(src), str(tmp_path / "o.wav"), "--plugin", "IR_test", "--stft", str(tmp_path / "o.f32"),
            "--comm-id", str(idf), "--world", "2", "--rank", "1", "--device", "0"]
    r = run(*args, env=env)
    assert r.returncode != 0 and "no communicator id" in r.stderr, r.stderr
    idf.write_bytes(bytes(128) + b"run-A")           # fresh, but another run's id
    r = run(*args, "--run-id", "run-B", env=env)
    assert r.returncode != 0 and "no communicator id" in r.stderr, r.stderr
