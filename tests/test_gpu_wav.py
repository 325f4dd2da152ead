"""WAV decode / encode on the GPU vs the oracle (bit-exact), through the C ABI.

The oracle's converters are pinned to the reference's own
convertInt16/24/32ToFloat (tests/test_wav.py); here the GPU kernels are
checked against the oracle: every int16 and int24 code, 2^20 int32 codes,
mono / stereo / 3-channel (generic path) interleaved payloads, unaligned
frame offsets, host and device buffers, and float / PCM encode.
"""
import numpy as np
import pytest

import dspbench as d
from wavutil import samples_bytes, wav_code_sets, wav_image

pytestmark = pytest.mark.gpu


def _info(bits, channels, frames, is_float=False):
    i = d._lib.dsp_wav_info()
    i.format = 3 if is_float else 1
    i.channels = channels
    i.sample_rate = 48000
    i.bits_per_sample = bits
    i.block_align = channels * bits // 8
    i.frames = frames
    i.data_bytes = frames * i.block_align
    i.n_data_chunks = 1
    return i


@pytest.mark.parametrize("bits", [16, 24, 32])
def test_decode_every_code(torch_cuda, oracle, bits):
    raw = wav_code_sets()[bits]
    n = raw.size // (bits // 8)
    got = d.wav.decode(raw, _info(bits, 1, n), device="cuda").cpu().numpy()[0]
    assert np.array_equal(got.view(np.uint32), oracle.pcm_to_float(raw, bits).view(np.uint32))


@pytest.mark.parametrize("channels", [1, 2, 3])
@pytest.mark.parametrize("bits,is_float", [(16, False), (24, False), (32, False), (32, True)])
# frame0 sets the payload start's alignment, so the tiled mono / stereo decode
# takes its 16-, 8- and 4-byte load paths (e.g. int16 stereo: 0 and 4 -> 16 B,
# 2 -> 8 B, 1 / 3 -> 4 B); 10_007 and 3001 end in a partial 4-frame group
@pytest.mark.parametrize("frame0,frames", [(0, 10_007), (1, 5000), (3, 4), (0, 1), (2, 9_999), (4, 3001),
                                           (0, 4 * 256 * 4 + 4)])
def test_decode_interleaved(torch_cuda, oracle, channels, bits, is_float, frame0, frames):
    rng = np.random.default_rng(channels * 100 + bits)
    total = frame0 + frames + 5
    raw = samples_bytes(rng, total * channels, bits, is_float)
    ref = oracle.deinterleave(oracle.pcm_to_float(raw, bits, is_float), channels)[:, frame0:frame0 + frames]
    info = _info(bits, channels, total, is_float)
    got = d.wav.decode(raw, info, frame0, frames, device="cuda").cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    host = d.wav.decode(raw, info, frame0, frames)                     # host-buffer mode
    assert np.array_equal(host.view(np.uint32), ref.view(np.uint32))


def test_load_file_with_extensible_and_two_data_chunks(torch_cuda, oracle, tmp_path):
    rng = np.random.default_rng(9)
    raw = bytes(samples_bytes(rng, 2 * 3001, 24))
    img = wav_image(raw, fmt=1, channels=2, bits=24, style="extensible",
                    split_data=[(0, 6 * 1000), (6 * 1000, len(raw))])
    p = tmp_path / "x.wav"
    p.write_bytes(img)
    x, info = d.wav.load(str(p), device="cuda")
    ref = oracle.deinterleave(oracle.pcm_to_float(np.frombuffer(raw, np.uint8), 24), 2)
    assert info.frames == 3001 and np.array_equal(x.cpu().numpy(), ref)


@pytest.mark.parametrize("bits,is_float", [(16, False), (24, False), (32, False), (32, True)])
@pytest.mark.parametrize("channels", [1, 2, 5])
def test_encode_matches_oracle_and_round_trips(torch_cuda, oracle, bits, is_float, channels):
    torch = torch_cuda
    rng = np.random.default_rng(bits + channels)
    x = (rng.random((channels, 3333), dtype=np.float32) * 2.2 - 1.1).astype(np.float32)   # clips
    fmt = 3 if is_float else 1
    got = d.wav.encode(torch.from_numpy(x).cuda(), fmt, bits).cpu().numpy()
    inter = np.ascontiguousarray(x.T).ravel()
    assert np.array_equal(got, oracle.float_to_pcm(inter, bits, is_float))
    assert np.array_equal(d.wav.encode(x, fmt, bits), got)                 # host mode
    back = d.wav.decode(got, _info(bits, channels, 3333, is_float), device="cuda").cpu().numpy()
    if is_float:
        assert np.array_equal(back, x)


def test_save_load_render_pipeline(torch_cuda, oracle, tmp_path):
    """WAV file -> GPU decode -> IR_test/gain render + STFT -> float WAV out."""
    torch = torch_cuda
    rng = np.random.default_rng(4)
    raw = bytes(samples_bytes(rng, 2 * 50_000, 16))
    p = tmp_path / "in.wav"
    p.write_bytes(wav_image(raw, channels=2, bits=16))
    x, info = d.wav.load(str(p), device="cuda")
    out, mag = d.render_stft(x.contiguous(), 2, 512, float(info.sample_rate), d.Plugin.gain_test(0.2))
    ref_in = oracle.deinterleave(oracle.pcm_to_float(np.frombuffer(raw, np.uint8), 16), 2)
    ref = oracle.render_offline([ref_in[0], ref_in[1]], 2, 512, 48000.0, oracle.restated_plugin("gain_test"))
    assert np.array_equal(out.cpu().numpy(), ref)
    q = tmp_path / "out.wav"
    d.wav.save(str(q), out, info.sample_rate)
    y, info2 = d.wav.load(str(q))
    assert info2.format == 3 and np.array_equal(y, ref)


@pytest.mark.parametrize("bits,is_float", [(16, False), (24, False), (32, False), (32, True)])
@pytest.mark.parametrize("channels", [1, 2])
@pytest.mark.parametrize("frames", [4, 4099, 70_000])
@pytest.mark.parametrize("poff", [0, 4, 8])
def test_encode_tile_path(torch_cuda, oracle, bits, is_float, channels, frames, poff):
    """The mono / stereo encode tile (16-byte aligned planar rows; payload
    stores 16, 8 or 4 bytes wide from its alignment; the last partial group
    byte by byte), through the C ABI, against the oracle's converters."""
    import ctypes as C
    torch = torch_cuda
    rng = np.random.default_rng(bits * 7 + channels + frames + poff)
    x = (rng.random((channels, frames), dtype=np.float32) * 2.2 - 1.1).astype(np.float32)
    rows = torch.zeros((channels, frames + 64), device="cuda")[:, :frames]   # 16-byte aligned rows
    rows.copy_(torch.from_numpy(x))
    nbytes = frames * channels * bits // 8
    buf = torch.full((nbytes + 32,), 0xA5, dtype=torch.uint8, device="cuda")
    ex = d._lib.dsp_exec(torch.cuda.current_device(), d._lib.DSP_EXEC_SYNC,
                         C.c_void_p(torch.cuda.current_stream().cuda_stream), 0)
    ptrs = d._lib.chan_table([rows[c].data_ptr() for c in range(channels)])
    st = d.lib().dsp_wav_encode(ptrs, channels, frames, 3 if is_float else 1, bits,
                                C.c_void_p(buf.data_ptr() + poff), C.byref(ex))
    assert st == 0
    got = buf.cpu().numpy()
    inter = np.ascontiguousarray(x.T).ravel()
    want = np.asarray(oracle.float_to_pcm(inter, bits, is_float)).view(np.uint8).ravel()
    assert np.array_equal(got[poff:poff + nbytes], want)
    assert np.all(got[:poff] == 0xA5) and np.all(got[poff + nbytes:] == 0xA5)   # nothing outside the payload
