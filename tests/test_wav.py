"""WAV input/output on CPU (include/dspbench/wav.h).

  * the oracle's restated converters vs the reference's own
    convertInt16/24/32ToFloat (audio.h:66-110): exhaustive int16 / int24 and
    2^20 int32 codes, against the golden hashes made from the reference;
  * dsp_wav_parse on the chunk layouts the reference reads and on the ones
    it mis-reads (fmt > 16 bytes, EXTENSIBLE, odd chunks, several data
    chunks, streamed data size);
  * dsp_wav_write_header round trips through the parser.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import dspbench as d
from wavutil import chunk, samples_bytes, wav_code_sets, wav_image

HERE = os.path.dirname(os.path.abspath(__file__))
META = json.load(open(os.path.join(HERE, "golden", "golden_v1.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("bits", [16, 24, 32])
def test_oracle_decode_matches_reference_converters(oracle, bits):
    raw = wav_code_sets()[bits]
    out = oracle.pcm_to_float(raw, bits)
    g = META["wav_decode"][str(bits)]
    assert out.size == g["n"] and sha(out) == g["sha256"]
    if oracle.ref_audio_available():
        assert np.array_equal(out.view(np.uint32), oracle.ref_convert(raw, bits).view(np.uint32))


def test_decode_edge_values(oracle):
    i16 = np.array([0x8000, 0x7fff, 0, 1], "<u2").view(np.uint8)
    assert list(oracle.pcm_to_float(i16, 16)) == [-1.0, float.fromhex("0x1.fffcp-1"), 0.0, 2.0 ** -15]
    i24 = np.array([0xff, 0xff, 0x7f, 0x00, 0x00, 0x80], np.uint8)
    assert list(oracle.pcm_to_float(i24, 24)) == [float.fromhex("0x1.fffffcp-1"), -1.0]
    i32 = np.array([0x7fffffff, 0x80000000], "<u4").view(np.uint8)
    assert list(oracle.pcm_to_float(i32, 32)) == [1.0, -1.0]   # int -> float rounds first


def test_pcm_encode_decode_round_trip(oracle):
    rng = np.random.default_rng(3)
    for bits in (16, 24):
        raw = rng.integers(0, 256, 3000 * (bits // 8), dtype=np.uint8)
        x = oracle.pcm_to_float(raw, bits)
        assert np.array_equal(oracle.float_to_pcm(x, bits), raw)
    x = np.array([1.5, -1.5, 0.5 / 32768, 1.5 / 32768], np.float32)   # clip, round half even
    assert list(oracle.pcm_to_float(oracle.float_to_pcm(x, 16), 16) * 32768) == [32767, -32768, 0, 2]


def _parse(img):
    return d.wav.parse(np.frombuffer(img, np.uint8))


@pytest.mark.parametrize("style", ["plain", "cbsize", "extensible"])
@pytest.mark.parametrize("fmt,bits", [(1, 16), (1, 24), (1, 32), (3, 32)])
def test_parse_fmt_layouts(style, fmt, bits):
    data = bytes(range(256)) * 3 + bytes(range(36))   # 804 bytes
    img = wav_image(data, fmt=fmt, channels=2, sr=44100, bits=bits, style=style)
    i = _parse(img)
    assert (i.format, i.channels, i.sample_rate, i.bits_per_sample) == (fmt, 2, 44100, bits)
    assert i.n_data_chunks == 1 and i.data_bytes == len(data)
    assert i.frames == len(data) // (2 * bits // 8)
    off = i.data_offset[0]
    assert img[off:off + len(data)] == data


def test_parse_skips_odd_chunks_and_concatenates_data_chunks():
    data = bytes(np.random.default_rng(1).integers(0, 256, 4000, dtype=np.uint8))
    img = wav_image(data, extra_before=chunk(b"LIST", b"INFOabc") + chunk(b"junk", b"x" * 5),
                    split_data=[(0, 1000), (1000, 4000)])
    i = _parse(img)
    assert i.n_data_chunks == 2 and i.data_bytes == 4000 and i.frames == 1000
    got = b"".join(img[i.data_offset[k]:i.data_offset[k] + i.data_size[k]] for k in range(2))
    assert got == data
    assert np.array_equal(d.wav.payload(np.frombuffer(img, np.uint8), i), np.frombuffer(data, np.uint8))


def test_parse_streamed_data_size_is_clamped():
    data = bytes(400)
    img = wav_image(data, data_size=0xFFFFFFFF)
    i = _parse(img)
    assert i.data_bytes == 400 and i.frames == 100


@pytest.mark.parametrize("img,status", [
    (b"RIFX" + bytes(40), -1),
    (b"RIFF\x00\x00\x00\x00WAVE", -1),                       # no fmt, no data
    (wav_image(bytes(16), fmt=1, bits=8), -3),                # 8-bit PCM: Wav_Invalid_Format
    (wav_image(bytes(16), fmt=6, bits=8), -3),                # A-law
    (wav_image(bytes(16), fmt=3, bits=64), -3),               # float64
])
def test_parse_rejects(img, status):
    info = d._lib.dsp_wav_info()
    buf = np.frombuffer(img, np.uint8)
    assert d.lib().dsp_wav_parse(buf.ctypes.data, buf.size, info) == status


@pytest.mark.parametrize("fmt,bits", [(1, 16), (1, 24), (1, 32), (3, 32)])
def test_header_round_trip(fmt, bits):
    h = d.wav.header(fmt, 3, 96000, bits, 1234)
    assert len(h) == (46 if fmt == 3 else 44)
    img = h + bytes(1234 * 3 * bits // 8)
    i = _parse(img)
    assert (i.format, i.channels, i.sample_rate, i.bits_per_sample, i.frames) == (fmt, 3, 96000, bits, 1234)
    assert struct.unpack("<I", h[4:8])[0] == len(img) - 8


def test_big_file_sizes_are_64_bit():
    """A data chunk past 4 GiB cannot be built in a unit test; the RIFF size
    clamps and frames stay 64-bit in the header writer."""
    h = d.wav.header(1, 2, 48000, 16, 2_000_000_000)   # 8 GB of payload
    assert struct.unpack("<I", h[4:8])[0] == 0xFFFFFFFF
    assert struct.unpack("<I", h[40:44])[0] == 0xFFFFFFFF


def test_samples_helper_shapes():
    rng = np.random.default_rng(0)
    assert samples_bytes(rng, 10, 24).size == 30 and samples_bytes(rng, 10, 32, True).size == 40
