"""WAV image builders and code sets shared by the CPU and GPU WAV tests."""
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden import wav_code_sets  # noqa: E402,F401

SUBTYPE_TAIL = bytes([0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80, 0x00, 0x00, 0xAA, 0x00, 0x38, 0x9B, 0x71])


def chunk(cid: bytes, payload: bytes, size=None) -> bytes:
    n = len(payload) if size is None else size
    return cid + struct.pack("<I", n) + payload + (b"\0" if len(payload) & 1 else b"")


def fmt_chunk(fmt, channels, sr, bits, style="plain"):
    ba = channels * bits // 8
    base = struct.pack("<HHIIHH", fmt if style != "extensible" else 0xFFFE, channels, sr, sr * ba, ba, bits)
    if style == "plain":
        return chunk(b"fmt ", base)
    if style == "cbsize":
        return chunk(b"fmt ", base + struct.pack("<H", 0))
    ext = struct.pack("<HHI", 22, bits, 0) + struct.pack("<H", fmt) + SUBTYPE_TAIL
    return chunk(b"fmt ", base + ext)


def wav_image(data: bytes, fmt=1, channels=2, sr=48000, bits=16, style="plain", extra_before=b"",
              split_data=None, data_size=None) -> bytes:
    body = b"WAVE" + fmt_chunk(fmt, channels, sr, bits, style) + extra_before
    if split_data:
        for a, b in split_data:
            body += chunk(b"data", data[a:b])
    else:
        body += chunk(b"data", data, data_size)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def samples_bytes(rng, n_samples, bits, is_float=False):
    if is_float:
        return (rng.random(n_samples, dtype=np.float32) * 2 - 1).astype("<f4").view(np.uint8)
    return rng.integers(0, 256, n_samples * (bits // 8), dtype=np.uint8)
