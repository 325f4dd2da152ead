"""wav.py -- WAV load / save through libdspbench (include/dspbench/wav.h).

``load`` replaces the reference's windows_load_wav (wav_reader.h:57-205):
the file is memory-mapped, its chunks are walked by ``dsp_wav_parse`` (64-bit
offsets, fmt > 16 bytes, WAVE_FORMAT_EXTENSIBLE), the data chunks are
uploaded and ``dsp_wav_decode`` converts + deinterleaves on the GPU,
bit-exact with convertInt16/24/32ToFloat (audio.h:66-110).  ``save`` is the
inverse (interleave, audio.h:123-133).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import check, chan_table, dsp_wav_info
from .api import _exec, _is_torch


def parse(image) -> dsp_wav_info:
    """Chunk walk of a file image (bytes / numpy uint8 / memmap)."""
    buf = np.frombuffer(image, dtype=np.uint8) if not isinstance(image, np.ndarray) else image
    info = dsp_wav_info()
    check(L.lib().dsp_wav_parse(buf.ctypes.data, buf.size, C.byref(info)), "dsp_wav_parse")
    return info


def payload(image, info: dsp_wav_info) -> np.ndarray:
    """The data chunks, concatenated (a view when there is one chunk)."""
    buf = np.frombuffer(image, dtype=np.uint8) if not isinstance(image, np.ndarray) else image
    parts = [buf[info.data_offset[i]:info.data_offset[i] + info.data_size[i]]
             for i in range(info.n_data_chunks)]
    return parts[0] if len(parts) == 1 else np.concatenate(parts)


def decode(data, info: dsp_wav_info, frame0: int = 0, frames: int | None = None, device=None):
    """Payload -> [channels, frames] float32.  `data` may be a numpy uint8
    array (host) or a torch uint8 CUDA tensor; with `device` the output is a
    torch tensor on that device (the payload is uploaded first if needed)."""
    frames = info.frames - frame0 if frames is None else frames
    if device is not None:
        import torch
        if not _is_torch(data):
            import warnings
            with warnings.catch_warnings():  # read-only memmap: only read, never written
                warnings.simplefilter("ignore", UserWarning)
                data = torch.from_numpy(np.ascontiguousarray(data)).to(device)
        out = torch.empty((info.channels, max(frames, 1)), dtype=torch.float32, device=data.device)
        ptrs = [out[c].data_ptr() for c in range(info.channels)]
        ex = _exec(out)
        src = data.data_ptr()
    else:
        data = np.ascontiguousarray(data)
        out = np.empty((info.channels, max(frames, 1)), np.float32)
        ptrs = [out[c].ctypes.data for c in range(info.channels)]
        ex = _exec(None)
        src = data.ctypes.data
    check(L.lib().dsp_wav_decode(C.c_void_p(src), C.byref(info), frame0, frames, chan_table(ptrs),
                                 C.byref(ex)), "dsp_wav_decode")
    return out[:, :frames]


def load(path: str, device=None):
    """Read a WAV file: returns (samples [channels, frames] float32, info)."""
    image = np.memmap(path, dtype=np.uint8, mode="r")
    info = parse(image)
    return decode(payload(image, info), info, device=device), info


def encode(x, fmt: int = L.DSP_WAV_FORMAT_FLOAT, bits: int = 32):
    """[channels, frames] float32 (numpy or torch CUDA) -> interleaved
    payload (numpy uint8, or a torch uint8 tensor on x's device)."""
    Cn, n = int(x.shape[0]), int(x.shape[1])
    nbytes = n * Cn * (bits // 8)
    if _is_torch(x):
        import torch
        out = torch.empty(max(nbytes, 4), dtype=torch.uint8, device=x.device)
        ptrs = [x[c].data_ptr() for c in range(Cn)]
        dst, ex = out.data_ptr(), _exec(x)
    else:
        x = np.ascontiguousarray(x, np.float32)
        out = np.empty(max(nbytes, 4), np.uint8)
        ptrs = [x[c].ctypes.data for c in range(Cn)]
        dst, ex = out.ctypes.data, _exec(None)
    check(L.lib().dsp_wav_encode(chan_table(ptrs), Cn, n, fmt, bits, C.c_void_p(dst), C.byref(ex)),
          "dsp_wav_encode")
    return out[:nbytes]


def header(fmt: int, channels: int, sample_rate: int, bits: int, frames: int) -> bytes:
    buf = (C.c_uint8 * 64)()
    n = L.lib().dsp_wav_write_header(buf, 64, fmt, channels, sample_rate, bits, frames)
    if n < 0:
        check(n, "dsp_wav_write_header")
    return bytes(buf[:n])


def save(path: str, x, sample_rate: int, fmt: int = L.DSP_WAV_FORMAT_FLOAT, bits: int = 32) -> None:
    """Write [channels, frames] float32 as a WAV file."""
    data = encode(x, fmt, bits)
    if _is_torch(data):
        data = data.cpu().numpy()
    with open(path, "wb") as f:
        f.write(header(fmt, int(x.shape[0]), sample_rate, bits, int(x.shape[1])))
        f.write(memoryview(data))
        if data.size & 1:
            f.write(b"\0")


def render_stft_wav(data, info: dsp_wav_info, C_out: int, B: int, sr: float, plugin, stft: bool = True,
                    N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN, K: int | None = None,
                    chunk: int = 1 << 22, out=None, mag=None, device: int = -1, stream=None):
    """The end-to-end path (wav.h dsp_render_stft_wav): a WAV payload in host
    memory -> per chunk H2D, GPU decode, render (+ STFT), D2H into host rows.
    `out` / `mag` (host float32, [C_out, ceil(L/B)B] / [C_out, F, K]) may be
    given pinned (torch.empty(..., pin_memory=True)) for direct DMA.
    Returns (out, mag | None) as numpy / the given host tensors."""
    from .api import Plugin  # noqa: F401
    K = K if K is not None else N // 2 + 1
    Lp = -(-info.frames // B) * B
    F = (Lp - N) // H + 1 if stft and Lp >= N else 0
    out = np.empty((C_out, max(Lp, 1)), np.float32) if out is None else out
    if stft and mag is None:
        mag = np.empty((C_out, max(F, 1), K), np.float32)
    ptr = (lambda a, c: a[c].data_ptr()) if _is_torch(out) else (lambda a, c: a[c].ctypes.data)
    optrs = chan_table([ptr(out, c) for c in range(C_out)])
    mptrs = chan_table([ptr(mag, c) for c in range(C_out)]) if stft else None
    src = data.data_ptr() if _is_torch(data) else np.ascontiguousarray(data).ctypes.data
    ex = L.dsp_exec(device, 0, C.c_void_p(stream) if stream else None, 0)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    check(L.lib().dsp_render_stft_wav(C.c_void_p(src), C.byref(info), C_out, B, sr,
                                      C.byref(ps) if ps is not None else None, N, H, window, K, optrs, mptrs, K,
                                      chunk, C.byref(ex)), "dsp_render_stft_wav")
    return out, (mag if stft else None)
