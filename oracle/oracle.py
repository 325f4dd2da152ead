"""oracle.py -- Python face of the CPU restatement.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It loads

  * oracle/liboracle.so       -- the C restatement (oracle.c)
  * oracle/_ref/libref_*.so   -- reference stock plugins compiled from their
                                 own sources (oracle/Makefile)

and adds float64 numpy restatements used to pin the C code:

  * ``np_window``      ippsWinHamming_32f / Hann  (ref dsp.cpp:69-72)
  * ``np_ir_magnitude`` fft_perform_and_get_magnitude (ref dsp.cpp:53-66)
  * ``np_stft_mag``    window -> fft_forward -> pythagore_array per frame
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")

WIN_HAMMING, WIN_HANN, WIN_RECT = 0, 1, 2

CALLBACK_T = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.POINTER(C.POINTER(C.c_float)),
                         C.c_uint, C.c_uint, C.c_float)

_lib = None


def lib() -> C.CDLL:
    """Load liboracle.so (built by ``make -C oracle``)."""
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        u64, u32, f32, vp = C.c_uint64, C.c_uint32, C.c_float, C.c_void_p
        fpp = C.POINTER(C.POINTER(C.c_float))
        L.oracle_render_offline.restype = u64
        L.oracle_render_offline.argtypes = [fpp, u32, u64, fpp, u32, u32, f32, vp, vp, vp]
        L.oracle_render_loop.restype = u64
        L.oracle_render_loop.argtypes = [fpp, u32, u64, u64, fpp, u32, u32, u64, f32, vp, vp, vp]
        L.oracle_window_f64.argtypes = [C.c_int, u32, vp]
        L.oracle_window_f32.argtypes = [C.c_int, u32, vp]
        L.oracle_fft_f64.argtypes = [vp, vp, u32, C.c_int]
        L.oracle_fft_f32.argtypes = [vp, vp, u32, C.c_int]
        L.oracle_fft_forward_f64.argtypes = [vp, vp, vp, u32]
        L.oracle_fft_reverse_f64.argtypes = [vp, vp, vp, u32]
        L.oracle_ir_magnitude_f64.argtypes = [vp, u32, vp]
        L.oracle_stft_frames.restype = u64
        L.oracle_stft_frames.argtypes = [u64, u32, u32]
        L.oracle_stft_mag_f64.argtypes = [vp, u64, u32, u32, C.c_int, u32, u64, vp]
        L.oracle_stft_mag_f32.argtypes = [vp, u64, u32, u32, C.c_int, u32, u64, vp, C.c_int]
        L.oracle_stft_mag_f32_r4.argtypes = [vp, u64, u32, u32, C.c_int, u32, u64, vp, C.c_int]
        L.oracle_normalize_int.restype = f32
        L.oracle_normalize_int.argtypes = [C.c_int32, C.c_int32, f32]
        L.oracle_denormalize_int.restype = C.c_int32
        L.oracle_denormalize_int.argtypes = [C.c_int32, C.c_int32, f32]
        L.oracle_normalize_float.restype = f32
        L.oracle_normalize_float.argtypes = [f32, f32, C.c_int, f32]
        L.oracle_denormalize_float.restype = f32
        L.oracle_denormalize_float.argtypes = [f32, f32, C.c_int, f32]
        L.oracle_normalize_enum_index.restype = f32
        L.oracle_normalize_enum_index.argtypes = [u32, C.c_int32]
        L.oracle_denormalize_enum_index.restype = u32
        L.oracle_denormalize_enum_index.argtypes = [u32, f32]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _chan_ptrs(arrs):
    t = (C.POINTER(C.c_float) * len(arrs))()
    for i, a in enumerate(arrs):
        assert a.dtype == np.float32 and a.flags.c_contiguous
        t[i] = a.ctypes.data_as(C.POINTER(C.c_float))
    return t


# --------------------------------------------------------------------------
# plugins
# --------------------------------------------------------------------------

@dataclass
class OraclePlugin:
    """A plugin callback + its parameter/state blobs, as the host holds them
    (ref plugin.h:95-113: parameters_holder / state_holder)."""
    callback: int          # address of audio_callback_type_wrapper-like fn
    params: np.ndarray     # uint8 blob
    state: np.ndarray      # uint8 blob
    keep: object = None    # keeps the CDLL alive

    def params_ptr(self):
        return _ptr(self.params) if self.params.size else None

    def state_ptr(self):
        return _ptr(self.state) if self.state.size else None


def _blob(values, fmt) -> np.ndarray:
    import struct
    b = struct.pack(fmt, *values) if values else b""
    return np.frombuffer(b, dtype=np.uint8).copy() if b else np.zeros(1, np.uint8)


def restated_plugin(name: str, params=None, state=None) -> OraclePlugin:
    """The C restatement of a stock plugin body (oracle.c)."""
    L = lib()
    table = {
        "gain_test": ("oracle_cb_gain_test", params if params is not None else [0.2], "<f", [], "<"),
        "static_gain_plugin": ("oracle_cb_static_gain", [], "<", state if state is not None else [0.1], "<f"),
        "IR_test": ("oracle_cb_ir_test", params if params is not None else [0.9, 0.002], "<ff", [], "<"),
        "no_op": ("oracle_cb_no_op", [], "<", [], "<"),
    }
    sym, pv, pf, sv, sf = table[name]
    fn = C.cast(getattr(L, sym), C.c_void_p).value
    return OraclePlugin(fn, _blob(pv, pf), _blob(sv, sf), L)


def ref_available() -> bool:
    return os.path.exists(os.path.join(REF_DIR, "libref_gain_test.so"))


class RefPlugin:
    """A reference stock plugin compiled from its own source (oracle/_ref).

    Mirrors plugin_populate_from_descriptor (ref plugin.cpp:335-364):
    default_parameters -> initialize_state."""

    def __init__(self, name: str, num_channels: int = 2, sample_rate: float = 48000.0, prefix: str = "libref_"):
        # prefix "libplug_": one of this repository's plugins (plugins/, tests/plugins/)
        # built for the CPU the way the reference's JIT builds a plugin (oracle/Makefile)
        path = os.path.join(REF_DIR, f"{prefix}{name}.so")
        self.lib = C.CDLL(path)
        self.lib.ref_sizeof_parameters.restype = C.c_ulong
        self.lib.ref_sizeof_state.restype = C.c_ulong
        self.lib.default_parameters_type_wrapper.argtypes = [C.c_void_p]
        self.lib.initialize_state_error_wrapper.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_float, C.c_void_p]
        self.lib.initialize_state_error_wrapper.restype = C.c_int
        self.params = np.zeros(max(1, self.lib.ref_sizeof_parameters()), np.uint8)
        self.state = np.zeros(max(1, self.lib.ref_sizeof_state()), np.uint8)
        self.lib.default_parameters_type_wrapper(_ptr(self.params))
        self.init_state(num_channels, sample_rate)

    def init_state(self, num_channels, sample_rate):
        err = self.lib.initialize_state_error_wrapper(_ptr(self.params), _ptr(self.state),
                                                      num_channels, sample_rate, None)
        assert err == 0

    @property
    def callback(self) -> int:
        return C.cast(self.lib.audio_callback_type_wrapper, C.c_void_p).value

    def as_oracle(self) -> OraclePlugin:
        return OraclePlugin(self.callback, self.params, self.state, self.lib)


# --------------------------------------------------------------------------
# render
# --------------------------------------------------------------------------

def render_offline(file_chans, C_out: int, B: int, sr: float, plugin: OraclePlugin | None,
                   L: int | None = None):
    """render_audio back to back, one-shot, until EOF (ref audio.cpp:13-175).
    Returns an array [C_out, ceil(L/B)*B]."""
    file_chans = [np.ascontiguousarray(x, dtype=np.float32) for x in file_chans]
    L_ = L if L is not None else (len(file_chans[0]) if file_chans else 0)
    nb = (L_ + B - 1) // B
    out = np.empty((C_out, max(nb * B, 1)), np.float32)
    outs = [out[c] for c in range(C_out)]
    lib().oracle_render_offline(_chan_ptrs(file_chans) if file_chans else None, len(file_chans), L_,
                                _chan_ptrs(outs), C_out, B, sr,
                                plugin.callback if plugin else None,
                                plugin.params_ptr() if plugin else None,
                                plugin.state_ptr() if plugin else None)
    return out[:, : nb * B]


def render_loop(file_chans, C_out: int, B: int, nblocks: int, sr: float, plugin, cursor: int = 0):
    file_chans = [np.ascontiguousarray(x, dtype=np.float32) for x in file_chans]
    out = np.empty((C_out, nblocks * B), np.float32)
    outs = [out[c] for c in range(C_out)]
    cur = lib().oracle_render_loop(_chan_ptrs(file_chans), len(file_chans), len(file_chans[0]), cursor,
                                   _chan_ptrs(outs), C_out, B, nblocks, sr, plugin.callback,
                                   plugin.params_ptr(), plugin.state_ptr())
    return out, cur


def callback_once(plugin: OraclePlugin, bufs: np.ndarray, sr: float = 44100.0) -> np.ndarray:
    """One audio_callback call on [C, n] float32 buffers, in place."""
    bufs = np.ascontiguousarray(bufs, dtype=np.float32)
    rows = [bufs[c] for c in range(bufs.shape[0])]
    fn = CALLBACK_T(plugin.callback)
    fn(plugin.params_ptr(), plugin.state_ptr(), C.cast(_chan_ptrs(rows), C.POINTER(C.POINTER(C.c_float))),
       bufs.shape[0], bufs.shape[1], sr)
    return bufs


# --------------------------------------------------------------------------
# spectral
# --------------------------------------------------------------------------

def np_window(kind: int, n: int) -> np.ndarray:
    if n == 1:
        return np.ones(1)
    a, b = {WIN_HAMMING: (0.54, 0.46), WIN_HANN: (0.5, 0.5), WIN_RECT: (1.0, 0.0)}[kind]
    return a - b * np.cos(2.0 * np.pi * np.arange(n) / (n - 1))


def c_window_f32(kind: int, n: int) -> np.ndarray:
    w = np.empty(n, np.float32)
    lib().oracle_window_f32(kind, n, _ptr(w))
    return w


def np_ir_magnitude(ir0: np.ndarray, ir_len: int = 2048) -> np.ndarray:
    """fft_perform_and_get_magnitude (ref dsp.cpp:53-66), float64."""
    x = np.zeros(4 * ir_len)
    x[:ir_len] = ir0[:ir_len].astype(np.float64) * np_window(WIN_HAMMING, ir_len)
    return np.abs(np.fft.fft(x)) / np.sqrt(4 * ir_len)


def c_ir_magnitude(ir0: np.ndarray, ir_len: int = 2048) -> np.ndarray:
    m = np.empty(4 * ir_len, np.float64)
    lib().oracle_ir_magnitude_f64(_ptr(np.ascontiguousarray(ir0, np.float32)), ir_len, _ptr(m))
    return m


def stft_frames(L_: int, N: int, H: int) -> int:
    return 0 if L_ < N else (L_ - N) // H + 1


def np_stft_mag(x: np.ndarray, N: int, H: int, win: int, K: int) -> np.ndarray:
    F = stft_frames(len(x), N, H)
    w = np_window(win, N)
    out = np.empty((F, K))
    for f0 in range(0, F, 256):
        f1 = min(F, f0 + 256)
        idx = (np.arange(f0, f1)[:, None] * H + np.arange(N)[None, :])
        fr = x[idx].astype(np.float64) * w
        out[f0:f1] = np.abs(np.fft.rfft(fr, axis=1))[:, :K] / np.sqrt(N) if K <= N // 2 + 1 else \
            (np.abs(np.fft.fft(fr, axis=1))[:, :K] / np.sqrt(N))
    return out


def c_stft_mag_f64(x: np.ndarray, N: int, H: int, win: int, K: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    F = stft_frames(len(x), N, H)
    m = np.empty((max(F, 1), K), np.float64)
    lib().oracle_stft_mag_f64(_ptr(x), len(x), N, H, win, K, K, _ptr(m))
    return m[:F]


def c_stft_mag_f32(x: np.ndarray, N: int, H: int, win: int, K: int, nthreads: int = 0) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    F = stft_frames(len(x), N, H)
    m = np.empty((max(F, 1), K), np.float32)
    lib().oracle_stft_mag_f32(_ptr(x), len(x), N, H, win, K, K, _ptr(m), nthreads)
    return m[:F]


def c_stft_mag_f32_r4(x: np.ndarray, N: int, H: int, win: int, K: int, nthreads: int = 0) -> np.ndarray:
    """The CPU baseline's fp32 STFT (radix-4 Stockham real FFT, OpenMP over frames)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    F = stft_frames(len(x), N, H)
    m = np.empty((max(F, 1), K), np.float32)
    lib().oracle_stft_mag_f32_r4(_ptr(x), len(x), N, H, win, K, K, _ptr(m), nthreads)
    return m[:F]


def c_fft_f64(re: np.ndarray, im: np.ndarray, direction: int = -1):
    re = np.ascontiguousarray(re, np.float64).copy()
    im = np.ascontiguousarray(im, np.float64).copy()
    lib().oracle_fft_f64(_ptr(re), _ptr(im), len(re), direction)
    return re, im


def ir_ramp_reference(gain: float, step: float, n: int) -> np.ndarray:
    """Sequential double recurrence of build/IR_test.cpp:47-58, in Python."""
    g = float(np.float32(gain))
    s = float(np.float32(step))
    out = np.empty(n, np.float32)
    for i in range(n):
        out[i] = np.float32(g)
        g = g - s
    return out


# --------------------------------------------------------------------------
# WAV sample decode (ref audio.h:66-133)
# --------------------------------------------------------------------------

def pcm_to_float(raw: np.ndarray, bits: int, is_float: bool = False) -> np.ndarray:
    """oracle_pcm_to_float over a byte array (restated converters)."""
    raw = np.ascontiguousarray(raw, np.uint8)
    n = raw.size // (bits // 8)
    out = np.empty(n, np.float32)
    L = lib()
    L.oracle_pcm_to_float.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64]
    L.oracle_pcm_to_float(bits, int(is_float), _ptr(raw), _ptr(out), n)
    return out


def float_to_pcm(x: np.ndarray, bits: int, is_float: bool = False) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(x.size * (bits // 8), np.uint8)
    L = lib()
    L.oracle_float_to_pcm.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64]
    L.oracle_float_to_pcm(bits, int(is_float), _ptr(x), _ptr(out), x.size)
    return out


def deinterleave(x: np.ndarray, channels: int) -> np.ndarray:
    return np.ascontiguousarray(x.reshape(-1, channels).T)


def ref_audio_available() -> bool:
    return os.path.exists(os.path.join(REF_DIR, "libref_audio.so"))


def ref_convert(raw: np.ndarray, bits: int) -> np.ndarray:
    """The reference's own convertInt{16,24,32}ToFloat (oracle/_ref/libref_audio.so)."""
    raw = np.ascontiguousarray(raw, np.uint8)
    n = raw.size // (bits // 8)
    out = np.empty(n, np.float32)
    R = C.CDLL(os.path.join(REF_DIR, "libref_audio.so"))
    fn = getattr(R, f"ref_convert_int{bits}")
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    fn(_ptr(raw), _ptr(out), n)
    return out


# --------------------------------------------------------------------------
# display reductions (ref opengl.h:877-890)
# --------------------------------------------------------------------------

def minmax_decimate(x: np.ndarray, pixels: int):
    x = np.ascontiguousarray(x, np.float32)
    vmax = np.empty(pixels, np.float32)
    vmin = np.empty(pixels, np.float32)
    L = lib()
    L.oracle_minmax_decimate.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    L.oracle_minmax_decimate(_ptr(x), x.size, pixels, _ptr(vmax), _ptr(vmin))
    return vmax, vmin


def spectrogram_decimate(mag: np.ndarray, pixels: int) -> np.ndarray:
    mag = np.ascontiguousarray(mag, np.float32)
    F, K = mag.shape
    out = np.empty((pixels, K), np.float32)
    L = lib()
    L.oracle_spectrogram_decimate.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32,
                                              C.c_void_p]
    L.oracle_spectrogram_decimate(_ptr(mag), F, K, K, pixels, _ptr(out))
    return out


def biquad_f64(x, coef, Ly: int | None = None):
    """The biquad cascade (rows b0 b1 b2 a1 a2) over x zero-padded to Ly,
    float64 (oracle.c oracle_biquad_f64).  Returns (y, lmax[S]): lmax[k] =
    max_n of section k's |b0 v| + |b1 v1| + |b2 v2| + |a1 y1| + |a2 y2|."""
    c = np.ascontiguousarray(np.asarray(coef, np.float32).reshape(-1, 5))
    x = np.ascontiguousarray(x, np.float32) if x is not None else None
    L_ = 0 if x is None else x.size
    Ly = L_ if Ly is None else Ly
    y = np.empty(max(Ly, 1), np.float64)
    lm = np.zeros(4, np.float64)
    Lb = lib()
    Lb.oracle_biquad_f64.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                                     C.c_void_p]
    Lb.oracle_biquad_f64(_ptr(x) if x is not None else None, L_, Ly, _ptr(c), c.shape[0], _ptr(y), _ptr(lm))
    return y[:Ly], lm[:c.shape[0]]


def biquad_f32(x, coef, Ly: int | None = None) -> np.ndarray:
    """The serial fp32 cascade, evaluated as plugins/biquad.cpp writes it
    (left to right, no contraction): oracle.c oracle_biquad_f32."""
    c = np.ascontiguousarray(np.asarray(coef, np.float32).reshape(-1, 5))
    x = np.ascontiguousarray(x, np.float32) if x is not None else None
    L_ = 0 if x is None else x.size
    Ly = L_ if Ly is None else Ly
    y = np.empty(max(Ly, 1), np.float32)
    Lb = lib()
    Lb.oracle_biquad_f32.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p]
    Lb.oracle_biquad_f32(_ptr(x) if x is not None else None, L_, Ly, _ptr(c), c.shape[0], _ptr(y))
    return y[:Ly]


def biquad_impulse_l1(coef, tol: float = 1e-13, max_len: int = 1 << 22):
    """Per section: (||h||_1, ||g||_1) of the section's impulse response h
    (b over a) and of its all-pole part g = 1 / (1 + a1 z^-1 + a2 z^-2), summed
    in float64 until the tail is below tol relative (or max_len)."""
    out = []
    for b0, b1, b2, a1, a2 in np.asarray(coef, np.float64).reshape(-1, 5):
        sums = []
        for b in ((b0, b1, b2), (1.0, 0.0, 0.0)):
            x1 = x2 = y1 = y2 = 0.0
            acc, n, quiet = 0.0, 0, 0
            while n < max_len:
                v = 1.0 if n == 0 else 0.0
                y = b[0] * v + b[1] * x1 + b[2] * x2 - a1 * y1 - a2 * y2
                x2, x1, y2, y1 = x1, v, y1, y
                acc += abs(y)
                n += 1
                quiet = quiet + 1 if abs(y) <= tol * max(acc, 1e-300) else 0
                if quiet > 64:
                    break
            sums.append(acc)
        out.append(tuple(sums))
    return out


def biquad_error_bound(coef, lmax, K: float = 16.0) -> float:
    """A bound on |y_gpu - y64| for the cascade: section k's own roundings
    (at most K u relative to its magnitude terms, u = 2^-24, K covering the
    fp32 recurrence's five roundings and the block scan's state rounding) pass
    through its all-pole part, and every earlier section's error through the
    whole later sections:  e_k <= ||h_k||_1 e_(k-1) + K u ||g_k||_1 lmax_k."""
    u = 2.0 ** -24
    e = 0.0
    for (h1, g1), lm in zip(biquad_impulse_l1(coef), lmax):
        e = h1 * e + K * u * g1 * lm
    return e


def fir_f64(x, taps, Ly: int | None = None) -> np.ndarray:
    """y[n] = sum_k taps[k] x[n - k] (x = 0 outside the file), float64."""
    x = np.ascontiguousarray(x, np.float32) if x is not None else None
    h = np.ascontiguousarray(taps, np.float32)
    L_ = 0 if x is None else x.size
    Ly = L_ if Ly is None else Ly
    y = np.empty(max(Ly, 1), np.float64)
    Lb = lib()
    Lb.oracle_fir_f64.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]
    Lb.oracle_fir_f64(_ptr(x) if x is not None else None, L_, _ptr(h), h.size, _ptr(y), Ly)
    return y[:Ly]
