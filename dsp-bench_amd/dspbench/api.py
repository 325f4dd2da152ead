"""Python host mirror of the DSP-Bench hot path over libdspbench.

Buffers are either torch CUDA tensors (device-resident: the fast path, the
call is enqueued on the tensor's current HIP stream) or numpy arrays (host
buffers: the library stages them through HBM and synchronises).  Every
computation happens in the HIP kernels of libdspbench; this module only
marshals pointers.

Interface mirror (reference odecaux/DSP-Bench):
  Plugin.gain_test / ir_test / static_gain / no_op  stock plugins with their
      Parameters / State blobs laid out as the plugin structs
      (build/gain_test.cpp:14-16, build/IR_test.cpp:14-17,
      test/static_gain_plugin.cpp:7-9)
  render_offline   render_audio pumped block by block (audio.cpp:13-175)
  render_loop      the same with the file looping (audio.cpp:100-132)
  stft_magnitude   windowing -> fft_forward -> pythagore_array per frame
  render_stft      both, fused
  ir_analysis      compute_IR + fft_perform_and_get_magnitude
                   (plugin.cpp:17-58, dsp.cpp:53-66)
  fft_forward / fft_reverse   dsp.cpp:74-132
"""
from __future__ import annotations

import ctypes as C
import struct
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from ._lib import check, chan_table, dsp_exec, dsp_plugin

IR_BUFFER_LENGTH = 2048  # ref hardcoded_values.h:27
MAX_FFT_ORDER = 13       # ref hardcoded_values.h:6


@dataclass
class Plugin:
    kind: int
    params: bytes = b""
    state: bytes = b""
    name: str = ""
    module: object = None
    exec_flags: int = 0  # DSP_EXEC_* bits every call with this plugin adds (per call, no global)
    _keep: list = field(default_factory=list, repr=False)

    @staticmethod
    def gain_test(gain: float = 0.2) -> "Plugin":
        return Plugin(L.DSP_PLUGIN_GAIN, struct.pack("<f", gain), b"", "gain_test")

    @staticmethod
    def ir_test(gain: float = 0.9, step: float = 0.002) -> "Plugin":
        return Plugin(L.DSP_PLUGIN_IR_RAMP, struct.pack("<ff", gain, step), b"", "IR_test")

    @staticmethod
    def static_gain(gain: float = 0.1) -> "Plugin":
        return Plugin(L.DSP_PLUGIN_STATIC_GAIN, b"", struct.pack("<f", gain), "static_gain_plugin")

    @staticmethod
    def no_op() -> "Plugin":
        return Plugin(L.DSP_PLUGIN_NOOP, b"", b"", "no_op")

    @staticmethod
    def fir(taps, direct: bool = False) -> "Plugin":
        """Build-defined FIR (cfg 3b): y[n] = sum_k taps[k] x[n - k].  The
        render uses FFT overlap-save for T <= 1025 taps unless `direct`
        (DSP_EXEC_FIR_DIRECT on every call with this plugin)."""
        t = np.ascontiguousarray(np.asarray(taps, dtype=np.float32))
        return Plugin(L.DSP_PLUGIN_FIR, t.tobytes(), b"", f"fir{t.size}",
                      exec_flags=L.DSP_EXEC_FIR_DIRECT if direct else 0)

    @staticmethod
    def biquad(sections) -> "Plugin":
        """Build-defined cascade of 1..4 direct-form-I biquads (DSP_PLUGIN_BIQUAD):
        `sections` = rows (b0, b1, b2, a1, a2), each y = b0 x + b1 x1 + b2 x2 -
        a1 y1 - a2 y2 (plugins/biquad.cpp's section), zero initial state, the
        whole file; rendered block-parallel by a state scan (iir.hip)."""
        c = np.ascontiguousarray(np.asarray(sections, dtype=np.float32).reshape(-1, 5))
        return Plugin(L.DSP_PLUGIN_BIQUAD, c.tobytes(), b"", f"biquad{c.shape[0]}")

    @staticmethod
    def biquad_lowpass_coefficients(cutoff: float = 1000.0, q: float = 0.7071, sr: float = 48000.0):
        """The coefficients plugins/biquad.cpp's initialize_state computes
        (RBJ cookbook low-pass in double, rounded to float), as one section row."""
        import math
        w0 = 2.0 * 3.14159265358979323846 * float(np.float32(cutoff)) / float(np.float32(sr))
        alpha = math.sin(w0) / (2.0 * float(np.float32(q)))
        c = math.cos(w0)
        a0 = 1.0 + alpha
        b0 = np.float32((1.0 - c) / 2.0 / a0)
        return np.array([[b0, np.float32((1.0 - c) / a0), b0, np.float32(-2.0 * c / a0),
                          np.float32((1.0 - alpha) / a0)]], np.float32)

    def as_struct(self) -> dsp_plugin:
        p = C.create_string_buffer(self.params, max(1, len(self.params)))
        s = C.create_string_buffer(self.state, max(1, len(self.state)))
        self._keep = [p, s]
        mod = self.module.handle if self.module is not None else None
        return dsp_plugin(self.kind, len(self.params), C.cast(p, C.c_void_p) if self.params else None,
                          len(self.state), C.cast(s, C.c_void_p) if self.state else None, mod)


# --------------------------------------------------------------------------
# buffer plumbing
# --------------------------------------------------------------------------

def _is_torch(x) -> bool:
    return hasattr(x, "data_ptr") and hasattr(x, "is_cuda")


def _rows(x):
    """Row pointers of a [C, L] buffer (torch CUDA or numpy)."""
    if x is None:
        return [], None
    if _is_torch(x):
        assert x.dtype.itemsize == 4 and x.dim() == 2 and x.stride(1) == 1
        return [x[c].data_ptr() for c in range(x.shape[0])], x
    x = np.asarray(x)
    assert x.dtype == np.float32 and x.ndim == 2 and x.strides[1] == 4
    return [x[c].ctypes.data for c in range(x.shape[0])], x


def _exec(ref, sample_offset: int = 0, stream=None, sync: bool = False) -> dsp_exec:
    if ref is not None and _is_torch(ref):
        import torch
        dev = ref.device.index if ref.device.index is not None else torch.cuda.current_device()
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        return dsp_exec(dev, L.DSP_EXEC_SYNC if sync else 0, C.c_void_p(st), sample_offset)
    return dsp_exec(-1, L.DSP_EXEC_HOST_BUFFERS | L.DSP_EXEC_SYNC, None, sample_offset)


def _alloc_like(ref, shape):
    if ref is not None and _is_torch(ref):
        import torch
        return torch.empty(shape, dtype=torch.float32, device=ref.device)
    return np.empty(shape, dtype=np.float32)


def stft_frames(L_: int, N: int, H: int) -> int:
    return int(L.lib().dsp_stft_frame_count(L_, N, H))


def num_blocks(L_: int, B: int) -> int:
    return (L_ + B - 1) // B


# --------------------------------------------------------------------------
# entry points
# --------------------------------------------------------------------------

_tls = threading.local()


def last_result() -> int:
    """dsp_exec.result of this thread's last render_offline / render_stft /
    render_loop / render_stft_host (DSP_RESULT_CLASS / _VERIFIED / _RERENDERED
    bits; the chunked driver ORs its chunks' bits)."""
    return getattr(_tls, "result", 0)


def _track(ex):
    r = C.c_uint32(0)
    ex.result = C.pointer(r)
    return r


def render_offline(file, C_out: int, B: int, sr: float, plugin: Plugin | None,
                   out=None, sample_offset: int = 0, L_file: int | None = None, stream=None):
    """Offline one-shot render.  file: [Cin, L] (Cin may be 0 / None).
    Returns out: [C_out, ceil(L/B)*B]."""
    in_ptrs, ref = _rows(file)
    L_ = L_file if L_file is not None else (file.shape[1] if file is not None else 0)
    nb = num_blocks(L_, B)
    if out is None:
        out = _alloc_like(ref, (C_out, max(nb * B, 1)))
    out_ptrs, oref = _rows(out)
    ex = _exec(oref, sample_offset, stream)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    res = _track(ex)
    st = L.lib().dsp_render_offline(chan_table(in_ptrs) if in_ptrs else None, len(in_ptrs), L_,
                                    chan_table(out_ptrs), C_out, B, sr,
                                    C.byref(ps) if ps is not None else None, C.byref(ex))
    check(st, "dsp_render_offline")
    _tls.result = res.value
    return out[:, : nb * B]


def render_loop(file, C_out: int, B: int, nblocks: int, sr: float, plugin: Plugin | None,
                cursor: int = 0, out=None, sample_offset: int = 0, stream=None):
    """Loop-mode render (audio.cpp:100-132): the file wraps from `cursor`.
    Device tensors only.  Returns (out [C_out, nblocks*B], next cursor)."""
    in_ptrs, ref = _rows(file)
    L_ = file.shape[1] if file is not None else 0
    if out is None:
        out = _alloc_like(ref, (C_out, max(nblocks * B, 1)))
    out_ptrs, oref = _rows(out)
    ex = _exec(oref, sample_offset, stream)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    res = _track(ex)
    cur = C.c_uint64()
    st = L.lib().dsp_render_loop(chan_table(in_ptrs) if in_ptrs else None, len(in_ptrs), L_, cursor,
                                 chan_table(out_ptrs), C_out, B, nblocks, sr,
                                 C.byref(ps) if ps is not None else None, C.byref(cur), C.byref(ex))
    check(st, "dsp_render_loop")
    _tls.result = res.value
    return out[:, : nblocks * B], cur.value


def stft_magnitude(x, N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN,
                   K: int | None = None, ld: int | None = None, out=None, L_sig: int | None = None,
                   stream=None):
    """STFT magnitudes of x: [C, L] -> [C, F, K]."""
    in_ptrs, ref = _rows(x)
    K = K if K is not None else N // 2 + 1
    ld = ld if ld is not None else K
    L_ = L_sig if L_sig is not None else x.shape[1]
    F = stft_frames(L_, N, H)
    if out is None:
        out = _alloc_like(ref, (len(in_ptrs), max(F, 1), ld))
    mag_ptrs = [out[c].data_ptr() if _is_torch(out) else out[c].ctypes.data for c in range(len(in_ptrs))]
    ex = _exec(ref, 0, stream)
    st = L.lib().dsp_stft_magnitude(chan_table(in_ptrs), len(in_ptrs), L_, N, H, window, K,
                                    chan_table(mag_ptrs), ld, C.byref(ex))
    check(st, "dsp_stft_magnitude")
    return out[:, :F, :K]


def render_stft(file, C_out: int, B: int, sr: float, plugin: Plugin | None,
                N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN, K: int | None = None,
                ld: int | None = None, out=None, mag=None, sample_offset: int = 0,
                L_file: int | None = None, ref=None, stream=None):
    """Render + STFT of the render.  Returns (out [C, nblocks*B], mag [C, F, K])."""
    in_ptrs, r = _rows(file)
    ref = r if r is not None else ref
    L_ = L_file if L_file is not None else (file.shape[1] if file is not None else 0)
    nb = num_blocks(L_, B)
    K = K if K is not None else N // 2 + 1
    ld = ld if ld is not None else K
    F = stft_frames(nb * B, N, H)
    if out is None:
        out = _alloc_like(ref, (C_out, max(nb * B, 1)))
    if mag is None:
        mag = _alloc_like(ref, (C_out, max(F, 1), ld))
    out_ptrs, oref = _rows(out)
    mag_ptrs = [mag[c].data_ptr() if _is_torch(mag) else mag[c].ctypes.data for c in range(C_out)]
    ex = _exec(oref, sample_offset, stream)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    res = _track(ex)
    st = L.lib().dsp_render_stft(chan_table(in_ptrs) if in_ptrs else None, len(in_ptrs), L_,
                                 chan_table(out_ptrs), C_out, B, sr,
                                 C.byref(ps) if ps is not None else None, N, H, window, K,
                                 chan_table(mag_ptrs), ld, C.byref(ex))
    check(st, "dsp_render_stft")
    _tls.result = res.value
    return out[:, : nb * B], mag[:, :F, :K]


def render_stft_host(x, C_out: int, B: int, sr: float, plugin: Plugin | None, stft: bool = True,
                     N: int = 8192, H: int = 4096, window: int = L.DSP_WIN_HANN, K: int | None = None,
                     chunk: int = 1 << 22, out=None, mag=None, sample_offset: int = 0, device: int = -1,
                     stream=None):
    """Host rows in, host rows out, streamed through HBM in chunks
    (dsp_render_stft_host).  x: numpy / pinned torch CPU [Cin, L] float32.
    Returns (out [C_out, ceil(L/B)B], mag [C_out, F, K] | None)."""
    K = K if K is not None else N // 2 + 1
    L_ = int(x.shape[1]) if x is not None else 0
    Lp = num_blocks(L_, B) * B
    F = stft_frames(Lp, N, H) if stft else 0
    out = np.empty((C_out, max(Lp, 1)), np.float32) if out is None else out
    if stft and mag is None:
        mag = np.empty((C_out, max(F, 1), K), np.float32)
    ptr = lambda a, c: a[c].data_ptr() if _is_torch(a) else a[c].ctypes.data  # noqa: E731
    in_ptrs = [ptr(x, c) for c in range(x.shape[0])] if x is not None else []
    ex = dsp_exec(device, 0, C.c_void_p(stream) if stream else None, sample_offset)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    res = _track(ex)
    st = L.lib().dsp_render_stft_host(chan_table(in_ptrs) if in_ptrs else None, len(in_ptrs), L_,
                                      chan_table([ptr(out, c) for c in range(C_out)]), C_out, B, sr,
                                      C.byref(ps) if ps is not None else None, N, H, window, K,
                                      chan_table([ptr(mag, c) for c in range(C_out)]) if stft else None, K, chunk,
                                      C.byref(ex))
    check(st, "dsp_render_stft_host")
    _tls.result = res.value
    return out[:, :Lp], (mag[:, :F] if stft else None)


def ir_analysis(plugin: Plugin | None, C_out: int = 2, sr: float = 48000.0,
                ir_len: int = IR_BUFFER_LENGTH, device=None):
    """compute_IR + fft_perform_and_get_magnitude.  Returns (ir [C, ir_len],
    mag [4*ir_len]) as torch tensors on `device`, or numpy when device is None."""
    if device is not None:
        import torch
        ir = torch.empty((C_out, ir_len), dtype=torch.float32, device=device)
        mag = torch.empty((4 * ir_len,), dtype=torch.float32, device=device)
        ir_ptrs = [ir[c].data_ptr() for c in range(C_out)]
        mptr = mag.data_ptr()
        ex = _exec(ir)
    else:
        ir = np.empty((C_out, ir_len), np.float32)
        mag = np.empty((4 * ir_len,), np.float32)
        ir_ptrs = [ir[c].ctypes.data for c in range(C_out)]
        mptr = mag.ctypes.data
        ex = _exec(None)
    ps = plugin.as_struct() if plugin is not None else None
    ex.flags |= plugin.exec_flags if plugin is not None else 0
    st = L.lib().dsp_ir_analysis(C.byref(ps) if ps is not None else None, C_out, sr, ir_len,
                                 chan_table(ir_ptrs), C.cast(C.c_void_p(mptr), L.FP), C.byref(ex))
    check(st, "dsp_ir_analysis")
    return ir, mag


def _fp(a):
    return C.cast(C.c_void_p(a.data_ptr() if _is_torch(a) else a.ctypes.data), L.FP)


def fft_forward(x):
    """fft_forward (dsp.cpp:74-103): real n -> (re, im), 1/sqrt(n) scaling."""
    n = x.shape[0]
    re, im = _alloc_like(x if _is_torch(x) else None, (n,)), _alloc_like(x if _is_torch(x) else None, (n,))
    ex = _exec(x if _is_torch(x) else None)
    check(L.lib().dsp_fft_forward(_fp(x), _fp(re), _fp(im), n, C.byref(ex)), "dsp_fft_forward")
    return re, im


def fft_reverse(re, im):
    """fft_reverse (dsp.cpp:106-132): Re(IDFT)/sqrt(n)."""
    n = re.shape[0]
    out = _alloc_like(re if _is_torch(re) else None, (n,))
    ex = _exec(re if _is_torch(re) else None)
    check(L.lib().dsp_fft_reverse(_fp(re), _fp(im), _fp(out), n, C.byref(ex)), "dsp_fft_reverse")
    return out


# --------------------------------------------------------------------------
# display reductions (long-file overviews)
# --------------------------------------------------------------------------

def minmax_decimate(x, pixels: int):
    """Per-pixel (max, min) of a 1-D signal, the reference's IR view
    (opengl.h:877-890).  Returns (vmax [pixels], vmin [pixels])."""
    ref = x if _is_torch(x) else None
    vmax = _alloc_like(ref, (max(pixels, 1),))
    vmin = _alloc_like(ref, (max(pixels, 1),))
    ex = _exec(ref)
    st = L.lib().dsp_minmax_decimate(_fp(x), x.shape[0], pixels, _fp(vmax), _fp(vmin), C.byref(ex))
    check(st, "dsp_minmax_decimate")
    return vmax[:pixels], vmin[:pixels]


def spectrogram_decimate(mag, pixels: int):
    """[F, K] magnitudes (row stride = mag's) -> [pixels, K] column maxima."""
    ref = mag if _is_torch(mag) else None
    F, K = int(mag.shape[0]), int(mag.shape[1])
    ld = (mag.stride(0) if _is_torch(mag) else mag.strides[0] // 4)
    out = _alloc_like(ref, (max(pixels, 1), K))
    ex = _exec(ref)
    st = L.lib().dsp_spectrogram_decimate(_fp(mag), F, K, ld, pixels, _fp(out), C.byref(ex))
    check(st, "dsp_spectrogram_decimate")
    return out[:pixels]
