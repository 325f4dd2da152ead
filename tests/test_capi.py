"""The C-ABI boundary on CPU: libdspbench.so loads, exports every function
include/dspbench/*.h declares, validates arguments, and -- with no GPU --
fails loudly instead of falling back to a CPU path.  The plugin-facing host
services (plugin_header.h) that run on the host are checked against libm /
numpy here; the GPU services (fft_forward/fft_reverse) in test_gpu_parity.py.
"""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

import dspbench as d
from dspbench import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# plugin_device.h defines the services inline for GPU-compiled plugins (it is
# handed to hiprtc as text, module.h): it declares nothing the library exports
HEADERS = sorted(h for h in glob.glob(os.path.join(REPO, "include", "dspbench", "*.h"))
                 if not h.endswith("plugin_device.h"))


def declared_functions(path):
    """Names of the function prototypes in a C header (comments and
    preprocessor lines stripped)."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    names = re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{}()]*(?:\([^;{}()]*\)[^;{}()]*)*\)\s*;", src)
    return sorted(set(n for n in names if n not in {"sizeof", "if", "while", "for", "return"}))


def test_headers_declare_the_boundary():
    names = {n for h in HEADERS for n in declared_functions(h)}
    for must in ("dsp_render_offline", "dsp_stft_magnitude", "dsp_render_stft", "dsp_ir_analysis",
                 "dsp_fft_forward", "dsp_fft_reverse", "fft_forward", "fft_reverse", "allocate_buffer",
                 "windowing_hamming", "pythagore_array", "sin_64", "tanh_32", "dsp_initializer_create"):
        assert must in names, must
    assert len(names) >= 94


@pytest.mark.parametrize("header", [os.path.basename(h) for h in HEADERS])
def test_library_exports_every_declared_symbol(header):
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions(os.path.join(REPO, "include", "dspbench", header))
               if not hasattr(lib, n)]
    assert not missing, f"{header}: declared but not exported: {missing}"


def test_abi_and_status_strings():
    L = d.lib()
    assert L.dsp_abi_version() == 3  # dspbench.h DSPBENCH_ABI_VERSION (bumped in round 5: facts.gain_table_form)
    for s, txt in [(0, b"ok"), (-1, b"invalid argument"), (-2, b"HIP runtime error"),
                   (-3, b"unsupported"), (-4, b"out of device memory"), (-5, b"no device"),
                   (-99, b"unknown status")]:
        L.dsp_status_string.restype = C.c_char_p
        assert L.dsp_status_string(s) == txt


@pytest.mark.parametrize("L_,N,H", [(0, 8192, 4096), (8191, 8192, 4096), (8192, 8192, 4096),
                                    (345_600_000, 8192, 4096), (10, 0, 1), (10, 4, 0), (9, 4, 2)])
def test_frame_count(L_, N, H):
    want = 0 if (N == 0 or H == 0 or L_ < N) else (L_ - N) // H + 1
    assert d.lib().dsp_stft_frame_count(L_, N, H) == want
    assert d.shard.stft_frames(L_, N, H) == want or N == 0


def _exec_host():
    ex = _lib.dsp_exec()
    ex.device = -1
    ex.flags = 0x3
    return ex


def test_invalid_arguments_rejected_before_device_use():
    L = d.lib()
    x = np.zeros((1, 1024), np.float32)
    rows = _lib.chan_table([x[0].ctypes.data])
    ex = _exec_host()
    assert L.dsp_render_offline(rows, 1, 1024, rows, 1, 0, 48000.0, None, C.byref(ex)) == -1  # B = 0
    assert L.dsp_render_offline(rows, 1, 1024, None, 1, 512, 48000.0, None, C.byref(ex)) == -1  # out NULL
    ex.sample_offset = 100
    assert L.dsp_render_offline(rows, 1, 1024, rows, 1, 512, 48000.0, None, C.byref(ex)) == -1
    L.dsp_last_error.restype = C.c_char_p
    assert b"sample_offset" in L.dsp_last_error()
    assert L.dsp_render_offline(rows, 1, 1024, rows, 0, 512, 48000.0, None, C.byref(ex)) == 0   # C = 0: no-op


@pytest.mark.parametrize("N,H,window,K,ld,what", [
    (8192, 4096, 7, 4097, 4097, b"window"),        # not a DSP_WIN_* kind
    (8192, 4096, -1, 4097, 4097, b"window"),
    (6000, 3000, 1, 3001, 3001, b"N="),            # not a power of two
    (16384, 4096, 1, 8193, 8193, b"N="),           # above 8192
    (8192, 0, 1, 4097, 4097, b"hop"),
    (8192, 4096, 1, 0, 4097, b"K="),
    (8192, 4096, 1, 5000, 5000, b"K="),            # neither <= N/2+1 nor N
    (8192, 4096, 1, 4097, 4096, b"ld="),           # rows overlap
])
def test_stft_arguments_rejected_before_device_use(N, H, window, K, ld, what):
    """dsp_stft_magnitude and dsp_render_stft refuse a bad shape before they
    touch a device (so this runs without one) and name the argument."""
    L = d.lib()
    L.dsp_last_error.restype = C.c_char_p
    x = np.zeros((1, 16384), np.float32)
    m = np.zeros((1, 8 * 8193), np.float32)
    rows, mrows = _lib.chan_table([x[0].ctypes.data]), _lib.chan_table([m[0].ctypes.data])
    ex = _exec_host()
    assert L.dsp_stft_magnitude(rows, 1, 16384, N, H, window, K, mrows, C.c_uint64(ld), C.byref(ex)) == -1
    assert what in L.dsp_last_error()
    assert L.dsp_render_stft(rows, 1, 16384, rows, 1, 512, C.c_float(48000.0), None, N, H, window, K, mrows,
                             C.c_uint64(ld), C.byref(ex)) == -1
    assert what in L.dsp_last_error()


def test_generic_ir_analysis_rejects_more_than_16_channels():
    """The generic driver's channel table holds 16 pointers: a GENERIC
    plugin's IR analysis with C = 17 is refused before any device or module
    use (the module handle here is never dereferenced)."""
    L = d.lib()
    bufs = np.zeros((17, 2048), np.float32)
    mag = np.zeros(8192, np.float32)
    rows = _lib.chan_table([bufs[c].ctypes.data for c in range(17)])
    plug = _lib.dsp_plugin(_lib.DSP_PLUGIN_GENERIC, 0, None, 0, None, C.c_void_p(0x1000))
    ex = _exec_host()
    st = L.dsp_ir_analysis(C.byref(plug), 17, 48000.0, 2048, rows, mag.ctypes.data_as(_lib.FP), C.byref(ex))
    assert st == -1
    L.dsp_last_error.restype = C.c_char_p
    assert b"1..16 channels" in L.dsp_last_error()


@pytest.mark.skipif(d.lib().dsp_device_count() > 0, reason="a GPU is visible")
def test_no_gpu_fails_loudly_no_cpu_fallback():
    """The product path has no CPU fallback: without a device every compute
    entry point returns DSP_ERR_NO_DEVICE (or a HIP error), never DSP_OK."""
    L = d.lib()
    x = np.ones((1, 8192), np.float32)
    y = np.zeros((1, 8192), np.float32)
    m = np.zeros((1, 4097), np.float32)
    xi, yo, mo = (_lib.chan_table([a[0].ctypes.data]) for a in (x, y, m))
    ex = _exec_host()
    for st in (L.dsp_render_offline(xi, 1, 8192, yo, 1, 512, 48000.0, None, C.byref(ex)),
               L.dsp_stft_magnitude(xi, 1, 8192, 8192, 4096, 1, 4097, mo, 4097, C.byref(ex)),
               L.dsp_fft_forward(*(a.ctypes.data_as(C.POINTER(C.c_float)) for a in (x, y, m)), 16, C.byref(ex))):
        assert st in (-5, -2), st
    with pytest.raises(d.DspError):
        d.render_offline(x, 1, 512, 48000.0, d.Plugin.gain_test(0.2))


# ---- plugin-facing host services (plugin_header.h) ----------------------------

@pytest.fixture(scope="module")
def svc():
    lib = C.CDLL(_lib.LIB_PATH)
    f, dbl = C.c_float, C.c_double
    for n in ("sin", "cos", "tan", "fabs", "ceil", "floor", "sqrt", "exp", "log10", "log", "asin", "acos",
              "atan", "sinh", "cosh", "tanh"):
        getattr(lib, n + "_32").restype, getattr(lib, n + "_32").argtypes = f, [f]
        getattr(lib, n + "_64").restype, getattr(lib, n + "_64").argtypes = dbl, [dbl]
    for n in ("pow", "fmod", "atan2"):
        getattr(lib, n + "_32").restype, getattr(lib, n + "_32").argtypes = f, [f, f]
        getattr(lib, n + "_64").restype, getattr(lib, n + "_64").argtypes = dbl, [dbl, dbl]
    lib.dsp_initializer_create.restype = C.c_void_p
    lib.dsp_initializer_create.argtypes = [C.c_size_t, C.c_int]
    lib.dsp_initializer_used.restype = C.c_size_t
    lib.dsp_initializer_used.argtypes = [C.c_void_p]
    lib.dsp_initializer_reset.argtypes = [C.c_void_p]
    lib.dsp_initializer_destroy.argtypes = [C.c_void_p]
    lib.allocate_buffer.restype = C.POINTER(C.c_float)
    lib.allocate_buffer.argtypes = [C.c_int, C.c_void_p]
    lib.allocate_buffers.restype = C.POINTER(C.POINTER(C.c_float))
    lib.allocate_buffers.argtypes = [C.c_int, C.c_int, C.c_void_p]
    lib.allocate_bytes.restype = C.c_void_p
    lib.allocate_bytes.argtypes = [C.c_int, C.c_void_p]
    for n in ("gain_32_array", "dc_offset_32_array"):
        getattr(lib, n).argtypes = [C.c_void_p, C.c_void_p, f, C.c_int]
    for n in ("sqrt", "abs", "ln", "log2", "log10", "to_db", "from_db"):
        getattr(lib, n + "_32_array").argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.set_array.argtypes = [f, C.c_void_p, C.c_int]
    for n in ("add_array", "product_array", "pythagore_array"):
        getattr(lib, n).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    lib.copy_array.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.zero_array.argtypes = [C.c_void_p, C.c_int]
    lib.windowing_hamming.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    return lib


def test_scalar_math_services(svc):
    import math
    for n, fn in [("sin", np.sin), ("cos", np.cos), ("exp", np.exp), ("sqrt", np.sqrt), ("tanh", np.tanh),
                  ("atan", np.arctan), ("log", np.log), ("log10", np.log10), ("floor", np.floor)]:
        for v in (0.25, 0.5, 1.5, 3.0):
            assert getattr(svc, n + "_64")(v) == getattr(math, n)(v)  # libm, as the reference
            assert getattr(svc, n + "_32")(v) == pytest.approx(float(fn(np.float32(v))), rel=2e-7)
    assert svc.pow_64(2.0, 10.0) == 1024.0 and svc.fmod_64(7.5, 2.0) == 1.5
    assert svc.atan2_32(1.0, 1.0) == pytest.approx(np.pi / 4, rel=1e-7)


def test_arena_allocators(svc):
    ini = svc.dsp_initializer_create(1 << 16, -1)
    assert ini
    b = svc.allocate_buffer(100, ini)
    assert C.addressof(b.contents) % 16 == 0
    bufs = svc.allocate_buffers(64, 3, ini)
    ptrs = [C.addressof(bufs[i].contents) for i in range(3)]
    assert all(p % 16 == 0 for p in ptrs) and len(set(ptrs)) == 3
    assert svc.allocate_bytes(7, ini) and svc.dsp_initializer_used(ini) >= 400 + 3 * 256
    svc.dsp_initializer_reset(ini)
    assert svc.dsp_initializer_used(ini) == 0
    svc.dsp_initializer_destroy(ini)


def test_array_services(svc):
    rng = np.random.default_rng(3)
    a = (rng.random(1000, dtype=np.float32) + 0.01).astype(np.float32)
    b = rng.random(1000, dtype=np.float32)
    out = np.empty_like(a)
    p = lambda z: z.ctypes.data  # noqa: E731
    svc.gain_32_array(p(a), p(out), 0.2, 1000)
    assert np.array_equal(out, a * np.float32(0.2))
    svc.dc_offset_32_array(p(a), p(out), 0.5, 1000)
    assert np.array_equal(out, a + np.float32(0.5))
    svc.add_array(p(a), p(b), p(out), 1000)
    assert np.array_equal(out, a + b)
    svc.product_array(p(a), p(b), p(out), 1000)
    assert np.array_equal(out, a * b)
    svc.pythagore_array(p(a), p(b), p(out), 1000)
    assert np.allclose(out, np.hypot(a, b), rtol=2e-7)
    svc.sqrt_32_array(p(a), p(out), 1000)
    assert np.array_equal(out, np.sqrt(a))
    svc.to_db_32_array(p(a), p(out), 1000)   # ln * 20/ln 10 (ref dsp.cpp:226-239)
    assert np.allclose(out, 20 * np.log10(a.astype(np.float64)), rtol=1e-5, atol=1e-5)
    svc.from_db_32_array(p(out), p(b), 1000)
    assert np.allclose(b, a, rtol=1e-5)
    svc.set_array(0.25, p(out), 1000)
    assert (out == 0.25).all()
    svc.copy_array(p(a), p(out), 1000)
    assert np.array_equal(out, a)
    svc.zero_array(p(out), 1000)
    assert not out.any()


def overlapping_copy_semantics(h, shift_right):
    """copy_array(h, h + 1, n - 1) / copy_array(h + 1, h, n - 1) as the device
    build's copy_array (plugin_device.h: element by element, first to last)
    does it."""
    h = h.copy()
    n = h.size
    if shift_right:
        for i in range(n - 1):
            h[i + 1] = h[i]
    else:
        for i in range(n - 1):
            h[i] = h[i + 1]
    return h


def test_copy_array_overlap_matches_the_device_build(svc):
    """Overlapping rows (a delay line shifted in place): the host build's
    copy_array copies first to last like the device build's, so the same
    plugin source renders the same on both (a shift right repeats h[0]; the
    GPU side: tests/test_gpu_parity.py::test_copy_array_overlap_on_the_device)."""
    h = np.arange(1, 65, dtype=np.float32)
    for right in (True, False):
        x = h.copy()
        base = x.ctypes.data
        if right:
            svc.copy_array(base, base + 4, 63)
        else:
            svc.copy_array(base + 4, base, 63)
        assert np.array_equal(x, overlapping_copy_semantics(h, right)), right


def test_windowing_hamming_service(svc, oracle):
    x = np.ones(2048, np.float32)
    y = np.empty_like(x)
    svc.windowing_hamming(x.ctypes.data, y.ctypes.data, 2048)
    assert np.max(np.abs(y - oracle.np_window(oracle.WIN_HAMMING, 2048))) <= 6e-8


def test_library_has_no_unresolved_internal_symbols():
    """Every symbol of the library's own namespace is defined in it (a
    kernel file missing from the Makefile shows up here, not at dlopen on
    the GPU box with immediate binding)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    bad = [l for l in out.splitlines() if "dspb" in l or " dsp_" in l]
    assert not bad, bad
    C.CDLL(_lib.LIB_PATH, mode=os.RTLD_NOW)


def test_render_loop_rejects_empty_file_and_bad_cursor():
    """Loop mode over an empty file would spin forever in the reference
    (audio.cpp:104); here it is refused before any device use, as is a cursor
    past the file."""
    L = d.lib()
    x = np.zeros((1, 100), np.float32)
    rows = _lib.chan_table([x[0].ctypes.data])
    ex = _lib.dsp_exec(-1, 0, None, 0)
    cur = C.c_uint64()
    assert L.dsp_render_loop(rows, 1, 0, 0, rows, 1, 64, 4, 48000.0, None, C.byref(cur), C.byref(ex)) == -1
    assert L.dsp_render_loop(rows, 1, 100, 100, rows, 1, 64, 4, 48000.0, None, C.byref(cur), C.byref(ex)) == -1
    # the next cursor is computed before anything runs
    L.dsp_render_loop(rows, 1, 100, 30, rows, 1, 64, 0, 48000.0, None, C.byref(cur), C.byref(ex))
    assert cur.value == 30
