"""module.py -- generic GPU dispatch of plugin sources (include/dspbench/module.h).

    code = compile_source(open("sine_test.cpp").read())     # hiprtc -> gfx950
    mod = Module(code)                                      # load on the GPU
    params = mod.default_parameters()
    mod.initialize_state(params, channels=2, sample_rate=48000.0)
    out = dspbench.render_offline(x, 2, 512, 48000.0, mod.plugin(params))
"""
from __future__ import annotations

import ctypes as C

from . import _lib as L
from ._lib import DspError, check


class CompileError(DspError):
    pass


def compile_source(source: str, name: str = "plugin.cpp") -> bytes:
    """Plugin C++ source -> gfx950 code object (no GPU needed)."""
    lib = L.lib()
    code, size = C.c_void_p(), C.c_uint64()
    log = C.create_string_buffer(1 << 16)
    st = lib.dsp_module_compile(source.encode(), name.encode(), C.byref(code), C.byref(size), log, len(log))
    if st != 0:
        raise CompileError(st, f"dsp_module_compile({name})", log.value.decode(errors="replace"))
    try:
        return C.string_at(code, size.value)
    finally:
        lib.dsp_module_free_code(code)


class Module:
    """A plugin's code object loaded on a GPU, with its device State."""

    def __init__(self, code: bytes, device: int = -1):
        self.handle = C.c_void_p()
        # bound now: at interpreter exit the module globals may already be gone
        self._destroy = L.lib().dsp_module_destroy
        self._code = C.create_string_buffer(code, len(code))
        check(L.lib().dsp_module_load(self._code, len(code), device, C.byref(self.handle)), "dsp_module_load")
        ps, ss, sl = C.c_uint32(), C.c_uint32(), C.c_int()
        check(L.lib().dsp_module_sizes(self.handle, C.byref(ps), C.byref(ss), C.byref(sl)), "dsp_module_sizes")
        self.params_size, self.state_size, self.stateless = ps.value, ss.value, bool(sl.value)

    def __del__(self):
        h = getattr(self, "handle", None)
        destroy = getattr(self, "_destroy", None)
        if h and destroy is not None:
            destroy(h)
            self.handle = None

    def default_parameters(self) -> bytes:
        buf = C.create_string_buffer(max(1, self.params_size))
        check(L.lib().dsp_module_default_parameters(self.handle, buf), "dsp_module_default_parameters")
        return buf.raw[:self.params_size]

    def initialize_state(self, params: bytes, channels: int, sample_rate: float,
                         arena_bytes: int = 16 << 20) -> None:
        buf = C.create_string_buffer(params, max(1, len(params)))
        check(L.lib().dsp_module_initialize_state(self.handle, buf, channels, sample_rate, arena_bytes),
              "dsp_module_initialize_state")

    def read_state(self) -> bytes:
        buf = C.create_string_buffer(max(1, self.state_size))
        check(L.lib().dsp_module_read_state(self.handle, buf), "dsp_module_read_state")
        return buf.raw[:self.state_size]

    def plugin(self, params: bytes, name: str = "generic"):
        from .api import Plugin
        return Plugin(L.DSP_PLUGIN_GENERIC, bytes(params), b"", name, self)
