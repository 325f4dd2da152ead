"""module.py -- generic GPU dispatch of plugin sources (include/dspbench/module.h).

    code = compile_source(open("sine_test.cpp").read())     # hiprtc -> gfx950
    mod = Module(code)                                      # load on the GPU
    params = mod.default_parameters()
    mod.initialize_state(params, channels=2, sample_rate=48000.0)
    out = dspbench.render_offline(x, 2, 512, 48000.0, mod.plugin(params))

The parameter descriptor (module.h) mirrors the reference's
Plugin_Descriptor (plugin.h:15-82): Descriptor.from_code(code) (no GPU) or
Module.descriptor; values <-> Parameters blob as
plugin_set_parameter_holder_from_values / _values_from_holder
(plugin.cpp:121-171); normalize / denormalize as plugin.h:173-233.
"""
from __future__ import annotations

import ctypes as C

from dataclasses import dataclass, field

from . import _lib as L
from ._lib import DspError, check

PARAM_TYPES = {L.DSP_PARAM_INT: "Int", L.DSP_PARAM_FLOAT: "Float", L.DSP_PARAM_ENUM: "Enum"}
DESC_ERRORS = ["Compiler_Success", "Compiler_Error_Recurse", "Compiler_Empty_Annotation",
               "Compiler_Invalid_Annotation", "Compiler_Missing_Min_Max", "Compiler_Min_Greater_Than_Max",
               "Compiler_Invalid_Min_Value", "Compiler_Invalid_Max_Value", "Compiler_Annotation_Type_Mismatch"]


@dataclass
class Param:
    """One annotated field of Parameters (Plugin_Descriptor_Parameter)."""
    name: str
    offset: int
    type: str                 # "Int" | "Float" | "Enum"
    error: str
    int_min: int = 0
    int_max: int = 0
    float_min: float = 0.0
    float_max: float = 0.0
    log: bool = False
    entries: list = field(default_factory=list)  # Enum: [(name, value), ...]
    _c: object = field(default=None, repr=False)

    def _enum_values(self):
        if not self.entries:
            return None
        return (C.c_int64 * len(self.entries))(*[v for _, v in self.entries])

    def _value(self, v) -> L.dsp_param_value:
        pv = L.dsp_param_value()
        if self.type == "Float":
            pv.float_value = float(v)
        elif self.type == "Int":
            pv.int_value = int(v)
        else:
            pv.enum_value = int(v)
        return pv

    def normalize(self, v) -> float:
        out = C.c_float()
        check(L.lib().dsp_param_normalize(C.byref(self._c), self._enum_values(), self._value(v), C.byref(out)),
              f"dsp_param_normalize({self.name})")
        return out.value

    def denormalize(self, x: float):
        out = L.dsp_param_value()
        check(L.lib().dsp_param_denormalize(C.byref(self._c), self._enum_values(), float(x), C.byref(out)),
              f"dsp_param_denormalize({self.name})")
        return out.float_value if self.type == "Float" else out.int_value


class Descriptor:
    """A plugin's parameter descriptor (module.h dsp_descriptor)."""

    def __init__(self, handle, owner=None):
        self.handle = handle
        self._owner = owner  # a Module keeps its descriptor alive; None: ours to free
        self._destroy = L.lib().dsp_descriptor_destroy
        info = L.dsp_plugin_descriptor()
        check(L.lib().dsp_descriptor_info(self.handle, C.byref(info)), "dsp_descriptor_info")
        self.params_size, self.params_align = info.params_size, info.params_align
        self.state_size, self.state_align = info.state_size, info.state_align
        self.error = DESC_ERRORS[info.error]
        self.parameters = []
        for i in range(info.num_parameters):
            p = L.dsp_param_desc()
            check(L.lib().dsp_descriptor_param(self.handle, i, C.byref(p)), "dsp_descriptor_param")
            ents = []
            for e in range(p.num_entries):
                v, nm = C.c_int64(), C.create_string_buffer(256)
                check(L.lib().dsp_descriptor_enum_entry(self.handle, i, e, C.byref(v), nm, 256), "enum entry")
                ents.append((nm.value.decode(), v.value))
            self.parameters.append(Param(p.name.decode(), p.offset, PARAM_TYPES[p.type], DESC_ERRORS[p.error],
                                         p.int_min, p.int_max, p.float_min, p.float_max, bool(p.float_log),
                                         ents, p))

    @staticmethod
    def from_code(code: bytes) -> "Descriptor":
        h = C.c_void_p()
        buf = C.create_string_buffer(code, len(code))
        check(L.lib().dsp_descriptor_from_code(buf, len(code), C.byref(h)), "dsp_descriptor_from_code")
        return Descriptor(h)

    def __del__(self):
        if getattr(self, "_owner", 1) is None and getattr(self, "handle", None):
            self._destroy(self.handle)
            self.handle = None

    def __getitem__(self, name: str) -> Param:
        for p in self.parameters:
            if p.name == name:
                return p
        raise KeyError(name)

    def params_from_values(self, values, holder: bytes = None) -> bytes:
        """values (one per parameter, or a {name: value} dict over a holder)
        -> the Parameters blob (plugin_set_parameter_holder_from_values)."""
        buf = C.create_string_buffer(bytes(holder) if holder is not None else b"", max(1, self.params_size))
        if isinstance(values, dict):
            cur = self.params_to_values(buf.raw[:self.params_size])
            values = [values.get(p.name, cur[i]) for i, p in enumerate(self.parameters)]
        arr = (L.dsp_param_value * max(1, len(self.parameters)))()
        for i, p in enumerate(self.parameters):
            arr[i] = p._value(values[i])
        check(L.lib().dsp_params_from_values(self.handle, arr, buf), "dsp_params_from_values")
        return buf.raw[:self.params_size]

    def params_to_values(self, holder: bytes) -> list:
        """The Parameters blob -> one value per parameter
        (plugin_set_parameter_values_from_holder)."""
        buf = C.create_string_buffer(bytes(holder), max(1, self.params_size))
        arr = (L.dsp_param_value * max(1, len(self.parameters)))()
        check(L.lib().dsp_params_to_values(self.handle, buf, arr), "dsp_params_to_values")
        return [arr[i].float_value if p.type == "Float" else arr[i].int_value
                for i, p in enumerate(self.parameters)]

    def __eq__(self, other) -> bool:
        return isinstance(other, Descriptor) and bool(L.lib().dsp_descriptor_equal(self.handle, other.handle))


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


def analyze_source(source: str) -> dict:
    """The facts dsp_module_compile stores for this source (dsp_plugin_analyze:
    the callback's LLVM IR read by the analysis; no GPU)."""
    f = L.dsp_callback_facts()
    check(L.lib().dsp_plugin_analyze(source.encode(), C.byref(f)), "dsp_plugin_analyze")
    return f.as_dict()


def analyze_source_shipped(source: str) -> dict:
    """The same analysis of the IR the module's own options (-O3, vectorised,
    unrolled) give (dsp_plugin_analyze_shipped; no GPU)."""
    f = L.dsp_callback_facts()
    check(L.lib().dsp_plugin_analyze_shipped(source.encode(), C.byref(f)), "dsp_plugin_analyze_shipped")
    return f.as_dict()


def code_facts(code: bytes) -> dict:
    """The facts a code object carries (dsp_code_facts; no GPU)."""
    f = L.dsp_callback_facts()
    buf = C.create_string_buffer(code, len(code))
    check(L.lib().dsp_code_facts(buf, len(code), C.byref(f)), "dsp_code_facts")
    return f.as_dict()


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

    @property
    def descriptor(self) -> "Descriptor":
        h = L.lib().dsp_module_descriptor(self.handle)
        if not h:
            raise DspError(L.DSP_ERR_INVALID, "Module.descriptor", "code object carries no descriptor")
        return Descriptor(C.c_void_p(h), owner=self)

    def plugin_from_values(self, values, name: str = "generic"):
        """A GENERIC plugin whose Parameters blob is built from parameter
        values over the defaults (plugin_populate_from_descriptor then
        plugin_set_parameter_holder_from_values, plugin.cpp:147-171,335-364)."""
        return self.plugin(self.descriptor.params_from_values(values, self.default_parameters()), name)

    @property
    def facts(self) -> dict:
        """What the callback's IR shows (dsp_module_facts): analyzed,
        reads_block, writes_state, input_control, gain_form, gain, why."""
        f = L.dsp_callback_facts()
        check(L.lib().dsp_module_facts(self.handle, C.byref(f)), "dsp_module_facts")
        return f.as_dict()

    def read_state(self) -> bytes:
        buf = C.create_string_buffer(max(1, self.state_size))
        check(L.lib().dsp_module_read_state(self.handle, buf), "dsp_module_read_state")
        return buf.raw[:self.state_size]

    def plugin(self, params: bytes, name: str = "generic", specialize: bool = True, verify: bool = False,
               serial_state: bool = False):
        """A GENERIC plugin over this module.  specialize=False runs the
        plugin's callback on every block (DSP_EXEC_NO_SPECIALIZE); by default
        a plugin whose block class its IR proves runs as that class
        (block_class).  verify=True checks blocks of every call against the
        callback (DSP_EXEC_VERIFY_CLASS; dspbench.api.last_result()).
        serial_state=True renders a State-writing callback as one chain
        (DSP_EXEC_SERIAL_STATE) instead of speculative segments (state_spec)."""
        from .api import Plugin
        flags = 0 if specialize else L.DSP_EXEC_NO_SPECIALIZE
        if verify:
            flags |= L.DSP_EXEC_VERIFY_CLASS
        if serial_state:
            flags |= L.DSP_EXEC_SERIAL_STATE
        return Plugin(L.DSP_PLUGIN_GENERIC, bytes(params), b"", name, self, exec_flags=flags)

    def state_spec(self) -> dict:
        """The module's last render of a State-writing callback in speculative
        segments (dsp_module_state_spec; waits for it): used, disabled,
        segments, blocks_per_segment, warmup_blocks, differed (pass 1, rerun 1,
        rerun 2), serial_reruns."""
        info = L.dsp_state_spec_info()
        check(L.lib().dsp_module_state_spec(self.handle, C.byref(info)), "dsp_module_state_spec")
        return info.as_dict()

    def debug_perturb_chain(self, block: int) -> None:
        """Test hook (dsp_module_debug DSP_MODULE_DEBUG_PERTURB_CHAIN): the
        next render that runs the State chain records a wrong State for
        `block`; its self-check must still render the serial chain's bits."""
        check(L.lib().dsp_module_debug(self.handle, 1, int(block)), "dsp_module_debug")

    def retired_tables(self) -> int:
        """Evicted TABLE-class blocks not freed yet (dsp_module_retired_tables)."""
        n = C.c_uint64()
        check(L.lib().dsp_module_retired_tables(self.handle, C.byref(n)), "dsp_module_retired_tables")
        return n.value

    def block_class(self, params: bytes, channels: int, block: int, sample_rate: float, stream=None):
        """(class, gain): "table" | "gain" | "gain_table" | "callback" (dsp_module_block_class),
        probing the plugin's callback on the current device if not known yet."""
        import torch
        buf = C.create_string_buffer(bytes(params), max(1, len(params)))
        cls, g = C.c_int32(), C.c_float()
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        ex = L.dsp_exec(-1, 0, C.c_void_p(st), 0)
        check(L.lib().dsp_module_block_class(self.handle, buf, len(params), channels, block, sample_rate,
                                             C.byref(cls), C.byref(g), C.byref(ex)), "dsp_module_block_class")
        return {L.DSP_BLOCK_TABLE: "table", L.DSP_BLOCK_GAIN: "gain",
                L.DSP_BLOCK_GAIN_TABLE: "gain_table"}.get(cls.value, "callback"), g.value
