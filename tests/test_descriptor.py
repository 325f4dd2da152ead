"""SURVEY 8 a8 through the product: the plugin parameter descriptor built by
dsp_module_compile (module.h; the reference's parse_plugin_descriptor,
compiler.cpp:944-1164), values <-> Parameters blob marshalling
(plugin.cpp:121-171) and normalisation (plugin.h:173-233).

Pinned by the reference's own tests: K3 (test/tests.cpp:102-212, the
plugin_with_parameters descriptor {Int[0,4]@0, Float[0,1]@4, Enum(4)@8},
defaults {0, 0.9f, A}, state {0.1f}) and K6 (test/tests.cpp:305-348,
normalisation round trips), and by the oracle's restated normalisation
(oracle/oracle.c).  The CPU tests need no GPU: the descriptor is read from
the code object's ELF; the GPU tests load the module and use the blobs.
"""
import os
import struct

import numpy as np
import pytest

import dspbench as d
from dspbench.module import Descriptor, compile_source

HERE = os.path.dirname(os.path.abspath(__file__))
MODS = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "modules")


def ref_code(name):
    p = os.path.join(MODS, f"mod_{name}.co")
    if not os.path.exists(p):
        pytest.skip("dsp-bench_amd/modules not built (tools/make_plugin_modules.py)")
    return open(p, "rb").read()


def desc_of(src):
    return Descriptor.from_code(compile_source(src, "t.cpp"))


# the stock plugins' annotations (build/*.cpp, test/*.cpp in the reference),
# as the descriptor must report them: name, type, range / enumerators, offset
STOCK = {
    "plugin_with_parameters": [("ish", "Int", (0, 4), 0), ("gain", "Float", (0.0, 1.0), 4),
                               ("truc", "Enum", [("A", 0), ("B", 1), ("C", 2), ("D", 3)], 8)],
    "gain_test": [("gain", "Float", (0.0, 2.0), 0)],
    "IR_test": [("gain", "Float", (0.0, 1.0), 0), ("step", "Float", (np.float32(0.001), np.float32(0.1)), 4)],
    "sine_test": [("gain", "Float", (0.0, 0.5), 0), ("frequency", "Float", (500.0, 20000.0), 4),
                  ("test_enum_param", "Enum", [("A", 0), ("B", 1), ("C", 2)], 8)],
    "handmade_test": [("initial_gain", "Float", (0.0, 1.0), 0),
                      ("slope", "Enum", [("linear", 0), ("logarythmic", 1)], 4),
                      ("step", "Float", (0.0, np.float32(0.1)), 8)],
    "buffer_test": [("dummy", "Float", (0.0, 1.0), 0)],
    "static_gain_plugin": [], "no_op": [], "template_plugin": [],
}


def check_params(D, want):
    assert D.error == "Compiler_Success"
    assert [p.name for p in D.parameters] == [w[0] for w in want]
    for p, (name, typ, rng, off) in zip(D.parameters, want):
        assert p.type == typ and p.offset == off and p.error == "Compiler_Success", p
        if typ == "Int":
            assert (p.int_min, p.int_max) == rng
        elif typ == "Float":
            assert (np.float32(p.float_min), np.float32(p.float_max)) == (np.float32(rng[0]), np.float32(rng[1]))
        else:
            assert p.entries == rng


def test_k3_descriptor_from_the_code_object():
    """K3 (test/tests.cpp:102-160) through the product, no GPU."""
    D = Descriptor.from_code(ref_code("plugin_with_parameters"))
    check_params(D, STOCK["plugin_with_parameters"])
    assert (D.params_size, D.params_align, D.state_size, D.state_align) == (12, 4, 4, 4)


@pytest.mark.parametrize("name", sorted(STOCK))
def test_stock_plugin_descriptors(name):
    check_params(Descriptor.from_code(ref_code(name)), STOCK[name])


def test_descriptor_forms_and_layout():
    """typedef'd struct, FLOAT_PARAM_LOG, enum class with explicit values,
    several declarators, unannotated and padded fields, a plugin's own
    annotation macros, raw annotate attributes."""
    src = r'''
#include "plugin_header.h"
#define MY_INT(a, b) __attribute__((annotate("Int " #a " " #b))) int
enum class Mode : int { Off = -1, Soft = 4, Hard = 40 };
typedef struct {
    double unannotated;                       // not a parameter (no annotation)
    FLOAT_PARAM_LOG(20.0f, 20000.0f) cutoff;
    MY_INT(-3,  7) semis, octave;
    char pad;
    ENUM_PARAM(Mode) mode;
    __attribute__((annotate("Float" " -1" " 1"))) float pan;
} Parameters;
struct State {};
Parameters default_parameters() { Parameters p{}; return p; }
State initialize_state(const Parameters&, const unsigned, const float, void*) { return State{}; }
void audio_callback(const Parameters&, State&, float**, const u32, const u32, const real32) {}
'''
    D = desc_of(src)
    assert D.error == "Compiler_Success"
    names = [p.name for p in D.parameters]
    assert names == ["cutoff", "semis", "octave", "mode", "pan"]
    c, s, o, m, pan = D.parameters
    assert (c.type, c.float_min, c.float_max, c.log, c.offset) == ("Float", 20.0, 20000.0, True, 8)
    assert (s.type, s.int_min, s.int_max, s.offset) == ("Int", -3, 7, 12)
    assert (o.type, o.int_min, o.int_max, o.offset) == ("Int", -3, 7, 16)
    assert (m.type, m.entries, m.offset) == ("Enum", [("Off", -1), ("Soft", 4), ("Hard", 40)], 24)
    assert (pan.type, pan.float_min, pan.float_max, pan.offset) == ("Float", -1.0, 1.0, 28)
    assert (D.params_size, D.params_align) == (32, 8)


@pytest.mark.parametrize("field,flag", [
    ('__attribute__((annotate("Int 4 0"))) int x;', "Compiler_Min_Greater_Than_Max"),
    ('__attribute__((annotate("Int 0 4"))) float x;', "Compiler_Annotation_Type_Mismatch"),
    ('__attribute__((annotate("Float 0 1"))) int x;', "Compiler_Annotation_Type_Mismatch"),
    ('__attribute__((annotate("Enum"))) int x;', "Compiler_Annotation_Type_Mismatch"),
    ('__attribute__((annotate("Float 0 1 lin"))) float x;', "Compiler_Invalid_Annotation"),
    ('__attribute__((annotate("Float 0"))) float x;', "Compiler_Missing_Min_Max"),
    ('__attribute__((annotate("Int 0 1 2"))) int x;', "Compiler_Missing_Min_Max"),
    ('__attribute__((annotate(""))) float x;', "Compiler_Empty_Annotation"),
    ('__attribute__((annotate("Bogus 0 1"))) float x;', "Compiler_Invalid_Annotation"),
])
def test_invalid_annotations_fail_the_compile(field, flag):
    """compiler.cpp:1009-1146: an invalid annotation is a compile error
    carrying the reference's flag."""
    src = ('#include "plugin_header.h"\nstruct Parameters { ' + field + ' };\nstruct State {};\n'
           'Parameters default_parameters() { return Parameters{}; }\n'
           'State initialize_state(const Parameters&, const unsigned, const float, void*) { return State{}; }\n'
           'void audio_callback(const Parameters&, State&, float**, const u32, const u32, const real32) {}\n')
    with pytest.raises(d.module.CompileError) as e:
        compile_source(src, "bad.cpp")
    assert flag in str(e.value)


def test_values_to_holder_and_back():
    """plugin_set_parameter_holder_from_values / _values_from_holder: 4-byte
    stores at the descriptor offsets, other bytes untouched."""
    D = Descriptor.from_code(ref_code("plugin_with_parameters"))
    holder = D.params_from_values([3, 0.25, 2], b"\xaa" * 12)
    assert holder == struct.pack("<ifi", 3, 0.25, 2)
    assert D.params_to_values(holder) == [3, 0.25, 2]
    h2 = D.params_from_values({"gain": 0.75}, holder)
    assert struct.unpack("<ifi", h2) == (3, 0.75, 2)


def test_descriptor_equal():
    a = Descriptor.from_code(ref_code("plugin_with_parameters"))
    b = Descriptor.from_code(ref_code("plugin_with_parameters"))
    c = Descriptor.from_code(ref_code("sine_test"))
    assert a == b and not (a == c)


def test_k6_normalisation_through_the_product(oracle):
    """K6 (test/tests.cpp:305-348) on dsp_param_normalize / _denormalize,
    and agreement with the oracle's restatement over random values."""
    D = desc_of(r'''
#include "plugin_header.h"
enum E { e0 = 0, e1 = 1, e256 = 256 };
struct Parameters { INT_PARAM(4, 8) i; FLOAT_PARAM(4.0f, 8.0f) f; ENUM_PARAM(E) e; FLOAT_PARAM_LOG(20.0f, 20000.0f) lg; };
struct State {};
Parameters default_parameters() { return Parameters{6, 6.0f, e256, 1000.0f}; }
State initialize_state(const Parameters&, const unsigned, const float, void*) { return State{}; }
void audio_callback(const Parameters&, State&, float**, const u32, const u32, const real32) {}
''')
    pi, pf, pe, pl = D.parameters
    assert pi.normalize(6) == 0.5 and pi.denormalize(0.5) == 6
    assert pf.normalize(6.0) == 0.5 and pf.denormalize(0.5) == 6.0
    assert pe.normalize(256) == 1.0 and pe.denormalize(pe.normalize(256)) == 256
    with pytest.raises(d.DspError):
        pe.normalize(7)  # no such enumerator (the reference asserts)
    L = oracle.lib()
    rng = np.random.default_rng(3)
    for v in rng.uniform(0.0, 10.0, 200).astype(np.float32):
        assert pf.normalize(v) == L.oracle_normalize_float(4.0, 8.0, 0, float(v))
        assert pl.normalize(v * 3000) == L.oracle_normalize_float(20.0, 20000.0, 1, float(v * 3000))
    for x in rng.uniform(0.0, 1.0, 200).astype(np.float32):
        assert pi.denormalize(x) == L.oracle_denormalize_int(4, 8, float(x))
        assert np.float32(pf.denormalize(x)) == np.float32(L.oracle_denormalize_float(4.0, 8.0, 0, float(x)))
        assert np.float32(pl.denormalize(x)) == np.float32(L.oracle_denormalize_float(20.0, 20000.0, 1, float(x)))
        assert pe.denormalize(x) == [0, 1, 256][L.oracle_denormalize_enum_index(3, float(x))]


@pytest.mark.gpu
def test_k3_module_defaults_and_state_through_the_descriptor(torch_cuda):
    """K3 (test/tests.cpp:163-212) through the loaded module: default_parameters
    read back through the descriptor, initialize_state's State."""
    mod = d.module.Module(ref_code("plugin_with_parameters"))
    D = mod.descriptor
    vals = D.params_to_values(mod.default_parameters())
    assert vals[0] == 0 and abs(vals[1] - 0.9) < 1e-3 and vals[2] == 0  # {0, 0.9f, A}
    mod.initialize_state(mod.default_parameters(), 1, 44100.0)
    assert abs(struct.unpack("<f", mod.read_state()[:4])[0] - 0.1) < 1e-3


@pytest.mark.gpu
def test_values_drive_the_gpu_render_and_ir_analysis(torch_cuda, oracle):
    """A host sets parameters by name (compute_IR's holder from values,
    plugin.cpp:36-39): gain_test's render and IR_test's IR analysis use the
    marshalled blob, bit-exact against the oracle."""
    mod = d.module.Module(ref_code("gain_test"))
    mod.initialize_state(mod.default_parameters(), 2, 48000.0)
    x = np.random.default_rng(9).uniform(-1, 1, (2, 10_000)).astype(np.float32)
    got = d.render_offline(torch_cuda.from_numpy(x).cuda(), 2, 512, 48000.0,
                           mod.plugin_from_values({"gain": 0.61})).cpu().numpy()
    want = oracle.render_offline([x[0], x[1]], 2, 512, 48000.0, oracle.restated_plugin("gain_test", [0.61]))
    assert np.array_equal(got, want)
    ir_mod = d.module.Module(ref_code("IR_test"))
    ir_mod.initialize_state(ir_mod.default_parameters(), 2, 48000.0)
    plug = ir_mod.plugin_from_values({"gain": 0.8, "step": 0.01})
    ir, _ = d.ir_analysis(plug, C_out=2, device="cuda")
    assert np.array_equal(ir.cpu().numpy()[1], oracle.ir_ramp_reference(0.8, 0.01, 2048))
