"""What a plugin's audio_callback does with its block, read from its own
LLVM IR (csrc/ir_proof.cpp; module.h dsp_callback_facts) -- CPU only: the
analysis compiles the plugin through comgr, no GPU.

The facts decide every fast path of a GENERIC plugin (module.cpp): a block
class (TABLE: reads no sample; GAIN: every store x * g at x's address, one g,
control flow free of samples) and parallel blocks (the State never written,
no global memory written).  The reference runs the callback on every block,
in order (audio.cpp:160-165), so each fact must be conservative: the test
plugins under tests/plugins/ are the cases a probe cannot see.
"""
import os

import pytest

import dspbench.module as dm

HERE = os.path.dirname(os.path.abspath(__file__))
PLUG = os.path.join(HERE, "plugins")
REF = "/root/reference"


def facts_of(path):
    with open(path) as f:
        return dm.analyze_source(f.read())


# (analyzed, reads_block, writes_state, input_control, gain_form) per plugin
STOCK = {
    "build/IR_test.cpp": (True, False, False, False, False),        # a table: the ramp, no sample read
    "build/handmade_test.cpp": (True, False, False, False, False),  # a table
    "build/gain_test.cpp": (True, True, False, False, True),        # x * param.gain
    "test/static_gain_plugin.cpp": (True, True, False, False, True),  # x * state.gain, State only read
    "test/no_op.cpp": (True, False, False, False, True),            # no store: the identity
    "build/template_plugin.cpp": (True, False, False, False, True),
    "test/plugin_with_parameters.cpp": (True, False, False, False, True),
    "build/sine_test.cpp": (True, False, True, False, False),       # writes its phase to State
    "build/buffer_test.cpp": (False, False, True, False, False),    # stores through arena pointers
}


@pytest.mark.parametrize("rel", sorted(STOCK))
def test_stock_plugin_facts(rel):
    path = os.path.join(REF, rel)
    if not os.path.exists(path):
        pytest.skip("reference sources not present")
    f = facts_of(path)
    got = (f["analyzed"], f["reads_block"], f["writes_state"], f["input_control"], f["gain_form"])
    assert got == STOCK[rel], (rel, f)
    # where g is read, so that the host knows it without the callback
    if rel.endswith("gain_test.cpp"):
        assert (f["gain_source"], f["gain_offset"]) == ("P", 0)  # Parameters.gain
    if rel.endswith("static_gain_plugin.cpp"):
        assert (f["gain_source"], f["gain_offset"]) == ("S", 0)  # State.gain
    if rel.endswith("no_op.cpp"):
        assert (f["gain_source"], f["gain_constant"]) == ("K", 1.0)  # no store: the identity


# test plugins (tests/plugins, written for these tests): what the probes of
# round 3 could not tell apart from a gain / a table
TEST = {
    "clip_beyond_2000.cpp": (True, True, False, False, False),   # stores a select on the sample
    "exact_value_branch.cpp": (True, True, False, False, False),  # x == 0.25 -> 7
    "gain_until_loud.cpp": (True, True, False, True, False),     # a branch on a sample: input control
    "static_counter.cpp": (False, True, False, False, False),    # a function-local static: global memory
    "fade_in.cpp": (True, True, False, False, False),            # g varies with the position
    "balance.cpp": (True, True, False, False, False),            # two different gains
    "gain_twice.cpp": (True, True, False, False, True),          # x * g twice: the probe of ones refuses it
    "half_block.cpp": (True, True, False, False, True),          # x * g on half the block: the probe refuses it
    "state_shaper.cpp": (True, True, False, False, False),       # State read only: parallel, no class
    "dc_level.cpp": (True, False, False, False, False),          # a table (set_array)
}


# the gain-table form (round 5): every element stored at most once as x * G
GAIN_TABLE = {"balance.cpp": True, "fade_in.cpp": True, "half_block.cpp": True, "gain_twice.cpp": False,
              "clip_beyond_2000.cpp": False, "exact_value_branch.cpp": False, "gain_until_loud.cpp": False,
              "state_shaper.cpp": False, "dc_level.cpp": False}


@pytest.mark.parametrize("name", sorted(GAIN_TABLE))
def test_gain_table_form_of_test_plugins(name):
    f = facts_of(os.path.join(PLUG, name))
    assert f["gain_table_form"] == GAIN_TABLE[name], (name, f)
    if not f["gain_table_form"]:
        assert f["table_why"], f


# bodies that store each element at most once as x * G (True), or not / not
# provably (False): the refusals are the cases a probe of ones cannot see
GT_SNIPPETS = {
    "pan_by_channel_loop": ("for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) "
                            "out[c][s] *= (c == 0 ? p.g : 1.0f - p.g);", True),
    "window_shape": ("for (u32 s = 0; s < B; ++s) { const float w = 0.5f - 0.5f * cosf(6.2831853f * s / B); "
                     "for (u32 c = 0; c < C; ++c) out[c][s] *= w; }", True),
    "repeat_loop": ("for (int r = 0; r < 2; ++r) for (u32 s = 0; s < B; ++s) out[0][s] *= p.g;", False),
    "same_channel_twice": ("for (u32 s = 0; s < B; ++s) out[0][s] *= p.g; "
                           "for (u32 s = 0; s < B; ++s) out[0][s] *= 0.5f;", False),
    "loop_and_const_channel": ("for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) out[c][s] *= p.g; "
                               "out[0][0] *= 2.0f;", False),
    "shifted_index": ("for (u32 s = 0; s + 1 < B; ++s) out[0][s + 1] *= p.g;", False),
    "gain_from_a_sample": ("for (u32 s = 0; s < B; ++s) out[0][s] *= out[1][0];", False),
    "channel_from_sample_loop": ("for (u32 s = 0; s < B && s < C; ++s) out[s][s] *= p.g;", False),
    # a cycle entered in its middle (no natural loop): refused whatever the index
    "irreducible_goto": ("u32 s = 0; if (C > 1) goto mid; top: out[0][s] *= p.g; mid: ++s; if (s < B) goto top;",
                         False),
    # an 8-bit index wraps within one run of its loop (B > 256 stores an
    # element twice): only i32 / i64 counters are induction variables
    "wrapping_u8_index": ("unsigned char i = 0; for (u32 n = 0; n < B; ++n, ++i) out[0][i] *= p.g;", False),
    "u32_index_same_loop": ("unsigned i = 0; for (u32 n = 0; n < B; ++n, ++i) out[0][i] *= p.g;", True),
}


@pytest.mark.parametrize("case", sorted(GT_SNIPPETS))
def test_gain_table_constructs(case):
    body, want = GT_SNIPPETS[case]
    f = dm.analyze_source(snippet("", body))
    assert f["gain_table_form"] == want, f


@pytest.mark.parametrize("name", sorted(TEST))
def test_test_plugin_facts(name):
    f = facts_of(os.path.join(PLUG, name))
    got = (f["analyzed"], f["reads_block"], f["writes_state"], f["input_control"], f["gain_form"])
    assert got == TEST[name], (name, f)
    if not f["analyzed"] or not f["gain_form"]:
        assert f["why"], f  # the reason is reported


def test_facts_travel_in_the_code_object():
    """dsp_module_compile stores the facts in the code object; dsp_code_facts
    reads them back without a GPU, equal to a fresh analysis."""
    src = open(os.path.join(PLUG, "gain_until_loud.cpp")).read()
    code = dm.compile_source(src, "gain_until_loud.cpp")
    f = dm.code_facts(code)
    assert f["present"] and f == dm.analyze_source(src)


SNIPPETS = {
    # an atomic on a global: outside the analysis
    "atomic": ("__device__ int hits; ", "atomicAdd(&hits, 1); out[0][0] *= p.g;", (False, None)),
    # a pointer into the block kept in private memory and used later
    "alias_local": ("", "float *q[2] = {out[0], out[0] + 1}; for (u32 s = 0; s + 1 < B; ++s) q[s & 1][s / 2] = 0.0f;",
                    (None, None)),
    # the block's address as a number decides the output
    "address": ("", "out[0][0] = (float)(((unsigned long long)out[0]) & 255);", (False, None)),
    # reads a neighbour: not a gain
    "neighbour": ("", "for (u32 s = 1; s < B; ++s) out[0][s] = out[0][s - 1] * p.g;", (True, False)),
    # a double-precision product rounded back: the optimiser proves it is the
    # float product (24 x 24 bits fit f64 exactly, one rounding), so a gain
    "f64": ("", "for (u32 s = 0; s < B; ++s) out[0][s] = (float)((double)out[0][s] * (double)p.g);", (True, True)),
    # products stored at another element's address
    "swap_channels": ("", "for (u32 s = 0; s < B; ++s) { float t = out[0][s]; out[0][s] = out[1][s] * p.g; "
                          "out[1][s] = t * p.g; }", (True, False)),
    "reverse": ("", "for (u32 s = 0; s < B / 2; ++s) { float t = out[0][s]; out[0][s] = out[0][B - 1 - s] * p.g; "
                    "out[0][B - 1 - s] = t * p.g; }", (True, False)),
    "sum_into_first": ("", "float acc = 0.0f; for (u32 s = 0; s < B; ++s) acc += out[0][s]; out[0][0] = acc * p.g;",
                       (True, False)),
    # a select / a conversion / a libm call on the sample
    "nan_select": ("", "for (u32 s = 0; s < B; ++s) out[0][s] = (out[0][s] != out[0][s]) ? 0.0f : out[0][s] * p.g;",
                   (True, False)),
    "int_roundtrip": ("", "for (u32 s = 0; s < B; ++s) out[0][s] = (float)(int)(out[0][s] * p.g);", (True, False)),
    "sin_of_sample": ("", "for (u32 s = 0; s < B; ++s) out[0][s] = sinf(out[0][s]) * p.g;", (True, False)),
    "sample_as_index": ("__device__ const float lut[4] = {0.1f, 0.2f, 0.3f, 0.4f}; ",
                        "for (u32 s = 0; s < B; ++s) out[0][s] = lut[((unsigned)out[0][s]) & 3u] * p.g;",
                        (True, False)),
    # a gain that is not one value read from Parameters / State or a constant
    "sr_dependent_gain": ("", "float g = sr > 44100.0f ? p.g : 0.5f * p.g; for (u32 c = 0; c < C; ++c) "
                              "for (u32 s = 0; s < B; ++s) out[c][s] *= g;", (True, False)),
    "gain_by_channel": ("", "for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) "
                            "out[c][s] *= (c ? p.g : 1.0f);", (True, False)),
    "block_length_gain": ("", "for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) out[c][s] *= (float)B;",
                          (True, False)),
    # writes outside the model: Parameters, the pointer table, inline asm
    "store_params": ("", "const_cast<Parameters &>(p).g = 1.0f; out[0][0] *= p.g;", (False, False)),
    "pointer_table_write": ("", "out[0] = out[1]; for (u32 s = 0; s < B; ++s) out[0][s] *= p.g;", (False, False)),
    "inline_asm": ("", "float v = out[0][0]; asm volatile(\"v_mov_b32 %0, %1\" : \"=v\"(v) : \"v\"(v)); "
                       "out[0][0] = v * p.g;", (False, False)),
}

# the gain forms that are gains: a constant, and the sample rate argument
GAIN_SOURCES = {
    "const_gain": ("for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) out[c][s] *= 0.5f;", ("K", 0.5)),
    "sr_gain": ("for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) out[c][s] *= sr;", ("R", None)),
    "param_gain": ("for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) out[c][s] *= p.g;", ("P", None)),
}


def snippet(pre, body):
    return ("#include \"plugin_header.h\"\n" + pre +
            "struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };\nstruct State {};\n"
            "Parameters default_parameters() { Parameters p = {0.5f}; return p; }\n"
            "State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) "
            "{ State s; return s; }\n"
            "void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, "
            "const real32 sr) {\n" + body + "\n}\n")


@pytest.mark.parametrize("case", sorted(GAIN_SOURCES))
def test_gain_sources(case):
    """Where the host reads g: a constant (K, its value), the sample-rate
    argument (R), a Parameters field (P, its byte offset)."""
    body, (src, k) = GAIN_SOURCES[case]
    f = dm.analyze_source(snippet("", body))
    assert f["analyzed"] and f["gain_form"] and f["gain_source"] == src, f
    if k is not None:
        assert f["gain_constant"] == k
    if src == "P":
        assert f["gain_offset"] == 0


@pytest.mark.parametrize("case", sorted(SNIPPETS))
def test_constructs_outside_the_model(case):
    pre, body, (want_analyzed, want_gain) = SNIPPETS[case]
    f = dm.analyze_source(snippet(pre, body))
    if want_analyzed is not None:
        assert f["analyzed"] == want_analyzed, f
    if want_gain is not None:
        assert f["gain_form"] == want_gain, f
    # whatever the verdict, nothing unsafe is concluded: a block read is
    # seen, and no gain form for the bodies that are no gain
    if case in ("neighbour", "f64"):
        assert f["reads_block"]
    if case != "f64":
        assert not f["gain_form"]


def test_state_written_through_a_pure_calls_pointer():
    """a pointer a pure call returns (llvm.ptrmask, from
    __builtin_align_down) keeps the origin of its argument -- a State store
    through it is a State write (no parallel blocks), or the analysis stops;
    either way the blocks are not taken as independent."""
    src = ("#include \"plugin_header.h\"\n"
           "struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };\nstruct State { float z[8]; };\n"
           "Parameters default_parameters() { Parameters p = {0.5f}; return p; }\n"
           "State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) "
           "{ State s = {}; return s; }\n"
           "void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, "
           "const real32 sr) {\n"
           "    float *q = __builtin_align_down(&st.z[5], 16);\n"
           "    q[0] += out[0][0];\n"
           "    for (u32 s = 0; s < B; ++s) out[0][s] *= p.g + q[1];\n}\n")
    f = dm.analyze_source(src)
    assert (not f["analyzed"]) or f["writes_state"], f


def test_no_fixpoint_means_no_facts():
    """The analysis reports `analyzed` only when its dataflow settled; the
    stock and test plugins all settle (above)."""
    f = facts_of(os.path.join(PLUG, "state_shaper.cpp"))
    assert f["analyzed"] and f["why"] != "no fixpoint after 64 passes"


def test_numbered_types_do_not_hide_the_arguments():
    """A callback calling double-precision sin links device-library
    declarations that bring numbered types (%0 = type ...) into the module,
    spelled like the analysis kernel's unnamed arguments %0 (Parameters) and
    %1 (State).  The arguments must still be recognised: a State write is
    seen, and an input-free tone stays a table candidate (round 5: the
    Parameters / State pointers had lost their origins in such modules)."""
    def src(body):
        return ("#include \"plugin_header.h\"\n"
                "struct Parameters { FLOAT_PARAM(20.0f, 2000.0f) f; };\nstruct State { float phase; };\n"
                "Parameters default_parameters() { Parameters p = {375.0f}; return p; }\n"
                "State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) "
                "{ State s = {}; return s; }\n"
                "void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, "
                "const real32 sr) {\n" + body + "\n}\n")
    tone = ("for (u32 s = 0; s < B; ++s) { const float v = (float)sin(2.0 * 3.14159265358979 * (double)p.f * "
            "(double)s / (double)sr); for (u32 c = 0; c < C; ++c) out[c][s] = v; }")
    f = dm.analyze_source(src(tone))
    assert f["analyzed"] and not f["reads_block"] and not f["writes_state"], f
    osc = ("for (u32 s = 0; s < B; ++s) { const float v = (float)sin((double)st.phase); st.phase += p.f / sr; "
           "for (u32 c = 0; c < C; ++c) out[c][s] = v; }")
    f = dm.analyze_source(src(osc))
    assert (not f["analyzed"]) or f["writes_state"], f


def state_snippet(body):
    return ("#include \"plugin_header.h\"\n"
            "struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };\nstruct State { double ph; float env; };\n"
            "Parameters default_parameters() { Parameters p = {0.5f}; return p; }\n"
            "State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) "
            "{ State s = {0.0, 0.0f}; return s; }\n"
            "void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, "
            "const real32 sr) {\n" + body + "\n}\n")


# does a value stored to State (or a branch) depend on a block sample?
STATE_DEP = {
    "phase_only": ("for (u32 s = 0; s < B; ++s) { out[0][s] = (float)cos_64(st.ph); st.ph += 0.01; "
                   "if (st.ph > 6.28) st.ph -= 6.28; }", False),
    "tremolo": ("for (u32 s = 0; s < B; ++s) { out[0][s] *= (float)cos_64(st.ph); st.ph += 0.01; }", False),
    "envelope": ("for (u32 s = 0; s < B; ++s) { const float x = out[0][s]; st.env = st.env + 0.1f * (x - st.env); "
                 "out[0][s] = st.env; }", True),
    "branch_on_a_sample": ("for (u32 s = 0; s < B; ++s) if (out[0][s] > 0.5f) st.ph += 1.0;", True),
    # a block element read after the loop wrote it: any block load counts
    # (conservative; a store the compiler forwards to the load is no read)
    "reads_its_own_output": ("for (u32 s = 0; s < B; ++s) out[0][s] = (float)s; st.env = out[0][B / 2];", True),
    "forwarded_store": ("out[0][0] = 1.0f; st.env = out[0][0];", False),
    "state_not_written": ("for (u32 s = 0; s < B; ++s) out[0][s] *= p.g + st.env;", False),
}


@pytest.mark.parametrize("case", sorted(STATE_DEP))
def test_state_reads_block(case):
    """state_reads_block (module.h dsp_callback_facts): 0 only when no value
    stored to State and no branch depends on a block sample -- the State's
    trajectory is then the same whatever the block holds (an oscillator's
    phase, a tremolo's), the condition for rendering its State chain apart
    from its output."""
    body, want = STATE_DEP[case]
    f = dm.analyze_source(state_snippet(body))
    assert f["analyzed"], f
    assert f["state_reads_block"] == want, (case, f)


def test_state_reads_block_of_stock_plugins():
    """sine_test.cpp's phase ignores its block; biquad.cpp's filter State is
    its block's history."""
    bq = os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "plugins", "biquad.cpp")
    assert facts_of(bq)["state_reads_block"] is True
    sine = os.path.join(REF, "build/sine_test.cpp")
    if os.path.exists(sine):
        assert facts_of(sine)["state_reads_block"] is False


# ---- the analysis options against the shipped ones --------------------------
# dsp_module_compile analyses the callback compiled at -O2 without
# vectorisation or unrolling, and ships code compiled at -O3 with both.  The
# facts that choose a render path must be the same either way: the -O3 IR
# (dsp_plugin_analyze_shipped) gives the same facts for every plugin the tests
# render.
FACT_KEYS = ("analyzed", "reads_block", "writes_state", "input_control", "gain_form", "gain_table_form",
             "state_reads_block", "state_split")


def _sources_rendered_by_the_tests():
    import test_gpu_state_spec as ss
    srcs = {}
    for rel in sorted(STOCK):
        p = os.path.join(REF, rel)
        if os.path.exists(p):
            srcs[rel] = open(p).read()
    for name in sorted(os.listdir(PLUG)):
        if name.endswith(".cpp"):
            srcs["tests/plugins/" + name] = open(os.path.join(PLUG, name)).read()
    srcs["plugins/biquad.cpp"] = open(os.path.join(os.path.dirname(HERE), "dsp-bench_amd", "plugins",
                                                   "biquad.cpp")).read()
    for name in ("ONE_POLE_SRC", "COUNTER_SRC", "RUNNING_SUM_SRC", "OSC_SRC", "TREMOLO_SRC", "BIG_STATE_SRC",
                 "WAVETABLE_SRC"):
        srcs["state_spec/" + name] = getattr(ss, name)
    for name, body in sorted(ss.GEN_BODIES.items()):
        srcs["gen/" + name] = ss.GEN_HEAD + body
    return srcs


def test_analysis_facts_equal_the_shipped_o3_facts():
    """writes_state, state_reads_block and the block-class facts from the
    analysis compile (-O2, scalar, not unrolled) equal those read from the
    -O3 IR the module ships, for the reference's stock plugins, every test
    plugin, biquad.cpp and every State-writing plugin of the GPU tests."""
    diff = []
    srcs = _sources_rendered_by_the_tests()
    assert len(srcs) >= 25
    for name, src in srcs.items():
        a, b = dm.analyze_source(src), dm.analyze_source_shipped(src)
        if tuple(a[k] for k in FACT_KEYS) != tuple(b[k] for k in FACT_KEYS):
            diff.append((name, {k: (a[k], b[k]) for k in FACT_KEYS if a[k] != b[k]}, b["why"][:120]))
    assert not diff, diff


# ---- the State chain's IR edit (ir_proof.cpp strip_chain_block_stores) ------
CHAIN_IR = """define amdgpu_kernel void @dspb_seg_chain_c2(ptr addrspace(4) %G) {
entry:
  %dspb_chain_blk = alloca [1024 x float], align 4, addrspace(5)
  %slot = alloca ptr addrspace(5), align 8, addrspace(5)
  %st = alloca double, align 8, addrspace(5)
  %p = getelementptr inbounds float, ptr addrspace(5) %dspb_chain_blk, i64 3
  %q = getelementptr inbounds <2 x float>, ptr addrspace(5) %p, i64 1
  store float 1.000000e+00, ptr addrspace(5) %p, align 4, !nontemporal !1
  store float 2.000000e+00, ptr addrspace(5) %p, align 4
  store <2 x float> <float 1.000000e+00, float 2.000000e+00>, ptr addrspace(5) %q, align 8
  store double 3.000000e+00, ptr addrspace(5) %st, align 8
  STORE_OF_A_POINTER
  ret void
}
define amdgpu_kernel void @dspb_render(ptr addrspace(4) %G) {
entry:
  %dspb_chain_blk = alloca [4 x float], align 4, addrspace(5)
  store float 2.000000e+00, ptr addrspace(5) %dspb_chain_blk, align 4
  ret void
}
"""


def _strip(ir):
    import ctypes as C
    from dspbench import _lib as L
    out = C.create_string_buffer(len(ir) + 64)
    n = C.c_int32()
    assert L.lib().dsp_ir_strip_chain_stores(ir.encode(), out, len(out), C.byref(n)) == 0
    return n.value, out.value.decode()


def test_strip_chain_block_stores_deletes_only_block_stores():
    """Stores through pointers derived from the chain's private block are
    deleted (a scalar and a vector store, the vector's constant holding a
    comma), the non-temporal copy of the input and the State store are kept,
    and functions other than the chain kernels are left alone."""
    n, out = _strip(CHAIN_IR.replace("  STORE_OF_A_POINTER\n", ""))
    assert n == 2, out
    assert "store float 2.000000e+00, ptr addrspace(5) %p" not in out
    assert "%q, align 8" not in out
    assert "!nontemporal" in out and "store double 3.000000e+00, ptr addrspace(5) %st" in out
    assert "store float 2.000000e+00, ptr addrspace(5) %dspb_chain_blk" in out  # @dspb_render untouched


def test_strip_chain_block_stores_reads_the_address_operand():
    """A store whose VALUE is a pointer derived from the block and whose
    address is elsewhere (the round-5 parser took the first `ptr addrspace(5)
    %` of the line for the address, and deleted a store to another location):
    outside the pass's model, so nothing is edited (-1: the module keeps the
    hiprtc code)."""
    ir = CHAIN_IR.replace("STORE_OF_A_POINTER", "store ptr addrspace(5) %p, ptr addrspace(5) %slot, align 8")
    n, out = _strip(ir)
    assert n == -1
    assert out == ir


# ---- a State that splits by word (dsp_callback_facts.state_split) ----------
SPLIT = {
    # (State, callback body, the block-dependent words -- "T-" every word from
    # T on -- or False: no split)
    # an envelope (block-dependent) beside a block counter (independent)
    "counter": ("struct State { float env; unsigned blocks; };",
                "for (u32 s = 0; s < B; ++s) { const float x = out[0][s] < 0.0f ? -out[0][s] : out[0][s]; "
                "st.env = st.env + p.g * (x - st.env); out[0][s] = st.env * (float)(st.blocks & 3u); } "
                "st.blocks += 1u;", "0"),
    # a phase beside a running sum: the phase alone is independent
    "phase_and_sum": ("struct State { double ph; float sum; };",
                      "for (u32 s = 0; s < B; ++s) { st.sum += out[0][s]; st.ph += 0.01; out[0][s] = st.sum; }",
                      "2"),
    # every written word depends on the block: nothing to split
    "sum_only": ("struct State { float sum; float pad; };",
                 "for (u32 s = 0; s < B; ++s) { st.sum += out[0][s]; out[0][s] = st.sum; }", False),
    # the counter advances only when the block is loud (a branch on a sample): no split
    "counter_under_a_branch": ("struct State { float env; unsigned blocks; };",
                               "for (u32 s = 0; s < B; ++s) { if (out[0][s] > 0.5f) st.blocks += 1u; "
                               "st.env += out[0][s]; }", False),
    # the counter is read back into the envelope's update: still independent itself
    "counter_feeds_env": ("struct State { float env; unsigned blocks; };",
                          "for (u32 s = 0; s < B; ++s) st.env = st.env * 0.5f + out[0][s] * (float)st.blocks; "
                          "st.blocks += 1u;", "0"),
    # the envelope feeds the counter's increment: both depend on the block
    "env_feeds_counter": ("struct State { float env; unsigned blocks; };",
                          "for (u32 s = 0; s < B; ++s) st.env = st.env * 0.5f + out[0][s]; "
                          "st.blocks += (unsigned)(st.env > 0.0f ? 1 : 2);", False),
    # envelopes in an array indexed by the channel, the loop bounded by a
    # constant (c < 4): the offsets' range is the array's
    "indexed_words": ("struct State { float env[4]; unsigned blocks; };",
                      "for (u32 c = 0; c < C && c < 4u; ++c) for (u32 s = 0; s < B; ++s) st.env[c] += out[c][s]; "
                      "st.blocks += 1u;", "0,1,2,3"),
    # the same loop bounded by C alone: every word from the array on
    "indexed_unbounded": ("struct State { unsigned blocks; float env[4]; };",
                          "for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) st.env[c] += out[c][s]; "
                          "st.blocks += 1u;", "1-"),
    # ... which, before the counter, leaves nothing independent
    "indexed_unbounded_first": ("struct State { float env[4]; unsigned blocks; };",
                                "for (u32 c = 0; c < C; ++c) for (u32 s = 0; s < B; ++s) st.env[c] += out[c][s]; "
                                "st.blocks += 1u;", False),
    # a pointer stepped through the State by a loop (widened: no upper bound)
    "pointer_walk": ("struct State { unsigned blocks; float env[4]; };",
                     "float *e = st.env; for (u32 c = 0; c < C && c < 4u; ++c, ++e) "
                     "for (u32 s = 0; s < B; ++s) *e += out[c][s]; st.blocks += 1u;", "1-"),
    # a channel loop whose exit test sits under a branch (not run every
    # iteration): no bound from it
    "exit_test_under_a_branch": ("struct State { unsigned blocks; float env[4]; };",
                                 "for (u32 c = 0; ; ++c) { for (u32 s = 0; s < B; ++s) st.env[c] += out[0][s]; "
                                 "if (p.g > 0.25f) { if (c + 1 >= 4u) break; } else if (c + 1 >= 2u) break; } "
                                 "st.blocks += 1u;", "1-"),
}


def split_snippet(state, body):
    return ("#include \"plugin_header.h\"\n"
            "struct Parameters { FLOAT_PARAM(0.0f, 1.0f) g; };\n" + state + "\n"
            "Parameters default_parameters() { Parameters p = {0.5f}; return p; }\n"
            "State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) "
            "{ State s = {}; return s; }\n"
            "void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, "
            "const real32 sr) {\n" + body + "\n}\n")


@pytest.mark.parametrize("case", sorted(SPLIT))
def test_state_split_by_word(case):
    """state_split: the State's 4-byte words split into those a store of a
    block-dependent value may hit and written others, with no branch on a
    sample and every dependent store at an offset the analysis names.  The
    speculative segments then start each warm-up from the others' State chain
    (DESIGN 4.6); a wrong split could only cost reruns (every segment is
    checked bit for bit), so these cases pin the analysis, not the output."""
    state, body, want = SPLIT[case]
    f = dm.analyze_source(split_snippet(state, body))
    assert f["analyzed"] and f["writes_state"] and f["state_reads_block"], (case, f)
    assert f["state_split"] == bool(want), (case, f)
    if want:
        assert f["state_dep_words"] == want, (case, f)


def test_state_split_under_the_comgr_torch_brings():
    """A process that imports PyTorch first resolves comgr and hiprtc to the
    copies PyTorch ships (an older LLVM, `torch/lib/libamd_comgr.so`): its IR
    keeps array GEPs ([N x T], 0, i) where the system's folds them to
    element GEPs -- the split analysis must name the same words from either
    (the GPU tests import torch before they compile; these tests do not)."""
    import subprocess
    import sys
    code = r'''
import sys, json
import torch
sys.path.insert(0, %r); sys.path.insert(0, %r)
import test_ir_proof as ti, test_gpu_state_spec as ss
import dspbench.module as dm
maps = [l.split()[-1] for l in open("/proc/self/maps") if "comgr" in l]
out = {"comgr": sorted(set(maps))}
for n, (st, body, want) in ti.SPLIT.items():
    a = dm.analyze_source(ti.split_snippet(st, body))
    out[n] = [a["state_split"], a["state_dep_words"]]
for n in ss.GEN_SPLIT:
    a = dm.analyze_source(ss.GEN_HEAD + ss.GEN_BODIES[n])
    out["gen/" + n] = [a["state_split"], a["state_dep_words"]]
print(json.dumps(out))
''' % (HERE, os.path.join(os.path.dirname(HERE), "dsp-bench_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, cwd=HERE)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    got = json.loads(r.stdout.strip().splitlines()[-1])
    for n, (st, body, want) in SPLIT.items():
        assert got[n] == [bool(want), want or ""], (n, got[n], got["comgr"])
    import test_gpu_state_spec as ss
    for n, want in ss.GEN_SPLIT.items():
        assert got["gen/" + n][0] == want, (n, got["gen/" + n], got["comgr"])
