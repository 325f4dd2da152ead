/*
 * module.h -- generic GPU dispatch of DSP-Bench plugins.
 *
 * The reference JIT-compiles a plugin's C++ source with clang/MCJIT for the
 * CPU (compiler.cpp:481-1203) and calls its audio_callback once per block.
 * Here the same source is compiled with hiprtc to a gfx950 code object:
 * `#include "plugin_header.h"` resolves to include/dspbench/plugin_device.h
 * (device definitions of every host service), the plugin body is wrapped in
 * `#pragma clang force_cuda_host_device`, and generated kernels call
 *
 *   default_parameters()                      -> the Parameters blob
 *   initialize_state(params, C, sr, context)  -> the State, on the device
 *                                                (context = device arena)
 *   audio_callback(params, state, out, C, B, sr) once per block, exactly as
 *       render_audio does (audio.cpp:13-175, one-shot: zero block, copy the
 *       file's channels, zero past EOF, callback in place)
 *
 * A plugin with an empty State renders every block in its own GPU thread;
 * a stateful plugin renders its blocks in order on one thread (the state
 * carries from block to block, as on the audio thread).  The State and the
 * arena it points into live in device memory and persist across renders,
 * like the reference's plugin handle (plugin.h:95-113).
 *
 * Parity: fp32/fp64 arithmetic is IEEE (no fast-math contraction); the
 * transcendental services are the device libm, which can differ from the
 * host libm in the last ulp.
 */
#ifndef DSPBENCH_MODULE_H
#define DSPBENCH_MODULE_H

#include <stddef.h>
#include <stdint.h>

#include "dspbench.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dsp_module dsp_module;

/* Compile plugin source text to a gfx950 code object (no GPU needed).
 * *code is malloc'd (free with dsp_module_free_code).  The compiler log
 * (errors, warnings) is written to log (NUL-terminated, truncated to
 * log_cap).  DSP_ERR_INVALID on a compile error. */
int dsp_module_compile(const char *source, const char *name, void **code, uint64_t *code_size,
                       char *log, uint64_t log_cap);
void dsp_module_free_code(void *code);

/* Load a code object on `device` (-1: current). */
int dsp_module_load(const void *code, uint64_t code_size, int device, dsp_module **out);
void dsp_module_destroy(dsp_module *m);

/* sizeof(Parameters), sizeof(State), and whether blocks render independently
 * (1: State is empty, or the callback provably never writes it -- see
 * dsp_module_facts; such a plugin renders its blocks in parallel and may be
 * time-sharded). */
int dsp_module_sizes(const dsp_module *m, uint32_t *params_size, uint32_t *state_size, int *stateless);

/* default_parameters() into a host blob of params_size bytes
 * (plugin_populate_from_descriptor, plugin.cpp:335-364). */
int dsp_module_default_parameters(dsp_module *m, void *params);

/* initialize_state(params, C, sr, context) into the module's device State,
 * with a fresh device arena of arena_bytes as the context. */
int dsp_module_initialize_state(dsp_module *m, const void *params, uint32_t C, float sr,
                                uint64_t arena_bytes);

/* Copy the device State to a host blob of state_size bytes (pointers in it
 * are device addresses). */
int dsp_module_read_state(const dsp_module *m, void *state);

/* ---- parameter descriptor -------------------------------------
 * The reference's JIT parses the `annotate` attributes of struct Parameters
 * into a Plugin_Descriptor (compiler.cpp:944-1164; plugin.h:15-82) and
 * marshals parameter values into the Parameters blob at the fields' byte
 * offsets (plugin_set_parameter_holder_from_values, plugin.cpp:147-171).
 * dsp_module_compile builds the same descriptor -- names and annotations from
 * the source text, offsets / sizes / types / enumerator values evaluated by
 * the device compiler -- stores it in the code object, and fails (with the
 * reference's error flag in the log) when an annotation is invalid.
 * Reading it needs no GPU. */
enum dsp_param_type { DSP_PARAM_INT = 0, DSP_PARAM_FLOAT = 1, DSP_PARAM_ENUM = 2 }; /* plugin.h:15-19 */

enum dsp_desc_error { /* errors.inc:1-19 */
    DSP_DESC_SUCCESS = 0,               /* Compiler_Success */
    DSP_DESC_ERROR_RECURSE = 1,         /* Compiler_Error_Recurse: some parameter has an error */
    DSP_DESC_EMPTY_ANNOTATION = 2,      /* Compiler_Empty_Annotation */
    DSP_DESC_INVALID_ANNOTATION = 3,    /* Compiler_Invalid_Annotation */
    DSP_DESC_MISSING_MIN_MAX = 4,       /* Compiler_Missing_Min_Max */
    DSP_DESC_MIN_GREATER_THAN_MAX = 5,  /* Compiler_Min_Greater_Than_Max */
    DSP_DESC_INVALID_MIN = 6,           /* Compiler_Invalid_Min_Value */
    DSP_DESC_INVALID_MAX = 7,           /* Compiler_Invalid_Max_Value */
    DSP_DESC_TYPE_MISMATCH = 8          /* Compiler_Annotation_Type_Mismatch */
};

#define DSP_PARAM_NAME_MAX 64

typedef struct dsp_param_desc { /* Plugin_Descriptor_Parameter (plugin.h:47-55) */
    char name[DSP_PARAM_NAME_MAX]; /* field name, NUL-terminated (truncated) */
    uint32_t offset;               /* byte offset in the Parameters blob */
    int32_t type;                  /* dsp_param_type */
    int32_t error;                 /* dsp_desc_error */
    int32_t int_min, int_max;      /* Int */
    float float_min, float_max;    /* Float */
    int32_t float_log;             /* Float: "log" annotation */
    uint32_t num_entries;          /* Enum: enumerators (dsp_descriptor_enum_entry) */
} dsp_param_desc;

typedef struct dsp_plugin_descriptor { /* Plugin_Descriptor (plugin.h:57-74) */
    uint64_t params_size, params_align;
    uint64_t state_size, state_align;
    uint32_t num_parameters; /* annotated fields of Parameters, in declaration order */
    int32_t error;           /* dsp_desc_error */
} dsp_plugin_descriptor;

typedef union dsp_param_value { /* Plugin_Parameter_Value (plugin.h:76-82) */
    int32_t int_value;
    float float_value;
    int32_t enum_value;
} dsp_param_value;

typedef struct dsp_descriptor dsp_descriptor;

/* The descriptor stored in a code object (no GPU).  Free with
 * dsp_descriptor_destroy.  DSP_ERR_INVALID when the code object has none. */
int dsp_descriptor_from_code(const void *code, uint64_t code_size, dsp_descriptor **out);
void dsp_descriptor_destroy(dsp_descriptor *d);
/* The descriptor of a loaded module (owned by the module), or NULL. */
const dsp_descriptor *dsp_module_descriptor(const dsp_module *m);

int dsp_descriptor_info(const dsp_descriptor *d, dsp_plugin_descriptor *out);
int dsp_descriptor_param(const dsp_descriptor *d, uint32_t index, dsp_param_desc *out);
/* Enum parameter `index`, enumerator `entry`: value and name (NUL-terminated,
 * truncated to name_cap; name may be NULL). */
int dsp_descriptor_enum_entry(const dsp_descriptor *d, uint32_t index, uint32_t entry, int64_t *value,
                              char *name, uint32_t name_cap);

/* values[i] -> the holder at parameter i's offset: int / float / enum as a
 * 4-byte int (plugin_set_parameter_holder_from_values, plugin.cpp:147-171).
 * Bytes of the holder that are no parameter are left as they are. */
int dsp_params_from_values(const dsp_descriptor *d, const dsp_param_value *values, void *holder);
/* the reverse (plugin_set_parameter_values_from_holder, plugin.cpp:121-145) */
int dsp_params_to_values(const dsp_descriptor *d, const void *holder, dsp_param_value *values);
/* 1 when two descriptors describe the same layout and parameters
 * (plugin_descriptor_compare, plugin.cpp:66-105: sizes, alignments, and per
 * parameter offset, type, name, ranges, enumerators), else 0. */
int dsp_descriptor_equal(const dsp_descriptor *a, const dsp_descriptor *b);

/* Normalisation (plugin.h:173-233) of one parameter's value to [0, 1] and
 * back.  Int: (v - min) / (max - min); Float: clamped, linear or log;
 * Enum: the index of the enumerator whose value is v over num_entries - 1
 * (enum_values = the parameter's enumerator values in declaration order).
 * dsp_param_normalize returns DSP_ERR_INVALID for an enum value that is no
 * enumerator (the reference asserts, plugin.h:222-231). */
int dsp_param_normalize(const dsp_param_desc *p, const int64_t *enum_values, dsp_param_value v, float *out);
int dsp_param_denormalize(const dsp_param_desc *p, const int64_t *enum_values, float x, dsp_param_value *out);

/* Render with a loaded module: dsp_render_offline / dsp_render_stft /
 * dsp_ir_analysis with plugin->kind = DSP_PLUGIN_GENERIC and plugin->module
 * = the module (plugin->params = the Parameters blob).  dsp_ir_analysis
 * initialises a separate scratch State per call (compute_IR,
 * plugin.cpp:17-58).
 *
 * Block classes.  A plugin whose blocks are independent -- an empty State,
 * or a State its callback never writes (dsp_module_facts) -- computes each
 * block from the block alone (it cannot tell where the block lies in the
 * file), so:
 *   DSP_BLOCK_TABLE  a callback that reads no sample of its block
 *                    (IR_test.cpp, build/IR_test.cpp:40-60) renders the same
 *                    block everywhere: the render is that block -- computed
 *                    once by the plugin's own callback -- tiled, and
 *                    dsp_render_stft runs the fused render + STFT kernel on
 *                    it as a block table;
 *   DSP_BLOCK_GAIN   a callback whose every block store is x * g at the
 *                    address x came from, with one g per call, under control
 *                    flow that reads no sample (gain_test.cpp,
 *                    static_gain_plugin.cpp; no store at all = the identity)
 *                    runs as the gain map with the g its callback gives x = 1.
 * A class is taken only when the callback's own LLVM IR proves it
 * (dsp_module_facts: dsp_module_compile analyses the plugin's code and stores
 * the facts in the code object) and probe blocks run through the callback
 * pin what the IR leaves open (which elements are written; the value of g),
 * once per (Parameters, C, B, sample rate) -- the first render with a new set
 * synchronises its stream once.  Anything else, including every code object
 * without facts, runs the callback on every block, as does
 * DSP_EXEC_NO_SPECIALIZE (dspbench.h). */
enum dsp_block_class { DSP_BLOCK_CALLBACK = 0, DSP_BLOCK_TABLE = 1, DSP_BLOCK_GAIN = 2, DSP_BLOCK_GAIN_TABLE = 3 };

/* The block class of `params` for C channels of B-sample blocks at sample
 * rate sr (probing on ex->stream if not known yet); *gain receives g for
 * DSP_BLOCK_GAIN (may be NULL). */
int dsp_module_block_class(dsp_module *m, const void *params, uint32_t params_size, uint32_t C, uint32_t B,
                           float sr, int32_t *block_class, float *gain, const dsp_exec *ex);

/* The class cache keeps 4 (Parameters, C, B, sr) sets.  An evicted TABLE
 * class's block is freed once no call holds it and every stream that read it
 * has passed its last use (an event recorded when each call returns); one a
 * captured graph used stays until dsp_module_destroy.  *n = evicted blocks not
 * freed yet (diagnostic; frees what can be freed first). */
int dsp_module_retired_tables(dsp_module *m, uint64_t *n);

/* ---- a State the callback writes: speculative segments -------------------
 * The reference runs such a callback block after block (audio.cpp:160-165);
 * one GPU lane running that chain is slower than a host core.  When the
 * analysis proved that the callback writes no memory but its State and its
 * block (dsp_callback_facts: analyzed, writes_state) and the State is at most
 * 1024 bytes, dsp_render_offline / dsp_render_stft (input and output rows
 * apart) cut the file into segments rendered at once, each from the live State
 * after a warm-up on the blocks before it, and keep a segment's output only
 * when the State it started from equals, bit for bit, the State the previous
 * segment ended with; the others are rendered again from that State (two
 * parallel passes, then serially in file order).  Output and final State are
 * the serial chain's, bit for bit, for any such callback.  It is fast when the
 * callback forgets its State (filters, envelopes, smoothers: trajectories
 * from different States meet exactly within a few hundred samples); when it
 * does not (an oscillator's phase) the call costs the serial chain plus one
 * pass per warm-up level tried (16x longer each, up to 4096 blocks, within
 * the same call); then -- within that call, and without speculation for
 * these Parameters from the next call on -- one lane runs the callback's State updates alone in file order
 * (its block a private array nothing reads, so the compiler drops the block
 * arithmetic) and records each block's State, then every segment renders from
 * its recorded State at once -- when the compiled chain kernel needs no
 * scratch for the block (a State that depends on the block renders serially;
 * for a callback that reads its block while its State ignores it,
 * dsp_callback_facts.state_reads_block = 0, dsp_module_compile builds the
 * chain kernels from the callback's IR with its block stores deleted).
 * DSP_EXEC_SERIAL_STATE (dspbench.h) forces the serial chain. */
typedef struct dsp_state_spec_info {
    int32_t used;                /* the module's last State-writing render ran in segments */
    int32_t disabled;            /* learned: serial for the current Parameters */
    uint32_t segments;           /* K of that render */
    uint32_t blocks_per_segment;
    uint32_t warmup_blocks;      /* the warm-up of the pass 1 that stood */
    uint32_t differed[3];        /* segments whose start State differed: that pass 1, rerun 1, rerun 2 */
    uint32_t serial_reruns;      /* segments the in-order walk rendered again */
    uint32_t levels;             /* pass 1 runs: the learnt warm-up, then 16x longer ones while more
                                    than 1/8 of the guessed segments started wrong (at most 4) */
    int32_t chain;               /* the render ran the State chain on one lane (the callback's block
                                    arithmetic dropped), then every segment from its recorded State
                                    in parallel: after its last warm-up level failed (decided on the
                                    GPU, within the call), or from the start once learnt (disabled) */
    /* The State chain is checked, not trusted: the exact rerun compares the
     * chain's record of every block's State with the State the callback
     * renders that block from, a check compares every segment's first State
     * with the State the segment before ended with, and the walk renders
     * serially from the true State whatever differs -- the call's output and
     * final State are the serial chain's either way.  Any difference also
     * makes these Parameters render serially from the next call on. */
    uint32_t chain_mismatch;     /* segments whose first State (the chain's record) differed from the
                                    State the segment before ended with: rendered again by the walk */
    uint32_t chain_records_differed;  /* blocks whose State in the exact rerun differed from the
                                         chain's record */
    int32_t split;               /* a split State (dsp_callback_facts.state_split): pass 1 started each
                                    warm-up from the block-independent words a State chain recorded
                                    there (a block counter), the others from the live State */
} dsp_state_spec_info;
/* Waits for the module's last speculative render and describes it. */
int dsp_module_state_spec(dsp_module *m, dsp_state_spec_info *out);

/* Test hooks (not for production use).  DSP_MODULE_DEBUG_PERTURB_CHAIN: the
 * module's next render that runs the State chain flips a high bit of the State
 * the chain records for block `value` (a wrong record, as a miscompiled chain
 * would make); the render must still come out equal to the serial chain, with
 * the mismatch reported in dsp_state_spec_info.  In a render of a split State
 * (dsp_state_spec_info.split) the same hook flips the low bit of the first
 * block-independent word recorded for segment `value` at the first warm-up
 * level: that segment starts wrong, its check fails and it is rendered again. */
enum { DSP_MODULE_DEBUG_PERTURB_CHAIN = 1 };
int dsp_module_debug(dsp_module *m, int what, uint64_t value);

/* Diagnostics (no GPU): the text pass dsp_module_compile applies to the LLVM
 * IR of the State chain kernels of a callback whose State never reads its
 * block (ir_proof.cpp strip_chain_block_stores).  *dropped = the stores
 * deleted (through a pointer derived from the chain's private block
 * `dspb_chain_blk`, other than the non-temporal copy of the input), or -1
 * when a store is outside the pass's model (the module then keeps the hiprtc
 * code); the edited text goes to out (out_cap bytes; NULL: not wanted). */
int dsp_ir_strip_chain_stores(const char *ir, char *out, uint64_t out_cap, int32_t *dropped);

/* Diagnostics: a module compiled with the environment variable
 * DSPB_SEG_TIMING set carries clocks of its speculative pass 1 (wave 0,
 * lane 0 of every workgroup, units of 16 shader clocks, summed over the
 * workgroups): out[0] staging + barrier, [1] the next round's loads issued,
 * [2] the callbacks, [3] the barrier after them, [4] copy-out + barrier,
 * [5] workgroups, [6] rounds.  Waits for the device; zeros otherwise. */
int dsp_module_seg_timing(dsp_module *m, uint32_t out[8]);

/* ---- what the callback does with its block (no GPU) ----------------------
 * dsp_module_compile compiles the plugin a second time into an analysis
 * kernel, dspb_proof(P, S, out, C, B, sr) { audio_callback(*P, *S, out, C, B,
 * sr); }, flattened, and reads its optimised LLVM IR: which memory every
 * load and store can touch (a block sample, the pointer table, Parameters,
 * State, private or global memory) and which values depend on a block sample
 * or differ between iterations.  A construct outside that model (a call that
 * may touch memory, an atomic, a store to a global or to Parameters, a
 * pointer stored to memory, an address used as a number) leaves `analyzed`
 * 0, and nothing is concluded from the IR. */
typedef struct dsp_callback_facts {
    int32_t present;       /* the code object carries facts (compiled with them) */
    int32_t analyzed;      /* every instruction of the callback was inside the analysis */
    int32_t reads_block;   /* loads a sample of its block (or copies from it) */
    int32_t writes_state;  /* stores through its State */
    int32_t input_control; /* a branch condition or a store address depends on a sample */
    int32_t gain_form;     /* every block store is x * g at x's address, one g per call
                              (or no block store: the identity) */
    int32_t gain_source;   /* gain_form: where g is read -- 'P' / 'S' a float at byte gain_offset
                              of Parameters / State, 'K' the constant gain_constant, 'R' the
                              sample rate; the host reads g from there (0: not known) */
    uint32_t gain_offset;
    float gain_constant;
    char gain[128];        /* g as the analysis wrote it (diagnostics) */
    char why[256];         /* why the analysis stopped, or why a property fails */
    int32_t gain_table_form; /* (ABI 3) every block store is x * G at x's address, G free of any
                              sample (it may vary with channel and position), and no element
                              is stored twice: the IR's loops (the CFG's natural loops and
                              their induction variables) give every store the address
                              (constant or loop channel, loop sample) */
    char table_why[128];   /* (ABI 3) why not gain_table_form */
    int32_t state_reads_block; /* (ABI 3) a value stored to State, or a branch condition, depends on
                              a block sample (1 unless the analysis completed and showed
                              otherwise): 0 = the State's trajectory is the same whatever the
                              block holds (an oscillator's phase, a tremolo's) */
    int32_t state_split;   /* state_reads_block, yet no branch depends on a sample and every store of
                              a block-dependent value has a known offset: the State's words split into
                              block-dependent ones and written block-independent ones (an envelope
                              beside a block counter).  The speculative segments then start each
                              warm-up from the independent words a State chain recorded there */
    char state_dep_words[64]; /* state_split: the block-dependent words, comma-separated word
                              indices, "T-" for every word from T on (diagnostics) */
} dsp_callback_facts;

/* The facts of a loaded module (present = 0 for a code object without). */
int dsp_module_facts(const dsp_module *m, dsp_callback_facts *out);
/* The facts stored in a code object (present = 0 when it has none; no GPU). */
int dsp_code_facts(const void *code, uint64_t code_size, dsp_callback_facts *out);
/* The same analysis of plugin source text, without building a module (no GPU). */
int dsp_plugin_analyze(const char *source, dsp_callback_facts *out);
/* Diagnostics (no GPU): the same analysis of IR compiled with the module's own
 * options (-O3, vectorisation and unrolling on) instead of the analysis
 * options (-O2 without them): the facts the shipped code would give, where
 * the analysis can read that IR (analyzed = 0 where it cannot). */
int dsp_plugin_analyze_shipped(const char *source, dsp_callback_facts *out);

#ifdef __cplusplus
}
#endif
#endif
