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

/* sizeof(Parameters), sizeof(State), whether State is empty. */
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

/* Render with a loaded module: dsp_render_offline / dsp_render_stft /
 * dsp_ir_analysis with plugin->kind = DSP_PLUGIN_GENERIC and plugin->module
 * = the module (plugin->params = the Parameters blob).  dsp_ir_analysis
 * initialises a separate scratch State per call (compute_IR,
 * plugin.cpp:17-58). */

#ifdef __cplusplus
}
#endif
#endif
