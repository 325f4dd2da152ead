/*
 * host.h -- host-side runtime of libdspbench (plain C ABI).
 *
 *   dsp_initializer   the opaque `initialization_context` / `allocator`
 *                     handed to a plugin's initialize_state (ref plugin.h:
 *                     117-120, Initializer{Arena*, IPP_FFT_Context*}): a
 *                     16-byte-aligned bump arena (ref memory.h:89-106) plus
 *                     the GPU the spectral services run on.
 */
#ifndef DSPBENCH_HOST_H
#define DSPBENCH_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dsp_initializer dsp_initializer;

dsp_initializer *dsp_initializer_create(size_t arena_bytes, int device);
void dsp_initializer_reset(dsp_initializer *ini);
size_t dsp_initializer_used(const dsp_initializer *ini);
void dsp_initializer_destroy(dsp_initializer *ini);

/* Print "<what>: <status> (<last error>)" to stderr. */
void dsp_host_report(const char *what, int status);

#ifdef __cplusplus
}
#endif
#endif
