// ref_audio.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Exposes the reference's own PCM converters and (de)interleavers
// (audio.h:66-133) with C linkage, compiled from the reference's sources
// where they lie (oracle/Makefile: -I$(REF) -DRELEASE, output only into
// oracle/_ref/libref_audio.so).  Used to generate and check the WAV decode
// golden vectors; never linked into the product.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "base.h"
#include "structs.h"
#include "memory.h"
#include "audio.h"

extern "C" {
void ref_convert_int16(const void *src, float *dst, int n) { convertInt16ToFloat(src, dst, n); }
void ref_convert_int24(const void *src, float *dst, int n) { convertInt24ToFloat(src, dst, n); }
void ref_convert_int32(const void *src, float *dst, int n) { convertInt32ToFloat(src, dst, n); }
void ref_deinterleave(float **dst, float *src, int frames, int channels) {
    deinterleave(dst, src, frames, channels);
}
void ref_interleave(float **in, float *out, uint64_t channels, uint64_t offset, uint64_t frames) {
    interleave(in, out, channels, offset, frames);
}
unsigned ref_next_power_of_two(unsigned v) { return next_power_of_two(v); }
}
