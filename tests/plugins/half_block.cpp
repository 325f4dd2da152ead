// Test plugin (not from the reference): every store is x * g at x's address,
// but only the first half of each block is stored; the second half keeps its
// input.  The IR's gain form holds, the probe of ones refuses the class
// (half the elements stay 1) unless g = 1.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B / 2; ++s) out[c][s] *= p.gain;
}
