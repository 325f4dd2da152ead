// Test plugin (not from the reference): arithmetic the reference JIT's
// -Ofast -ffast-math (compiler.cpp:507-515) may rewrite -- a four-term sum of
// a sample and its three predecessors in the block (reassociation), divided by
// a parameter (a reciprocal multiply under -freciprocal-math).  Stateless:
// the first three samples of a block have fewer terms.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.1f, 10.0f) div; };
struct State {};
Parameters default_parameters() { Parameters p = {3.0f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c) {
        float x1 = 0.0f, x2 = 0.0f, x3 = 0.0f;
        for (u32 s = 0; s < B; ++s) {
            const float x = out[c][s];
            out[c][s] = (((x + x1) + x2) + x3) / p.div;
            x3 = x2;
            x2 = x1;
            x1 = x;
        }
    }
}
