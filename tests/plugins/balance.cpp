// Test plugin (not from the reference): a different gain per channel.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) left; FLOAT_PARAM(0.0f, 2.0f) right; };
struct State {};
Parameters default_parameters() { Parameters p = {0.25f, 0.75f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        out[0][s] *= p.left;
        if (C > 1) out[1][s] *= p.right;
    }
}
