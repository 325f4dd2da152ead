// Test plugin (not from the reference): a per-position gain (a linear fade
// over the block) -- x * g(s), not one g per call.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.75f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 s = 0; s < B; ++s) {
        const float g = p.gain * (float)s / (float)B;
        for (u32 c = 0; c < C; ++c) out[c][s] *= g;
    }
}
