// Test plugin (not from the reference): an empty State, but a function-local
// static counts the calls, and every other block is attenuated -- state that
// lives outside State, so the blocks must run in order.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    static int calls = 0;
    ++calls;
    const float g = p.gain * ((calls % 2) ? 1.0f : 0.5f);
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) out[c][s] *= g;
}
