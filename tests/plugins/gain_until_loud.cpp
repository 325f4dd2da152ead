// Test plugin (not from the reference): a gain that stops at the first
// sample above 5000 and leaves the rest of the block as it is -- every store
// is x * g, but which samples are stored depends on the input (a branch on a
// sample), beyond the reach of every probe.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            if (out[c][s] > 5000.0f) break;
            out[c][s] *= p.gain;
        }
}
