// Test plugin (not from the reference): a gain that zeroes samples beyond
// +-2000.  Probe blocks within +-1000 cannot tell it from a gain; its IR
// stores a select on the sample, not x * g.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            const float x = out[c][s];
            out[c][s] = fabs_32(x) > 2000.0f ? 0.0f : x * p.gain;
        }
}
