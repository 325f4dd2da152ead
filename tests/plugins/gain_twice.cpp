// Test plugin (not from the reference): every store is x * g at x's address,
// but each sample is scaled twice (y = g^2 x): the probe of ones refuses the
// gain class unless g^2 = g.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (int pass = 0; pass < 2; ++pass)
        for (u32 c = 0; c < C; ++c)
            for (u32 s = 0; s < B; ++s) out[c][s] *= p.gain;
}
