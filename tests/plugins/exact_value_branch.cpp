// Test plugin (not from the reference): a gain, except that a sample of
// exactly 0.25 becomes 7 -- an exact-value branch no random probe hits.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 2.0f) gain; };
struct State {};
Parameters default_parameters() { Parameters p = {0.5f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            if (out[c][s] == 0.25f) out[c][s] = 7.0f;
            else out[c][s] *= p.gain;
        }
}
