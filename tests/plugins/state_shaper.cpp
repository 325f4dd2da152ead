// Test plugin (not from the reference): a waveshaper y = a x^3 + b x whose
// coefficients initialize_state puts in State; the callback only reads them,
// so the blocks are independent (rendered in parallel), but the map is no
// gain and no table.
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(0.0f, 1.0f) drive; };
struct State { float a, b; float unused[12]; };
Parameters default_parameters() { Parameters p = {0.3f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) {
    State s = {};
    s.a = -p.drive / 3.0f;
    s.b = 1.0f + p.drive;
    return s;
}
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c)
        for (u32 s = 0; s < B; ++s) {
            const float x = out[c][s];
            out[c][s] = st.a * x * x * x + st.b * x;
        }
}
