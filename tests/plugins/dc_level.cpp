// Test plugin (not from the reference): every sample set to a level from the
// Parameters -- a table (it reads no sample).
#include "plugin_header.h"
struct Parameters { FLOAT_PARAM(-1.0f, 1.0f) level; };
struct State {};
Parameters default_parameters() { Parameters p = {0.125f}; return p; }
State initialize_state(const Parameters &p, const unsigned C, const float sr, void *ctx) { State s; return s; }
void audio_callback(const Parameters &p, State &st, float **out, const u32 C, const u32 B, const real32 sr) {
    for (u32 c = 0; c < C; ++c) set_array(p.level, out[c], (i32)B);
}
