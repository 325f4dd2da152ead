// biquad.cpp -- a stateful example plugin for the generic GPU dispatch:
// RBJ-cookbook low-pass biquad, direct form I, one state set per channel.
// Written against plugin_header.h like any DSP-Bench plugin; it compiles for
// the CPU JIT and, through dsp_module_compile, for gfx950.
#include "plugin_header.h"

struct Parameters {
    FLOAT_PARAM_LOG(20.0f, 20000.0f) cutoff;
    FLOAT_PARAM(0.1f, 10.0f) q;
};

#define MAX_CH 16

struct State {
    float b0, b1, b2, a1, a2;
    float x1[MAX_CH], x2[MAX_CH], y1[MAX_CH], y2[MAX_CH];
};

Parameters default_parameters()
{
    Parameters p = {1000.0f, 0.7071f};
    return p;
}

State initialize_state(const Parameters& p, const unsigned int num_channels, const float sample_rate,
                       void* initialization_context)
{
    State s = {};
    const double w0 = 2.0 * 3.14159265358979323846 * p.cutoff / sample_rate;
    const double alpha = sin_64(w0) / (2.0 * p.q);
    const double c = cos_64(w0);
    const double a0 = 1.0 + alpha;
    s.b0 = (float)((1.0 - c) / 2.0 / a0);
    s.b1 = (float)((1.0 - c) / a0);
    s.b2 = s.b0;
    s.a1 = (float)(-2.0 * c / a0);
    s.a2 = (float)((1.0 - alpha) / a0);
    return s;
}

void audio_callback(const Parameters& p, State& s, float** out, const u32 num_channels,
                    const u32 num_samples, const real32 sample_rate)
{
    for (u32 c = 0; c < num_channels && c < MAX_CH; c++) {
        float x1 = s.x1[c], x2 = s.x2[c], y1 = s.y1[c], y2 = s.y2[c];
        for (u32 i = 0; i < num_samples; i++) {
            const float x = out[c][i];
            const float y = s.b0 * x + s.b1 * x1 + s.b2 * x2 - s.a1 * y1 - s.a2 * y2;
            x2 = x1; x1 = x;
            y2 = y1; y1 = y;
            out[c][i] = y;
        }
        s.x1[c] = x1; s.x2[c] = x2; s.y1[c] = y1; s.y2[c] = y2;
    }
}
