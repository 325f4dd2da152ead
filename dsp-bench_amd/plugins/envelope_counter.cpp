// envelope_counter.cpp -- an example plugin whose State splits: an envelope
// follower (forgets where it started within a few hundred samples) beside a
// block counter (never forgets, never reads the block) that steps a slow
// eight-block gain pattern.  The reference's audio thread runs such a plugin
// block after block (audio.cpp:160-165); compiled for the GPU its State
// splits (dsp_callback_facts.state_split): the counter's chain alone on one
// lane, then speculative segments started from it.
#include "plugin_header.h"

struct Parameters {
    FLOAT_PARAM(0.0f, 1.0f) release;
    FLOAT_PARAM(0.0f, 1.0f) depth;
};

struct State {
    float env;
    u32 blocks;
};

Parameters default_parameters()
{
    Parameters p = {0.01f, 0.5f};
    return p;
}

State initialize_state(const Parameters& p, const unsigned int num_channels, const float sample_rate,
                       void* initialization_context)
{
    State s = {0.0f, 0u};
    return s;
}

void audio_callback(const Parameters& p, State& s, float** out, const u32 num_channels, const u32 num_samples,
                    const real32 sample_rate)
{
    const float step = (float)(s.blocks & 7u) * 0.125f;
    for (u32 i = 0; i < num_samples; i++) {
        const float x = out[0][i] < 0.0f ? -out[0][i] : out[0][i];
        s.env = x > s.env ? x : s.env + p.release * (x - s.env);
        const float g = 1.0f - p.depth * s.env * step;
        for (u32 c = 0; c < num_channels; c++) out[c][i] = out[c][i] * g;
    }
    s.blocks += 1u;
}
