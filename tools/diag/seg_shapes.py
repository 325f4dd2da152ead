"""Time biquad.cpp (compiled unchanged) through the speculative segments at
several (C, B) shapes, 10 min of 48 kHz: which kernel instantiation each
shape gets and what it costs (tools/sessions/gpu_r05s.sh)."""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "dsp-bench_amd"))
import dspbench as d  # noqa: E402

with open(os.path.join(ROOT, "dsp-bench_amd", "modules", "mod_biquad.co"), "rb") as f:
    mod = d.module.Module(f.read())
params = mod.default_parameters()
L = 48000 * 600
for C, B in [(2, 512), (2, 256), (1, 512), (2, 1024), (4, 512)]:
    x = torch.rand((C, L), device="cuda") * 2 - 1
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params)
    out = torch.empty((C, (L + B - 1) // B * B), device="cuda")
    for _ in range(3):
        d.render_offline(x, C, B, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    print("  after warm-up:", mod.state_spec(), flush=True)
    t = time.perf_counter()
    n = 10
    for _ in range(n):
        d.render_offline(x, C, B, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / n * 1e3
    info = mod.state_spec()
    print(f"C={C} B={B}: {ms:.3f} ms per 10 min ({C * L / ms / 1e3:.0f} Msamples/s) segments={info['segments']} "
          f"seg={info['blocks_per_segment']} levels={info['levels']} differed={info['differed']}", flush=True)
