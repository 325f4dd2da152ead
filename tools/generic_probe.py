"""Generic plugin dispatch throughput: the reference's plugins (compiled by
the product's hiprtc path, oracle/_ref/mod_*.co) rendered on the GPU, beside
the same sources compiled for the CPU (oracle/_ref/libref_*.so) through the
oracle's render loop on one host core (skipped past 60 s of audio).

    python tools/generic_probe.py [seconds_of_audio] [plugin ...]

Stateless plugins: the median of 7 renders into one output buffer, timed
with HIP events (the call no longer synchronises).  DSPB_STATELESS_PATH =
0 (in-place wave), 1 (private arrays) or 3 (LDS blocks, the default) picks
the stateless driver path; the GPU output is checked against the first
path run in the same process when DSPB_PROBE_CHECK=1.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "dsp-bench_amd"))
sys.path.insert(0, ROOT)
import dspbench as d  # noqa: E402
from oracle import oracle  # noqa: E402

MODS = os.path.join(ROOT, "dsp-bench_amd", "modules")
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
names = sys.argv[2:] or ["sine_test", "handmade_test", "gain_test"]
L = int(secs * 48000)
g = torch.Generator(device="cuda").manual_seed(1)
xg = torch.rand((2, L), device="cuda", generator=g) * 2 - 1
path = os.environ.get("DSPB_STATELESS_PATH", "3 (default)")
for name in names:
    with open(os.path.join(MODS, f"mod_{name}.co"), "rb") as f:
        mod = d.module.Module(f.read())
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    plug = mod.plugin(params, name)
    out = d.render_offline(xg, 2, 512, 48000.0, plug)
    torch.cuda.synchronize()
    reps = 7 if mod.stateless else 1
    ts = []
    for _ in range(reps):  # into the same output buffer: no allocation in the loop
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.render_offline(xg, 2, 512, 48000.0, plug, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    tg = sorted(ts)[len(ts) // 2]
    cpu = ""
    if secs <= 60:
        x = xg.cpu().numpy()
        ref = oracle.RefPlugin(name, 2, 48000.0)
        t = time.perf_counter()
        want = oracle.render_offline([x[0], x[1]], 2, 512, 48000.0, ref.as_oracle())
        tc = time.perf_counter() - t
        tol = 1e-6 if name in ("sine_test", "buffer_test") else 0.0
        ok = np.max(np.abs(out.cpu().numpy() - want)) <= tol if mod.stateless else "n/a (state advanced)"
        cpu = f"   CPU 1 core {tc * 1e3:9.2f} ms ({2 * L / tc / 1e6:8.1f} Msamples/s)  parity {ok}"
    gbs = 2 * L * 8 / tg / 1e9
    print(f"{name:16s} path {path} stateless={mod.stateless}  {secs:g} s stereo: GPU {tg * 1e3:9.3f} ms "
          f"({2 * L / tg / 1e6:10.1f} Msamples/s, {gbs:7.1f} GB/s read+write){cpu}", flush=True)
