"""Generic plugin dispatch throughput: the reference's stateful plugins
(compiled by the product's hiprtc path, oracle/_ref/mod_*.co) rendered on the
GPU, beside the same sources compiled for the CPU (oracle/_ref/libref_*.so)
through the oracle's render loop on one host core.

    python tools/generic_probe.py [seconds_of_audio] [plugin ...]

Stateless plugins: the median of 7 renders into one output buffer.
DSPB_STATELESS_LDS=<bytes per wave> picks the staged path's LDS rows
(0: the in-HBM one-block-per-thread path).
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

REF = os.path.join(ROOT, "oracle", "_ref")
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
names = sys.argv[2:] or ["sine_test", "handmade_test", "gain_test"]
L = int(secs * 48000)
x = np.random.default_rng(1).uniform(-1, 1, (2, L)).astype(np.float32)
xg = torch.from_numpy(x).cuda()
for name in names:
    with open(os.path.join(REF, f"mod_{name}.co"), "rb") as f:
        mod = d.module.Module(f.read())
    params = mod.default_parameters()
    mod.initialize_state(params, 2, 48000.0)
    plug = mod.plugin(params, name)
    out = d.render_offline(xg, 2, 512, 48000.0, plug)
    torch.cuda.synchronize()
    reps = 7 if mod.stateless else 1
    ts = []
    for _ in range(reps):  # into the same output buffer: no allocation in the loop
        t = time.perf_counter()
        d.render_offline(xg, 2, 512, 48000.0, plug, out=out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    tg = sorted(ts)[len(ts) // 2]
    ref = oracle.RefPlugin(name, 2, 48000.0)
    t = time.perf_counter()
    want = oracle.render_offline([x[0], x[1]], 2, 512, 48000.0, ref.as_oracle())
    tc = time.perf_counter() - t
    print(f"{name:16s} stateless={mod.stateless}  {secs:g} s stereo: GPU {tg * 1e3:9.2f} ms "
          f"({2 * L / tg / 1e6:8.1f} Msamples/s)   CPU 1 core {tc * 1e3:9.2f} ms ({2 * L / tc / 1e6:8.1f} Msamples/s)",
          flush=True)
