"""Time a tremolo (tests/test_gpu_state_spec.py TREMOLO_SRC: reads its block,
its phase never depends on it) over 1 min of stereo: the State chain from
edited IR (the default once learnt) against the serial chain."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402
import test_gpu_state_spec as t  # noqa: E402

mod = t.module_of(t.TREMOLO_SRC, "tremolo_time")
params = mod.default_parameters()
x = torch.rand(2, 48000 * 60, device="cuda") * 2 - 1
for serial in (True, False):
    mod.initialize_state(params, 2, 48000.0)
    plug = mod.plugin(params, serial_state=serial)
    out = torch.empty_like(x)
    d.render_offline(x, 2, 512, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    first = time.perf_counter()
    d.render_offline(x, 2, 512, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    n, t0 = 5, time.perf_counter()
    for _ in range(n):
        d.render_offline(x, 2, 512, 48000.0, plug, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    info = mod.state_spec()
    print(f"{'serial chain' if serial else 'default'}: {ms:.2f} ms per 1 min stereo render "
          f"({2 * 48000 * 60 / ms / 1e3:.1f} Msamples/s); chain={info['chain']}")
