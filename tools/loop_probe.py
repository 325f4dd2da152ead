"""Loop-mode render throughput (dsp_render_loop, audio.cpp:100-132): 1 h of
48 kHz stereo rendered from a shorter file that wraps, gain_test, B = 512.
    python tools/loop_probe.py [file_seconds ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

B = 512
CURSOR = int(os.environ.get("CURSOR", "123"))
nb = 48_000 * 3600 // B
out = torch.empty((2, nb * B), device="cuda")
for secs in [float(a) for a in sys.argv[1:]] or [10.0, 600.0]:
    L = int(48_000 * secs)
    x = torch.rand((2, L), device="cuda")
    p = d.Plugin.gain_test(0.5)
    for _ in range(3):
        d.render_loop(x, 2, B, nb, 48000.0, p, cursor=CURSOR, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        d.render_loop(x, 2, B, nb, 48000.0, p, cursor=CURSOR, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    byt = 2 * nb * B * 8  # each output sample: one file read (cache or HBM) + one write
    print(f"cursor {CURSOR}, file {secs:6.1f} s: {ms:.4f} ms per stereo hour, {byt / ms / 1e6:7.1f} GB/s of render traffic", flush=True)
