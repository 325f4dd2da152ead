"""Per-file cost of many short renders: eager dsp_render_stft calls against
replays of one captured HIP graph (tests/test_gpu_graph.py checks the bits).
    python tools/graph_replay_probe.py [seconds_per_file ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

secs = [float(a) for a in sys.argv[1:]] or [0.2, 1.0, 10.0]
p = d.Plugin.ir_test(0.9, 0.002)
for s in secs:
    L = int(48_000 * s)
    x = torch.rand((2, L), device="cuda")
    nb = d.num_blocks(L, 512)
    out = torch.empty((2, nb * 512), device="cuda")
    mag = torch.empty((2, max(1, d.stft_frames(nb * 512, 8192, 4096)), 4097), device="cuda")
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(3):
            d.render_stft(x, 2, 512, 48000.0, p, out=out, mag=mag)
    torch.cuda.synchronize()
    n = 400
    with torch.cuda.stream(side):
        t0 = time.perf_counter()
        for _ in range(n):
            d.render_stft(x, 2, 512, 48000.0, p, out=out, mag=mag)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / n * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        d.render_stft(x, 2, 512, 48000.0, p, out=out, mag=mag)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / n * 1e3
    print(f"{s:6.2f} s stereo file: eager {eager:8.4f} ms/file, graph replay {graph:8.4f} ms/file "
          f"({2 * L / graph / 1e3:10.1f} Msamples/s replayed)", flush=True)
