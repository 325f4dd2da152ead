"""Which engine moves a pinned host <-> HBM copy, and what it costs the GPU.

    python tools/copy_engine_probe.py [MiB]

Prints the HSA/HIP copy knobs of the environment, then
  * H2D alone, D2H alone, and both at once on two streams (GB/s);
  * the fused IR_test render + STFT of one pipeline chunk (8 Mi samples of
    stereo, what dsp_render_stft_wav runs per chunk) alone, and while a D2H
    copy of the same size runs on another stream (ms per chunk).
Run it under rocprofv3 --kernel-trace --memory-copy-trace to see whether the
copies run as __amd_rocclr_copyBuffer kernels (on the CUs) or on SDMA.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

for k in sorted(os.environ):
    if k.startswith(("HSA_", "GPU_", "ROC_", "HIP_", "DEBUG_CLR", "AMD_")):
        print(f"env {k}={os.environ[k]}")

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = mib * (1 << 20) // 4
h_up = torch.empty(n, pin_memory=True)
h_dn = torch.empty(n, pin_memory=True)
d_up = torch.empty(n, device="cuda")
d_dn = torch.rand(n, device="cuda")
s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def up():
    with torch.cuda.stream(s1):
        d_up.copy_(h_up, non_blocking=True)


def down():
    with torch.cuda.stream(s2):
        h_dn.copy_(d_dn, non_blocking=True)


def both():
    up()
    down()


gb = n * 4 / 1e9
print(f"H2D {mib} MiB: {gb / timed(up):6.1f} GB/s")
print(f"D2H {mib} MiB: {gb / timed(down):6.1f} GB/s")
t = timed(both)
print(f"H2D + D2H at once, {mib} MiB each: {2 * gb / t:6.1f} GB/s total")

# one pipeline chunk of the end-to-end path
L = 1 << 23
x = torch.zeros((2, L), device="cuda")
out = torch.empty((2, L), device="cuda")
F = d.stft_frames(L, 8192, 4096)
mag = torch.empty((2, F, 4097), device="cuda")
plug = d.Plugin.ir_test()


def chunk(reps):
    with torch.cuda.stream(s3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            d.render_stft(x, 2, 512, 48000.0, plug, window=d.DSP_WIN_HANN, out=out, mag=mag)
        e1.record()
    return e0, e1


for _ in range(3):
    chunk(20)
torch.cuda.synchronize()
e0, e1 = chunk(50)
torch.cuda.synchronize()
print(f"chunk alone: {e0.elapsed_time(e1) / 50:.4f} ms")
for label, fn in (("D2H", down), ("H2D", up), ("H2D + D2H", both)):
    fn()
    e0, e1 = chunk(20)
    torch.cuda.synchronize()
    print(f"chunk with a {mib} MiB {label} copy in flight: {e0.elapsed_time(e1) / 20:.4f} ms")
