"""Interleaved A/B of the magnitude row pitch (ld) for the headline fused
render + STFT: the same 4097 bins per frame, rows padded to ld floats.
    python tools/ab_ld.py [rounds] [ld ...]"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

L_ = 48_000 * 3600
x = (torch.rand((2, L_), device="cuda") * 2 - 1) * 0.1
nb = d.num_blocks(L_, 512)
F = d.stft_frames(nb * 512, 8192, 4096)
out = torch.empty((2, nb * 512), device="cuda")
LDS = tuple(int(a) for a in sys.argv[2:]) or (4097, 4100, 4104, 4128, 4160)
mags = {ld: torch.empty((2, F, ld), device="cuda") for ld in LDS}
lib = d.lib()
res = {ld: [] for ld in LDS}
p = d.Plugin.ir_test()
for _ in range(60):  # settle the clock
    d.render_stft(x, 2, 512, 48000.0, p, out=out, mag=mags[LDS[0]], ld=LDS[0])
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    for ld in LDS:
        torch.cuda.synchronize()
        lib.dsp_kernel_timing(None, None, None)
        lib.dsp_kernel_timing_enable(1)
        for _ in range(10):
            d.render_stft(x, 2, 512, 48000.0, p, out=out, mag=mags[ld], ld=ld)
        torch.cuda.synchronize()
        lib.dsp_kernel_timing_enable(0)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
        lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
        res[ld].append(ms.value / n.value)
for ld, v in res.items():
    print(f"ld {ld}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms")
