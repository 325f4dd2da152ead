"""Interleaved in-process A/B of the two 8192-point STFT kernels
(cdna guide rule 24).  Prints per-variant median kernel time over rounds."""
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
mag = torch.empty((2, F, 4097), device="cuda")
lib = d.lib()
VARIANTS = tuple(int(a) for a in sys.argv[2:]) or (2, 4, 5)
res = {k: [] for v in VARIANTS for k in (v, f"mem{v}")}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    for v in VARIANTS:
        lib.dsp_stft_kernel_variant(v)
        for kind in ("fused", "mem"):
            for _ in range(2):  # warm
                if kind == "fused":
                    d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
                else:
                    d.stft_magnitude(x, out=mag)
            torch.cuda.synchronize()
            lib.dsp_kernel_timing(None, None, None)
            lib.dsp_kernel_timing_enable(1)
            for _ in range(5):
                if kind == "fused":
                    d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
                else:
                    d.stft_magnitude(x, out=mag)
            torch.cuda.synchronize()
            lib.dsp_kernel_timing_enable(0)
            ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
            lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
            key = v if kind == "fused" else f"mem{v}"
            res[key].append(ms.value / n.value)
for k, v in res.items():
    print(f"variant {k}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms")
