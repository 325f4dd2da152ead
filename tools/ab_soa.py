"""Interleaved in-process A/B of the kernel option bits (rule 24).
  usage: python tools/ab_soa.py ROUNDS [vVARIANT] [opts...]
variant 2: opts are dsp_stft_soa_options values; variant 5: opts are the
packed kernel's bits (passed as 14 | opt << 4)."""
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
args = sys.argv[2:]
variant = 2
if args and args[0].startswith("v"):
    variant, args = int(args[0][1:]), args[1:]
lib.dsp_stft_kernel_variant(variant)
opts = [int(a) for a in args] or (list(range(0, 16, 2)) if variant == 2 else list(range(8)))
res = {}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    for o in opts:
        lib.dsp_stft_soa_options(o if variant == 2 else 14 | (o << 4))
        for kind in ("fused", "mem"):
            def run():
                if kind == "fused":
                    d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
                else:
                    d.stft_magnitude(x, out=mag)
            run(); run()
            torch.cuda.synchronize()
            lib.dsp_kernel_timing(None, None, None)
            lib.dsp_kernel_timing_enable(1)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            lib.dsp_kernel_timing_enable(0)
            ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
            lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
            res.setdefault((kind, o), []).append(ms.value / n.value)
for (kind, o), v in sorted(res.items()):
    print(f"{kind:5s} opt {o}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms")
