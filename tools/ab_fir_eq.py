"""Bit-identity of two FIR render methods (dsp_fir_method) on 10 min of stereo:
python tools/ab_fir_eq.py M1 M2"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

m1, m2 = int(sys.argv[1]), int(sys.argv[2])
L_ = 48_000 * 600 + 12345
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.rand((2, L_), device="cuda", generator=g) * 2 - 1
ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=48000.0, device=torch.device("cuda"))
fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy())
nb = d.num_blocks(L_, 512)
outs = {}
for m in (m1, m2):
    d.lib().dsp_fir_method(m)
    o = torch.full((2, nb * 512), float("nan"), device="cuda")
    d.render_offline(x, 2, 512, 48000.0, fplug, out=o)
    torch.cuda.synchronize()
    outs[m] = o
d.lib().dsp_fir_method(0)
same = torch.equal(outs[m1], outs[m2])
print("bit-identical:", same, "nan:", bool(torch.isnan(outs[m2]).any()))
assert same
