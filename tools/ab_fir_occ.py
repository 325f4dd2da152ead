"""FIR overlap-save at two (method 2) vs three (method 3) waves per SIMD:
bit-identity of the render on 10 min of stereo, then the bench's timing for
both (run bench.py --workload fir1024 --fir-method M separately)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

L_ = 48_000 * 600 + 12345
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.rand((2, L_), device="cuda", generator=g) * 2 - 1
ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=48000.0, device=torch.device("cuda"))
fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy())
nb = d.num_blocks(L_, 512)
outs = {}
for m in (2, 3):
    d.lib().dsp_fir_method(m)
    o = torch.full((2, nb * 512), float("nan"), device="cuda")
    d.render_offline(x, 2, 512, 48000.0, fplug, out=o)
    torch.cuda.synchronize()
    outs[m] = o
d.lib().dsp_fir_method(0)
print("bit-identical:", torch.equal(outs[2], outs[3]), "nan:", bool(torch.isnan(outs[3]).any()))
assert torch.equal(outs[2], outs[3])
