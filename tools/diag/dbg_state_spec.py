import os, sys
import torch
ROOT="/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path.insert(0, os.path.join(ROOT, "dsp-bench_amd"))
import dspbench as d
with open(os.path.join(ROOT, "dsp-bench_amd", "modules", "mod_biquad.co"), "rb") as f:
    mod = d.module.Module(f.read())
params = mod.default_parameters()
for C, B, L in [(2, 512, 48000 * 60), (2, 256, 48000 * 60), (1, 512, 48000 * 30)]:
    x = torch.rand((C, L), device="cuda") * 2 - 1
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params)
    for i in range(3):
        y = d.render_offline(x, C, B, 48000.0, plug)
        torch.cuda.synchronize()
        print(C, B, i, mod.state_spec(), flush=True)
