"""Where the State chain path of a never-forgetting plugin departs from the
serial chain: per call, the first differing sample and the States."""
import sys
import os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "dsp-bench_amd"))
import dspbench as d
import test_gpu_state_spec as t

C, B, L = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (2, 512, 300_000)
mod = t.module_of(t.OSC_SRC, "osc_dbg")
params = mod.default_parameters()
x = t.noise(C, L, 11)
res = {}
for serial in (False, True):
    mod.initialize_state(params, C, 48000.0)
    plug = mod.plugin(params, serial_state=serial)
    xg = torch.from_numpy(x).cuda()
    outs = []
    for call in range(3):
        y = d.render_offline(xg, C, B, 48000.0, plug).cpu().numpy()
        outs.append((y, mod.read_state(), mod.state_spec() if not serial else None))
    res[serial] = outs
for call in range(3):
    a, sa, info = res[False][call]
    b, sb, _ = res[True][call]
    diff = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(axis=0))[0]
    print("call", call, "info", info)
    print("  states equal", sa == sb, np.frombuffer(sa, np.float64), np.frombuffer(sb, np.float64))
    if len(diff):
        print("  first diff sample", diff[0], "block", diff[0] // B, "count", len(diff), "last", diff[-1])
