import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "dsp-bench_amd"))
import numpy as np, torch
import dspbench as d
src = open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests/test_gpu_specialize.py")).read()
i = src.index("TONE_SRC = r'''"); j = src.index("'''", i + 15)
tone = src[i + 15:j]
code = d.module.compile_source(tone, "tone.cpp")
print("facts", d.module.code_facts(code))
mod = d.module.Module(code)
p = mod.default_parameters()
mod.initialize_state(p, 2, 44100.0)
print("stateless", mod.stateless)
print("class", mod.block_class(p, 2, 480, 44100.0))
x = torch.zeros((2, 4800), device="cuda")
a = d.render_offline(x, 2, 480, 44100.0, mod.plugin(p, "tone", specialize=False)).cpu().numpy()
b = d.render_offline(torch.rand((2, 4800), device="cuda"), 2, 480, 44100.0, mod.plugin(p, "tone", specialize=False)).cpu().numpy()
print("input-independent", np.array_equal(a, b), "channels equal", np.array_equal(a[0], a[1]), "blocks equal", np.array_equal(a[0, :480], a[0, 480:960]))
