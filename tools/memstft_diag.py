"""Does the memory-source STFT give the same bits for the same frames in
different buffers?  (diagnostic for the callback-path chunk mismatch)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

L = 8192 * 12
x = torch.rand((2, L), device="cuda") * 2 - 1
m0 = d.stft_magnitude(x).clone()
for tag, y in (("clone", x.clone()), ("slice", x[:, : 3 * 4096 + 4096].contiguous()),
               ("offset view", torch.cat([torch.zeros((2, 4096), device="cuda"), x], 1)[:, 4096:])):
    m = d.stft_magnitude(y)
    n = min(m.shape[1], m0.shape[1])
    print(tag, "rows", n, "equal", bool(torch.equal(m[:, :n], m0[:, :n])),
          "max diff", float((m[:, :n] - m0[:, :n]).abs().max()), flush=True)
m1 = d.stft_magnitude(x)
print("rerun equal", bool(torch.equal(m1, m0)))
