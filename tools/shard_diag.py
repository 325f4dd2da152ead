"""Where do a time shard's spectra differ from the whole-file call?
(diagnostic for tests/test_gpu_shard.py::test_loopback_sharded_driver_equals_whole_file)"""
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402
import dspbench.shard as sh  # noqa: E402

L, B, K, world = 8192 * 14 + 2345, 512, 4097, 2
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.rand((2, L), device="cuda", generator=g) * 2 - 1
plugin = d.Plugin.gain_test(0.3)
ref_out, ref_mag = d.render_stft(x, 2, B, 96000.0, plugin, window=d.DSP_WIN_HANN, L_file=L)
torch.cuda.synchronize()


def cmp(tag, mag, f0, nf):
    m = mag[:, :nf]
    r = ref_mag[:, f0:f0 + nf]
    bad = (m != r).reshape(2, nf, -1).any(-1)
    print(f"{tag}: rows differ {bad.sum().item()} of {2 * nf}, max {(m - r).abs().max().item():.3g}", flush=True)


s = sh.plan(L, world, 0, B, 8192, 4096, True, 2, sh.TIME)
print(s)
# 1. one dsp_render_stft on rank 0's rows, as a view and as a copy
for tag, xin in (("view", x[:, :s.read_len]), ("copy", x[:, :s.read_len].contiguous())):
    o, m = d.render_stft(xin, 2, B, 96000.0, plugin, window=d.DSP_WIN_HANN, L_file=s.read_len)
    torch.cuda.synchronize()
    cmp(f"render_stft {tag}", m, 0, s.frames)
# 2. the sharded driver without a collective, sequential
out = torch.empty((2, -(-s.read_len // B) * B), device="cuda")
mag = torch.empty((2, s.frames, K), device="cuda")
for chunk in (0, 3 * 4096):
    sh.render_stft_sharded(x[:, :s.read_len].contiguous(), L, 2, B, 96000.0, plugin, s, out, mag, comm=None,
                           gather=False, chunk=chunk)
    torch.cuda.synchronize()
    cmp(f"sharded chunk={chunk} sequential", mag, 0, s.frames)
# 3. the same on two threads at once, each on its own stream
res = {}


def run(r):
    torch.cuda.set_device(0)
    sr = sh.plan(L, world, r, B, 8192, 4096, True, 2, sh.TIME)
    o = torch.empty((2, -(-sr.read_len // B) * B), device="cuda")
    m = torch.empty((2, sr.frames, K), device="cuda")
    st = torch.cuda.Stream()
    xl = x[:, sr.start:sr.start + sr.read_len].contiguous()
    st.wait_stream(torch.cuda.default_stream())
    for _ in range(3):
        sh.render_stft_sharded(xl, L, 2, B, 96000.0, plugin, sr, o, m, comm=None, gather=False, chunk=3 * 4096,
                               stream=st.cuda_stream)
    st.synchronize()
    res[r] = (sr, m)


ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
for t in ts:
    t.start()
for t in ts:
    t.join()
for r in range(world):
    sr, m = res[r]
    cmp(f"threads rank {r}", m, sr.frame0, sr.frames)
