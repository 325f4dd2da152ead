"""Interleaved A/B of two builds of libdspbench.so at the headline shape:
each round runs every library in a fresh subprocess (settled: 60 warm + 200
timed launches) and prints the median kernel time.

    python tools/ab_lib.py [--fir|--mem] ROUNDS LIB_A LIB_B ...
(--fir: the fir1024 workload, 10 min stereo overlap-save; --mem: the stft96k
memory-source STFT)
"""
import os
import statistics
import subprocess
import sys

CHILD = r'''
import ctypes as C, os, sys, torch
sys.path.insert(0, os.path.join(%r, "dsp-bench_amd"))
os.environ["DSPBENCH_LIB"] = %r
import dspbench as d
lib = d.lib()
MODE = %r
L_ = 48_000 * (600 if MODE == "fir" else 7200 if MODE == "mem" else 3600)
x = torch.rand((2, L_), device="cuda") - 0.5
# fir: 4 input copies in rotation (a 230 MB input would stay in the Infinity Cache)
xs = [x] + ([x.clone() for _ in range(3)] if MODE == "fir" else [])
it = [0]
def nx():
    it[0] += 1
    return xs[it[0] %% len(xs)]
nb = d.num_blocks(L_, 512)
F = d.stft_frames(nb * 512, 8192, 4096)
out = torch.empty((2, nb * 512), device="cuda"); mag = torch.empty((2, F, 4097), device="cuda")
if MODE == "fir":
    ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=48000.0, device=torch.device("cuda"))
    fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy())
def step():
    if MODE == "fir": d.render_offline(nx(), 2, 512, 48000.0, fplug, out=out)
    elif MODE == "mem": d.stft_magnitude(x, N=8192, H=4096, window=d.DSP_WIN_HANN, K=4097, out=mag)
    else: d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
for _ in range(60): step()
torch.cuda.synchronize()
lib.dsp_kernel_timing(None, None, None); lib.dsp_kernel_timing_enable(1)
for _ in range(200): step()
torch.cuda.synchronize(); lib.dsp_kernel_timing_enable(0)
ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
print(ms.value / n.value)
'''
repo = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
argv = sys.argv[1:]
mode = "headline"
if argv and argv[0] in ("--fir", "--mem"):
    mode = argv.pop(0)[2:]
rounds = int(argv[0])
libs = argv[1:]
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        o = subprocess.run([sys.executable, "-c", CHILD % (repo, os.path.abspath(l), mode)], capture_output=True,
                           text=True, timeout=120)
        res[l].append(float(o.stdout.strip().splitlines()[-1]))
for l, v in res.items():
    print(f"{l}: median {statistics.median(v):.4f} ms  all {' '.join(f'{t:.4f}' for t in v)}")
