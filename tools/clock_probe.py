"""Clock / power of the headline kernel per option bit set: each option runs
back to back for ~2.5 s while rocm-smi samples sclk and socket power twice
(read-only queries).  Tells a power-capped kernel (lower sclk) from a
stalled one.

    python tools/clock_probe.py OPT [OPT ...]   (stft_pk.hpp kPk* bits)
    python tools/clock_probe.py fir             (the fir1024 workload instead)
    python tools/clock_probe.py mem [OPT ...]   (the stft96k workload: STFT from HBM)
"""
import os
import re
import statistics
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
# the A/B options live in the tools build only (make -C dsp-bench_amd ab)
os.environ.setdefault("DSPBENCH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "dsp-bench_amd", "build", "ab", "libdspbench_ab.so"))
import dspbench as d  # noqa: E402

FIR = sys.argv[1:2] == ["fir"]
MEM = sys.argv[1:2] == ["mem"]
L_ = 48_000 * (600 if FIR else 7200 if MEM else 3600)
x = torch.zeros((2, L_), device="cuda")
nb = d.num_blocks(L_, 512)
F = d.stft_frames(nb * 512, 8192, 4096)
out = torch.empty((2, nb * 512), device="cuda")
mag = torch.empty((2, d.stft_frames(L_, 8192, 4096) if MEM else F, 4097), device="cuda")
lib = d.lib()
if FIR:
    ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=48000.0, device=torch.device("cuda"))
    fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy())
    x.uniform_(-0.1, 0.1)
if MEM:
    x.uniform_(-0.1, 0.1)


def step():
    if FIR:
        d.render_offline(x, 2, 512, 48000.0, fplug, out=out)
    elif MEM:
        d.stft_magnitude(x, N=8192, H=4096, window=d.DSP_WIN_HANN, K=4097, out=mag)
    else:
        d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)


def smi(samples):
    for delay in (1.0, 0.7):
        time.sleep(delay)
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True)
        samples.append(r.stdout)


for o in ([0] if FIR else [int(a) for a in sys.argv[2:]] or [0] if MEM else [int(a) for a in sys.argv[1:]] or [0]):
    lib.dsp_stft_pk_ab_options(o)
    samples = []
    th = threading.Thread(target=smi, args=(samples,))
    t0 = time.time()
    th.start()
    n = 0
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    ts = []
    while time.time() - t0 < 2.5:
        e0.record()
        for _ in range(20):
            step()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20)
        n += 20
    th.join()
    sclk = [m for s in samples for m in re.findall(r"sclk.*?\((\d+)Mhz\)", s)]
    pw = [m for s in samples for m in re.findall(r"Socket Graphics Package Power \(W\): ([\d.]+)", s)]
    print(f"opt {o:4d}: {n} launches, {statistics.median(ts[2:]):.4f} ms/launch settled, sclk {sclk} MHz, "
          f"power {pw} W", flush=True)
lib.dsp_stft_pk_ab_options(0)
