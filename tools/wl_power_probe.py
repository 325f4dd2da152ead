"""Clock and package power of one bench workload's kernel, settled: the
workload's step runs back to back for ~3 s while rocm-smi samples sclk and
socket power (read-only queries).  Tells a power-capped kernel (sclk pulled
below its idle-boost clock at the package limit) from an issue- or
memory-bound one (full clock, power below the cap).

    python tools/wl_power_probe.py stft96k|gain_stft|headline [seconds]

Product library only (no A/B options)."""
import os
import re
import statistics
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

wl = sys.argv[1]
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
sr = 96_000 if wl == "stft96k" else 48_000
L = sr * 3600
x = (torch.rand((2, L), device="cuda") * 2 - 1) * 0.1
nb = d.num_blocks(L, 512)
F = d.stft_frames(L if wl == "stft96k" else nb * 512, 8192, 4096)
out = None if wl == "stft96k" else torch.empty((2, nb * 512), device="cuda")
mag = torch.empty((2, F, 4097), device="cuda")
plug = d.Plugin.gain_test(0.2) if wl == "gain_stft" else d.Plugin.ir_test(0.9, 0.002)


def step():
    if wl == "stft96k":
        d.stft_magnitude(x, N=8192, H=4096, window=d.DSP_WIN_HANN, K=4097, out=mag)
    else:
        d.render_stft(x, 2, 512, float(sr), plug, N=8192, H=4096, window=d.DSP_WIN_HANN, K=4097,
                      out=out, mag=mag)


def smi(samples, stop):
    time.sleep(1.0)
    while not stop.is_set():
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True)
        samples.append(r.stdout)
        time.sleep(0.4)


for _ in range(5):
    step()
torch.cuda.synchronize()
samples, stop = [], threading.Event()
th = threading.Thread(target=smi, args=(samples, stop))
th.start()
t0 = time.time()
ts = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
while time.time() - t0 < secs:
    e0.record()
    for _ in range(10):
        step()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
stop.set()
th.join()
sclk = [int(m) for s in samples for m in re.findall(r"sclk.*?\((\d+)Mhz\)", s)]
pw = [float(m) for s in samples for m in re.findall(r"Socket Graphics Package Power \(W\): ([\d.]+)", s)]
print(f"{wl}: {len(ts) * 10} launches, settled {statistics.median(ts[len(ts) // 3:]):.4f} ms/launch "
      f"(first {ts[0]:.4f}), sclk MHz {sclk}, package W {pw}", flush=True)
