"""First-call (cold) latency of library entry points: each translation unit's
code object is loaded on the first launch of one of its kernels.
    python tools/first_call_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

x = torch.zeros((2, 48000 * 10), device="cuda")
torch.cuda.synchronize()


def t(name, f, n=2):
    for i in range(n):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        print(f"{name:28s} call {i}: {(time.perf_counter() - t0) * 1e3:8.3f} ms", flush=True)


t("minmax_decimate (display.o)", lambda: d.minmax_decimate(x[0], 1000))
t("render_offline (render.o)", lambda: d.render_offline(x, 2, 512, 48000.0, d.Plugin.gain_test()))
t("render_stft (stft_pk.o)", lambda: d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test()))
t("stft hamming (stft_pk.o)", lambda: d.stft_magnitude(x, N=8192, H=4096, window=d.DSP_WIN_HAMMING, K=4097))
t("ir_analysis", lambda: d.ir_analysis(d.Plugin.ir_test(), C_out=2, device="cuda"))
t("fft_forward 1024 (spectral.o)", lambda: d.fft_forward(x[0, :1024]))
