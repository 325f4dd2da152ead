"""The end-to-end path alone (bench.py's `end_to_end`): 1 h of 16-bit stereo
WAV payload in pinned host memory -> dsp_render_stft_wav (8 Mi-sample chunks:
H2D, GPU decode, fused IR_test render + STFT, D2H of render + spectra into
pinned host rows).  Prints each call's time and host-link rate; under
rocprofv3 --kernel-trace --memory-copy-trace every chunk kernel and copy of
the three calls is in the trace (tools/e2e_trace.py summarises it).

    python tools/e2e_probe.py [minutes]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402
from dspbench import wav as dwav  # noqa: E402

minutes = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
SR, CH, B = 48_000, 2, 512
L = int(minutes * 60 * SR)
L -= L % 4096
nb = d.num_blocks(L, B)
F = d.stft_frames(nb * B, 8192, 4096)
pay = torch.randint(-32768, 32768, (CH * L,), dtype=torch.int16).view(torch.uint8).pin_memory()
info = d._lib.dsp_wav_info(format=1, channels=CH, sample_rate=SR, bits_per_sample=16, block_align=CH * 2,
                           frames=L, data_bytes=pay.numel(), n_data_chunks=1)
h_out = torch.empty((CH, nb * B), pin_memory=True)
h_mag = torch.empty((CH, F, 4097), pin_memory=True)
plugin = d.Plugin.ir_test(0.9, 0.002)
stream = torch.cuda.current_stream()
moved = pay.numel() + (h_out.numel() + h_mag.numel()) * 4
for i in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dwav.render_stft_wav(pay, info, CH, B, float(SR), plugin, out=h_out, mag=h_mag, chunk=1 << 23,
                         stream=stream.cuda_stream)
    ms = (time.perf_counter() - t0) * 1e3
    print(f"call {i}: {ms:.2f} ms, {CH * L / ms / 1e3:.1f} Msamples/s, host link {moved / ms / 1e6:.1f} GB/s "
          f"({pay.numel() / 1e9:.2f} GB up, {(moved - pay.numel()) / 1e9:.2f} GB down)", flush=True)
# spot check: the render of the last call is IR_test's B-periodic ramp
ref, _ = d.render_stft(torch.zeros((CH, 8192), device="cuda"), CH, B, float(SR), plugin)
assert torch.equal(h_out[:, :8192], ref.cpu()), "end-to-end render differs"
print("render spot check ok")
