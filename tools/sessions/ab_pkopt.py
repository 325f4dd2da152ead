"""Interleaved in-process A/B of stft8192_pk_kernel store options at the
headline shape (IR_test B = 512 fused render + Hann STFT, 1 h of 48 kHz stereo).

    python tools/ab_pkopt.py ROUNDS OPT [OPT ...]     (OPT = stft_pk.hpp kPk* bits)

Each round runs every option for 20 back-to-back launches after 10 warm ones
(the settled, power-capped state the bench measures) and records the average
launch time from libdspbench's own HIP events."""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
# the A/B options live in the tools build only (make -C dsp-bench_amd ab)
os.environ.setdefault("DSPBENCH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "dsp-bench_amd", "build", "ab", "libdspbench_ab.so"))
import dspbench as d  # noqa: E402

L_ = 48_000 * 3600
x = (torch.rand((2, L_), device="cuda") * 2 - 1) * 0.1
nb = d.num_blocks(L_, 512)
F = d.stft_frames(nb * 512, 8192, 4096)
out = torch.empty((2, nb * 512), device="cuda")
mag = torch.empty((2, F, 4097), device="cuda")
lib = d.lib()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
OPTS = tuple(int(a) for a in sys.argv[2:]) or (0, 32)
res = {o: [] for o in OPTS}
ref = None
for rnd in range(rounds):
    for o in OPTS:
        lib.dsp_stft_pk_ab_options(o)
        for _ in range(10):
            d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
        torch.cuda.synchronize()
        if rnd == 0:  # every option must produce the same bits
            m = mag.clone()
            if ref is None:
                ref = m
            else:  # a different split order may change the last bit, not more
                err = ((m - ref).abs().amax(dim=2) / ref.amax(dim=2)).max().item()
                print(f"opt {o}: max peak-relative difference to opt {OPTS[0]}: {err:.2e}")
                assert err < 1e-6, f"option {o} changed the output"

        lib.dsp_kernel_timing(None, None, None)
        lib.dsp_kernel_timing_enable(1)
        for _ in range(20):
            d.render_stft(x, 2, 512, 48000.0, d.Plugin.ir_test(), out=out, mag=mag)
        torch.cuda.synchronize()
        lib.dsp_kernel_timing_enable(0)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
        lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
        res[o].append(ms.value / n.value)
lib.dsp_stft_pk_ab_options(0)
byt = b.value / n.value
for o, v in res.items():
    med = statistics.median(v)
    print(f"opt {o:3d}: median {med:.4f} ms  min {min(v):.4f} ms  ({byt / med / 1e6:.1f} GB/s)")
