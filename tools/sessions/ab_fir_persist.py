"""Interleaved in-process A/B of the overlap-save FIR (bench workload
fir1024: 1024 taps = compute_IR(IR_test)[0:1024], stereo 48 kHz): the
product's one-wave-per-frame fir_fft_kernel (opt 0) against the tools
build's persistent grids (kernels.hpp kFirAb*: 262144 = 4-wave groups,
524288 = 8-wave groups, + (n << 20) = the SIMD's second wave sleeps n x 8128
cycles first).

    python tools/ab_fir_persist.py ROUNDS MINUTES [OPT ...]

Each round runs each option for 20 launches after 10 warm ones, rotating 4
inputs as bench.py does, and records the average launch time from
libdspbench's own HIP events; round 0 checks the renders against opt 0.
The variants were measured and removed (profiles/r03_fir_persist_ab.txt,
r03_fir_pair_ab.txt -- the pair kernel is now the product's): the
persistent grids are in commit 91c8a58's tools build, the 3-waves-per-SIMD
build was never committed (fir_fft.hip at 12-wave groups with the stage
twiddles loaded inside each transform)."""
import ctypes as C
import hashlib
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
os.environ.setdefault("DSPBENCH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "dsp-bench_amd", "build", "ab", "libdspbench_ab.so"))
import dspbench as d  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
minutes = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
OPTS = tuple(int(o) for o in sys.argv[3:]) or (0, 262144, 524288)
SR, B, CH = 48_000, 512, 2
L = int(minutes * 60 * SR)
L -= L % B
dev = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(7)
xs = [torch.rand((CH, L), device="cuda", generator=g) * 2 - 1 for _ in range(4)]
out = torch.empty((CH, L), device="cuda")
ir, _ = d.ir_analysis(d.Plugin.ir_test(0.9, 0.002), C_out=1, sr=float(SR), device=dev)
fplug = d.Plugin.fir(ir[0, :1024].cpu().numpy())
lib = d.lib()
# a product build (DSPBENCH_LIB=...libdspbench.so variant) has no A/B switch: option 0 only
set_opt = getattr(lib, "dsp_stft_pk_ab_options", None) if hasattr(lib, "dsp_stft_pk_ab_options") else None
if set_opt is None:
    assert OPTS == (0,), "option switches need the tools build"
    set_opt = lambda o: 0  # noqa: E731
res = {o: [] for o in OPTS}
ref = None
k = 0


def step():
    global k
    k = (k + 1) % 4
    d.render_offline(xs[k], CH, B, float(SR), fplug, out=out)


for rnd in range(rounds):
    for o in OPTS:
        set_opt(o)
        if rnd == 0:
            d.render_offline(xs[0], CH, B, float(SR), fplug, out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
                print(f"opt {o}: render sha1 {hashlib.sha1(ref.cpu().numpy().tobytes()).hexdigest()[:16]}", flush=True)
            else:
                same = torch.equal(out, ref)
                rel = float((out - ref).abs().max() / ref.abs().max())
                nbad = int((out != ref).sum())
                print(f"opt {o}: bit-identical to opt {OPTS[0]}: {same} (peak-relative max diff {rel:.3g}, "
                      f"{nbad} samples differ)", flush=True)
                assert rel <= 2e-6, f"option {o} changed the render beyond the overlap-save bar"
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        lib.dsp_kernel_timing(None, None, None)
        lib.dsp_kernel_timing_enable(1)
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        lib.dsp_kernel_timing_enable(0)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
        lib.dsp_kernel_timing(C.byref(ms), C.byref(n), C.byref(b))
        res[o].append(ms.value / n.value)
    print(f"round {rnd}: " + "  ".join(f"{o}: {res[o][-1]:.4f} ms" for o in OPTS), flush=True)
set_opt(0)
byt = b.value / n.value
for o, v in res.items():
    med = statistics.median(v)
    print(f"opt {o:8d}: median {med:.4f} ms  min {min(v):.4f} ms  ({byt / med / 1e6:.1f} GB/s, "
          f"{byt / med / 8e9:.3f} of 8 TB/s)")
