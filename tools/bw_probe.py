"""HBM bandwidth probes on the box: pure write (fill), read+write (copy),
read-only (sum), each on ~2.8 GB, timed with HIP events (median of 10)."""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

n = 2 * 48_000 * 3600 * 2  # floats (2.76 GB)
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
a.uniform_()
lib = d.lib()
ex = d.api._exec(a)


def t(fn, reps=10):
    ts = []
    for _ in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts[2:])


FP = d._lib.FP
pa, pb = C.cast(C.c_void_p(a.data_ptr()), FP), C.cast(C.c_void_p(b.data_ptr()), FP)
res = {
    "torch fill (write)": (t(lambda: b.fill_(1.0)), n * 4),
    "dsp_set (write)": (t(lambda: lib.dsp_set(1.0, pb, n, C.byref(ex))), n * 4),
    "torch copy (r+w; a device memcpy)": (t(lambda: b.copy_(a)), 2 * n * 4),
    "dsp_gain (r+w)": (t(lambda: lib.dsp_gain(pa, pb, 0.5, n, C.byref(ex))), 2 * n * 4),
    "dsp_copy (r+w)": (t(lambda: lib.dsp_copy(pa, pb, n, C.byref(ex))), 2 * n * 4),
    "dsp_magnitude (2r+w)": (t(lambda: lib.dsp_magnitude(pa, pa, pb, n, C.byref(ex))), 3 * n * 4),
    "torch sum (read)": (t(lambda: a.sum()), n * 4),
}
for k, (ms, byt) in res.items():
    print(f"{k:22s} {ms:8.4f} ms  {byt / ms / 1e6:8.1f} GB/s")
