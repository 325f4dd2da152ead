"""IR-analysis latency: the Python face (allocating its
outputs) vs the bare C call on preallocated device buffers, back to back and
synchronised after every call.

    python tools/ir_latency.py [calls]
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-bench_amd"))
import dspbench as d  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
dev = torch.device("cuda", 0)
plug = d.Plugin.ir_test(0.9, 0.002)
ir = torch.empty((2, 2048), device=dev)
mag = torch.empty((8192,), device=dev)
lib = d.lib()
ps = plug.as_struct()
tab = d._lib.chan_table([ir[0].data_ptr(), ir[1].data_ptr()])
mp = C.cast(C.c_void_p(mag.data_ptr()), d._lib.FP)
ex = d.api._exec(ir)


def bare():
    d._lib.check(lib.dsp_ir_analysis(C.byref(ps), 2, 48000.0, 2048, tab, mp, C.byref(ex)), "dsp_ir_analysis")


def face():
    d.ir_analysis(plug, C_out=2, sr=48000.0, ir_len=2048, device=dev)


for name, fn in (("python face", face), ("bare C call", bare)):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t) / n
    t = time.perf_counter()
    for _ in range(n):
        fn()
        torch.cuda.synchronize()
    ts = (time.perf_counter() - t) / n
    print(f"{name:12s}: back to back {tb * 1e6:7.2f} us/call, synchronised {ts * 1e6:7.2f} us/call", flush=True)

# the one-frame STFT, bare call
for _ in range(200):
    bare()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(n):
    bare()
torch.cuda.synchronize()
print(f"one-frame STFT: back to back {(time.perf_counter() - t) / n * 1e6:7.2f} us/call", flush=True)
