"""GPU check of tools/diag/ir_chain_proto.py's code objects: both chain
kernels (compiled from source; from the edited IR) run the tremolo's State
chain over the same blocks, and the recorded States are compared bit for bit
with each other and with numpy's float64 restatement of the phase update.
  usage: python tools/diag/ir_chain_gpu_check.py <proto out dir>   (on a GPU box)"""
import ctypes as C
import struct
import sys
import time

import numpy as np
import torch

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/chain_proto"
hip = C.CDLL("libamdhip64.so")
torch.zeros(1, device="cuda")  # context
nblocks, rate, depth, sr = 20_000, 5.0, 0.5, 48000.0
prm = torch.tensor(list(np.frombuffer(struct.pack("ff", rate, depth), np.uint8)), dtype=torch.uint8, device="cuda")
x = torch.rand(2, nblocks * 512, device="cuda")
res = {}
for tag in ("source", "edited"):
    mod, fn = C.c_void_p(), C.c_void_p()
    data = open(f"{out}/tremolo_{tag}.co", "rb").read()
    assert hip.hipModuleLoadData(C.byref(mod), data) == 0
    assert hip.hipModuleGetFunction(C.byref(fn), mod, b"dspb_chain") == 0
    st = torch.zeros(8, dtype=torch.uint8, device="cuda")
    blk = torch.zeros(nblocks * 8, dtype=torch.uint8, device="cuda")
    args = [C.c_void_p(prm.data_ptr()), C.c_void_p(st.data_ptr()), C.c_void_p(blk.data_ptr()),
            C.c_void_p(x[0].data_ptr()), C.c_void_p(x[1].data_ptr()), C.c_uint64(nblocks), C.c_float(sr)]
    ptrs = (C.c_void_p * len(args))(*[C.cast(C.pointer(a), C.c_void_p) for a in args])
    torch.cuda.synchronize()
    t = time.perf_counter()
    assert hip.hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, None, ptrs, None) == 0
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    res[tag] = (blk.cpu().numpy().view(np.float64).copy(), st.cpu().numpy().view(np.float64)[0], ms)
    print(f"{tag}: {ms:.2f} ms for {nblocks} blocks ({ms * 1e3 / nblocks:.2f} us per block)")
two_pi = float(np.float32(6.283185))
step = two_pi * rate / sr
ph, want = 0.0, np.empty(nblocks)
for b in range(nblocks):
    want[b] = ph
    for _ in range(512):
        ph += step
        if ph > two_pi:
            ph -= two_pi
a, b_ = res["source"][0], res["edited"][0]
print("source == edited:", np.array_equal(a.view(np.uint64), b_.view(np.uint64)),
      "edited == numpy:", np.array_equal(b_.view(np.uint64), want.view(np.uint64)),
      "final:", res["edited"][1] == ph)
