"""The headline's output buffers (render rows and spectra) allocated three
ways -- hipMalloc (torch's caching allocator), hipExtMallocWithFlags fine
grained (1) and uncached (3) -- and the headline call timed on each:
25 launches (the driver's command: 5 untimed, 20 timed) and then 200 settled
launches, alternating the allocation kinds.  Question: does the write path's
cache policy change the energy per frame (the kernel is held by the 1400 W
package cap)?  Results are checked bit for bit against the
default allocation.

    python tools/alloc_probe.py [rounds]
"""
import ctypes as C
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dsp-bench_amd"))
import dspbench as d  # noqa: E402
from dspbench import shard  # noqa: E402

hip = shard._hip_runtime()
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipFree.argtypes = [C.c_void_p]


class DevBuf:
    """A raw device allocation seen by torch through __cuda_array_interface__."""

    def __init__(self, shape, flags):
        n = 4
        for s in shape:
            n *= s
        p = C.c_void_p()
        st = hip.hipExtMallocWithFlags(C.byref(p), n, flags)
        assert st == 0, f"hipExtMallocWithFlags({flags}) = {st}"
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "<f4", "data": (self.ptr, False),
                                         "version": 3, "strides": None}

    def free(self):
        hip.hipFree(C.c_void_p(self.ptr))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    SR, CH, B = 48000, 2, 512
    L = 60 * 60 * SR
    L -= L % 4096
    dev = torch.device("cuda", 0)
    x = torch.zeros((CH, L), device=dev)
    nb = d.num_blocks(L, B)
    F = d.stft_frames(nb * B, 8192, 4096)
    plug = d.Plugin.ir_test(0.9, 0.002)
    kinds = {"hipMalloc": None, "finegrained": 1, "uncached": 3}
    bufs = {}
    for k, fl in kinds.items():
        if fl is None:
            bufs[k] = (torch.empty((CH, nb * B), device=dev), torch.empty((CH, F, 4097), device=dev), None)
        else:
            o, m = DevBuf((CH, nb * B), fl), DevBuf((CH, F, 4097), fl)
            bufs[k] = (torch.as_tensor(o, device=dev), torch.as_tensor(m, device=dev), (o, m))
    s = torch.cuda.current_stream()

    def run(k, n):
        out, mag, _ = bufs[k]
        for _ in range(n):
            d.render_stft(x, CH, B, float(SR), plug, out=out, mag=mag)

    # parity: every kind writes the same bits
    for k in kinds:
        run(k, 1)
    torch.cuda.synchronize()
    ref_o, ref_m, _ = bufs["hipMalloc"]
    for k in kinds:
        o, m, _ = bufs[k]
        assert torch.equal(o, ref_o) and torch.equal(m, ref_m), k
    print("parity: identical outputs for every allocation kind", flush=True)
    for r in range(rounds):
        for k in kinds:
            torch.cuda.synchronize()
            time.sleep(1.0)  # an idle second: each kind starts from a similar clock state
            run(k, 5)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            run(k, 20)
            e1.record(s)
            torch.cuda.synchronize()
            drv = e0.elapsed_time(e1) / 20
            run(k, 100)
            e0.record(s)
            run(k, 200)
            e1.record(s)
            torch.cuda.synchronize()
            settled = e0.elapsed_time(e1) / 200
            print(f"round {r} {k:12s} driver-shape {drv:.4f} ms  settled {settled:.4f} ms", flush=True)
    for k in kinds:
        if bufs[k][2]:
            for b in bufs[k][2]:
                b.free()


if __name__ == "__main__":
    main()
