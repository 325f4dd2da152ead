"""Which pinned host allocations make a D2H hipMemcpyAsync run on SDMA, and
which make CLR use a blit kernel (__amd_rocclr_copyBuffer, on the CUs).

    rocprofv3 --kernel-trace --memory-copy-trace --stats -d DIR -- python tools/pinned_kind_probe.py

Each case copies 64 MiB device -> host with hipMemcpyAsync on its own
non-blocking stream, in the order printed; the trace tells which engine ran
each copy (a copyBuffer kernel, or a MEMORY_COPY_DEVICE_TO_HOST record).
"""
import ctypes as C
import os
import time

import torch

torch.cuda.init()
# the runtime torch already loaded (by soname), not a second copy from /opt/rocm
hip = C.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostGetFlags.argtypes = [C.POINTER(C.c_uint), C.c_void_p]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]

for line in open("/proc/self/maps"):  # which HIP runtime(s) this process has mapped
    if "libamdhip64" in line and "r-xp" in line:
        print("mapped:", line.split()[-1], flush=True)

NB = 64 << 20
src = torch.rand(NB // 4, device="cuda")
torch.cuda.synchronize()
st = C.c_void_p()
assert hip.hipStreamCreateWithFlags(C.byref(st), 1) == 0


def copy(label, ptr, keep=None):
    flags = C.c_uint(0)
    r = hip.hipHostGetFlags(C.byref(flags), C.c_void_p(ptr))
    t0 = time.perf_counter()
    for _ in range(3):
        assert hip.hipMemcpyAsync(C.c_void_p(ptr), C.c_void_p(src.data_ptr()), NB, 2, st) == 0
    assert hip.hipStreamSynchronize(st) == 0
    dt = (time.perf_counter() - t0) / 3
    print(f"{label:40s} hipHostGetFlags rc={r} flags=0x{flags.value:x}  {NB / dt / 1e9:6.1f} GB/s", flush=True)
    time.sleep(0.05)  # a gap in the trace between cases


t = torch.empty(NB // 4, pin_memory=True)
copy("torch pin_memory=True", t.data_ptr())
for name, fl in [("hipHostMallocDefault", 0), ("hipHostMallocPortable", 1), ("hipHostMallocMapped", 2),
                 ("hipHostMallocWriteCombined", 4), ("hipHostMallocCoherent", 0x40000000),
                 ("hipHostMallocNonCoherent", 0x80000000)]:
    p = C.c_void_p()
    rc = hip.hipHostMalloc(C.byref(p), NB, fl)
    if rc:
        print(f"{name}: hipHostMalloc rc={rc}")
        continue
    copy(name, p.value)
buf = (C.c_char * (NB + 4096))()
base = (C.addressof(buf) + 4095) // 4096 * 4096
rc = hip.hipHostRegister(C.c_void_p(base), NB, 0)
print(f"hipHostRegister rc={rc}")
if rc == 0:
    copy("malloc + hipHostRegister", base)
