"""Host link bandwidth with pinned memory: H2D alone, D2H alone, and both at
once on two streams (the ceiling of the end-to-end pipeline, which moves a
WAV payload up and the render + spectra down).
    python tools/host_link_probe.py [MiB]"""
import sys
import time

import torch

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = mib * (1 << 20) // 4
h_up = torch.empty(n, pin_memory=True)
h_dn = torch.empty(n, pin_memory=True)
d_up = torch.empty(n, device="cuda")
d_dn = torch.rand(n, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def up():
    with torch.cuda.stream(s1):
        d_up.copy_(h_up, non_blocking=True)


def down():
    with torch.cuda.stream(s2):
        h_dn.copy_(d_dn, non_blocking=True)


def both():
    up()
    down()


gb = n * 4 / 1e9
t = timed(up)
print(f"H2D {mib} MiB: {gb / t:6.1f} GB/s")
t = timed(down)
print(f"D2H {mib} MiB: {gb / t:6.1f} GB/s")
t = timed(both)
print(f"H2D + D2H concurrently, {mib} MiB each: {2 * gb / t:6.1f} GB/s total ({gb / t:6.1f} per direction)")
