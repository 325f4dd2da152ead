"""Summarise a rocprofv3 trace of tools/e2e_probe.py: per call, the chunk
kernels' durations (stft8192_pk), the blit-kernel copies
(__amd_rocclr_copyBuffer) and the SDMA copies (memory-copy trace).

    python tools/e2e_trace.py <rocprof output dir (…/run_kernel_trace.csv)>
"""
import csv
import os
import statistics
import sys

d = sys.argv[1]
kern = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
mc_path = os.path.join(d, "run_memory_copy_trace.csv")
mc = list(csv.DictReader(open(mc_path))) if os.path.exists(mc_path) else []
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
stft = [r for r in kern if "stft8192_pk" in r["Kernel_Name"]]
blit = [r for r in kern if "copyBuffer" in r["Kernel_Name"]]
print(f"chunk kernels: {len(stft)}, median {statistics.median(map(dur, stft)):.4f} ms, "
      f"max {max(map(dur, stft)):.4f} ms, mean {statistics.mean(map(dur, stft)):.4f} ms")
print(f"blit-kernel copies (copyBuffer): {len(blit)}" +
      (f", mean {statistics.mean(map(dur, blit)):.3f} ms" if blit else ""))
kinds = {}
for r in mc:
    kinds.setdefault(r.get("Direction", r.get("Kind", "?")), []).append(r)
for k, rs in kinds.items():
    b = sum(int(r.get("Bytes", 0) or 0) for r in rs)
    print(f"memory copies {k}: {len(rs)}, {b / 1e9:.2f} GB, mean {statistics.mean(map(dur, rs)):.3f} ms")
# the slowest chunk kernels, for the record
for r in sorted(stft, key=dur)[-3:]:
    print(f"  slowest: {dur(r):.4f} ms")
