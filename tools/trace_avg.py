"""Average kernel duration over the timed launches of a rocprofv3 kernel trace.

bench.py times its last --steps launches; rocprofv3 --stats averages all of
them, warmup included, so the two agree only over the same launches:

    python tools/trace_avg.py <run_kernel_trace.csv> <kernel substring> [last_n]
"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    d = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                d.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    d.sort()
    ns = [x[1] for x in d]
    tail = ns[-last:]
    print(f"{name}: {len(ns)} launches, all-launch avg {sum(ns) / len(ns) / 1e6:.5f} ms, "
          f"last {len(tail)} avg {sum(tail) / len(tail) / 1e6:.5f} ms, "
          f"min {min(ns) / 1e6:.5f} ms, max {max(ns) / 1e6:.5f} ms")


if __name__ == "__main__":
    main()
