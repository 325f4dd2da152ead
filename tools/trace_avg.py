"""Average kernel duration over the timed launches of a rocprofv3 kernel trace.

bench.py times --steps launches after --warmup ones (then runs up to 50 more
for the per-step distribution); rocprofv3 --stats averages all of them, so the
two agree only over the same launches:

    python tools/trace_avg.py <run_kernel_trace.csv> <kernel substring> [timed_n [skip_n]]

timed_n launches after the first skip_n (default: the last timed_n).
"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else None
    d = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                d.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    d.sort()
    ns = [x[1] for x in d]
    tail = ns[-last:] if skip is None else ns[skip:skip + last]
    which = f"last {len(tail)}" if skip is None else f"launches {skip}..{skip + len(tail) - 1}"
    print(f"{name}: {len(ns)} launches, all-launch avg {sum(ns) / len(ns) / 1e6:.5f} ms, "
          f"{which} (the timed ones) avg {sum(tail) / len(tail) / 1e6:.5f} ms, "
          f"min {min(ns) / 1e6:.5f} ms, max {max(ns) / 1e6:.5f} ms")


if __name__ == "__main__":
    main()
