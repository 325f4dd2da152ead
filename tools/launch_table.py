"""Per-launch duration table of one kernel from a rocprofv3 kernel trace.

    python tools/launch_table.py <run_kernel_trace.csv> <kernel substring> <warmup> <timed>

Prints every launch (index, start offset from the first launch, duration, gap
to the previous launch), then the averages over the warmup launches, the
timed launches [warmup, warmup + timed) -- the ones bench.py's step timing
covers -- and the rest (bench.py's per-step distribution pass).
"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    warm, timed = int(sys.argv[3]), int(sys.argv[4])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    t0 = rows[0][0]
    print(f"# {name}: {len(rows)} launches; idx, start_ms (from launch 0), dur_ms, gap_us (to previous end)")
    prev_end = None
    for i, (s, e) in enumerate(rows):
        gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:9.1f}"
        print(f"{i:4d} {(s - t0) / 1e6:10.3f} {(e - s) / 1e6:9.5f} {gap}")
        prev_end = e
    dur = [(e - s) / 1e6 for s, e in rows]

    def avg(a):
        return sum(a) / len(a) if a else float("nan")
    print(f"# warmup launches 0..{warm - 1}: avg {avg(dur[:warm]):.5f} ms")
    print(f"# timed launches {warm}..{warm + timed - 1}: avg {avg(dur[warm:warm + timed]):.5f} ms")
    rest = dur[warm + timed:]
    if rest:
        print(f"# later launches {warm + timed}..{len(dur) - 1}: avg {avg(rest):.5f} ms, "
              f"median {sorted(rest)[len(rest) // 2]:.5f} ms")


if __name__ == "__main__":
    main()
