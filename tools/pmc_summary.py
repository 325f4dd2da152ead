"""Summarise rocprofv3 --pmc counter CSVs: per kernel, mean per dispatch, and
per-wave / derived figures (quad-cycle counters -> cycles)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k)
    for c, v in sorted(m.items()):
        print(f"   {c:26s} {v:.4g}")
    w = m.get("SQ_WAVES")
    if w:
        for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in m:
                print(f"   per wave {c:22s} {4 * m[c] / w:10.0f} cycles")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if c in m:
                print(f"   per wave {c:22s} {m[c] / w:10.0f}")
    if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
        f = m.get("FETCH_SIZE", 0) * 1024 * 2  # gfx950: FETCH_SIZE reads 1/2 of streamed bytes
        wr = m.get("WRITE_SIZE", 0) * 1024
        print(f"   HBM bytes (FETCH x2 + WRITE) = {f + wr:.4g}  (fetch {f:.4g}, write {wr:.4g})")
