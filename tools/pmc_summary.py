"""Summarise rocprofv3 --pmc counter CSVs: per kernel, mean per dispatch, and
per-wave / derived figures (quad-cycle counters -> cycles).
  usage: python tools/pmc_summary.py <pmc dir> [--json out.json]
--json writes {kernel: {counter means..., "hbm_bytes", "fetch_bytes",
"write_bytes"}} with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
FETCH_SIZE (KiB) x 2, WRITE_SIZE (KiB) as is.

Dispatches of one instantiation with different grid sizes (a bench line's
full-size launches beside the end-to-end pass's chunk launches) are separate
entries, keyed "<instantiation> [grid G]"; each entry also records the
dispatch ids it averages (first, last, count)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
summary = {}


def kname(n):
    """The kernel's name with its full template argument list (the
    instantiation), without the parameter list."""
    n = n.strip()
    if n.endswith(")"):
        depth = 0
        for i in range(len(n) - 1, -1, -1):
            depth += n[i] == ")"
            depth -= n[i] == "("
            if depth == 0:
                return n[:i]
    return n

agg = collections.defaultdict(lambda: collections.defaultdict(list))
ids = collections.defaultdict(list)
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        key = f"{kname(r['Kernel_Name'])} [grid {r.get('Grid_Size', '?')}]"
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        ids[key].append(int(r["Dispatch_Id"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    m["dispatch_ids"] = [min(ids[k]), max(ids[k]), len(set(ids[k]))]
    print(k)
    for c, v in sorted(m.items()):
        print(f"   {c:26s} {v:.4g}" if not isinstance(v, list) else f"   {c:26s} {v}")
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
        m.update(hbm_bytes=f + wr, fetch_bytes=f, write_bytes=wr)
    m["dispatches"] = max(len(v) for v in d.values())
    summary[k] = m
if js:
    json.dump({"source": root, "note": "per-dispatch means; FETCH_SIZE x2 (gfx950), WRITE_SIZE exact",
               "kernels": summary}, open(js, "w"), indent=1)
