#!/bin/bash
# round 3, session q: the round's closing numbers -- the bench's default line
# (CPU baseline, end to end), the driver's command three times, every workload
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03q; mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/headline.log 2>&1 || { echo "headline rc=$?"; tail -5 $o/headline.log; exit 1; }
tail -1 $o/headline.log > $o/headline.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $o/driver_$i.log 2>&1 || { echo "driver rc=$?"; exit 1; }
  tail -1 $o/driver_$i.log >> $o/driver.jsonl
done
bash tools/bench_all.sh > $o/bench_all.txt 2>&1 || { echo "bench_all rc=$?"; tail -5 $o/bench_all.txt; exit 1; }
cp gpurun_out/bench_all.jsonl $o/bench_all.jsonl
python3 - <<'PY'
import json
for f in ("gpurun_out/r03q/headline.jsonl", "gpurun_out/r03q/driver.jsonl"):
    for line in open(f):
        l = json.loads(line)
        print(f.split("/")[-1], l["value"], l["ms_per_step"], l["roofline"]["frac"], l["config"].get("settled_step_ms_p50"),
              (l.get("cpu_baseline") or {}).get("value"), (l["config"].get("end_to_end") or {}).get("end_to_end_ms"))
PY
cat $o/bench_all.txt | tail -14
