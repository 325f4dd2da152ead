#!/bin/bash
# round 3, session aa: bench.py times any step the library records as one
# launch by the region's stream events (no per-launch events in the timed
# region): every workload at the bench's defaults, then cfg 3's FIR at 10 min
# and 1 h
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03aa; mkdir -p $o
timeout -k 10 1000 bash tools/bench_all.sh > $o/bench_all.txt 2>&1 || { echo "bench_all rc=$?"; tail -20 $o/bench_all.txt; exit 1; }
cp gpurun_out/bench_all.jsonl $o/
cat $o/bench_all.txt
for m in 10 60.01; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 50 --warmup 20 --workload fir1024 --minutes $m --no-cpu-baseline > $o/fir_$m.log 2>&1 || { echo "fir $m rc=$?"; tail -5 $o/fir_$m.log; exit 1; }
  echo "fir $m min $(tail -1 $o/fir_$m.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"], c["settled_step_ms_p50"], c["timed_launches_per_call"])')"
done
