#!/bin/bash
# round 3: the pair FIR kernel at 10 min (cfg 3's bench shape: 9375 frames,
# 4.58 waves per wave slot) and at 1 h (56,250 frames, 27.5 per slot),
# alternated twice on one box
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03fir; mkdir -p $o
for r in 1 2; do
for m in 10 60.01; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 50 --warmup 20 --workload fir1024 --minutes $m --no-cpu-baseline > $o/fir_${m}_$r.log 2>&1 || { echo "fir $m rc=$?"; tail -5 $o/fir_${m}_$r.log; exit 1; }
  echo "fir $r $m min $(tail -1 $o/fir_${m}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"], c["settled_step_ms_p50"], c["samples_per_gpu"])')" | tee -a $o/fir.txt
done
done
