#!/bin/bash
# round 5, session r: HEAD's bench line at the defaults and under the
# driver's command (--gpus 1 --steps 20 --warmup 5)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05r; mkdir -p $o
timeout -k 10 400 python3 bench.py > $o/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_default.log; exit 1; }
grep -h '"metric"' $o/bench_default.log > $o/bench_default.jsonl
cut -c1-300 $o/bench_default.jsonl
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_driver.log; exit 1; }
grep -h '"metric"' $o/bench_driver.log > $o/bench_driver.jsonl
cut -c1-300 $o/bench_driver.jsonl
echo done
