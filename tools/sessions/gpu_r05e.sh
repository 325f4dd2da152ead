#!/bin/bash
# round 5, session e: the whole GPU suite after the gain-table class, the
# class-table holds and the driver result plumbing; then the gain-table
# plugins' render + STFT lines
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05e; mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for a in "--workload generic_stft --plugin balance" "--workload generic_stft --plugin fade_in" \
         "--workload generic --plugin balance" "--workload generic_stft --plugin balance --no-specialize"; do
  timeout -k 10 300 python3 bench.py $a --no-cpu-baseline >> $o/bench.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench.jsonl | cut -c1-300
done
echo done
