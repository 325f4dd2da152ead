#!/bin/bash
# round 5, session p: the stateless LDS-blocks driver with the callback on
# every block (gain_test.cpp / IR_test.cpp, --no-specialize), render and
# render + STFT, twice each -- before / after a change of lanes per round
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05p; mkdir -p $o
tag=${1:-run}
for i in 1 2; do
  for a in "--workload generic --plugin gain_test --no-specialize" "--workload generic --plugin IR_test --no-specialize" \
           "--workload generic_stft --plugin IR_test --no-specialize"; do
    timeout -k 10 300 python3 bench.py $a --no-cpu-baseline >> $o/bench_$tag.jsonl 2>> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
    echo "$tag $(tail -1 $o/bench_$tag.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:50], d["ms_per_step"], d["roofline"]["frac"])')"
  done
done
echo done
