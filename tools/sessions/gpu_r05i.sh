#!/bin/bash
# round 5, session i: speculative segments for State-writing plugins -- the
# bit-exactness suite against the serial chain, the stateful module tests,
# then biquad.cpp / sine_test.cpp compiled unchanged through the segments
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05i; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_state_spec.py tests/test_gpu_module.py -x -v --timeout 120 \
  --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for a in "--workload biquad_src" "--workload biquad_src --minutes 1" "--workload sine_src --steps 5 --warmup 2"; do
  timeout -k 10 400 python3 bench.py $a >> $o/bench.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench.jsonl | cut -c1-250
done
echo done
