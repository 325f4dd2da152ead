#!/bin/bash
# round 5, session g: the gain-table row staged in LDS in the fused kernel,
# the IR prover's numbered-type fix (proof/specialize/biquad suites), and the
# gain-table plugins' fused lines
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05g; mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_proof.py tests/test_gpu_specialize.py tests/test_gpu_biquad.py -x -q --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for a in "--workload generic_stft --plugin balance" "--workload generic_stft --plugin fade_in" \
         "--workload gain_stft"; do
  timeout -k 10 300 python3 bench.py $a --no-cpu-baseline >> $o/bench.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench.jsonl | cut -c1-250
done
echo done
