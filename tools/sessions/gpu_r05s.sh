#!/bin/bash
# round 5, session s: gain-table rows in registers for B <= 512 -- the
# gain-table GPU tests, the balance / fade_in bench lines and their kernel stats
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05s; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_proof.py > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for p in balance fade_in gain_test; do
  timeout -k 10 300 python3 bench.py --workload generic_stft --plugin $p > $o/bench_$p.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_$p.log; exit 1; }
  grep -h '"metric"' $o/bench_$p.log | cut -c1-260
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --workload generic_stft --plugin fade_in --steps 50 --warmup 20 > $o/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $o/prof.log; exit 1; }
find $o/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $o/kernel_stats.csv
cut -c1-200 $o/kernel_stats.csv | head -5
echo done
