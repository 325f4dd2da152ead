#!/bin/bash
# round 5, session u: the State chain within the first render -- state-spec
# GPU tests, sine_src (1 min, 1 h: first call and steady state), biquad_src
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05u; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_state_spec.py > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python3 bench.py --workload sine_src > $o/bench_sine_1min.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_sine_1min.log; exit 1; }
grep -h '"metric"' $o/bench_sine_1min.log | cut -c1-200
timeout -k 10 300 python3 bench.py --workload sine_src --minutes 59.99 --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_sine_1h.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_sine_1h.log; exit 1; }
grep -h '"metric"' $o/bench_sine_1h.log | cut -c1-200
timeout -k 10 300 python3 bench.py --workload biquad_src > $o/bench_biquad_src.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_biquad_src.log; exit 1; }
grep -h '"metric"' $o/bench_biquad_src.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --workload sine_src --steps 20 --warmup 5 --no-cpu-baseline > $o/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $o/prof.log; exit 1; }
find $o/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $o/kernel_stats.csv
cut -c1-160 $o/kernel_stats.csv | head -8
echo done
