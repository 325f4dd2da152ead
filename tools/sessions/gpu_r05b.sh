#!/bin/bash
# round 5, session b: DSP_PLUGIN_BIQUAD's first GPU run -- its tests, then the
# stateful bench lines (the kind at 1 and 2 sections, biquad.cpp and
# sine_test.cpp compiled unchanged on the serial chain)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05b; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_biquad.py -x -v --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for a in "--workload biquad" "--workload biquad --sections 2" "--workload biquad_src --steps 5 --warmup 2" \
         "--workload sine_src --steps 5 --warmup 2"; do
  timeout -k 10 300 python3 bench.py $a >> $o/bench.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench.jsonl | cut -c1-400
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --workload biquad --steps 20 --warmup 5 --no-cpu-baseline > $o/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $o/prof.log; exit 1; }
head -4 $o/prof/run_kernel_stats.csv | cut -c1-200
echo done
