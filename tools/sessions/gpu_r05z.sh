#!/bin/bash
# round 5, session z: warm-up levels capped at 1/16 of the file when a State
# chain can take over -- state-spec GPU tests, sine_src first call (1 min, 1 h)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05z; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_state_spec.py > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python3 bench.py --workload sine_src --no-cpu-baseline > $o/bench_sine_1min.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_sine_1min.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"first_call_ms": [0-9.]*' $o/bench_sine_1min.log
timeout -k 10 300 python3 bench.py --workload sine_src --minutes 59.99 --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_sine_1h.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_sine_1h.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"first_call_ms": [0-9.]*' $o/bench_sine_1h.log
timeout -k 10 300 python3 bench.py --workload biquad_src --no-cpu-baseline > $o/bench_biquad_src.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_biquad_src.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"first_call_ms": [0-9.]*' $o/bench_biquad_src.log
echo done
