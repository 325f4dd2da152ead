#!/bin/bash
# round 3, session u (re-entry): the GPU suite and the driver's command at HEAD
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03u; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $o/gpu_tests.log; exit 1; }
tail -3 $o/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log | cut -c1-400
