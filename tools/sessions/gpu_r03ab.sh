#!/bin/bash
# round 3, session ab: the GPU suite with the random-Parameters IR_test.cpp tests
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03ab; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
