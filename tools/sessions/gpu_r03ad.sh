#!/bin/bash
# round 3, session ad: the source-plugin headline across channel counts /
# offsets and under channel shards
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03ad; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
