#!/bin/bash
# round 3, closing check: the GPU suite, smoke and the driver's bench command
# on the final tree
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03af; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d[\"config\"]; print(d[\"value\"], d[\"ms_per_step\"], d[\"roofline\"][\"frac\"], c[\"input_reading_companion\"], c[\"end_to_end\"][\"end_to_end_ms\"], d[\"cpu_baseline\"][\"value\"])"
