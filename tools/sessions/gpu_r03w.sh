#!/bin/bash
# round 3, session w: table-class blocks in a verified closed form
# (module.cpp affine_ramp): the specialization tests, then the driver's
# command alternated between IR_test.cpp (source) and the enum restatement
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03w; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_module.py -x -q --timeout 120 --timeout-method thread > $o/spec_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/spec_tests.log; exit 1; }
tail -1 $o/spec_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for r in 1 2 3; do
for v in source enum; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --ir-plugin $v --no-cpu-baseline --no-e2e > $o/drv_${v}_$r.log 2>&1 || { echo "drv $v rc=$?"; tail -5 $o/drv_${v}_$r.log; exit 1; }
  echo "$r $v $(tail -1 $o/drv_${v}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], c["settled_step_ms_p50"], c["first_call_ms"], c["block_class"])')" | tee -a $o/drv.txt
done
done
