#!/bin/bash
# round 4, session b: block classes and parallel blocks from the callback's
# IR (csrc/ir_proof.cpp): the new proof tests first, then the whole GPU suite
# and smoke()
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04b; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_proof.py tests/test_gpu_specialize.py -x -v --timeout 120 --timeout-method thread > $o/proof.log 2>&1 || { echo "proof rc=$?"; tail -60 $o/proof.log; exit 1; }
tail -1 $o/proof.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
cat $o/smoke.log
