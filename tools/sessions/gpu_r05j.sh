#!/bin/bash
# round 5, session j: the whole GPU suite and smoke() after the speculative
# segments for State-writing plugins
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05j; mkdir -p $o
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -3 $o/smoke.log
echo done
