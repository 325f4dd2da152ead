#!/bin/bash
# round 4, session a: the whole GPU suite under the driver's own command shape
# (rank harness now FileStore + daemon ranks), smoke(), and the --gpus 2
# launcher rehearsal on one GPU (DSPB_BENCH_REHEARSAL=1: both ranks on cuda:0,
# gloo as the transport)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04a; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
cat $o/smoke.log
DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 3 --minutes 10 > $o/rehearsal2.jsonl 2> $o/rehearsal2.err || { echo "rehearsal rc=$?"; tail -30 $o/rehearsal2.err; exit 1; }
cat $o/rehearsal2.jsonl
