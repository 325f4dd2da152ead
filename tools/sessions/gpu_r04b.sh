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
# static_gain_plugin.cpp compiled unchanged (a State its callback only reads):
# 1 h stereo through the generic dispatch, its proven block class
timeout -k 10 300 python bench.py --workload generic --plugin static_gain_plugin --steps 100 --warmup 50 > $o/bench_static_gain.jsonl 2> $o/bench_static_gain.err || { echo "bench rc=$?"; tail -20 $o/bench_static_gain.err; exit 1; }
cat $o/bench_static_gain.jsonl
# headline A/B: HEAD's build (build/base) against the working tree's
timeout -k 10 400 python tools/ab_lib.py 4 dsp-bench_amd/build/base/libdspbench.so dsp-bench_amd/libdspbench.so > $o/ab_headline.txt 2>&1 || { echo "ab rc=$?"; tail -20 $o/ab_headline.txt; exit 1; }
cat $o/ab_headline.txt
