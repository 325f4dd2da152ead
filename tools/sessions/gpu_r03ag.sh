#!/bin/bash
# round 3, session ag: the two-wave 8192-point channel-pair FIR kernel
# (fir_pair2w_kernel): the FIR GPU tests through the product dispatch, then
# interleaved A/B against HEAD's build (build/base: the one-wave pair kernel)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03ag; mkdir -p $o
R=$PWD/dsp-bench_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 400 python tools/ab_lib.py --fir 4 $R/build/base/libdspbench.so $R/libdspbench.so > $o/ab_fir.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_fir.txt; exit 1; }
cat $o/ab_fir.txt
