#!/bin/bash
# round 4, session c: the stage twiddles whole from a table (DSPB_PK_TWT=1,
# build/twt) -- parity of the headline kernel with that build, then the
# interleaved headline A/B: HEAD~2 (build/base), the W4 window fusion
# (the tree's build), W4 + the twiddle table (build/twt)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04c; mkdir -p $o
R=$PWD/dsp-bench_amd
DSPBENCH_LIB=$R/build/twt/libdspbench.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_specialize.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $o/twt_tests.log 2>&1 || { echo "twt tests rc=$?"; tail -40 $o/twt_tests.log; exit 1; }
tail -1 $o/twt_tests.log
timeout -k 10 600 python tools/ab_lib.py 5 $R/build/base/libdspbench.so $R/libdspbench.so $R/build/twt/libdspbench.so > $o/ab_headline.txt 2>&1 || { echo "ab rc=$?"; tail -20 $o/ab_headline.txt; exit 1; }
cat $o/ab_headline.txt
