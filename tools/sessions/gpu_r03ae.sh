#!/bin/bash
# round 3, session ae: the window multiply written as fused with the first
# radix-2 stage (x2dft32 PRE) against HEAD's build (build/base): parity tests,
# then interleaved settled A/B on the headline and the memory STFT
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03ae; mkdir -p $o
R=$PWD/dsp-bench_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_specialize.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 500 python tools/ab_lib.py 4 $R/build/base/libdspbench.so $R/libdspbench.so > $o/ab_headline.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_headline.txt; exit 1; }
cat $o/ab_headline.txt
timeout -k 10 500 python tools/ab_lib.py --mem 4 $R/build/base/libdspbench.so $R/libdspbench.so > $o/ab_mem.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_mem.txt; exit 1; }
cat $o/ab_mem.txt
