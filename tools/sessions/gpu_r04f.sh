#!/bin/bash
# round 4, session f: FIR channel pairs as 8192-point frames over two waves,
# decimated in frequency (fir_dif2_kernel, -DDSPB_FIR_DIF2=1 in build/dif2):
# the FIR GPU tests through that build, then the interleaved 10-minute fir1024
# A/B against the one-wave pair kernel (the tree's build)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04f; mkdir -p $o
R=$PWD/dsp-bench_amd
DSPBENCH_LIB=$R/build/dif2/libdspbench.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread > $o/fir_tests.log 2>&1 || { echo "fir tests rc=$?"; tail -40 $o/fir_tests.log; exit 1; }
tail -1 $o/fir_tests.log
timeout -k 10 400 python tools/ab_lib.py --fir 5 $R/libdspbench.so $R/build/dif2/libdspbench.so > $o/ab_fir.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_fir.txt; exit 1; }
cat $o/ab_fir.txt
