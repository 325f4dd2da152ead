#!/bin/bash
# round 4, session g: fir_dif2_kernel with its frame and H loads in fewer
# batches (DSPB_DIF2_LB / _HB: 16/16, 32/32 = no batching, 8/8) against the
# one-wave pair kernel (the tree's build), fir1024 10 min
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04g; mkdir -p $o
R=$PWD/dsp-bench_amd
DSPBENCH_LIB=$R/build/dif2_16_16/libdspbench.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread > $o/fir_tests.log 2>&1 || { echo "fir tests rc=$?"; tail -40 $o/fir_tests.log; exit 1; }
tail -1 $o/fir_tests.log
timeout -k 10 500 python tools/ab_lib.py --fir 4 $R/libdspbench.so $R/build/dif2_16_16/libdspbench.so $R/build/dif2_32_32/libdspbench.so $R/build/dif2_8_8/libdspbench.so > $o/ab_fir.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_fir.txt; exit 1; }
cat $o/ab_fir.txt
