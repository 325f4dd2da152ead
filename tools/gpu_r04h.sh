#!/bin/bash
# round 4, session h: DSP_EXEC_VERIFY_CLASS (tests/test_gpu_proof.py), then
# fir_dif2_kernel with fewer load batches against the pair kernel
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04h; mkdir -p $o
R=$PWD/dsp-bench_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_proof.py tests/test_gpu_specialize.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $o/proof.log 2>&1 || { echo "proof rc=$?"; tail -40 $o/proof.log; exit 1; }
tail -1 $o/proof.log
DSPBENCH_LIB=$R/build/dif2_16_16/libdspbench.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread > $o/fir_tests.log 2>&1 || { echo "fir tests rc=$?"; tail -40 $o/fir_tests.log; exit 1; }
tail -1 $o/fir_tests.log
timeout -k 10 500 python tools/ab_lib.py --fir 4 $R/libdspbench.so $R/build/dif2_16_16/libdspbench.so $R/build/dif2_32_32/libdspbench.so $R/build/dif2_8_8/libdspbench.so > $o/ab_fir.txt 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_fir.txt; exit 1; }
cat $o/ab_fir.txt
# the magnitude rows staged in LDS and stored as aligned non-temporal dwordx4
# (kPkMagStage | kPkNtMag on the PER kernels, build/magst) under the driver's
# command: round 3 measured it settled only (less energy per frame, +0.6% time)
timeout -k 10 900 python -u tools/ab_driver.py 4 --pause 8 $R/libdspbench.so $R/build/magst/libdspbench.so > $o/ab_driver_magst.txt 2>&1 || { echo "ab rc=$?"; tail -20 $o/ab_driver_magst.txt; exit 1; }
tail -2 $o/ab_driver_magst.txt
