#!/bin/bash
# round 4, session h: DSP_EXEC_VERIFY_CLASS (tests/test_gpu_proof.py, incl.
# the in-place case) with the specialize / graph suites and the FIR suite on
# the tree's build, then the magnitude-staging variant under the driver's command
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04h; mkdir -p $o
R=$PWD/dsp-bench_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_proof.py tests/test_gpu_specialize.py tests/test_gpu_graph.py tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread > $o/proof.log 2>&1 || { echo "proof rc=$?"; tail -40 $o/proof.log; exit 1; }
tail -1 $o/proof.log
# the magnitude rows staged in LDS and stored as aligned non-temporal dwordx4
# (kPkMagStage | kPkNtMag on the PER kernels, build/magst) under the driver's
# command: round 3 measured it settled only (less energy per frame, +0.6% time)
if [ -f $R/build/magst/libdspbench.so ]; then
  timeout -k 10 900 python -u tools/ab_driver.py 4 --pause 8 $R/libdspbench.so $R/build/magst/libdspbench.so > $o/ab_driver_magst.txt 2>&1 || { echo "ab rc=$?"; tail -20 $o/ab_driver_magst.txt; exit 1; }
  tail -2 $o/ab_driver_magst.txt
fi
