#!/bin/bash
# round 4, session d: the driver's own command (20 steps after 5 warmup: the
# power-cap clock dip) alternated between HEAD~ (build/base) and the W4 build
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r04d; mkdir -p $o
R=$PWD/dsp-bench_amd
timeout -k 10 900 python -u tools/ab_driver.py 4 --pause 8 $R/build/base/libdspbench.so $R/libdspbench.so > $o/ab_driver.txt 2>&1 || { echo "ab rc=$?"; tail -20 $o/ab_driver.txt; exit 1; }
cat $o/ab_driver.txt
