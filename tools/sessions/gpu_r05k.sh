#!/bin/bash
# round 5, session k: kernel trace of biquad.cpp through the speculative
# segments (pass 1, checks, reruns, walk per launch)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05k; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- \
  python3 bench.py --workload biquad_src --steps 20 --warmup 5 --no-cpu-baseline > $o/prof.log 2>&1 \
  || { echo "rocprof rc=$?"; tail -20 $o/prof.log; exit 1; }
grep -h '"metric"' $o/prof.log | cut -c1-200
head -12 $o/prof/run_kernel_stats.csv | cut -c1-220
echo done
