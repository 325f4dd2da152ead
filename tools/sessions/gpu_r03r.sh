#!/bin/bash
# round 3, session r: rocprofv3 kernel-trace summaries of the closing state --
# the headline under the driver's command and fir1024 (the pair kernel)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03r; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/driver -o run --output-format csv \
  -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $o/driver.log 2>&1 || { echo "driver rc=$?"; tail -5 $o/driver.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/fir -o run --output-format csv \
  -- python bench.py --workload fir1024 --no-cpu-baseline > $o/fir.log 2>&1 || { echo "fir rc=$?"; tail -5 $o/fir.log; exit 1; }
for d in driver fir; do
  echo "== $d"; tail -1 $o/$d.log | cut -c1-200
  f=$(ls $o/$d/run_kernel_stats.csv 2>/dev/null || find $o/$d -name '*kernel_stats.csv' | head -1)
  head -4 "$f" | cut -c1-220
done
python3 tools/trace_avg.py $(find $o/driver -name '*kernel_trace.csv' | head -1) stft8192_pk 20 5 | tee $o/driver_trace_avg.txt
