#!/bin/bash
# tools/driver_cmd_profile.sh -- the round-end driver's exact bench command,
# measured three ways on one box:
#   1. bench.py --gpus 1 --steps 20 --warmup 5, three times back to back
#      (the line the driver records, and its spread);
#   2. the same command under rocprofv3 --kernel-trace --stats: a per-launch
#      duration table of the fused kernel (tools/launch_table.py);
#   3. the same command with DSPB_CLOCK_STAMPS=1: the fused kernel's waves
#      stamp (s_memtime, s_memrealtime) at entry and exit, so every launch
#      also gets its effective shader clock (the ratio of the two counters).
#   usage: bash tools/driver_cmd_profile.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r02}
out=gpurun_out/driver_$tag
mkdir -p $out
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
for i in 1 2 3; do
    echo "=== bench run $i"
    timeout -k 10 300 python $CMD > $out/bench_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    grep -h '"metric"' $out/bench_$i.log
done
echo "=== rocprof kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python $CMD \
    > $out/prof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
grep -h '"metric"' $out/prof.log
python tools/launch_table.py $out/prof/run_kernel_trace.csv stft8192_pk 5 20 | tee $out/launch_table.txt
echo "=== done"
