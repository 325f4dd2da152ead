#!/bin/bash
# round 5, session a: HEAD's roofline evidence under the driver's exact command
# (bench.py --gpus 1 --steps 20 --warmup 5): two bench lines, a rocprofv3
# kernel trace + stats (launch table of the fused kernel), FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes; then counters + clock/power of the two
# input-reading kernels (stft96k = cfg 4, gain_stft)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05a; mkdir -p $o
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
for i in 1 2; do
  timeout -k 10 300 python3 $CMD > $o/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_$i.log; exit 1; }
  grep -h '"metric"' $o/bench_$i.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 $CMD \
  > $o/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $o/prof.log; exit 1; }
grep -h '"metric"' $o/prof.log > $o/prof_bench.jsonl
python3 tools/launch_table.py $o/prof/run_kernel_trace.csv "stft8192_pk_kernel<1, 0, (dspb::MapKind)3" 5 20 > $o/launch_table.txt
tail -4 $o/launch_table.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex stft8192 -d $o/pmc_headline/p_$c -o run \
    --output-format csv -- python3 $CMD > $o/pmc_$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -20 $o/pmc_$c.log; exit 1; }
done
python3 tools/pmc_summary.py $o/pmc_headline --json $o/pmc_headline.json > $o/pmc_headline.txt
grep -A3 "MapKind)3, true, true, 4" $o/pmc_headline.txt | tail -4
# counters of the two input-reading kernels (short runs; one group per pass)
for wl in stft96k gain_stft; do
  i=0
  while read -r group; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $group --kernel-include-regex stft8192 -d $o/pmc_$wl/p$i -o run \
      --output-format csv -- python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline \
      > $o/pmc_${wl}_$i.log 2>&1 || { echo "pmc $wl $i rc=$?"; tail -20 $o/pmc_${wl}_$i.log; exit 1; }
  done < tools/pmc_sq.txt
  python3 tools/pmc_summary.py $o/pmc_$wl --json $o/pmc_$wl.json > $o/pmc_$wl.txt
  timeout -k 10 120 python3 tools/wl_power_probe.py $wl 4 > $o/power_$wl.txt 2>&1 || { echo "power $wl rc=$?"; exit 1; }
  cat $o/power_$wl.txt
done
timeout -k 10 120 python3 tools/wl_power_probe.py headline 4 > $o/power_headline.txt 2>&1 && cat $o/power_headline.txt
echo done
