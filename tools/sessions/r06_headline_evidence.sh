# round 6 at HEAD: the headline's roofline evidence under the driver's command
# (bench.py --gpus 1 --steps 20 --warmup 5): the bench line, a rocprofv3
# kernel trace + stats with the launch table of the fused kernel, HBM
# traffic from FETCH_SIZE and WRITE_SIZE in separate --pmc passes;
# profiles/r06_headline_*
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r06h; mkdir -p $o
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 python3 $CMD > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
grep -h '"metric"' $o/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 $CMD \
  > $o/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $o/prof.log; exit 1; }
grep -h '"metric"' $o/prof.log > $o/prof_bench.jsonl
python3 tools/launch_table.py $o/prof/run_kernel_trace.csv "stft8192_pk_kernel<1, 0, (dspb::MapKind)3" 5 20 > $o/launch_table.txt
tail -4 $o/launch_table.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex stft8192 -d $o/pmc/p_$c -o run \
    --output-format csv -- python3 $CMD > $o/pmc_$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -20 $o/pmc_$c.log; exit 1; }
done
python3 tools/pmc_summary.py $o/pmc --json $o/pmc_headline.json > $o/pmc_headline.txt
grep -A3 "MapKind)3, true, true, 4" $o/pmc_headline.txt | tail -4
