#!/bin/bash
# round 5, session f: the whole GPU suite (gain-table class, channel-pair
# biquad tiles), the gain-table plugins' lines, and the biquad A/B: channel
# pairs per wave (packed) at one section (build/ab_pair1) against the
# product's single-channel tiles, alternated; 2 and 4 sections (pairs)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05f; mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for a in "--workload generic_stft --plugin balance" "--workload generic_stft --plugin fade_in" \
         "--workload generic --plugin balance" "--workload generic_stft --plugin balance --no-specialize" \
         "--workload biquad --sections 2" "--workload biquad --sections 4"; do
  timeout -k 10 300 python3 bench.py $a --no-cpu-baseline >> $o/bench.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench.jsonl | cut -c1-250
done
R=$PWD/dsp-bench_amd
for i in 1 2; do
  for lib in $R/libdspbench.so $R/build/ab_pair1/libdspbench.so; do
    DSPBENCH_LIB=$lib timeout -k 10 300 python3 bench.py --workload biquad --no-cpu-baseline >> $o/ab_pair1.jsonl 2>> $o/bench_err.log || { echo "ab rc=$?"; exit 1; }
    echo "$lib $(tail -1 $o/ab_pair1.jsonl | cut -c1-160)"
  done
done
echo done
