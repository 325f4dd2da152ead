#!/bin/bash
# round 5, session d: the N = 8 path rehearsed on one GPU (8 ranks on cuda:0,
# gloo as the gather's transport) for the headline and cfg 5's ch96k; BIQUAD
# with the chain mode split off; the class-cache and proof suites
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05d; mkdir -p $o
( while sleep 30; do echo "tick $(date +%T)"; done ) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_biquad.py tests/test_gpu_proof.py -x -q --timeout 120 \
  --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for a in "--workload biquad" "--workload biquad --sections 2 --no-cpu-baseline" "--workload biquad --sections 4 --no-cpu-baseline"; do
  timeout -k 10 300 python3 bench.py $a >> $o/bench_biquad.jsonl 2> $o/bench_err.log || { echo "bench '$a' rc=$?"; tail -20 $o/bench_err.log; exit 1; }
  tail -1 $o/bench_biquad.jsonl | cut -c1-300
done
for wl in headline ch96k; do
  DSPB_BENCH_REHEARSAL=1 timeout -k 10 900 python3 bench.py --gpus 8 --workload $wl --steps 20 --warmup 5 \
    --gather-timeout 600 > $o/rehearsal_$wl.jsonl 2> $o/rehearsal_$wl.err || { echo "rehearsal $wl rc=$?"; tail -30 $o/rehearsal_$wl.err; exit 1; }
  cut -c1-300 $o/rehearsal_$wl.jsonl
done
echo done
