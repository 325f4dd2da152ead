#!/bin/bash
# round 5, session v: traffic of the gain-table fused kernel with the gain pairs in
# registers (balance.cpp, B = 512): FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes, plus a kernel
# trace + stats of each command
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05v; mkdir -p $o
run() {  # name, kernel regex, bench args
  local n=$1 re=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_$n -o run --output-format csv -- \
    python3 bench.py "$@" > $o/prof_$n.log 2>&1 || { echo "rocprof $n rc=$?"; tail -20 $o/prof_$n.log; exit 1; }
  grep -h '"metric"' $o/prof_$n.log | cut -c1-200
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$re" -d $o/pmc_$n/p_$c -o run \
      --output-format csv -- python3 bench.py "$@" > $o/pmc_${n}_$c.log 2>&1 || { echo "pmc $n $c rc=$?"; tail -20 $o/pmc_${n}_$c.log; exit 1; }
  done
  python3 tools/pmc_summary.py $o/pmc_$n --json $o/pmc_$n.json > $o/pmc_$n.txt
  cat $o/pmc_$n.txt
}
run generic_stft_gain_table stft8192 --workload generic_stft --plugin balance --steps 20 --warmup 5 --no-cpu-baseline
echo done
