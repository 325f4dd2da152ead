#!/bin/bash
# round 3, session y: the spectra's row stride (--mag-ld) under the driver's
# command and settled: 4097 (packed rows, every row at another 4-byte phase
# of the 128-byte line), 4100 (16-byte aligned rows), 4128 (128-byte aligned)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03y; mkdir -p $o
for r in 1 2; do
for ld in 4097 4128 4100; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --mag-ld $ld --no-cpu-baseline --no-e2e > $o/drv_${ld}_$r.log 2>&1 || { echo "drv $ld rc=$?"; tail -5 $o/drv_${ld}_$r.log; exit 1; }
  echo "drv $r $ld $(tail -1 $o/drv_${ld}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], c["settled_step_ms_p50"])')" | tee -a $o/ld.txt
done
done
for r in 1 2; do
for ld in 4097 4128; do
  for wl in headline stft96k gain_stft; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 100 --workload $wl --mag-ld $ld --no-cpu-baseline --no-e2e > $o/set_${wl}_${ld}_$r.log 2>&1 || { echo "set $ld rc=$?"; tail -5 $o/set_${wl}_${ld}_$r.log; exit 1; }
  echo "settled $wl $r $ld $(tail -1 $o/set_${wl}_${ld}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], c["settled_step_ms_p50"])')" | tee -a $o/ld.txt
  done
done
done
