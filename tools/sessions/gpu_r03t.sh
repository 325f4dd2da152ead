#!/bin/bash
# round 3, session t: persistent headline kernel A/B (build/persist1: computed
# window, build/persist2: window table in LDS) -- parity against the product,
# interleaved settled A/B, and the driver's command per library
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03t; mkdir -p $o
R=$PWD/dsp-bench_amd
for v in prod persist1 persist2; do
  lib=$R/libdspbench.so; [[ $v != prod ]] && lib=$R/build/$v/libdspbench.so
  DSPBENCH_LIB=$lib timeout -k 10 120 python tools/persist_check.py /tmp/chk_$v > $o/chk_$v.log 2>&1 || { echo "check $v failed"; tail -5 $o/chk_$v.log; exit 1; }
done
python tools/persist_cmp.py /tmp/chk_prod /tmp/chk_persist1 /tmp/chk_persist2 | tee $o/cmp.txt
timeout -k 10 600 python tools/ab_lib.py 3 $R/libdspbench.so $R/build/persist1/libdspbench.so $R/build/persist2/libdspbench.so 2>&1 | tee $o/ab_settled.txt || exit 1
for r in 1 2; do
for v in prod persist1 persist2; do
  lib=$R/libdspbench.so; [[ $v != prod ]] && lib=$R/build/$v/libdspbench.so
  DSPBENCH_LIB=$lib timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $o/drv_$v.log 2>&1 || { echo "drv $v failed"; tail -5 $o/drv_$v.log; exit 1; }
  echo "$r $v $(tail -1 $o/drv_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"], d["config"]["settled_step_ms_p50"])')" | tee -a $o/drv.txt
done
done
