#!/bin/bash
# round 3, session v: the headline through IR_test.cpp compiled unchanged
# (bench.py --ir-plugin source, now the default) against the enum
# restatement: parity test, the driver's command alternated, the N = 2
# rehearsal (gather) for headline and ch96k, and a kernel trace of the
# source headline (same instantiation as the enum one)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03v; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_specialize.py -x -q --timeout 120 --timeout-method thread > $o/spec_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/spec_tests.log; exit 1; }
tail -1 $o/spec_tests.log
for r in 1 2; do
for v in source enum; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --ir-plugin $v --no-cpu-baseline > $o/drv_${v}_$r.log 2>&1 || { echo "drv $v rc=$?"; tail -5 $o/drv_${v}_$r.log; exit 1; }
  echo "$r $v $(tail -1 $o/drv_${v}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], c["settled_step_ms_p50"], c["first_call_ms"], c["block_class"], c["end_to_end"]["end_to_end_ms"])')" | tee -a $o/drv.txt
done
done
for wl in headline ch96k; do
    DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --minutes 5 \
        --no-cpu-baseline --workload $wl > $o/rehearsal_$wl.txt 2>&1 || { echo "rehearsal $wl rc=$?"; tail -20 $o/rehearsal_$wl.txt; exit 1; }
    grep '"metric"' $o/rehearsal_$wl.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$wl', l['value'], l['config']['block_class'], l['config']['render_gather_ms'], l['config']['render_gather_error'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $o/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $o/prof.log; exit 1; }
head -4 $o/prof/run_kernel_stats.csv | cut -c1-300
