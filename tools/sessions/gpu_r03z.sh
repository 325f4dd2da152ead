#!/bin/bash
# round 3, session z: the N > 1 bench path rehearsed at world 4 on one GPU
# (gloo for the barrier / max-reduce and as the gather transport), headline
# and cfg 5, with IR_test.cpp compiled unchanged as the plugin
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03z; mkdir -p $o
for wl in headline ch96k; do
    DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 5 --warmup 2 --minutes 5 \
        --no-cpu-baseline --workload $wl > $o/rehearsal4_$wl.txt 2>&1 || { echo "rehearsal $wl rc=$?"; tail -20 $o/rehearsal4_$wl.txt; exit 1; }
    grep '"metric"' $o/rehearsal4_$wl.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); c=l['config']; print('$wl', l['n_gpus'], l['value'], c['block_class'], c['ir_plugin'], c['render_gather_ms'], c['render_gather_error'])"
done
# the pair FIR kernel at 10 min (the cfg 3 bench shape: 9375 frames, 4.58
# waves per wave slot) and at 1 h (56,250 frames, 27.5 per slot)
for m in 10 60.01; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 50 --warmup 20 --workload fir1024 --minutes $m --no-cpu-baseline > $o/fir_$m.log 2>&1 || { echo "fir $m rc=$?"; tail -5 $o/fir_$m.log; exit 1; }
  echo "fir $m min $(tail -1 $o/fir_$m.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"], c["settled_step_ms_p50"])')"
done
