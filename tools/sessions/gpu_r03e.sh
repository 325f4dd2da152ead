#!/bin/bash
# round 3, session e: the pinned-memory kind probe (which D2H copies run on
# SDMA) and the N > 1 bench path rehearsed on one GPU (gather on by default)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03e
mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/prof -o run --output-format csv \
    -- python tools/pinned_kind_probe.py > $o/probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
grep -v "^W2026\|^E2026" $o/probe.txt
for wl in headline ch96k; do
    DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --minutes 5 \
        --no-cpu-baseline --workload $wl > $o/rehearsal_$wl.txt 2>&1 || { echo "rehearsal $wl rc=$?"; tail -20 $o/rehearsal_$wl.txt; exit 1; }
    grep '"metric"' $o/rehearsal_$wl.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$wl', l['value'], l['config']['render_gather_ms'], l['config']['render_gather'])"
done
