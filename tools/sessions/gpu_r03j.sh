#!/bin/bash
# round 3, session j: the full GPU suite, smoke, the bench (defaults and the
# driver's command) and the driver command's kernel trace
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03j
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.txt 2>&1 \
    || { echo "gpu tests rc=$?"; grep -E "FAIL|Error" $o/gpu_tests.txt | head; tail -5 $o/gpu_tests.txt; exit 1; }
tail -2 $o/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { echo "smoke rc=$?"; cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python bench.py > $o/bench_default.txt 2>&1 || { echo "bench rc=$?"; tail $o/bench_default.txt; exit 1; }
grep '"metric"' $o/bench_default.txt > $o/bench_default.jsonl
for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver_$i.txt 2>&1 || { echo "bench drv rc=$?"; exit 1; }
    grep '"metric"' $o/bench_driver_$i.txt >> $o/bench_driver.jsonl
done
python3 - $o <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_default.jsonl", "bench_driver.jsonl"):
    for line in open(f"{o}/{f}"):
        l = json.loads(line)
        print(f, l["value"], l["ms_per_step"], l["roofline"]["frac"], l["roofline"]["kernel_avg_ms"],
              (l["config"].get("end_to_end") or {}).get("end_to_end_ms"), l["roofline"].get("traffic_over_algorithmic"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $o/prof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
python tools/launch_table.py $o/prof/run_kernel_trace.csv stft8192_pk 5 20 > $o/launch_table.txt
tail -3 $o/launch_table.txt
