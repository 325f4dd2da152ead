#!/bin/bash
# round 3, session i: block classes of stateless plugins (tests + generic bench lines)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03i
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_specialize.py \
    tests/test_gpu_module.py tests/test_gpu_fuzz.py tests/test_gpu_graph.py > $o/tests.txt 2>&1 \
    || { echo "tests rc=$?"; grep -E "FAIL|Error|assert" $o/tests.txt | head -30; tail -5 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
for args in "--workload generic_stft" "--workload generic_stft --no-specialize" "--workload generic" \
            "--workload generic --no-specialize" "--workload generic_stft --plugin gain_test"; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 20 --no-cpu-baseline $args > $o/b.txt 2>&1 \
        || { echo "bench $args rc=$?"; tail -5 $o/b.txt; exit 1; }
    grep '"metric"' $o/b.txt >> $o/bench.jsonl
    grep '"metric"' $o/b.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$args', l['ms_per_step'], r['kernel_avg_ms'], r['frac'], l['config']['block_class'])"
done
