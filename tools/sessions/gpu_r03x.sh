#!/bin/bash
# round 3, session x: closing evidence with IR_test.cpp compiled unchanged as
# the headline plugin -- the GPU suite, smoke, the driver's command three
# times, its rocprofv3 kernel trace (launch table), and the HBM PMC of the
# headline kernel under that command
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03x; mkdir -p $o
step() {  # step <name> <timeout> <cmd...>: stop the session on any failure
    local name=$1 t=$2; shift 2
    echo "=== $name"
    timeout -k 10 "$t" "$@" > "$o/$name.txt" 2>&1
    local rc=$?
    tail -n 3 "$o/$name.txt" | cut -c1-300
    if [[ $rc -ne 0 ]]; then echo "FATAL: $name rc=$rc"; exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step bench_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5; done
step prof 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5
python tools/launch_table.py $o/prof/run_kernel_trace.csv stft8192_pk 5 20 > $o/launch_table.txt 2>&1 || true
tail -3 $o/launch_table.txt
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e"
for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_headline_$c 200 rocprofv3 --pmc $c --kernel-include-regex stft8192 -d $o/pmc_headline/p_$c -o run \
        --output-format csv -- python $CMD
done
echo "=== session done"
