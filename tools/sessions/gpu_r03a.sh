#!/bin/bash
# round 3, session a: copy-engine probe (which engine moves the pipeline's
# host copies) and the HBM PMC of the HEAD kernels under the driver's command.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03a
mkdir -p $o
step() {  # step <name> <timeout> <cmd...>: stop the session on any failure
    local name=$1 t=$2; shift 2
    echo "=== $name"
    timeout -k 10 "$t" "$@" > "$o/$name.txt" 2>&1
    local rc=$?
    tail -n 12 "$o/$name.txt"
    if [[ $rc -ne 0 ]]; then echo "FATAL: $name rc=$rc"; exit $rc; fi
}
step copy_default 150 python tools/copy_engine_probe.py 256
step copy_prof 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/prof_copy -o run --output-format csv \
    -- python tools/copy_engine_probe.py 256
step copy_sdma1 150 env HSA_ENABLE_SDMA=1 python tools/copy_engine_probe.py 256
step copy_limitwg 150 env DEBUG_CLR_LIMIT_BLIT_WG=4 python tools/copy_engine_probe.py 256
step copy_blit3 150 env GPU_BLIT_ENGINE_TYPE=3 python tools/copy_engine_probe.py 256
step copy_blit2 150 env GPU_BLIT_ENGINE_TYPE=2 python tools/copy_engine_probe.py 256
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e"
for wl in headline gain_stft stft96k; do
    for c in FETCH_SIZE WRITE_SIZE; do
        step pmc_${wl}_$c 200 rocprofv3 --pmc $c --kernel-include-regex stft8192 -d $o/pmc_${wl}_$c -o run \
            --output-format csv -- python $CMD --workload $wl
    done
done
echo "=== session done"
