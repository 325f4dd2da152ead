#!/bin/bash
# tools/gpu_session.sh -- one gpurun session: GPU tests, smoke, bench, profile.
# Every GPU step has its own time limit; a crash / abort / timeout ends the
# session (no further GPU work), a plain test failure (exit 1) does not.
#   usage: bash tools/gpu_session.sh [tests|bench|prof|all|others|full] [tag]
#   (others: one bench line per non-headline workload; full: all + others)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mode=${1:-all}
tag=${2:-r02}
out=gpurun_out
mkdir -p $out

fatal() {  # exit codes that mean the GPU step crashed or hung
    case $1 in 0|1|5) return 1;; *) return 0;; esac
}

run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "$out/$name.log"
    if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
    return 0
}

[[ $mode == full ]] && mode=all && others=1 || others=0
if [[ $mode == tests || $mode == all ]]; then
    run pytest_gpu 900 python -m pytest tests -m gpu -q -x --timeout=600
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $mode == bench || $mode == all || $mode == prof ]]; then
    run bench 600 python bench.py
fi
if [[ $mode == prof || $mode == all ]]; then
    # the bench's own launch count (100 warmup + 200 timed + 50 for the
    # per-step distribution), so the trace's average over launches 100..299
    # is the number bench.py reports as kernel_avg_ms
    run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run --output-format csv -- python bench.py --no-cpu-baseline
    python tools/trace_avg.py $out/prof_$tag/run_kernel_trace.csv stft8192_pk 200 100 | tee $out/prof_$tag/trace_avg.txt
fi
if [[ $mode == others || $others == 1 ]]; then
    for wl in gain10min stft96k ch96k fir1024 wav16 wav24 ir generic generic_stft gain_stft; do
        run bench_$wl 300 python bench.py --workload $wl --no-cpu-baseline
    done
    run bench_generic_stft_gain 300 python bench.py --workload generic_stft --plugin gain_test --no-cpu-baseline
fi
echo "=== done"
