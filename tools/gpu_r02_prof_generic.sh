set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pg -o run --output-format csv -- python bench.py --workload generic_stft --no-cpu-baseline --steps 5 --warmup 3 > gpurun_out/pg.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pr -o run --output-format csv -- python bench.py --workload generic --no-cpu-baseline --steps 5 --warmup 3 > gpurun_out/pr.log 2>&1 || exit $?
find gpurun_out/pg gpurun_out/pr -name "*.csv" | head
