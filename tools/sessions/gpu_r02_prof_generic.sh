# rocprofv3 kernel trace of the generic render + STFT bench (fused kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pg -o run --output-format csv -- python bench.py --workload generic_stft --no-cpu-baseline --steps 5 --warmup 3 > gpurun_out/pg.log 2>&1 || exit $?
KREGEX=dspb_rstft timeout -k 10 600 bash tools/pmc.sh gstft --workload generic_stft --steps 3 --warmup 1 --no-cpu-baseline || exit $?
python tools/pmc_summary.py gpurun_out/pmc_gstft > gpurun_out/pmc_gstft/summary.txt 2>&1; head -40 gpurun_out/pmc_gstft/summary.txt
