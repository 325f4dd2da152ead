# kernel traces of the stateful bench lines (biquad_src, envelope_src) at
# the role-split pass 1: per-kernel time (rocprofv3 --kernel-trace --stats);
# profiles/r06_seg_roles_kernel_stats_*.csv
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in biquad_src envelope_src; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- \
    python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/prof_$wl.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_$wl -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kernel_stats_$wl.csv
  head -8 gpurun_out/kernel_stats_$wl.csv | cut -c1-200
done
