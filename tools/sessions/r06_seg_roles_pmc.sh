# SQ counters of the role-split pass 1 (dspb_seg_c2b512) for biquad_src, the
# same groups as round 5's profiles/r05_pmc_state_segments.txt (one group per
# rocprofv3 --pmc pass, short runs); profiles/r06_pmc_seg_roles.{txt,json}
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r06_pmc_roles; mkdir -p $o
i=0
while read -r group; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $group --kernel-include-regex "dspb_seg_c2b512$" -d $o/p$i -o run \
    --output-format csv -- python3 bench.py --workload biquad_src --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
    > $o/pmc_$i.log 2>&1 || { echo "pmc $i rc=$?"; tail -20 $o/pmc_$i.log; exit 1; }
done < tools/pmc_sq.txt
python3 tools/pmc_summary.py $o --json $o/pmc.json > $o/pmc.txt
cat $o/pmc.txt
