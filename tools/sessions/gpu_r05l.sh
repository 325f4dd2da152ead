#!/bin/bash
# round 5, session l: SQ counters of the speculative segments' pass 1
# (dspb_seg_c2b512) on biquad.cpp, one counter group per pass
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r05l; mkdir -p $o
i=0
while read -r group; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $group --kernel-include-regex dspb_seg -d $o/pmc_seg/p$i -o run \
    --output-format csv -- python3 bench.py --workload biquad_src --steps 5 --warmup 2 --no-cpu-baseline \
    > $o/pmc_seg_$i.log 2>&1 || { echo "pmc $i rc=$?"; tail -20 $o/pmc_seg_$i.log; exit 1; }
done < tools/pmc_sq.txt
python3 tools/pmc_summary.py $o/pmc_seg --json $o/pmc_seg.json > $o/pmc_seg.txt
cat $o/pmc_seg.txt
echo done
