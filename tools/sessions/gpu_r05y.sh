#!/bin/bash
# round 5, session y: SQ counters of the State chain kernel (sine_test.cpp,
# 1 min of stereo): is the one lane issue-bound on its dependent float64 chain?
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
PMC_GROUPS=tools/pmc_sq.txt KREGEX=dspb_seg_chain timeout -k 10 400 bash tools/pmc.sh sine_chain \
  --workload sine_src --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/pmc_sine_chain.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/pmc_sine_chain.log; exit 1; }
tail -8 gpurun_out/pmc_sine_chain.log
python3 tools/pmc_summary.py gpurun_out/pmc_sine_chain --json gpurun_out/pmc_sine_chain.json > gpurun_out/pmc_sine_chain.txt
cat gpurun_out/pmc_sine_chain.txt
echo done
