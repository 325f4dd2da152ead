#!/bin/bash
# round 4, session e: evidence for the W4 headline kernel -- the driver's
# command three times, the same under rocprofv3 --kernel-trace --stats (launch
# table), the HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the
# headline and of the memory STFT (cfg 4), and the settled bench
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/driver_cmd_profile.sh r04e || { echo "driver profile failed"; exit 1; }
PMC_GROUPS=tools/pmc_hbm.txt bash tools/pmc.sh r04e_headline --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-companion || { echo "pmc failed"; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_r04e_headline --json gpurun_out/pmc_r04e_headline/summary.json > gpurun_out/pmc_r04e_headline/summary.txt
PMC_GROUPS=tools/pmc_hbm.txt bash tools/pmc.sh r04e_stft96k --workload stft96k --steps 3 --warmup 1 --no-cpu-baseline || { echo "pmc failed"; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_r04e_stft96k --json gpurun_out/pmc_r04e_stft96k/summary.json > gpurun_out/pmc_r04e_stft96k/summary.txt
o=gpurun_out/r04e; mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench_settled.jsonl 2> $o/bench_settled.err || { echo "bench rc=$?"; tail -20 $o/bench_settled.err; exit 1; }
cat $o/bench_settled.jsonl | cut -c1-400
