#!/bin/bash
# round 3, session n: SQ counters of the overlap-save FIR kernels (product
# fir_fft_kernel vs the channel-pair kernel, tools build), two passes each
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03n; mkdir -p $o
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for opt in 0 262144; do
  i=0; mkdir -p $o/o$opt
  for g in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "fir_" -d $o/o${opt}/p$i -o run --output-format csv \
      -- python tools/ab_fir_persist.py 1 10 $opt > $o/o${opt}/p$i.log 2>&1 || { echo "opt $opt pass $i rc=$?"; tail -5 $o/o${opt}/p$i.log; exit 1; }
  done
done
echo done
for opt in 0 262144; do echo "== opt $opt"; python3 tools/pmc_summary.py $o/o$opt | grep -E "fir_|per wave|SQ_BUSY|GRBM"; done
