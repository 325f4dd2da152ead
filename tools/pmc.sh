#!/bin/bash
# tools/pmc.sh -- PMC counter passes (one rocprofv3 run per counter group,
# --pmc never combined with sys/runtime traces).
#   usage: [PMC_GROUPS=file] pmc.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
args=${*:---steps 3 --warmup 1 --no-cpu-baseline}
out=gpurun_out/pmc_$tag
mkdir -p $out
DEFAULT_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
"
if [[ -n "${PMC_GROUPS:-}" ]]; then group_text=$(cat "$PMC_GROUPS"); else group_text=$DEFAULT_GROUPS; fi
i=0
while read -r group; do
    [[ -z "$group" || "$group" == \#* ]] && continue
    i=$((i+1))
    echo "=== pass $i: $group"
    timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "${KREGEX:-stft8192|render_vec}" \
        -d $out/p$i -o run --output-format csv -- python bench.py $args > $out/p$i.log 2>&1
    rc=$?
    echo "rc=$rc"; grep -h '"metric"' $out/p$i.log | cut -c1-120
    case $rc in 0|1) ;; *) echo "FATAL: stopping"; exit $rc;; esac
done <<< "$group_text"
echo "=== pmc done"
