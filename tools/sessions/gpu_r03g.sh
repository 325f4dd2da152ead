#!/bin/bash
# round 3, session g: SDMA engine choice for the end-to-end downloads
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03g
mkdir -p $o
for m in pref 1 2 4 6 f; do
    if [[ $m == pref ]]; then unset DSPB_SDMA_ENGINES; else export DSPB_SDMA_ENGINES=$m; fi
    timeout -k 10 150 python tools/e2e_probe.py > $o/e2e_$m.txt 2>&1 || { echo "e2e $m rc=$?"; tail $o/e2e_$m.txt; exit 1; }
    echo "engines $m: $(grep 'call 2' $o/e2e_$m.txt)"
done
unset DSPB_SDMA_ENGINES
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_sdma -o run --output-format csv \
    -- python tools/e2e_probe.py > $o/prof_sdma.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python tools/e2e_trace.py $o/prof_sdma | tee $o/trace_sdma.txt
DSPB_NO_SDMA=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_blit -o run --output-format csv \
    -- python tools/e2e_probe.py > $o/prof_blit.log 2>&1 || { echo "prof blit rc=$?"; exit 1; }
python tools/e2e_trace.py $o/prof_blit | tee $o/trace_blit.txt
