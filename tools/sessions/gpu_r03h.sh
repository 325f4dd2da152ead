#!/bin/bash
# round 3, session h: SDMA engine masks and repeated e2e A/B of the D2H engine
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03h
mkdir -p $o
timeout -k 10 30 ./tools/d2h_probe 16 masks
for rep in 1 2 3; do
    for m in 4 6 8 c 10 pref blit; do
        unset DSPB_SDMA_ENGINES DSPB_NO_SDMA
        case $m in pref) ;; blit) export DSPB_NO_SDMA=1;; *) export DSPB_SDMA_ENGINES=$m;; esac
        timeout -k 10 150 python tools/e2e_probe.py > $o/e2e_${m}_$rep.txt 2>&1 || { echo "e2e $m rc=$?"; tail $o/e2e_${m}_$rep.txt; exit 1; }
        echo "rep $rep engines $m: $(grep 'call 1' $o/e2e_${m}_$rep.txt | cut -c1-60) | $(grep 'call 2' $o/e2e_${m}_$rep.txt | cut -c1-60)"
    done
done
