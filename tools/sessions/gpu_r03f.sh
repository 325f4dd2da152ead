#!/bin/bash
# round 3, session f: the end-to-end pipeline with SDMA downloads (and the
# HIP runtime's blit-kernel downloads, DSPB_NO_SDMA=1, for the A/B)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03f
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py \
    tests/test_gpu_wav.py > $o/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 150 python tools/e2e_probe.py > $o/e2e_sdma.txt 2>&1 || { echo "e2e rc=$?"; tail $o/e2e_sdma.txt; exit 1; }
cat $o/e2e_sdma.txt
DSPB_NO_SDMA=1 timeout -k 10 150 python tools/e2e_probe.py > $o/e2e_blit.txt 2>&1 || { echo "e2e blit rc=$?"; exit 1; }
cat $o/e2e_blit.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/prof_sdma -o run --output-format csv \
    -- python tools/e2e_probe.py > $o/prof_sdma.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python tools/e2e_trace.py $o/prof_sdma | tee $o/trace_sdma.txt
python tools/host_link_probe.py 1024 > $o/host_link.txt 2>&1 && cat $o/host_link.txt
