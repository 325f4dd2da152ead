#!/bin/bash
# round 3, session ac: output buffers' allocation kind vs the headline's time
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r03ac; mkdir -p $o
timeout -k 10 300 python -u tools/alloc_probe.py 3 > $o/alloc_probe.txt 2>&1 || { echo "probe rc=$?"; tail -20 $o/alloc_probe.txt; exit 1; }
grep -v "^W20\|^E20\|amdgpu.ids" $o/alloc_probe.txt
