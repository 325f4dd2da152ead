#!/bin/bash
# round 5, session aa: the IR-level State chain prototype on the GPU
# (tools/diag/ir_chain_proto.py builds the code objects on this box's CPU)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag/ir_chain_proto.py gpurun_out/chain_proto > gpurun_out/chain_proto.log 2>&1 || { echo "proto rc=$?"; tail -20 gpurun_out/chain_proto.log; exit 1; }
cat gpurun_out/chain_proto.log
timeout -k 10 200 python3 tools/diag/ir_chain_gpu_check.py gpurun_out/chain_proto > gpurun_out/chain_check.log 2>&1 || { echo "check rc=$?"; tail -20 gpurun_out/chain_check.log; exit 1; }
cat gpurun_out/chain_check.log
