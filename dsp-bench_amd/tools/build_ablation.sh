#!/bin/bash
# Build the phase-ablation set of the stamped SoA kernel (tools/stamps.hip):
# build/stamps_ab<mask> skips the phases in <mask> (stft_soa.hip kAb*).
#   usage: bash tools/build_ablation.sh [STAMP_OPT]
set -e
cd "$(dirname "$0")/.."
opt=${1:-0}
for ab in 0 1 2 4 8 16 32 64 127; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DDSPB_STAMPS \
        -DDSPB_ABLATE=$ab -DSTAMP_OPT=$opt -I../include -Icsrc tools/stamps.hip -o build/stamps_ab$ab &
done
wait
