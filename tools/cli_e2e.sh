#!/bin/bash
# tools/cli_e2e.sh -- end-to-end offline render through the C++ CLI: a
# synthetic 16-bit stereo WAV of M minutes -> dspbench_render (parse, H2D,
# GPU decode, IR_test render + STFT, GPU encode, D2H, write).
#   usage: bash tools/cli_e2e.sh [minutes]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
m=${1:-10}
d=$(mktemp -d)
python - "$d/in.wav" "$m" <<'PY'
import struct, sys
import numpy as np
path, minutes = sys.argv[1], float(sys.argv[2])
L = int(minutes * 60 * 48000)
raw = np.random.default_rng(1).integers(-32768, 32768, size=2 * L, dtype=np.int64).astype("<i2").tobytes()
fmt = struct.pack("<HHIIHH", 1, 2, 48000, 48000 * 4, 4, 16)
body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(raw)) + raw
open(path, "wb").write(b"RIFF" + struct.pack("<I", len(body)) + body)
PY
ls -la "$d/in.wav"
for p in gain_test IR_test; do
    ./dsp-bench_amd/dspbench_render "$d/in.wav" "$d/out.wav" --plugin $p
    ./dsp-bench_amd/dspbench_render "$d/in.wav" "$d/out.wav" --plugin $p --stft "$d/mag.f32"
done
rm -rf "$d"
