# A/B two builds of libdspbench on one workload, one process per run:
#   bash tools/ab_libs_stft.sh ROUNDS WORKLOAD name... (dsp-bench_amd/build/var/<name>/libdspbench.so)
# first: the memory STFT of a seeded hour through each build (sha1 of the spectra), then bench lines
set -o pipefail
R=$1; W=$2; shift 2
for v in "$@"; do
  DSPBENCH_LIB=dsp-bench_amd/build/var/$v/libdspbench.so timeout -k 10 120 python - <<'PY' || exit 1
import hashlib, os, sys, torch
sys.path.insert(0, "dsp-bench_amd")
import dspbench as d
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.rand((2, 96000 * 600), device="cuda", generator=g) * 2 - 1
m = d.stft_magnitude(x)
torch.cuda.synchronize()
print(os.environ["DSPBENCH_LIB"].split("/")[-2], "spectra sha1", hashlib.sha1(m.cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
PY
done
for r in $(seq 1 $R); do
  for v in "$@"; do
    DSPBENCH_LIB=dsp-bench_amd/build/var/$v/libdspbench.so timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline > /tmp/ab_$v.log 2>&1 || exit 1
    tail -1 /tmp/ab_$v.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('round $r $v', l['ms_per_step'], l['roofline']['kernel_avg_ms'], l['roofline']['frac'])"
  done
done
