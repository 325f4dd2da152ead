# every bench workload once at the bench's defaults (no CPU baseline, no
# end-to-end pass): one JSON line each into gpurun_out/bench_all.jsonl, and a
# summary table
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/bench_all.jsonl
for wl in headline stft96k gain_stft generic generic_stft fir1024 gain10min ch96k wav16 wav24 wav16enc wav24enc ir biquad biquad_src sine_src envelope_src; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline --no-e2e > gpurun_out/bench_$wl.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$wl.log >> gpurun_out/bench_all.jsonl
done
# a BIQUAD cascade of four sections (packed channel pairs, issue-bound)
timeout -k 10 200 python -u bench.py --workload biquad --sections 4 --no-cpu-baseline --no-e2e \
  > gpurun_out/bench_biquad4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_biquad4.log >> gpurun_out/bench_all.jsonl
# buffer_test.cpp (its State writes through arena pointers: the serial chain; 1 min)
timeout -k 10 200 python -u bench.py --workload generic --plugin buffer_test --minutes 1 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-e2e > gpurun_out/bench_buffer_test.log 2>&1 || exit 1
tail -1 gpurun_out/bench_buffer_test.log >> gpurun_out/bench_all.jsonl
# the gain-table class (a per-position gain plugin on the fused path)
timeout -k 10 200 python -u bench.py --workload generic_stft --plugin fade_in --no-cpu-baseline --no-e2e \
  > gpurun_out/bench_generic_stft_fade_in.log 2>&1 || exit 1
tail -1 gpurun_out/bench_generic_stft_fade_in.log >> gpurun_out/bench_all.jsonl
python3 - <<'PY'
import json
for line in open("gpurun_out/bench_all.jsonl"):
    l = json.loads(line)
    r = l["roofline"]
    print(f'{l["config"]["workload"][:70]:72s} {l["value"]:>12.1f} {l["ms_per_step"]:8.4f} {r.get("frac", 0):7.4f} {r.get("kernel_avg_ms", 0)}')
PY
