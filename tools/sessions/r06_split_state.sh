# the split State (envelope beside a block counter): GPU tests and bench lines
set -e
mkdir -p gpurun_out/r06f
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_state_spec.py ${SS_K:+-k "$SS_K"} > gpurun_out/r06f/state_spec.log 2>&1
for w in ${WLS:-envelope_src biquad_src sine_src}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 >> gpurun_out/r06f/bench.jsonl 2> gpurun_out/r06f/bench_$w.err
done
