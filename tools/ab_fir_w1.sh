# FIR overlap-save, four-wave workgroups with H in LDS (method 2) vs one-wave
# workgroups with H from L2 (method 3): bit-identity, then alternated bench runs
mkdir -p gpurun_out
rm -f gpurun_out/ab_fir_w1.txt
timeout -k 10 120 python -u tools/ab_fir_eq.py 2 3 > gpurun_out/fir_w1_eq.log 2>&1 || exit 1
for r in 1 2 3; do
 for m in 2 3; do
  timeout -k 10 120 python -u bench.py --workload fir1024 --fir-method $m --no-cpu-baseline --no-e2e --steps 100 --warmup 50 > gpurun_out/abl.log 2>&1 || exit 1
  echo "$r 10min method$m $(tail -1 gpurun_out/abl.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])')" >> gpurun_out/ab_fir_w1.txt
 done
done
for m in 2 3; do
  timeout -k 10 200 python -u bench.py --workload fir1024 --minutes 59.99 --fir-method $m --no-cpu-baseline --no-e2e --steps 50 --warmup 30 > gpurun_out/abl.log 2>&1 || exit 1
  echo "1 1h method$m $(tail -1 gpurun_out/abl.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])')" >> gpurun_out/ab_fir_w1.txt
done
