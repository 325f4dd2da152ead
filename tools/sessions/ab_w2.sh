mkdir -p gpurun_out
for r in 1 2; do
 for wl in stft96k gain_stft; do
  for lib in build/ab_opt0/libdspbench.so libdspbench.so; do
   DSPBENCH_LIB=$GRAFT_REPO_ROOT/dsp-bench_amd/$lib timeout -k 10 120 python -u bench.py --workload $wl --no-cpu-baseline --no-e2e --steps 100 --warmup 50 > gpurun_out/abl.log 2>&1 || exit 1
   echo "$r $wl $lib $(tail -1 gpurun_out/abl.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])')" >> gpurun_out/ab_w2.txt
  done
 done
done
