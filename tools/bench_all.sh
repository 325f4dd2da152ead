# every bench workload once at the bench's defaults (no CPU baseline, no
# end-to-end pass): one JSON line each into gpurun_out/bench_all.jsonl
mkdir -p gpurun_out
rm -f gpurun_out/bench_all.jsonl
for wl in stft96k gain_stft generic generic_stft fir1024 gain10min ch96k wav16 wav16enc; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline --no-e2e > gpurun_out/bench_$wl.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$wl.log >> gpurun_out/bench_all.jsonl
done
