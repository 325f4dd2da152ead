#!/bin/bash
# tools/power_probe.sh -- sample GPU power / clocks / temperature (read-only
# rocm-smi queries) while a long bench run keeps the fused kernel busy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/power
mkdir -p $out
rocm-smi --showpower --showclocks --showtemp > $out/idle.txt 2>&1
timeout -k 10 120 python bench.py --steps ${1:-2000} --warmup 5 --no-cpu-baseline > $out/bench.log 2>&1 &
pid=$!
for i in $(seq 1 12); do
    sleep 0.5
    rocm-smi --showpower --showclocks --showtemp > $out/s$i.txt 2>&1
done
wait $pid
echo "bench rc=$?"
grep -h -E "Socket|Power|sclk|mclk|fclk|Temperature" $out/idle.txt $out/s*.txt | sort | uniq -c | sort -rn | head -40
grep -o '"ms_per_step": [0-9.]*' $out/bench.log
