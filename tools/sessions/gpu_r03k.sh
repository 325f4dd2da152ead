set -u -o pipefail
o=gpurun_out/r03k; mkdir -p $o
DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --minutes 5 --no-cpu-baseline --workload headline --gather-timeout 0.01 > $o/dog.txt 2>&1 || { echo "dog rc=$?"; tail -20 $o/dog.txt; exit 1; }
grep '"metric"' $o/dog.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('dog', l['value'], l['config']['render_gather_ms'], l['config']['render_gather_error'])"
exit 0
DSPB_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --minutes 5 --no-cpu-baseline --workload ch96k > $o/ch.txt 2>&1 || { echo "ch rc=$?"; tail -20 $o/ch.txt; exit 1; }
grep '"metric"' $o/ch.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('ch96k', l['value'], l['config']['render_gather_ms'], l['config']['render_gather_error'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/n1.txt 2>&1 || { echo "n1 rc=$?"; tail -20 $o/n1.txt; exit 1; }
grep '"metric"' $o/n1.txt | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('n1', l['value'], l['roofline']['frac'], l['config']['render_gather_ms'])"
