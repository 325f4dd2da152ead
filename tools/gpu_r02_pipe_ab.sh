# A/B of the generic render + STFT schedules (fused kernel off)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-cpu-baseline --workload generic_stft --steps 50 --warmup 20 > gpurun_out/$tag.log 2>&1 || exit $?; python -c "
import json; l=[x for x in open('gpurun_out/$tag.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$tag', j['ms_per_step'], j['roofline']['kernel_avg_ms'], j['roofline']['frac'])"; }
run serial DSPB_GENERIC_FUSED=0 DSPB_PIPE_CHUNK_BYTES=100000000000
run one64 DSPB_GENERIC_FUSED=0 DSPB_PIPE_STREAMS=1 DSPB_PIPE_CHUNK_BYTES=67108864
run one256 DSPB_GENERIC_FUSED=0 DSPB_PIPE_STREAMS=1 DSPB_PIPE_CHUNK_BYTES=268435456
run two64 DSPB_GENERIC_FUSED=0 DSPB_PIPE_CHUNK_BYTES=67108864
run two256 DSPB_GENERIC_FUSED=0 DSPB_PIPE_CHUNK_BYTES=268435456
timeout -k 10 300 python bench.py --no-cpu-baseline --workload stft96k --minutes 30 --steps 50 --warmup 20 > gpurun_out/stft48.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/stft48.log
