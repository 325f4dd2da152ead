# GPU session: generic-driver module tests + generic benches (render only,
# render + STFT)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_module.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_module.log 2>&1; rc=$?; tail -5 gpurun_out/t_module.log; [ $rc -le 1 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$tag.log 2>&1 || exit $?; python -c "
import json; l=[x for x in open('gpurun_out/$tag.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$tag', j['ms_per_step'], j['roofline']['kernel_avg_ms'], j['roofline']['frac'], j['value'])"; }
run b_generic --workload generic
run b_generic_ir --workload generic --plugin IR_test
run b_gstft_ir --workload generic_stft
run b_gstft_gain --workload generic_stft --plugin gain_test
