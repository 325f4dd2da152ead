set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_module.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_module.log 2>&1; rc=$?; tail -5 gpurun_out/t_module.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload generic --no-cpu-baseline > gpurun_out/b_generic.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload generic --plugin IR_test --no-cpu-baseline > gpurun_out/b_generic_ir.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload generic_stft --no-cpu-baseline > gpurun_out/b_gstft_ir.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload generic_stft --plugin gain_test --no-cpu-baseline > gpurun_out/b_gstft_gain.log 2>&1 || exit $?
for f in b_generic b_generic_ir b_gstft_ir b_gstft_gain; do python -c "
import json,sys; l=[x for x in open('gpurun_out/$f.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$f', j['ms_per_step'], j['roofline']['kernel_avg_ms'], j['roofline']['frac'], j['value'])"; done
