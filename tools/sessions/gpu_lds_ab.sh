# A/B of the LDS-blocks render variants (tools/build_lds_variants.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in 77824_2 53248_3 38912_4; do
  for p in gain_test IR_test; do
    DSPBENCH_LIB=$PWD/ablibs/lds_$v/libdspbench.so DSPB_MODULES_DIR=$PWD/ablibs/lds_$v/modules timeout -k 10 120 python bench.py --workload generic --plugin $p --no-cpu-baseline --steps 100 --warmup 50 > gpurun_out/lds_$v.log 2>&1 || exit $?
    python -c "
import json; l=[x for x in open('gpurun_out/lds_$v.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$v $p', j['roofline']['kernel_avg_ms'], j['roofline']['frac'])"
  done
done
done
