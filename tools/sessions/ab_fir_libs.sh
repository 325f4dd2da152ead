# alternate product-library variants (tools/build_fir_variants.sh) on the
# fir1024 workload, one process per run: bash tools/ab_fir_libs.sh ROUNDS MINUTES name...
set -o pipefail
R=$1; M=$2; shift 2
for r in $(seq 1 $R); do
  for v in "$@"; do
    echo "== round $r variant $v"
    DSPBENCH_LIB=dsp-bench_amd/build/var/$v/libdspbench.so timeout -k 10 120 python -u tools/ab_fir_persist.py 3 $M 0 | grep -E "sha1|median" || exit 1
  done
done
