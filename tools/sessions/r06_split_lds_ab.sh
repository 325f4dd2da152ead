# split_y2's partner exchange through LDS float4 slots (DSPB_SPLIT_LDS=1,
# build/ab_split) against the product's ds_bpermute + per-value lane-0
# selects: the STFT parity tests on the variant, then the driver's command
# interleaved (tools/ab_driver.py), then the input-reading STFTs (cfg 4 and
# gain_stft) alternating; profiles/r06_split_lds_ab.txt
set -o pipefail
mkdir -p gpurun_out
V=dsp-bench_amd/build/ab_split/libdspbench.so
P=dsp-bench_amd/libdspbench.so
DSPBENCH_LIB=$PWD/$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/split_lds_parity.txt 2>&1 || exit 1
tail -2 gpurun_out/split_lds_parity.txt
timeout -k 10 600 python -u tools/ab_driver.py 5 $P $V > gpurun_out/split_lds_ab_driver.txt 2>&1 || exit 1
for r in 1 2 3; do
  for L in $P $V; do
    for wl in stft96k gain_stft; do
      DSPBENCH_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline --no-e2e \
        > gpurun_out/split_lds_$wl.log 2>&1 || exit 1
      echo "round $r $L $wl $(tail -1 gpurun_out/split_lds_$wl.log)" >> gpurun_out/split_lds_wl.txt
    done
  done
done
