# A/B of DSP_PLUGIN_BIQUAD library variants (bench.py --workload biquad, 1 h stereo)
set -e
mkdir -p gpurun_out/r06b
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_biquad.py > gpurun_out/r06b/biquad_tests.log 2>&1
for S in ${SECTIONS:-1 2 4}; do
 for rep in 1 2; do
  for lib in ${LIBS:-new head}; do
   if [ $lib = new ]; then unset DSPBENCH_LIB; else export DSPBENCH_LIB=$PWD/dsp-bench_amd/build/ab_$lib/libdspbench.so; fi
   echo "S=$S lib=$lib rep=$rep" >> gpurun_out/r06b/ab.txt
   timeout -k 10 120 python bench.py --workload biquad --sections $S --no-cpu-baseline --no-e2e --no-companion >> gpurun_out/r06b/ab.txt 2>&1
  done
 done
done
