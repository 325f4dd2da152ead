# A/B: plugin modules compiled with hiprtc's default unrolling against
# -mllvm -unroll-count=16 / 32 (module code objects built by a patched
# compiler into dsp-bench_amd/build/ab_uN/modules; the library is HEAD's)
set -e
mkdir -p gpurun_out/r06i
for rep in 1 2; do
 for v in base u16 u32; do
  if [ $v = base ]; then unset DSPB_MODULES_DIR; else export DSPB_MODULES_DIR=$PWD/dsp-bench_amd/build/ab_$v/modules; fi
  for w in biquad_src envelope_src; do
   echo "v=$v w=$w rep=$rep" >> gpurun_out/r06i/ab.txt
   timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e >> gpurun_out/r06i/ab.txt 2>/dev/null
  done
  echo "v=$v w=generic_nospec rep=$rep" >> gpurun_out/r06i/ab.txt
  timeout -k 10 200 python bench.py --workload generic --no-specialize --no-cpu-baseline --no-e2e >> gpurun_out/r06i/ab.txt 2>/dev/null
 done
done
