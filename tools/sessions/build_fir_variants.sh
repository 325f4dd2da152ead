# Product-library variants that differ only in how fir_fft.hip is compiled
# (scheduler strategy): dsp-bench_amd/build/var/<name>/libdspbench.so, linked
# from the product objects (make first) with fir_fft.o rebuilt.  A/B with
# tools/ab_fir_persist.py under DSPBENCH_LIB=<that library>.
#
#   bash tools/build_fir_variants.sh name "extra hipcc flags" [...]
set -e
cd "$(dirname "$0")/../dsp-bench_amd"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Wall -Wno-unused-function -fno-slp-vectorize"
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  d=build/var/$name
  mkdir -p $d
  $HIPCC $FLAGS $extra -c csrc/fir_fft.hip -o $d/fir_fft.o
  objs=$(ls build/obj/*.o | grep -v '/fir_fft.o$')
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/libdspbench.so $objs $d/fir_fft.o -lhiprtc -ldl
  echo "built $d/libdspbench.so ($extra)"
done
