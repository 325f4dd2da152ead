#!/bin/bash
# tools/build_lds_variants.sh -- A/B libraries of the stateless LDS-blocks
# render (round bytes x workgroups per CU): ablibs/lds_<R>_<W>/libdspbench.so
# + modules/, loaded with DSPBENCH_LIB / DSPB_MODULES_DIR (tools only)
set -e
cd "$(dirname "$0")/../dsp-bench_amd"
make -j8 >/dev/null
for v in "$@"; do
    R=${v%_*}; W=${v#*_}
    out=../ablibs/lds_$v; mkdir -p $out/modules
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -Ibuild/gen -Wall \
        -Wno-unused-function -DDSPB_LDS_ROUND=$R -DDSPB_LDS_WGS=$W -x hip -c csrc/module.cpp -o $out/module.o
    objs=$(ls build/obj/*.o | grep -v '/module.o$')
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libdspbench.so $objs $out/module.o -lhiprtc -ldl
    DSPBENCH_LIB=$PWD/$out/libdspbench.so DSPB_MODULES_DIR=$PWD/$out/modules python3 ../tools/make_plugin_modules.py
done
