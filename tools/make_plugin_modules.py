#!/usr/bin/env python3
"""make_plugin_modules.py -- the reference's stock plugins as gfx950 modules.

Compiles the reference's stock plugins, from their sources where they lie
under /root/reference, with the product's plugin compiler
(dsp_module_compile, hiprtc -> gfx950) into
dsp-bench_amd/modules/mod_<name>.co: what a user of the reference gets by
pointing the product at those plugin sources.  The GPU tests and bench.py
load these code objects on a box that has no /root/reference.  Outputs are
git-ignored build products (they travel to the GPU box with the tree).

Usage: python tools/make_plugin_modules.py [REF_DIR]
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "dsp-bench_amd"))

PLUGINS = ["build/gain_test", "build/IR_test", "build/sine_test", "build/buffer_test",
           "build/handmade_test", "build/template_plugin", "test/static_gain_plugin", "test/no_op",
           "test/plugin_with_parameters"]


LIB = os.environ.get("DSPBENCH_LIB", os.path.join(ROOT, "dsp-bench_amd", "libdspbench.so"))
OUT = os.environ.get("DSPB_MODULES_DIR", os.path.join(ROOT, "dsp-bench_amd", "modules"))


# this repository's own example plugins (no reference needed)
OWN = [os.path.join(ROOT, "dsp-bench_amd", "plugins", "biquad.cpp"),
       # a split State (an envelope beside a block counter): the bench's envelope_src
       os.path.join(ROOT, "dsp-bench_amd", "plugins", "envelope_counter.cpp"),
       # test plugins the bench times (the gain-table class: per-channel / per-position gains)
       os.path.join(ROOT, "tests", "plugins", "balance.cpp"), os.path.join(ROOT, "tests", "plugins", "fade_in.cpp")]


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import dspbench.module as m
    out = OUT
    os.makedirs(out, exist_ok=True)
    srcs = [os.path.join(ref, p + ".cpp") for p in PLUGINS] if os.path.isdir(os.path.join(ref, "build")) else []
    for src in srcs + OWN:
        p = os.path.splitext(src)[0]
        dst = os.path.join(out, f"mod_{os.path.basename(p)}.co")
        # the driver kernels (csrc/module.cpp) are compiled into every module:
        # rebuild when the library is newer too
        newest = max(os.path.getmtime(src), os.path.getmtime(LIB)) if os.path.exists(LIB) else os.path.getmtime(src)
        if os.path.exists(dst) and os.path.getmtime(dst) >= newest:
            continue
        code = m.compile_source(open(src).read(), os.path.basename(p))
        with open(dst, "wb") as f:
            f.write(code)
        print(f"make_plugin_modules: {dst} ({len(code)} bytes)")


if __name__ == "__main__":
    main()
