"""Prototype: a State chain for a callback that reads its block
while its State does not depend on it (state_reads_block = 0, a tremolo).

The chain kernel below hands the callback a private block filled from the
input with non-temporal stores.  Compiled from source the callback's own
stores keep that block alive (its loads read it), so the output arithmetic
stays.  Here the kernel is compiled to LLVM IR text, the callback's stores
to the block (every store through a pointer derived from the block's alloca
that is not one of the copy's non-temporal stores) are deleted, and the text
is code-generated at -O3 through comgr (tools/diag/ir_codegen_probe).  The
check: the code object's chain kernel keeps no private memory and no longer
calls the cosine.  CPU only.

  usage: python tools/diag/ir_chain_proto.py [out_dir]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "dsp-bench_amd"))
LLVM = "/opt/rocm/lib/llvm/bin"

CHAIN = r'''
extern "C" __global__ void dspb_chain(const Parameters *P, State *S, State *st_blk, const float *in0,
                                      const float *in1, unsigned long long nblocks, float sr) {
    if (threadIdx.x != 0) return;
    const Parameters prm = *P;
    State st = *S;
    for (unsigned long long b = 0; b < nblocks; ++b) {
        st_blk[b] = st;
        float dspb_chain_blk[2 * 512];
        float *ptrs[2] = {dspb_chain_blk, dspb_chain_blk + 512};
        for (unsigned i = 0; i < 512; ++i) {
            __builtin_nontemporal_store(in0[b * 512 + i], &dspb_chain_blk[i]);
            __builtin_nontemporal_store(in1[b * 512 + i], &dspb_chain_blk[512 + i]);
        }
        audio_callback(prm, st, ptrs, 2, 512, sr);
    }
    *S = st;
}
'''


def tu(src_name):
    return ("#include <hip/hip_runtime.h>\n#include \"plugin_header.h\"\n"
            "#pragma clang force_cuda_host_device begin\n#define annotate(...)\n#define __annotate__(...)\n"
            f"#include \"{src_name}\"\n#undef annotate\n#undef __annotate__\n"
            "#pragma clang force_cuda_host_device end\n" + CHAIN)


def derived(ir_fn, root):
    """SSA names of pointers derived from `root` (GEPs, phis, selects, casts)."""
    names = {root}
    grew = True
    while grew:
        grew = False
        for line in ir_fn:
            m = re.match(r"\s*(%[\w.]+) = (getelementptr|phi|select|addrspacecast|bitcast)\b(.*)", line)
            if not m or m.group(1) in names:
                continue
            ops = set(re.findall(r"%[\w.]+", m.group(3)))
            if ops & names:
                names.add(m.group(1))
                grew = True
    return names


def strip_block_stores(ir):
    lines = ir.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("define") and "@dspb_chain(" in l)
    end = next(i for i in range(start, len(lines)) if lines[i] == "}")
    fn = lines[start:end + 1]
    root = next(re.match(r"\s*(%[\w.]+) = alloca", l).group(1) for l in fn
                if re.match(r"\s*%dspb_chain_blk[\w.]* = alloca", l))
    names = derived(fn, root)
    kept, dropped = [], 0
    for l in fn:
        m = re.match(r"\s*store [^,]+, ptr addrspace\(5\) (%[\w.]+)", l)
        if m and m.group(1) in names and "!nontemporal" not in l:
            dropped += 1
            continue
        kept.append(l)
    return "\n".join(lines[:start] + kept + lines[end + 1:]), dropped


def main():
    import test_gpu_state_spec as t
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/chain_proto"
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(REPO, "include/dspbench/plugin_device.h")) as f:
        open(os.path.join(out, "plugin_header.h"), "w").write(f.read())
    for name, src in (("tremolo", t.TREMOLO_SRC),):
        open(os.path.join(out, f"{name}.cpp"), "w").write(src)
        open(os.path.join(out, f"{name}_tu.hip"), "w").write(tu(f"{name}.cpp"))
        ll = os.path.join(out, f"{name}.ll")
        subprocess.run([f"{LLVM}/clang", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-emit-llvm", "-O2", "-std=c++20", "-ffp-contract=off", "-w", "-fno-discard-value-names",
                        "-I", out, os.path.join(out, f"{name}_tu.hip"), "-o", ll], check=True)
        ir = open(ll).read()
        edited, dropped = strip_block_stores(ir)
        open(os.path.join(out, f"{name}_edited.ll"), "w").write(edited)
        probe = os.path.join(out, "probe")
        subprocess.run(["g++", "-O1", "-std=c++17", "-I/opt/rocm/include",
                        os.path.join(REPO, "tools/diag/ir_codegen_probe.cpp"), "-L/opt/rocm/lib", "-lamd_comgr",
                        "-Wl,-rpath,/opt/rocm/lib", "-o", probe], check=True)
        for tag, text in (("source", ll), ("edited", os.path.join(out, f"{name}_edited.ll"))):
            co = os.path.join(out, f"{name}_{tag}.co")
            r = subprocess.run([probe, text, co], capture_output=True, text=True)
            if r.returncode:
                print(tag, "codegen failed", r.stdout[-800:])
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            priv = re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)
            asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True).stdout
            body = asm[asm.find("<dspb_chain>:"):]
            print(f"{name} {tag}: block stores dropped {dropped if tag == 'edited' else 0}, private {priv}, "
                  f"instructions {body.count(chr(10))}, v_fma_f64 {body.count('v_fma_f64')}, "
                  f"scratch ops {len(re.findall(r'scratch_|buffer_store|buffer_load', body))}")


if __name__ == "__main__":
    main()
