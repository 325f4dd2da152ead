# diagnostics: a split State's facts as the analysis, the code object and the
# loaded module report them (one process, GPU visible)
import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "dsp-bench_amd")
import test_gpu_state_spec as ss
import dspbench.module as dm
for n in ("split_counter_tail", "split_phase_env"):
    src = ss.GEN_HEAD + ss.GEN_BODIES[n]
    a = dm.analyze_source(src)
    code = dm.compile_source(src, f"gen_{n}.cpp")
    f = dm.code_facts(code)
    mod = dm.Module(code)
    g = mod.facts
    print(n, a["state_split"], a["state_dep_words"], f["state_split"], f["state_dep_words"],
          g["state_split"], g["state_dep_words"], g["present"], flush=True)
