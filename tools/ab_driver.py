"""Interleaved A/B of libdspbench.so builds under the driver's own bench
command (python bench.py --gpus 1 --steps 20 --warmup 5: the timed launches
sit in the clock dip after the kernel first meets the power cap), each run a
fresh process after an idle pause, the line's ms_per_step and roofline frac.

    python tools/ab_driver.py ROUNDS [--pause S] LIB_A LIB_B ...
"""
import json
import os
import statistics
import subprocess
import sys
import time

repo = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
argv = sys.argv[1:]
rounds = int(argv.pop(0))
pause = 8.0
if argv and argv[0] == "--pause":
    argv.pop(0)
    pause = float(argv.pop(0))
libs = argv
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        time.sleep(pause)
        env = dict(os.environ, DSPBENCH_LIB=os.path.abspath(l))
        o = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "1", "--steps", "20",
                            "--warmup", "5", "--no-cpu-baseline", "--no-e2e", "--no-companion"],
                           capture_output=True, text=True, timeout=300, env=env, cwd=repo)
        line = json.loads([s for s in o.stdout.splitlines() if s.startswith("{")][-1])
        res[l].append((line["ms_per_step"], line["roofline"]["frac"]))
        print(f"round {r} {os.path.relpath(l, repo)}: {line['ms_per_step']:.4f} ms frac {line['roofline']['frac']:.4f}",
              flush=True)
for l, v in res.items():
    print(f"{os.path.relpath(l, repo)}: median {statistics.median(t for t, _ in v):.4f} ms, "
          f"frac {statistics.median(f for _, f in v):.4f}")
