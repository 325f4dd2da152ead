"""Instruction mix of the kernels in a hipcc -save-temps .s file.

    python tools/isa_hist.py <file.s> [kernel substring] [--top N]
"""
import collections
import re
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.startswith('.Lfunc_end'):
            yield cur, body
            cur = None
            continue
        if cur:
            t = line.strip()
            if t and not t.startswith(('.', ';', 's_nop')) and not t.endswith(':'):
                body.append(t.split()[0])


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith('--') else ''
    top = int(sys.argv[sys.argv.index('--top') + 1]) if '--top' in sys.argv else 0
    for name, ins in kernels(path):
        if sub not in name:
            continue
        c = collections.Counter(ins)
        grp = lambda p: sum(v for k, v in c.items() if k.startswith(p))
        print(f"{name[:100]}\n  total {len(ins)}  valu {grp('v_')}  (pk {grp('v_pk_')}, fma {grp('v_fma')}, "
              f"cndmask {grp('v_cndmask')}, mov {grp('v_mov')})  ds {grp('ds_')}  global {grp('global_')}  "
              f"buffer {grp('buffer_')}  salu {grp('s_')}")
        if top:
            for k, v in c.most_common(top):
                print(f"    {v:5d} {k}")


if __name__ == "__main__":
    main()
