"""(CPU) The Python ctypes mirrors of the C ABI's structs (dspbench/_lib.py,
dspbench/shard.py) against the headers in include/dspbench: every mirrored
field at the offset the C compiler gives it and every struct of the size it
gives, so a field added on one side only (module.h dsp_state_spec_info grew
`chain` in round 5) fails here rather than as a silently shifted read."""
import ctypes as C
import json
import os
import shutil
import subprocess

import pytest

import dspbench._lib as L
import dspbench.shard as S

HERE = os.path.dirname(os.path.abspath(__file__))
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

MIRRORS = [L.dsp_plugin, L.dsp_exec, L.dsp_wav_info, L.dsp_param_desc, L.dsp_plugin_descriptor,
           L.dsp_param_value, L.dsp_callback_facts, L.dsp_state_spec_info, S.dsp_gather_piece,
           S.dsp_comm_transport, S.dsp_shard]


def c_layout(tmp_path):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dspbench/dspbench.h"',
             '#include "dspbench/module.h"', '#include "dspbench/shard.h"', '#include "dspbench/wav.h"',
             'int main(void) {', '  printf("{");']
    first = True
    for cls in MIRRORS:
        name = cls.__name__
        kw = "union" if issubclass(cls, C.Union) else "struct"
        sep = "" if first else ","
        first = False
        lines.append(f'  printf("{sep}\\"{name}\\": {{\\"size\\": %zu", sizeof({kw} {name}));')
        for fname, *_ in cls._fields_:
            lines.append(f'  printf(", \\"{fname}\\": %zu", offsetof({kw} {name}, {fname}));')
        lines.append('  printf("}");')
    lines += ['  printf("}\\n");', '  return 0;', '}']
    src = tmp_path / "layout.c"
    exe = tmp_path / "layout"
    src.write_text("\n".join(lines))
    subprocess.run([cc, "-std=c11", "-I", INCLUDE, str(src), "-o", str(exe)], check=True)
    return json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)


def test_ctypes_mirrors_match_the_headers(tmp_path):
    got = c_layout(tmp_path)
    for cls in MIRRORS:
        want = got[cls.__name__]
        assert C.sizeof(cls) == want["size"], (cls.__name__, C.sizeof(cls), want["size"])
        for fname, *_ in cls._fields_:
            assert getattr(cls, fname).offset == want[fname], (cls.__name__, fname)
