"""Compare persist_check.py outputs: python tools/persist_cmp.py REF_DIR DIR..."""
import glob
import os
import sys

import numpy as np

ref = sys.argv[1]
for d in sys.argv[2:]:
    for f in sorted(glob.glob(os.path.join(ref, "*.npy"))):
        a, b = np.load(f), np.load(os.path.join(d, os.path.basename(f)))
        if a.shape != b.shape:
            print(d, os.path.basename(f), "SHAPE", a.shape, b.shape)
            continue
        eq = np.array_equal(a, b)
        peak = np.abs(a).max(axis=-1, keepdims=True) + 1e-30
        rel = float((np.abs(a.astype(np.float64) - b) / peak).max())
        print(d, os.path.basename(f), "bit-exact" if eq else f"max peak-rel diff {rel:.3e}")
