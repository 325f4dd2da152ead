#!/usr/bin/env python3
"""make_golden.py -- regenerate tests/golden/golden_v1.npz + golden_v1.json.

TEST INFRASTRUCTURE.  Run in the build container, where oracle/_ref holds
the reference's own stock plugins compiled from their sources with the JIT's
flags (oracle/Makefile, ref compiler.cpp:507-515).  The fixtures are DATA:
inputs are regenerated from seeds (numpy PCG64) by the tests; outputs are
stored as arrays or as a SHA-256 of the float32 bytes (bit-exact targets).

Where each vector comes from:
  K1  static_gain_plugin on x[i] = i, 1 ch x 512       ref test/tests.cpp:255-303
  K2  no_op is the identity on x[i] = i                 ref test/tests.cpp:215-252
  K3  plugin_with_parameters defaults {0, 0.9f, 0}, state {0.1f}
                                                        ref test/tests.cpp:175-212
  K4  IR analysis of gain_test (0.2): flat 0.2*0.08/sqrt(8192)   SURVEY 8(c)
  K5  IR analysis of IR_test (0.9, 0.002), all 8192 bins, float64 SURVEY 8(c)
  R1  render_audio one-shot, static_gain, 1 s mono @48 kHz, B = 256 (cfg 1)
  R2  render_audio one-shot, gain_test, 2 x 200000, B = 512 (cfg 2 shape)
  R3  render_audio one-shot, IR_test, 2 x 200000, B = 512 (cfg 3a shape)
  S1  5-frame Hann STFT (N 8192, H 4096, 4097 bins) of a seeded sweep + noise,
      float64 numpy (IPP is absent: DIV_BY_SQRTN and sqrt(re^2+im^2) restated)
  P1  sine_test (stateful) callback, 4 blocks of 512, 2 ch (generic dispatch)
  W1  WAV sample decode through the reference's own convertInt16/24/32ToFloat
      (audio.h:66-110, oracle/_ref/libref_audio.so): every int16 code, every
      int24 code, 2^20 seeded int32 codes + edges -- SHA-256 of the floats

Usage: python tests/golden/make_golden.py   (writes next to this file)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as o  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def signal_uniform(seed: int, shape) -> np.ndarray:
    """uniform[-1, 1) float32, the cfg 1/2 synthetic WAV."""
    return (np.random.default_rng(seed).random(shape) * 2.0 - 1.0).astype(np.float32)


def signal_sweep(seed: int, n: int, sr: float = 96000.0) -> np.ndarray:
    """20 Hz - 40 kHz log sweep + noise at -20 dBFS (cfg 4 style)."""
    t = np.arange(n) / sr
    T = n / sr
    f0, f1 = 20.0, 40000.0
    k = np.log(f1 / f0)
    ph = 2 * np.pi * f0 * T / k * (np.exp(t / T * k) - 1)
    noise = np.random.default_rng(seed).standard_normal(n) * 0.1
    return (0.1 * (np.sin(ph) + noise)).astype(np.float32)


def wav_code_sets() -> dict:
    """Little-endian sample bytes: all int16, all int24, 2^20 int32 (+ edges)."""
    c16 = np.arange(1 << 16, dtype=np.uint32).astype("<u2").view(np.uint8)
    c = np.arange(1 << 24, dtype=np.uint32)
    c24 = np.stack([c & 0xff, (c >> 8) & 0xff, (c >> 16) & 0xff], axis=1).astype(np.uint8).ravel()
    r = np.random.default_rng(5).integers(0, 1 << 32, 1 << 20, dtype=np.uint64).astype(np.uint32)
    r[:6] = [0, 1, 0x7fffffff, 0x80000000, 0xffffffff, 0x40000000]
    return {16: c16, 24: c24, 32: r.astype("<u4").view(np.uint8)}


def main():
    if not o.ref_available():
        sys.exit("oracle/_ref missing: run `make -C oracle` with /root/reference present")
    arrays, meta = {}, {"numpy": np.__version__}

    # K1 / K2 / K3 -- the reference's own unit tests
    x = np.arange(512, dtype=np.float32)[None, :]
    arrays["k1_out"] = o.callback_once(o.RefPlugin("static_gain_plugin", 1, 44100.0).as_oracle(),
                                       x.copy(), 44100.0)[0]
    arrays["k2_out"] = o.callback_once(o.RefPlugin("no_op", 1, 44100.0).as_oracle(), x.copy(), 44100.0)[0]
    pw = o.RefPlugin("plugin_with_parameters", 1, 44100.0)
    arrays["k3_params"] = pw.params.copy()
    arrays["k3_state"] = pw.state.copy()

    # IR buffers (compute_IR, ref plugin.cpp:17-58: impulse, one callback of 2048)
    for name in ("gain_test", "IR_test"):
        imp = np.zeros((2, 2048), np.float32)
        imp[:, 0] = 1.0
        ir = o.callback_once(o.RefPlugin(name, 2, 48000.0).as_oracle(), imp, 48000.0)
        arrays[f"ir_{name}"] = ir
    arrays["k4_mag"] = o.np_ir_magnitude(arrays["ir_gain_test"][0])
    arrays["k5_mag"] = o.np_ir_magnitude(arrays["ir_IR_test"][0])

    # R1-R3 -- one-shot offline render through the reference plugins
    renders = {
        "r1": ("static_gain_plugin", 1, 48000, 1, 256, 2),
        "r2": ("gain_test", 2, 200000, 2, 512, 2),
        "r3": ("IR_test", 2, 200000, 2, 512, 2),
    }
    meta["renders"] = {}
    for key, (name, cin, n, seed, B, cout) in renders.items():
        sig = signal_uniform(seed, (cin, n))
        plug = o.RefPlugin(name, cout, 48000.0).as_oracle()
        out = o.render_offline([sig[c] for c in range(cin)], cout, B, 48000.0, plug)
        meta["renders"][key] = {"plugin": name, "in_channels": cin, "L": n, "seed": seed, "B": B,
                                "out_channels": cout, "shape": list(out.shape), "sha256": sha(out)}
        arrays[f"{key}_head"] = out[:, :256]
        arrays[f"{key}_tail"] = out[:, -256:]

    # S1 -- STFT magnitudes, float64
    sw = signal_sweep(4, 8192 + 4 * 4096)
    arrays["s1_signal"] = sw
    arrays["s1_mag"] = o.np_stft_mag(sw, 8192, 4096, o.WIN_HANN, 4097).astype(np.float32)
    arrays["s1_mag_hamming_full"] = o.np_stft_mag(sw[:8192], 8192, 4096, o.WIN_HAMMING, 8192).astype(np.float32)

    # P1 -- a stateful plugin, block after block (state carried by the host)
    sp = o.RefPlugin("sine_test", 2, 48000.0)
    blocks = []
    for _ in range(4):
        blocks.append(o.callback_once(sp.as_oracle(), np.zeros((2, 512), np.float32), 48000.0))
    arrays["p1_sine_test"] = np.concatenate(blocks, axis=1)
    arrays["p1_sine_test_params"] = sp.params.copy()

    # W1 -- WAV decode through the reference's converters
    meta["wav_decode"] = {}
    for bits, raw in wav_code_sets().items():
        out = o.ref_convert(raw, bits)
        meta["wav_decode"][str(bits)] = {"n": int(out.size), "sha256": sha(out),
                                         "first": [float(v) for v in out[:4]]}

    meta["k4_flat"] = 0.2 * 0.08 / np.sqrt(8192.0)
    meta["k5_bins"] = {str(k): float(arrays["k5_mag"][k]) for k in (0, 1, 2, 4096, 8191)}
    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), **arrays)
    with open(os.path.join(HERE, "golden_v1.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", sorted(arrays), "\nK5:", meta["k5_bins"])


if __name__ == "__main__":
    main()
