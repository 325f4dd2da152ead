"""The host-side parsers under AddressSanitizer + UndefinedBehaviorSanitizer
(host code only: no GPU sanitizers exist on this pool).  tests/sanitize/
host_fuzz.cpp mutates valid WAV images, plugin sources and a compiled plugin
module and feeds them to dsp_wav_parse, the descriptor scanner and the
descriptor reader; any sanitizer report, hang or broken invariant fails.

Found and fixed by this harness: a 16-bit block-align overflow that divided
by zero (wav.cpp), two scanner loops that never advanced on malformed
annotations, unchecked ELF offset sums and descriptor field offsets outside
Parameters (descriptor.cpp).
"""
import ctypes as C
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "dsp-bench_amd")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("san") / "host_fuzz")
    cmd = [gxx, "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           f"-I{REPO}/include", f"-I{PKG}/csrc", f"{HERE}/sanitize/host_fuzz.cpp", f"{PKG}/host/wav.cpp",
           f"{PKG}/csrc/descriptor.cpp", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("the compiler has no sanitizer runtime")
    assert r.returncode == 0, r.stderr
    return exe


def _module():
    mods = os.path.join(PKG, "modules")
    for name in ("mod_gain_test.co", "mod_IR_test.co", "mod_biquad.co"):
        if os.path.exists(os.path.join(mods, name)):
            return os.path.join(mods, name)
    pytest.skip("no compiled plugin module (tools/make_plugin_modules.py)")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_host_parsers_fuzz(harness, seed):
    env = dict(os.environ, HOST_FUZZ_ITERS="20000", HOST_FUZZ_SEED=str(seed),
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([harness, f"{REPO}/include/dspbench/plugin_device.h", _module(),
                        f"{PKG}/plugins/biquad.cpp"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "host fuzz ok" in r.stdout


def test_wav_block_align_overflow_is_rejected():
    """16384 channels x 32-bit PCM: nBlockAlign would wrap to 0 (and the frame
    count divide by it); the parser refuses the header instead."""
    lib = C.CDLL(os.path.join(PKG, "libdspbench.so"))
    hdr = bytearray(44 + 64)
    hdr[0:4] = b"RIFF"
    hdr[4:8] = (len(hdr) - 8).to_bytes(4, "little")
    hdr[8:16] = b"WAVEfmt "
    hdr[16:20] = (16).to_bytes(4, "little")
    hdr[20:22] = (1).to_bytes(2, "little")        # PCM
    hdr[22:24] = (16384).to_bytes(2, "little")    # channels
    hdr[24:28] = (48000).to_bytes(4, "little")
    hdr[34:36] = (32).to_bytes(2, "little")       # bits
    hdr[36:40] = b"data"
    hdr[40:44] = (64).to_bytes(4, "little")
    info = (C.c_uint8 * 512)()
    buf = (C.c_uint8 * len(hdr)).from_buffer(hdr)
    st = lib.dsp_wav_parse(buf, C.c_uint64(len(hdr)), info)
    assert st != 0
