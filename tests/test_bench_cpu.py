"""bench.py's host-side helpers (CPU): the PMC traffic figure applies only to
a launch of the profiled size, and every workload with an instantiation
names a committed summary."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


HEADLINE_BYTES = 2 * 42186 * (4 * 4096 + 4 * 4097)  # C * F * (4H + 4K), 1 h stereo at 48 kHz


def test_pmc_traffic_of_the_profiled_launch(bench):
    t, src, inst = bench.pmc_traffic("headline", HEADLINE_BYTES)
    assert t is not None and src.startswith("profiles/") and inst
    assert 0.99 < t / HEADLINE_BYTES < 1.01


def test_pmc_traffic_refuses_another_size(bench):
    # a 5-minute run (one twelfth of the bytes) must not borrow the 1 h launch's figure
    t, src, inst = bench.pmc_traffic("headline", HEADLINE_BYTES / 12)
    assert t is None and "another size" in src and inst


def test_every_instantiation_has_a_summary(bench):
    for wl, inst in bench.PK_INST.items():
        _, src, got = bench.pmc_traffic(wl, 0)  # size 0: no figure, but the summary is found
        assert got == inst
        assert src is not None, f"{wl}: no committed PMC summary names {inst}"


def test_headline_plugin_defaults_to_the_source(bench, monkeypatch):
    # the headline measures IR_test.cpp compiled unchanged unless --ir-plugin enum
    monkeypatch.setattr("sys.argv", ["bench.py"])
    assert bench.parse().ir_plugin == "source"
    monkeypatch.setattr("sys.argv", ["bench.py", "--ir-plugin", "enum"])
    assert bench.parse().ir_plugin == "enum"
    name = bench.source_plugin_name("IR_test", "table")
    assert "IR_test.cpp" in name and "compiled unchanged" in name and "table" in name


def test_gpus_flag_launches_or_checks_the_world(bench):
    """--gpus N: unlaunched N > 1 starts N ranks (torch.distributed.run as a
    child, rendezvous on 127.0.0.1); under a launcher WORLD_SIZE must equal
    N; N = 1 unlaunched runs in place."""
    assert bench.check_world(1, {}) == ("run", None)
    assert bench.check_world(8, {}) == ("launch", None)
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == ("run", None)
    what, why = bench.check_world(8, {"WORLD_SIZE": "2"})
    assert what == "error" and "WORLD_SIZE=2" in why
    assert bench.check_world(0, {})[0] == "error"
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "5"])
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4" and "torch.distributed.run" in cmd
    assert "127.0.0.1:0" in cmd
    assert cmd[-5].endswith("bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_world_mismatch_exits_nonzero():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_gather_watchdog_prints_the_line_and_fails(bench):
    """A gather pass that never finishes: the watchdog prints the line (with
    the error) and exits with a non-zero status, so a hung gather shows in
    the run's rc."""
    import threading
    done = threading.Event()
    got = {}

    def emit(ms, err):
        got["line"] = (ms, err)

    def fake_exit(rc):
        got["rc"] = rc
        done.set()
    bench.start_gather_watchdog(0.05, 0, emit, exit_fn=fake_exit)
    assert done.wait(5.0)
    assert got["rc"] == bench.GATHER_TIMEOUT_RC != 0
    assert got["line"][0] is None and "timed out" in got["line"][1]


def test_gather_watchdog_cancelled_in_time(bench):
    called = []
    dog = bench.start_gather_watchdog(0.5, 0, lambda *a: called.append(a), exit_fn=lambda rc: called.append(rc))
    dog.cancel()
    import time
    time.sleep(0.7)
    assert called == []
