"""Shared test setup.

Markers:
  gpu  -- needs a real MI355X (run with `pytest -m gpu` on the GPU box).
Everything unmarked runs on the CPU-only build container.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "dsp-bench_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible (torch.cuda.is_available() is False)")
    return torch


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o
