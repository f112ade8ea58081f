"""Shared pytest setup: the `gpu` marker, the oracle (test infrastructure only)
and the golden fixtures produced from the real reference (tests/golden/make_golden.py)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def _gpu_available() -> bool:
    try:
        import twemproxy_amd as t

        return t.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Skip-free guard: a gpu-marked test must not silently pass without a GPU."""
    if not _gpu_available():
        pytest.fail("no GPU visible to libnc_gpuhash.so: gpu tests need the MI355X box")
    import torch

    torch.cuda.init()
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def corpus():
    z = np.load(os.path.join(GOLDEN, "corpus.npz"))
    return z["keys"], z["offsets"], z["expected"]


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def dist_fixture():
    with open(os.path.join(GOLDEN, "dist.json")) as f:
        return json.load(f)
