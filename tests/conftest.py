import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Start offsets for the restated time-based tests: the reference seeds them with
# System.currentTimeMillis(), so their assertions must hold for any start time.
OFFSETS = [0, 37, 199, 1_000, 1_700_000_000_000, 1_700_000_000_123, 1_700_000_000_999]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_oracle():
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "sentinel_oracle.c")
    if (not os.path.exists(so)) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_oracle()


@pytest.fixture(params=OFFSETS)
def t0(request):
    return request.param


@pytest.fixture(autouse=True, scope="session")
def _torch_hip_first(request):
    """GPU runs: torch's HIP runtime initialises before the library's (tests that hand torch device buffers to
    the library find no device when the library came first). Only when GPU tests were selected."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
