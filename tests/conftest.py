"""pytest configuration: the ``gpu`` marker and shared helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# One IPC configuration for every multi-process GPU run: the
# dma-buf IPC mode, which the host driver of this pool supports (the image
# and the GPU box export it; bench.py sets it for its N > 1 ranks).  Set here
# as well so a process started without it — and every worker the tests spawn,
# which inherits this environment — runs the same mode as the bench.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (runs via gpurun / the round-end GPU tier)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
