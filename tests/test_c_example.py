"""The C ABI used from plain C (no Python, no torch in the process):
examples/c_drop_in.c links liblfa.so + liblfa_coll.so against /opt/rocm's
HIP runtime and RCCL, the way a libfabric provider would, and checks the
synchronous table entry, the async form and a provider allreduce + CQ."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_drop_in_example():
    from libfabric_amd import build
    exe = build.build_example()
    assert exe and os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_drop_in: OK" in r.stdout
