"""The off_lfa offload-collective provider (libfabric_amd/csrc/off_lfa.c)
driven the way rxm drives an offload provider, by examples/off_lfa_host.c:
a minimal owner (peer AV / CQ / EQ / endpoint) built from libfabric's public
headers, loading liboff_lfa-fi.so through fi_prov_ini.

* CPU: discovery (FI_PEER_TRANSFER required, "off_" prefix), fi_domain2 with
  FI_PEER, rxm's capability probe (rxm_domain.c:878-893) giving the mask
  BARRIER|BROADCAST|ALLREDUCE|ALLGATHER|REDUCE_SCATTER|REDUCE|SCATTER, peer
  AV/CQ/EQ/endpoint contexts, options, av_set algebra, errors before join.
* GPU: world join through the peer EQ, every collective on device and host
  buffers with completions delivered through the owner's peer CQ (carrying
  the owner's context), av_set address, subset join — with the progress
  thread and with owner-driven progress through the util_ep slot.

Both binaries are compiled in the build container against libfabric's public
headers; the GPU box runs the prebuilt files.
"""
import os
import subprocess

import pytest

from libfabric_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binaries():
    if build.have_fabric_headers():
        build.build_all()
    lib, exe = build.LIB_OFF, build.OFF_HOST
    if not (os.path.exists(lib) and os.path.exists(exe)):
        pytest.fail("off_lfa provider / host driver not built (needs libfabric's "
                    "public headers at build time)")
    return lib, exe


def _run(*args, timeout=300):
    lib, exe = _binaries()
    env = dict(os.environ)
    env.pop("OFF_LFA_PROGRESS", None)
    r = subprocess.run([exe, lib, *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.strip().splitlines()[-1]    # RCCL prints a banner first


def test_provider_exports():
    lib, _ = _binaries()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert "fi_prov_ini" in syms
    assert os.path.basename(lib) == "liboff_lfa-fi.so"     # lib<name>-fi.so


@pytest.mark.parametrize("mode", [[], ["manual"]])
def test_host_driver_cpu(mode):
    assert _run("cpu", *mode).startswith("OK cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [[], ["manual"]])
def test_host_driver_gpu(mode):
    assert _run("gpu", *mode).startswith("OK gpu")
