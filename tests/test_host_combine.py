"""The product's HOST-memory combine (lfa_host_write / lfa_host_reduce_tree in
liblfa.so) on CPU: the kernels' own functors (lfa_ops.hpp) compiled for the
host, pinned to the reference-generated fixtures and to the oracle.

This path serves host-resident operands only (the synchronous table's small
host buckets and host-transport endpoints); device pointers always take the
gfx950 kernels (tests/test_combine_gpu.py).
"""
import json
import os

import numpy as np
import pytest

import oracle
from tests._cmp import assert_parity


@pytest.fixture(scope="module")
def lfa():
    from libfabric_amd import atomic, lib
    lib()
    return atomic


@pytest.fixture(scope="module")
def manifest(golden_dir):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        return json.load(f)


def test_golden_write_fixtures(lfa, manifest, golden_dir):
    """All 132 write-table entries, bit-exact vs the reference build."""
    for case in manifest["combine"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        d = np.ascontiguousarray(z["dst"]).view(np.uint8).copy()
        s = np.ascontiguousarray(z["src"]).view(np.uint8).copy()
        lfa.host_write(case["op"], case["dt"], d, s, case["n"])
        assert_parity(case["dt"], d, z["out"], case["file"])


def test_golden_allreduce_fixtures_tree(lfa, manifest, golden_dir):
    """The recursive-doubling tree on the multi-rank fixtures (N = 2,3,5,8)."""
    for case in manifest["allreduce"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        sends = [np.ascontiguousarray(x) for x in z["sends"]]
        out = np.empty_like(sends[0])
        lfa.host_reduce_tree(case["op"], case["dt"], out, sends)
        assert_parity(case["dt"], out.view(np.uint8), z["out"], case["file"])


def _rand(dt, n, rng):
    nd = oracle.DT_NP[dt]
    if nd.kind == "V":
        return rng.integers(0, 256, size=n * 16, dtype=np.uint8).view(nd)
    if nd.kind == "c":
        return rng.uniform(-2, 2, size=2 * n).astype(np.float32).view(np.complex64)
    if nd.kind == "f":
        return rng.uniform(-2, 2, size=n).astype(nd)
    info = np.iinfo(nd)
    return rng.integers(info.min, info.max, size=n, dtype=nd, endpoint=True)


CASES = [("SUM", "FLOAT"), ("MIN", "INT64"), ("BOR", "INT64"), ("PROD", "DOUBLE"),
         ("SUM", "INT8"), ("MAX", "UINT16"), ("PROD", "FLOAT_COMPLEX"),
         ("BXOR", "UINT128"), ("LXOR", "FLOAT"), ("ATOMIC_WRITE", "INT32")]


@pytest.mark.parametrize("opname,dtname", CASES)
def test_sizes_and_misalignment(lfa, opname, dtname):
    op, dt = oracle.OPS[opname], oracle.DT_CODE[dtname]
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(op * 7 + dt)
    for n in (0, 1, 7, 1000, 4099):
        for off in (0, 1, 3):
            raw_d = _rand(dt, n + 8, rng).view(np.uint8).copy()
            raw_s = _rand(dt, n + 8, rng).view(np.uint8).copy()
            # byte offsets: off=1/3 are not even element-aligned
            d = raw_d[off:off + n * esz]
            s = raw_s[off:off + n * esz]
            want = d.copy().view(oracle.DT_NP[dt])
            oracle.write(op, dt, want, s.copy().view(oracle.DT_NP[dt]))
            from libfabric_amd import lib
            rc = lib().lfa_host_write(op, dt, d.ctypes.data, s.ctypes.data, n)
            assert rc == 0
            assert_parity(dt, d, want.view(np.uint8), f"{opname} {dtname} n={n} off={off}")


@pytest.mark.parametrize("n", list(range(1, 33)))
def test_tree_every_fan_in(lfa, n):
    rng = np.random.default_rng(n)
    for op, dt in ((2, 8), (3, 9), (0, 6), (9, 5), (2, 10)):
        sends = [_rand(dt, 777, rng) for _ in range(n)]
        want = oracle.allreduce(op, dt, sends)[0]
        out = np.empty_like(sends[0])
        lfa.host_reduce_tree(op, dt, out, sends)
        assert_parity(dt, out.view(np.uint8), want.view(np.uint8), f"n={n} op={op} dt={dt}")
        # in place: dst aliases an input
        alias = [x.copy() for x in sends]
        lfa.host_reduce_tree(op, dt, alias[n // 2], alias)
        assert_parity(dt, alias[n // 2].view(np.uint8), want.view(np.uint8), "aliased")


def test_errors(lfa):
    from libfabric_amd import lib
    L = lib()
    a = np.zeros(4, np.float32)
    assert L.lfa_host_write(6, 8, a.ctypes.data, a.ctypes.data, 4) == -95   # BOR float
    assert L.lfa_host_write(2, 8, None, a.ctypes.data, 4) == -22
    assert L.lfa_host_write(2, 8, None, None, 0) == 0
    assert L.lfa_host_write(10, 8, a.ctypes.data, a.ctypes.data, 4) == -95  # ATOMIC_READ


# ----------------------------------- synchronous tables, host pointers ----
# prov/coll's REDUCE items hand the table HOST memory (coll_coll.c:758-768,
# :364, :1058).  The table classifies each pointer (hipPointerGetAttributes;
# on a machine without a GPU every pointer is host) and runs buckets up to
# lfa_host_small_bytes() on the host; tests/test_combine_gpu.py covers the
# staged (HBM) path above it and device pointers.

_RW = None


def _tables():
    import ctypes
    from libfabric_amd import lib
    L = lib()
    w = (ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_write_handlers")
    rw = (ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_readwrite_handlers")
    sw = (ctypes.c_void_p * (7 * 16)).in_dll(L, "lfa_atomic_swap_handlers")
    W = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
    R = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_size_t)
    S = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_void_p, ctypes.c_size_t)
    return (lambda op, dt: W(w[op * 16 + dt]) if w[op * 16 + dt] else None,
            lambda op, dt: R(rw[op * 16 + dt]) if rw[op * 16 + dt] else None,
            lambda op, dt: S(sw[(op - 12) * 16 + dt]) if sw[(op - 12) * 16 + dt] else None)


def test_sync_write_table_host_pointers(lfa, manifest, golden_dir):
    from libfabric_amd import lib
    assert lib().lfa_host_small_bytes() >= 1 << 16
    wt, _, _ = _tables()
    for case in manifest["combine"]:
        fn = wt(case["op"], case["dt"])
        assert fn is not None
        z = np.load(os.path.join(golden_dir, case["file"]))
        d = np.ascontiguousarray(z["dst"]).view(np.uint8).copy()
        s = np.ascontiguousarray(z["src"]).view(np.uint8).copy()
        fn(d.ctypes.data, s.ctypes.data, case["n"])    # coll_coll.c:763 order
        assert_parity(case["dt"], d, z["out"], case["file"])
    # the void table reports its failures per thread: none here
    assert lib().lfa_atomic_last_error() == 0


def test_sync_fetch_and_compare_tables_host_pointers(lfa, manifest, golden_dir):
    _, rt, st = _tables()
    for case in manifest["readwrite"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        d = np.ascontiguousarray(z["dst"]).view(np.uint8).copy()
        s = np.ascontiguousarray(z["src"]).view(np.uint8).copy()
        r = np.zeros_like(d)
        rt(case["op"], case["dt"])(d.ctypes.data, s.ctypes.data, r.ctypes.data, case["n"])
        assert_parity(case["dt"], d, z["out"], case["file"])
        assert_parity(case["dt"], r, z["res"], case["file"] + " res")
    for case in manifest["swap"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        nd = oracle.DT_NP[case["dt"]]
        want_d = z["dst"].view(nd).copy()
        want_r = np.zeros_like(want_d)
        oracle.swap(case["op"], case["dt"], want_d, z["src"].view(nd).copy(),
                    z["cmp"].view(nd).copy(), want_r, oracle.CAS)
        d = np.ascontiguousarray(z["dst"]).view(np.uint8).copy()
        s = np.ascontiguousarray(z["src"]).view(np.uint8).copy()
        c = np.ascontiguousarray(z["cmp"]).view(np.uint8).copy()
        r = np.zeros_like(d)
        st(case["op"], case["dt"])(d.ctypes.data, s.ctypes.data, c.ctypes.data,
                                   r.ctypes.data, case["n"])
        assert np.array_equal(d, want_d.view(np.uint8)), case["file"]
        assert np.array_equal(r, want_r.view(np.uint8)), case["file"]
