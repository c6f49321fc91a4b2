"""CPU-side checks of the native boundary (no GPU compute calls).

* liblfa.so / liblfa_coll.so load and export every function and table that
  include/*.h declares;
* the host-only entry points (datatype size, atomic_valid, table membership)
  agree with the oracle restatement of util_atomic.c;
* argument validation errors come back as negative errno values.
"""
import ctypes
import os
import re

import pytest

import oracle
from libfabric_amd import _native
from libfabric_amd.enums import DT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def _declared(header: str) -> list[str]:
    text = open(os.path.join(INC, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(lfa_[a-z0-9_]+)\s*\(", text)
    names += re.findall(r"extern\s+[^;]*?\b(lfa_[a-z0-9_]+)\s*\[", text)
    return sorted(set(n for n in names if not n.endswith("_fn")))


def _lib_or_skip(name):
    try:
        return _native.lib(name)
    except _native.NativeLibraryMissing as e:
        pytest.fail(str(e))


def test_lfa_exports_every_declared_symbol():
    L = _lib_or_skip("lfa")
    for sym in _declared("lfa_atomic.h"):
        assert hasattr(L, sym), sym


@pytest.mark.skipif(not os.path.exists(os.path.join(INC, "lfa_coll.h")),
                    reason="no lfa_coll.h yet")
def test_coll_exports_every_declared_symbol():
    L = _lib_or_skip("coll")
    for sym in _declared("lfa_coll.h"):
        assert hasattr(L, sym), sym


def test_table_membership_matches_oracle():
    from libfabric_amd import atomic
    for op in range(12):
        for dt in range(16):
            assert (atomic.write_handler(op, dt) is not None) == \
                oracle.has_handler(op, dt), (op, dt)


def test_fetch_compare_tables_match_oracle():
    L = _lib_or_skip("lfa")
    rw = (ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_readwrite_handlers")
    sw = (ctypes.c_void_p * (7 * 16)).in_dll(L, "lfa_atomic_swap_handlers")
    for op in range(12):
        for dt in range(16):
            assert bool(rw[op * 16 + dt]) == oracle.has_readwrite(op, dt), (op, dt)
    for op in range(12, 19):
        for dt in range(16):
            assert bool(sw[(op - 12) * 16 + dt]) == oracle.has_swap(op, dt), (op, dt)


def test_valid_and_size_match_oracle():
    from libfabric_amd import atomic
    flags_set = [0, 1 << 3, 1 << 58, 1 << 59, (1 << 58) | (1 << 59),
                 (1 << 3) | (1 << 58), 1 << 40]
    for op in range(20):
        for dt in range(18):
            for fl in flags_set:
                assert atomic.atomic_valid(dt, op, fl) == \
                    oracle.atomic_valid(dt, op, fl), (op, dt, fl)
    for dt in range(17):
        assert atomic.datatype_size(dt) == oracle.datatype_size(dt)


def test_async_argument_errors():
    L = _lib_or_skip("lfa")
    # unsupported (op, dt): float BOR → -EOPNOTSUPP, before touching the GPU
    assert L.lfa_atomic_write_async(6, int(DT.FLOAT), None, None, 0, None) == -95
    # null buffers with cnt > 0 → -EINVAL
    assert L.lfa_atomic_write_async(2, int(DT.FLOAT), None, None, 4, None) == -22
    # tree: nsrc out of range → -EINVAL
    arr = (ctypes.c_void_p * 1)(None)
    assert L.lfa_reduce_tree_async(2, int(DT.FLOAT), None, arr, 0, 0, None) == -22
    assert L.lfa_reduce_tree_async(2, int(DT.FLOAT), None, arr, 33, 0, None) == -22
    assert L.lfa_reduce_tree_async(11, int(DT.FLOAT), None, arr, 1, 0, None) == -95
    # cnt == 0 is a no-op success
    assert L.lfa_atomic_write_async(2, int(DT.FLOAT), None, None, 0, None) == 0


def test_version_string():
    L = _lib_or_skip("lfa")
    assert b"gfx950" in L.lfa_version()


def test_param_layer():
    """lfa_param / lfa_param_set (include/lfa_atomic.h): a set value wins over
    the environment, NULL removes it (the environment shows through again),
    names and values past the slot sizes are -EINVAL.  The off_lfa provider
    feeds fi_param_get's values through this (tests/test_off_lfa.py)."""
    import errno
    L = _lib_or_skip("lfa")
    L.lfa_param.restype = ctypes.c_char_p
    L.lfa_param.argtypes = [ctypes.c_char_p]
    L.lfa_param_set.restype = ctypes.c_int
    L.lfa_param_set.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    name = b"LFA_TEST_PARAM_LAYER"
    os.environ.pop(name.decode(), None)
    assert L.lfa_param(name) is None
    os.environ[name.decode()] = "from-env"
    try:
        assert L.lfa_param(name) == b"from-env"
        assert L.lfa_param_set(name, b"12345") == 0
        assert L.lfa_param(name) == b"12345"
        assert L.lfa_param_set(name, b"678") == 0
        assert L.lfa_param(name) == b"678"
        assert L.lfa_param_set(name, None) == 0
        assert L.lfa_param(name) == b"from-env"
    finally:
        del os.environ[name.decode()]
    assert L.lfa_param_set(b"", b"x") == -errno.EINVAL
    assert L.lfa_param_set(b"L" * 64, b"x") == -errno.EINVAL
    assert L.lfa_param_set(name, b"v" * 200) == -errno.EINVAL
