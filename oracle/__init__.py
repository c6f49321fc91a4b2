"""ORACLE — test infrastructure only (see oracle/oracle_atomic.c header).

ctypes access to
  * ``liboracle.so``          — our C restatement of the reference combine
    tables (CAS and plain variants) and of prov/coll's recursive-doubling
    allreduce (prov/coll/src/coll_coll.c:349-449);
  * ``_ref/libft_atomic.so``  — the reference's own fabtests restatement
    (fabtests/common/ofi_atomic.c), compiled from /root/reference by
    oracle/Makefile.  Used only to pin the restatement.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this package.  The product package ``libfabric_amd`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libft_atomic.so")

CAS, PLAIN = 0, 1

# enum fi_datatype (include/rdma/fi_domain.h:224-247) -> numpy storage dtype
DATATYPES = {
    "INT8": (0, np.dtype(np.int8)),
    "UINT8": (1, np.dtype(np.uint8)),
    "INT16": (2, np.dtype(np.int16)),
    "UINT16": (3, np.dtype(np.uint16)),
    "INT32": (4, np.dtype(np.int32)),
    "UINT32": (5, np.dtype(np.uint32)),
    "INT64": (6, np.dtype(np.int64)),
    "UINT64": (7, np.dtype(np.uint64)),
    "FLOAT": (8, np.dtype(np.float32)),
    "DOUBLE": (9, np.dtype(np.float64)),
    "FLOAT_COMPLEX": (10, np.dtype(np.complex64)),
    "INT128": (14, np.dtype("V16")),
    "UINT128": (15, np.dtype("V16")),
}
DT_CODE = {k: v[0] for k, v in DATATYPES.items()}
DT_NP = {v[0]: v[1] for v in DATATYPES.values()}
DT_NAME = {v[0]: k for k, v in DATATYPES.items()}

# enum fi_op (include/rdma/fi_domain.h:249-273)
OPS = {"MIN": 0, "MAX": 1, "SUM": 2, "PROD": 3, "LOR": 4, "LAND": 5,
       "BOR": 6, "BAND": 7, "LXOR": 8, "BXOR": 9, "ATOMIC_READ": 10,
       "ATOMIC_WRITE": 11}
OP_NAME = {v: k for k, v in OPS.items()}

_lib = None
_ref = None


def build() -> None:
    """Compile liboracle.so (and _ref/ when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_datatype_size.restype = ctypes.c_size_t
        L.oracle_datatype_size.argtypes = [ctypes.c_int]
        L.oracle_write.restype = ctypes.c_int
        L.oracle_write.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t]
        L.oracle_write_handler.restype = ctypes.c_void_p
        L.oracle_write_handler.argtypes = [ctypes.c_int] * 3
        L.oracle_atomic_valid.restype = ctypes.c_int
        L.oracle_atomic_valid.argtypes = [ctypes.c_int, ctypes.c_int,
                                          ctypes.c_uint64]
        L.oracle_allreduce.restype = ctypes.c_int
        L.oracle_allreduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.c_size_t]
        L.oracle_has_readwrite.restype = ctypes.c_int
        L.oracle_has_readwrite.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_has_swap.restype = ctypes.c_int
        L.oracle_has_swap.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_readwrite.restype = ctypes.c_int
        L.oracle_readwrite.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_size_t]
        L.oracle_swap.restype = ctypes.c_int
        L.oracle_swap.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 4 + [ctypes.c_size_t]
        L.oracle_allreduce_sched_len.restype = ctypes.c_int
        L.oracle_allreduce_sched_len.argtypes = [ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref() -> ctypes.CDLL:
    """The reference's fabtests restatement (plain-loop semantics)."""
    global _ref
    if _ref is None:
        if not ref_available():
            build()
        _ref = ctypes.CDLL(REF_PATH)
    return _ref


_WRITE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_size_t)


def ref_handler(op: int, dt: int):
    """ofi_atomic_write_handlers[op][dt] from the reference build, or None."""
    tbl = (ctypes.c_void_p * (12 * 16)).in_dll(ref(), "ofi_atomic_write_handlers")
    p = tbl[op * 16 + dt]
    return _WRITE_FN(p) if p else None


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def datatype_size(dt: int) -> int:
    return lib().oracle_datatype_size(dt)


def has_handler(op: int, dt: int) -> bool:
    return bool(lib().oracle_write_handler(PLAIN, op, dt))


def write(op: int, dt: int, dst: np.ndarray, src: np.ndarray,
          variant: int = PLAIN) -> None:
    """dst[i] = dst[i] OP src[i] in place (ofi_atomic_write_handler)."""
    assert dst.flags.c_contiguous and src.flags.c_contiguous
    assert dst.nbytes == src.nbytes
    n = dst.nbytes // datatype_size(dt)
    rc = lib().oracle_write(variant, op, dt, _ptr(dst), _ptr(src), n)
    if rc:
        raise ValueError(f"oracle_write({op},{dt}) -> {rc}")


_RW_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_size_t)
_SW_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_size_t)
SWAP_OPS = {"CSWAP": 12, "CSWAP_NE": 13, "CSWAP_LE": 14, "CSWAP_LT": 15,
            "CSWAP_GE": 16, "CSWAP_GT": 17, "MSWAP": 18}


def ref_readwrite_handler(op: int, dt: int):
    tbl = (ctypes.c_void_p * (12 * 16)).in_dll(ref(), "ofi_atomic_readwrite_handlers")
    p = tbl[op * 16 + dt]
    return _RW_FN(p) if p else None


def ref_swap_handler(op: int, dt: int):
    tbl = (ctypes.c_void_p * (7 * 16)).in_dll(ref(), "ofi_atomic_swap_handlers")
    p = tbl[(op - 12) * 16 + dt]
    return _SW_FN(p) if p else None


def has_readwrite(op: int, dt: int) -> bool:
    return bool(lib().oracle_has_readwrite(op, dt))


def has_swap(op: int, dt: int) -> bool:
    return bool(lib().oracle_has_swap(op, dt))


def readwrite(op, dt, dst, src, res, variant=PLAIN):
    rc = lib().oracle_readwrite(variant, op, dt, _ptr(dst), _ptr(src), _ptr(res),
                                dst.nbytes // datatype_size(dt))
    if rc:
        raise ValueError(f"oracle_readwrite({op},{dt}) -> {rc}")


def swap(op, dt, dst, src, cmp, res, variant=CAS):
    rc = lib().oracle_swap(variant, op, dt, _ptr(dst), _ptr(src), _ptr(cmp), _ptr(res),
                           dst.nbytes // datatype_size(dt))
    if rc:
        raise ValueError(f"oracle_swap({op},{dt}) -> {rc}")


def ref_write(op: int, dt: int, dst: np.ndarray, src: np.ndarray) -> None:
    fn = ref_handler(op, dt)
    if fn is None:
        raise ValueError(f"reference has no handler for op={op} dt={dt}")
    fn(_ptr(dst), _ptr(src), dst.nbytes // datatype_size(dt))


def atomic_valid(dt: int, op: int, flags: int = 0) -> int:
    return lib().oracle_atomic_valid(dt, op, flags)


def allreduce(op: int, dt: int, sends: list[np.ndarray]) -> list[np.ndarray]:
    """Every rank's fi_allreduce result, recursive-doubling order."""
    n = len(sends)
    cnt = sends[0].nbytes // datatype_size(dt)
    results = [np.empty_like(s) for s in sends]
    sp = (ctypes.c_void_p * n)(*[_ptr(s) for s in sends])
    rp = (ctypes.c_void_p * n)(*[_ptr(r) for r in results])
    rc = lib().oracle_allreduce(op, dt, n, sp, rp, cnt)
    if rc:
        raise ValueError(f"oracle_allreduce -> {rc}")
    return results


def reduce_scatter(op: int, dt: int, sends: list[np.ndarray]) -> list[np.ndarray]:
    """Slice r of the allreduce result for every rank r.

    The build's definition (no reference code: coll_ep.c:75-76 is
    fi_coll_no_reduce_scatter; semantics man/fi_collective.3.md:354-385):
    ``count`` input elements per rank, rank r receives the block
    [off(r), off(r+1)) where the first ``count % N`` ranks hold one extra
    element (block-contiguous, = ncclReduceScatter layout when N | count).
    """
    n = len(sends)
    full = allreduce(op, dt, sends)[0]
    return [full[a:b].copy() for a, b in slice_bounds(full.shape[0], n)]


def slice_bounds(count: int, n: int) -> list[tuple[int, int]]:
    base, extra = divmod(count, n)
    out, off = [], 0
    for r in range(n):
        ln = base + (1 if r < extra else 0)
        out.append((off, off + ln))
        off += ln
    return out


def tree_reference_order(n: int) -> str:
    """Human-readable association order of the N-rank allreduce result."""
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    leaves = []
    for i in range(pof2):
        leaves.append(f"(x{2*i+1}.x{2*i})" if i < rem else f"x{i+rem}")
    m = 1
    while m < pof2:
        leaves = [f"({leaves[i+1]}.{leaves[i]})" if len(leaves) > 1 else leaves[i]
                  for i in range(0, len(leaves), 2)]
        m *= 2
    return leaves[0]
