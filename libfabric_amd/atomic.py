"""Tensor-level access to the gfx950 combine kernels (liblfa.so).

Mirrors the reference's L4 combine interface (include/ofi_atomic.h:45-90):

  datatype_size(dt)                 ofi_datatype_size        util_atomic.c:58
  atomic_valid(dt, op, flags)       ofi_atomic_valid         util_atomic.c:1088
  write_handler(op, dt)             ofi_atomic_write_handlers[op][dt]
  write(op, dt, dst, src, cnt)      ofi_atomic_write_handler(op, dt, dst, src, cnt)
                                    — asynchronous on a HIP stream
  reduce_tree(op, dt, dst, srcs)    prov/coll's log2(N) REDUCE items fused into
                                    one pass (coll_coll.c:349-449 order)

Tensors are raw device storage: ``dt`` says how the bytes are interpreted,
``cnt`` defaults to ``dst.nbytes // datatype_size(dt)``.  Errors raise
``LfaError`` carrying the negative errno the C ABI returned.
"""
from __future__ import annotations

import ctypes

import torch

from ._native import lib
from .enums import DT, OP

LFA_EOPNOTSUPP = 95
LFA_EINVAL = 22


class LfaError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} failed: {rc}")
        self.rc = rc


def datatype_size(dt: int) -> int:
    return int(lib().lfa_datatype_size(int(dt)))


def atomic_valid(dt: int, op: int, flags: int = 0) -> int:
    return int(lib().lfa_atomic_valid(int(dt), int(op), int(flags)))


_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


def write_handler(op: int, dt: int):
    """The synchronous table entry lfa_atomic_write_handlers[op][dt] or None."""
    tbl = (ctypes.c_void_p * (12 * 16)).in_dll(lib(), "lfa_atomic_write_handlers")
    p = tbl[int(op) * 16 + int(dt)]
    return _FN(p) if p else None


def _stream_handle(stream) -> int | None:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _check_dev(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def write(op: int, dt: int, dst: torch.Tensor, src: torch.Tensor,
          cnt: int | None = None, stream=None) -> None:
    """dst[i] = dst[i] OP src[i] on the GPU (enqueued, not waited for)."""
    _check_dev(dst, "dst")
    _check_dev(src, "src")
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    if cnt * esz > dst.nbytes or cnt * esz > src.nbytes:
        raise ValueError("cnt exceeds buffer size")
    rc = lib().lfa_atomic_write_async(int(op), int(dt), dst.data_ptr(),
                                      src.data_ptr(), cnt,
                                      _stream_handle(stream))
    if rc:
        raise LfaError(rc, f"lfa_atomic_write_async({OP(op).name},{DT(dt).name})")


def write_ptr(op: int, dt: int, dst: int, src: int, cnt: int,
              stream=None) -> int:
    """Raw-pointer form (returns the C return code)."""
    return int(lib().lfa_atomic_write_async(int(op), int(dt), dst, src, cnt,
                                            _stream_handle(stream)))


def readwrite(op: int, dt: int, dst: torch.Tensor, src: torch.Tensor | None,
              res: torch.Tensor, cnt: int | None = None, stream=None) -> None:
    """res = dst; dst = dst OP src (ofi_atomic_readwrite_handler; ATOMIC_READ
    ignores src, ATOMIC_WRITE exchanges)."""
    _check_dev(dst, "dst")
    _check_dev(res, "res")
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    rc = lib().lfa_atomic_readwrite_async(
        int(op), int(dt), dst.data_ptr(), src.data_ptr() if src is not None else None,
        res.data_ptr(), cnt, _stream_handle(stream))
    if rc:
        raise LfaError(rc, f"lfa_atomic_readwrite_async({op},{DT(dt).name})")


def swap(op: int, dt: int, dst: torch.Tensor, src: torch.Tensor, cmp: torch.Tensor,
         res: torch.Tensor, cnt: int | None = None, stream=None) -> None:
    """res = dst; dst = src where (cmp OP dst) (ofi_atomic_swap_handler)."""
    for name, t in (("dst", dst), ("src", src), ("cmp", cmp), ("res", res)):
        _check_dev(t, name)
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    rc = lib().lfa_atomic_swap_async(int(op), int(dt), dst.data_ptr(), src.data_ptr(),
                                     cmp.data_ptr(), res.data_ptr(), cnt,
                                     _stream_handle(stream))
    if rc:
        raise LfaError(rc, f"lfa_atomic_swap_async({op},{DT(dt).name})")


def reduce_tree(op: int, dt: int, dst: torch.Tensor, srcs: list[torch.Tensor],
                cnt: int | None = None, stream=None) -> None:
    """dst = recursive-doubling tree of srcs (rank order = list order)."""
    _check_dev(dst, "dst")
    for i, s in enumerate(srcs):
        _check_dev(s, f"srcs[{i}]")
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    if any(cnt * esz > s.nbytes for s in srcs) or cnt * esz > dst.nbytes:
        raise ValueError("cnt exceeds buffer size")
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    rc = lib().lfa_reduce_tree_async(int(op), int(dt), dst.data_ptr(), arr,
                                     len(srcs), cnt, _stream_handle(stream))
    if rc:
        raise LfaError(rc, f"lfa_reduce_tree_async({OP(op).name},{DT(dt).name})")


def reduce_tree_put(op: int, dt: int, dsts: list[torch.Tensor], srcs: list[torch.Tensor],
                    cnt: int | None = None, stream=None) -> None:
    """Every dsts[j] = recursive-doubling tree of srcs, one pass, system-scope
    accesses (lfa_reduce_tree_put_async, the LFA_ALGO_P2P kernel)."""
    for i, t in enumerate(list(dsts) + list(srcs)):
        _check_dev(t, f"operand {i}")
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dsts[0].nbytes // esz
    if any(cnt * esz > t.nbytes for t in list(dsts) + list(srcs)):
        raise ValueError("cnt exceeds buffer size")
    sa = (ctypes.c_void_p * len(srcs))(*[t.data_ptr() for t in srcs])
    da = (ctypes.c_void_p * len(dsts))(*[t.data_ptr() for t in dsts])
    rc = lib().lfa_reduce_tree_put_async(int(op), int(dt), da, len(dsts), sa, len(srcs),
                                         cnt, _stream_handle(stream))
    if rc:
        raise LfaError(rc, f"lfa_reduce_tree_put_async({OP(op).name},{DT(dt).name})")


# ------------------------------------------------------- host-memory forms --

def _host_ptr(a) -> int:
    if isinstance(a, torch.Tensor):
        if a.is_cuda:
            raise ValueError("host form called with a device tensor")
        return a.data_ptr()
    return a.ctypes.data


def host_write(op: int, dt: int, dst, src, cnt: int | None = None) -> None:
    """dst[i] = dst[i] OP src[i] for HOST buffers (numpy arrays or CPU
    tensors), lfa_host_write: the kernels' functors run on the host."""
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    rc = lib().lfa_host_write(int(op), int(dt), _host_ptr(dst), _host_ptr(src), cnt)
    if rc:
        raise LfaError(rc, f"lfa_host_write({op},{dt})")


def host_reduce_tree(op: int, dt: int, dst, srcs, cnt: int | None = None) -> None:
    """dst = prov/coll's recursive-doubling tree of HOST buffers srcs."""
    esz = datatype_size(dt)
    if cnt is None:
        cnt = dst.nbytes // esz
    arr = (ctypes.c_void_p * len(srcs))(*[_host_ptr(s) for s in srcs])
    rc = lib().lfa_host_reduce_tree(int(op), int(dt), _host_ptr(dst), arr, len(srcs), cnt)
    if rc:
        raise LfaError(rc, f"lfa_host_reduce_tree({op},{dt})")
