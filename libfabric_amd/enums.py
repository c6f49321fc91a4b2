"""ABI enum values (identical to include/lfa_fabric.h and libfabric's
include/rdma/fi_domain.h:224-289)."""
import enum

import torch

LFA_TREE_MAX = 32


class DT(enum.IntEnum):
    INT8 = 0
    UINT8 = 1
    INT16 = 2
    UINT16 = 3
    INT32 = 4
    UINT32 = 5
    INT64 = 6
    UINT64 = 7
    FLOAT = 8
    DOUBLE = 9
    FLOAT_COMPLEX = 10
    DOUBLE_COMPLEX = 11
    LONG_DOUBLE = 12
    LONG_DOUBLE_COMPLEX = 13
    INT128 = 14
    UINT128 = 15


class OP(enum.IntEnum):
    MIN = 0
    MAX = 1
    SUM = 2
    PROD = 3
    LOR = 4
    LAND = 5
    BOR = 6
    BAND = 7
    LXOR = 8
    BXOR = 9
    ATOMIC_READ = 10
    ATOMIC_WRITE = 11


class COLL(enum.IntEnum):
    BARRIER = 0
    BROADCAST = 1
    ALLTOALL = 2
    ALLREDUCE = 3
    ALLGATHER = 4
    REDUCE_SCATTER = 5
    REDUCE = 6
    SCATTER = 7
    GATHER = 8


SIZES = {DT.INT8: 1, DT.UINT8: 1, DT.INT16: 2, DT.UINT16: 2, DT.INT32: 4,
         DT.UINT32: 4, DT.INT64: 8, DT.UINT64: 8, DT.FLOAT: 4, DT.DOUBLE: 8,
         DT.FLOAT_COMPLEX: 8, DT.DOUBLE_COMPLEX: 16, DT.LONG_DOUBLE: 16,
         DT.LONG_DOUBLE_COMPLEX: 32, DT.INT128: 16, DT.UINT128: 16}

_TORCH = {
    torch.int8: DT.INT8, torch.uint8: DT.UINT8, torch.int16: DT.INT16,
    torch.uint16: DT.UINT16, torch.int32: DT.INT32, torch.uint32: DT.UINT32,
    torch.int64: DT.INT64, torch.uint64: DT.UINT64, torch.float32: DT.FLOAT,
    torch.float64: DT.DOUBLE, torch.complex64: DT.FLOAT_COMPLEX,
    torch.complex128: DT.DOUBLE_COMPLEX,
}
_TORCH_INV = {v: k for k, v in _TORCH.items()}


def datatype_of_torch(dtype: torch.dtype) -> DT:
    try:
        return _TORCH[dtype]
    except KeyError:
        raise TypeError(f"no fi_datatype for {dtype}") from None


def torch_dtype_of(dt: int) -> torch.dtype:
    """Storage dtype for a datatype (128-bit ints are carried as uint8)."""
    return _TORCH_INV.get(DT(dt), torch.uint8)
