"""libfabric_amd — MI355X-native libfabric collective reduction path.

The product is native code:
  * ``liblfa.so``       gfx950 combine kernels behind a C ABI
                        (include/lfa_atomic.h — the ofi_atomic_write_handlers
                        drop-in, prov/util/src/util_atomic.c:907-922);
  * ``liblfa_coll.so``  the C host provider behind the fi_ops_collective
                        surface (include/lfa_coll.h — prov/coll's allreduce /
                        reduce / reduce_scatter / query / join / barrier).
This Python package only loads them (ctypes) and adapts torch tensors for
tests and bench.py.  There is no CPU fallback: without the built libraries
every entry point raises ``NativeLibraryMissing``.
"""
from .enums import (DT, OP, COLL, LFA_TREE_MAX, datatype_of_torch,  # noqa: F401
                    torch_dtype_of)
from ._native import NativeLibraryMissing, lib, lib_path  # noqa: F401
from . import atomic  # noqa: F401

__all__ = ["DT", "OP", "COLL", "atomic", "lib", "lib_path",
           "NativeLibraryMissing", "datatype_of_torch", "torch_dtype_of"]
