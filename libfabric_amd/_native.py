"""ctypes binding of the native libraries.  Fails loudly when missing.

``import torch`` happens first on purpose: torch bundles its own
libamdhip64.so / librccl.so with the same SONAMEs as /opt/rocm's.  Loading
torch first makes liblfa*.so bind to the already-loaded runtime, so device
pointers from torch's allocator and our kernels share one HIP context.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL loads below)

PKG = os.path.dirname(os.path.abspath(__file__))
_LIBS = {"lfa": "liblfa.so", "coll": "liblfa_coll.so",
         "tune": "liblfa_tune.so",    # tuning forms: bench.py --tune* only
         "bench": "liblfa_bench.so"}  # C latency loop: bench.py only
_loaded = {}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name: str = "lfa") -> str:
    return os.path.join(PKG, _LIBS[name])


def _bind_lfa(L):
    c_int, c_size_t, c_void_p, c_uint64 = (ctypes.c_int, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_uint64)
    L.lfa_datatype_size.restype = c_size_t
    L.lfa_datatype_size.argtypes = [c_int]
    L.lfa_atomic_valid.restype = c_int
    L.lfa_atomic_valid.argtypes = [c_int, c_int, c_uint64]
    L.lfa_atomic_last_error.restype = c_int
    L.lfa_atomic_last_error.argtypes = []
    L.lfa_atomic_write_async.restype = c_int
    L.lfa_atomic_write_async.argtypes = [c_int, c_int, c_void_p, c_void_p,
                                         c_size_t, c_void_p]
    L.lfa_reduce_tree_async.restype = c_int
    L.lfa_reduce_tree_async.argtypes = [c_int, c_int, c_void_p,
                                        ctypes.POINTER(c_void_p), c_int,
                                        c_size_t, c_void_p]
    L.lfa_reduce_tree_put_async.restype = c_int
    L.lfa_reduce_tree_put_async.argtypes = [c_int, c_int, ctypes.POINTER(c_void_p), c_int,
                                            ctypes.POINTER(c_void_p), c_int, c_size_t,
                                            c_void_p]
    L.lfa_atomic_readwrite_async.restype = c_int
    L.lfa_atomic_readwrite_async.argtypes = [c_int, c_int, c_void_p, c_void_p,
                                             c_void_p, c_size_t, c_void_p]
    L.lfa_atomic_swap_async.restype = c_int
    L.lfa_atomic_swap_async.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_size_t, c_void_p]
    L.lfa_atomic_write_staged.restype = c_int
    L.lfa_atomic_write_staged.argtypes = [c_int, c_int, c_void_p, c_void_p, c_size_t,
                                          c_size_t]
    L.lfa_version.restype = ctypes.c_char_p
    L.lfa_host_small_bytes.restype = c_size_t
    L.lfa_host_write.restype = c_int
    L.lfa_host_write.argtypes = [c_int, c_int, c_void_p, c_void_p, c_size_t]
    L.lfa_host_reduce_tree.restype = c_int
    L.lfa_host_reduce_tree.argtypes = [c_int, c_int, c_void_p, ctypes.POINTER(c_void_p),
                                       c_int, c_size_t]


def _bind_tune(L):
    c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    L.lfa__tune_tree_f32.restype = c_int
    L.lfa__tune_tree_f32.argtypes = [c_int, c_void_p, ctypes.POINTER(c_void_p),
                                     c_int, c_size_t, c_void_p]
    L.lfa__tune_treeput_f32.restype = c_int
    L.lfa__tune_treeput_f32.argtypes = [c_int, ctypes.POINTER(c_void_p), c_int,
                                        ctypes.POINTER(c_void_p), c_int, c_size_t, c_void_p]
    L.lfa__tp_probe.restype = c_int
    L.lfa__tp_probe.argtypes = [c_int, ctypes.POINTER(c_void_p), c_int,
                                ctypes.POINTER(c_void_p), c_int, c_size_t, c_void_p]
    L.lfa__tune_treeput_u.restype = c_int
    L.lfa__tune_treeput_u.argtypes = [c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_int,
                                      ctypes.POINTER(c_void_p), c_int, c_size_t, c_void_p]
    for fn in (L.lfa__tune_sum_f32, L.lfa__tune2_sum_f32, L.lfa__tune3_sum_f32):
        fn.restype = c_int
        fn.argtypes = [c_int, c_void_p, c_void_p, c_size_t, c_void_p]
    L.lfa__tune_fetch_f32.restype = c_int
    L.lfa__tune_fetch_f32.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_size_t, c_void_p]
    L.lfa__tune_stream.restype = c_int
    L.lfa__tune_stream.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    L.lfa__tune_read_n.restype = c_int
    L.lfa__tune_read_n.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p, c_size_t,
                                   c_void_p]


def lib(name: str = "lfa") -> ctypes.CDLL:
    """The loaded native library; raises NativeLibraryMissing if not built."""
    if name in _loaded:
        return _loaded[name]
    path = lib_path(name)
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} is not built: run `python -m libfabric_amd.build` "
            "(there is no CPU fallback for the combine path)")
    if name == "coll":
        lib("lfa")
    if name == "bench":
        lib("coll")
    L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    if name == "lfa":
        _bind_lfa(L)
    elif name == "tune":
        _bind_tune(L)
    elif name == "bench":
        c = ctypes
        L.lfa_bench_loop.restype = c.c_int
        L.lfa_bench_loop.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_size_t,
                                     c.c_int, c.c_int, c.c_int, c.c_uint64, c.c_int, c.c_int,
                                     c.POINTER(c.c_double)]
        L.lfa_bench_samples.restype = c.c_int
        L.lfa_bench_samples.argtypes = L.lfa_bench_loop.argtypes
    _loaded[name] = L
    return L
