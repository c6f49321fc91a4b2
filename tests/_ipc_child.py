"""Child process of test_coll_gpu.py::test_p2p_kernel_on_ipc_mapped_memory.

Maps the parent's device buffer through hipIpcOpenMemHandle (the mapping
LFA_ALGO_P2P builds between ranks) and runs the P2P kernel,
lfa_reduce_tree_put_async, on it: inputs read from, outputs written to the
parent's allocation.  argv: handle-hex nsrc ndst count dt op in_stride out_off
"""
import ctypes
import sys


class IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def main() -> int:
    from libfabric_amd import _native
    L = _native.lib()
    h = IpcHandle()
    ctypes.memmove(ctypes.byref(h), bytes.fromhex(sys.argv[1]), 64)
    nsrc, ndst, count, dt, op, stride, out_off = map(int, sys.argv[2:9])
    base = ctypes.c_void_p()
    L.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle,
                                      ctypes.c_uint]
    rc = L.hipIpcOpenMemHandle(ctypes.byref(base), h, 1)  # LazyEnablePeerAccess
    if rc != 0:
        print(f"hipIpcOpenMemHandle -> {rc}", flush=True)
        return 3
    b = base.value
    srcs = (ctypes.c_void_p * nsrc)(*[b + k * stride for k in range(nsrc)])
    dsts = (ctypes.c_void_p * ndst)(*[b + out_off + j * stride for j in range(ndst)])
    rc = L.lfa_reduce_tree_put_async(op, dt, dsts, ndst, srcs, nsrc, count, None)
    sync = L.hipDeviceSynchronize()
    L.hipIpcCloseMemHandle(ctypes.c_void_p(b))
    print(f"tree_put rc={rc} sync={sync}", flush=True)
    return 0 if rc == 0 and sync == 0 else 4


if __name__ == "__main__":
    sys.exit(main())
