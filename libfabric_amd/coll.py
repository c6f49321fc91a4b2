"""ctypes front end of the collective provider (liblfa_coll.so, include/lfa_coll.h).

The provider is C; this module only marshals arguments:

  plan(...)        lfa_coll_plan — a rank's schedule as data (host only)
  block(...)       lfa_coll_block — reduce_scatter block bounds
  host_chunks(...) lfa_coll_host_chunk — host-buffer staging geometry
  loopback(...)    lfa_coll_loopback — all ranks' schedules on ONE GPU
  Endpoint         domain + endpoint over RCCL; fi_ops_collective calls
                   (allreduce, reduce_scatter, reduce, allgather, broadcast,
                   barrier), join, query, cq_read — prov/coll's surface
                   (include/rdma/fi_collective.h:92-139).

Bootstrap: rank 0 creates the RCCL unique id (lfa_coll_get_unique_id) and
ships it to the other ranks over torch.distributed's store/gloo group.
"""
from __future__ import annotations

import ctypes
import sys
from dataclasses import dataclass

import numpy as np
import torch

from ._native import lib as _lib
from .enums import COLL, DT, OP, SIZES

c_int, c_size_t, c_void_p, c_uint64, c_uint32, c_int32 = (
    ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64,
    ctypes.c_uint32, ctypes.c_int32)
c_ssize_t = ctypes.c_ssize_t

ALGO_TREE, ALGO_RD, ALGO_RCCL, ALGO_TREE_COLL, ALGO_P2P, ALGO_AUTO = 0, 1, 2, 3, 4, 5
GROUP_CHUNK_AUTO = (1 << 64) - 1   # lfa_coll.h LFA_GROUP_CHUNK_AUTO, the default
AUTO_CHUNK_BYTES = 32 << 20        # lfa_coll.h LFA_AUTO_CHUNK_BYTES
(STEP_SEND, STEP_RECV, STEP_GROUP_END, STEP_REDUCE, STEP_TREE, STEP_COPY,
 STEP_ALLTOALL, STEP_ALLGATHER, STEP_BARRIER, STEP_TREE_PUT, STEP_ONESHOT) = range(11)
BUF_SEND, BUF_RESULT, BUF_TMP, BUF_SYM_IN, BUF_SYM_OUT = 0, 1, 2, 3, 4
ADDR_NOTAVAIL = (1 << 64) - 1
EAGAIN, EIO = 11, 5
JOIN_COMPLETE = 6
UNIQUE_ID_BYTES = 128


class Ref(ctypes.Structure):
    _fields_ = [("buf", c_int32), ("rank", c_uint32), ("off", c_uint64)]


class Step(ctypes.Structure):
    _fields_ = [("type", c_int32), ("peer", c_int32), ("count", c_uint64),
                ("dst", Ref), ("src", Ref), ("first", c_uint32),
                ("nsrc", c_uint32)]


class AtomicAttr(ctypes.Structure):
    _fields_ = [("count", c_size_t), ("size", c_size_t)]


class CollectiveAttr(ctypes.Structure):
    _fields_ = [("op", c_int), ("datatype", c_int),
                ("datatype_attr", AtomicAttr), ("max_members", c_size_t),
                ("mode", c_uint64)]


class CqEntry(ctypes.Structure):
    _fields_ = [("op_context", c_void_p), ("flags", c_uint64), ("len", c_size_t),
                ("buf", c_void_p), ("data", c_uint64)]


class CqErrEntry(ctypes.Structure):
    _fields_ = [("op_context", c_void_p), ("flags", c_uint64), ("err", c_int),
                ("prov_errno", c_int)]


class EqEntry(ctypes.Structure):
    _fields_ = [("fid", c_void_p), ("context", c_void_p), ("data", c_uint64)]


_bound = False


def lib() -> ctypes.CDLL:
    global _bound
    L = _lib("coll")
    if _bound:
        return L
    P = ctypes.POINTER
    L.lfa_coll_plan.restype = c_int
    L.lfa_coll_plan.argtypes = [c_int, c_int, c_int, c_int, c_int, c_size_t,
                                c_size_t, P(Step), P(c_size_t), P(Ref),
                                P(c_size_t), P(c_size_t)]
    L.lfa_coll_host_chunk.restype = c_int
    L.lfa_coll_host_chunk.argtypes = [c_int, c_size_t, c_int, c_size_t, c_size_t,
                                      c_size_t, P(HostChunk)]
    L.lfa_coll_block.restype = None
    L.lfa_coll_block.argtypes = [c_size_t, c_int, c_int, P(c_size_t), P(c_size_t)]
    L.lfa_coll_loopback.restype = c_int
    L.lfa_coll_loopback.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_size_t, P(c_void_p), P(c_void_p), c_void_p]
    L.lfa_coll_get_unique_id.restype = c_int
    L.lfa_coll_get_unique_id.argtypes = [c_void_p, c_size_t]
    L.lfa_coll_domain_open.restype = c_int
    L.lfa_coll_domain_open.argtypes = [c_int, c_int, c_int, c_void_p, c_size_t,
                                       P(c_void_p)]
    L.lfa_coll_domain_open_host.restype = c_int
    L.lfa_coll_domain_open_host.argtypes = [c_int, c_int, P(PeerXferOps), c_void_p,
                                            P(c_void_p)]
    L.lfa_coll_domain_open_peer.restype = c_int
    L.lfa_coll_domain_open_peer.argtypes = [c_int] + L.lfa_coll_domain_open_host.argtypes
    L.lfa_mc_group_id.restype = c_int
    L.lfa_mc_group_id.argtypes = [c_void_p]
    L.lfa_mc_counters.restype = c_int
    L.lfa_mc_counters.argtypes = [c_void_p, c_uint64, P(McCounters)]
    L.lfa_mc_seed_ticket.restype = c_int
    L.lfa_mc_seed_ticket.argtypes = [c_void_p, c_uint64, c_uint64]
    L.lfa_mc_ws_info.restype = c_int
    L.lfa_mc_ws_info.argtypes = [c_void_p, c_uint64, P(WsInfo)]
    L.lfa_coll_ep_test_solo.restype = c_int
    L.lfa_coll_ep_test_solo.argtypes = [c_void_p, c_size_t]
    L.lfa_coll_ws_mem.restype = c_int
    L.lfa_coll_ws_mem.argtypes = []
    L.lfa_coll_ep_test_word.restype = c_int
    L.lfa_coll_ep_test_word.argtypes = [c_void_p, c_int, ctypes.c_long, c_int]
    L.lfa_coll_ep_uses_direct.restype = c_int
    L.lfa_coll_ep_uses_direct.argtypes = [c_void_p]
    L.lfa_coll_ep_word_ops.restype = c_uint64
    L.lfa_coll_ep_word_ops.argtypes = [c_void_p]
    L.lfa_coll_domain_close.restype = c_int
    L.lfa_coll_domain_close.argtypes = [c_void_p]
    L.lfa_coll_domain_comm_count.restype = c_int
    L.lfa_coll_domain_comm_count.argtypes = [c_void_p, P(c_int)]
    L.lfa_coll_ep_open.restype = c_int
    L.lfa_coll_ep_open.argtypes = [c_void_p, P(c_void_p)]
    L.lfa_coll_ep_close.restype = c_int
    L.lfa_coll_ep_close.argtypes = [c_void_p]
    L.lfa_coll_ep_stream.restype = c_void_p
    L.lfa_coll_ep_stream.argtypes = [c_void_p]
    L.lfa_coll_ep_set_algo.restype = c_int
    L.lfa_coll_ep_set_algo.argtypes = [c_void_p, c_int]
    L.lfa_coll_ep_set_chunk.restype = c_int
    L.lfa_coll_ep_set_chunk.argtypes = [c_void_p, c_size_t]
    L.lfa_coll_ep_set_group_chunk.restype = c_int
    L.lfa_coll_ep_set_group_chunk.argtypes = [c_void_p, c_size_t]
    L.lfa_coll_auto_algo.restype = c_int
    L.lfa_coll_auto_algo.argtypes = [c_int, c_size_t, c_int, c_size_t, c_int]
    L.lfa_coll_auto_bulk.restype = c_int
    L.lfa_coll_auto_bulk.argtypes = []
    L.lfa_coll_member_chunk.restype = c_size_t
    L.lfa_coll_member_chunk.argtypes = [c_int, c_int, c_size_t, c_size_t]
    L.lfa_coll_group_chunk.restype = c_size_t
    L.lfa_coll_group_chunk.argtypes = [c_size_t, c_int, c_size_t]
    L.lfa_coll_ep_flush.restype = c_int
    L.lfa_coll_ep_flush.argtypes = [c_void_p]
    L.lfa_coll_ep_stage_bytes.restype = c_size_t
    L.lfa_coll_ep_stage_bytes.argtypes = [c_void_p]
    L.lfa_coll_ws_cached_bytes.restype = c_size_t
    L.lfa_coll_ws_cached_bytes.argtypes = []
    L.lfa_coll_ws_quarantined_bytes.restype = c_size_t
    L.lfa_coll_ws_quarantined_bytes.argtypes = []
    L.lfa_coll_world_addr.restype = c_uint64
    L.lfa_coll_world_addr.argtypes = [c_void_p]
    L.lfa_join_collective.restype = c_int
    L.lfa_join_collective.argtypes = [c_void_p, c_uint64, P(c_int), c_size_t,
                                      c_uint64, P(c_void_p), c_void_p]
    L.lfa_join_members.restype = c_int
    L.lfa_join_members.argtypes = L.lfa_join_collective.argtypes
    L.lfa_mc_addr.restype = c_uint64
    L.lfa_mc_addr.argtypes = [c_void_p]
    L.lfa_mc_close.restype = c_int
    L.lfa_mc_close.argtypes = [c_void_p]
    for name in ("lfa_allreduce", "lfa_reduce_scatter", "lfa_allgather"):
        f = getattr(L, name)
        f.restype = c_ssize_t
    L.lfa_allreduce.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                c_void_p, c_uint64, c_int, c_int, c_uint64, c_void_p]
    L.lfa_reduce_scatter.argtypes = L.lfa_allreduce.argtypes
    L.lfa_reduce.restype = c_ssize_t
    L.lfa_reduce.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                             c_void_p, c_uint64, c_uint64, c_int, c_int, c_uint64,
                             c_void_p]
    L.lfa_allgather.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                c_void_p, c_uint64, c_int, c_uint64, c_void_p]
    L.lfa_scatter.restype = c_ssize_t
    L.lfa_scatter.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                              c_void_p, c_uint64, c_uint64, c_int, c_uint64, c_void_p]
    L.lfa_broadcast.restype = c_ssize_t
    L.lfa_broadcast.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_uint64,
                                c_uint64, c_int, c_uint64, c_void_p]
    L.lfa_barrier.restype = c_ssize_t
    L.lfa_barrier.argtypes = [c_void_p, c_uint64, c_void_p]
    L.lfa_query_collective.restype = c_int
    L.lfa_query_collective.argtypes = [c_void_p, c_int, P(CollectiveAttr), c_uint64]
    L.lfa_cq_read.restype = c_ssize_t
    L.lfa_cq_read.argtypes = [c_void_p, P(CqEntry), c_size_t]
    L.lfa_cq_readerr.restype = c_ssize_t
    L.lfa_cq_readerr.argtypes = [c_void_p, P(CqErrEntry)]
    L.lfa_eq_read.restype = c_ssize_t
    L.lfa_eq_read.argtypes = [c_void_p, P(c_uint32), P(EqEntry)]
    _bound = True
    return L


XferPost = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, c_void_p, c_size_t, c_uint64,
                            ctypes.POINTER(c_void_p))
XferTest = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p)


class PeerXferOps(ctypes.Structure):
    """struct lfa_peer_xfer_ops: the owner's tagged transport (FI_PEER_TRANSFER)."""
    _fields_ = [("send", XferPost), ("recv", XferPost), ("test", XferTest)]


class HostChunk(ctypes.Structure):
    _fields_ = [("src_off", c_size_t), ("src_pitch", c_size_t), ("width", c_size_t),
                ("height", c_size_t), ("dev_count", c_size_t), ("dst_off", c_size_t)]


class CollError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} -> {rc}")
        self.rc = rc


def _chk(rc: int, what: str) -> int:
    if rc < 0:
        raise CollError(rc, what)
    return rc


# ------------------------------------------------------------- schedules --

@dataclass
class Plan:
    steps: list
    refs: list
    tmp_bytes: int


def plan(coll: int, algo: int, rank: int, nranks: int, root: int, count: int,
         esz: int) -> Plan:
    L = lib()
    ns, nr, tmp = c_size_t(0), c_size_t(0), c_size_t(0)
    _chk(L.lfa_coll_plan(coll, algo, rank, nranks, root, count, esz, None,
                         ctypes.byref(ns), None, ctypes.byref(nr),
                         ctypes.byref(tmp)), "lfa_coll_plan(size)")
    steps = (Step * max(ns.value, 1))()
    refs = (Ref * max(nr.value, 1))()
    _chk(L.lfa_coll_plan(coll, algo, rank, nranks, root, count, esz, steps,
                         ctypes.byref(ns), refs, ctypes.byref(nr),
                         ctypes.byref(tmp)), "lfa_coll_plan")
    def tup(r):
        # symmetric-workspace refs also name the owning group rank
        return (r.buf, r.off, r.rank) if r.buf in (BUF_SYM_IN, BUF_SYM_OUT) else (r.buf, r.off)

    out = []
    for s in steps[:ns.value]:
        out.append({"type": s.type, "peer": s.peer, "count": s.count,
                    "dst": tup(s.dst), "src": tup(s.src),
                    "first": s.first, "nsrc": s.nsrc})
    return Plan(out, [tup(r) for r in refs[:nr.value]], tmp.value)


def auto_algo(coll: int, count: int, nranks: int, esz: int, p2p_ok: bool = True) -> int:
    """lfa_coll_auto_algo: LFA_ALGO_AUTO's choice for one operation."""
    return lib().lfa_coll_auto_algo(coll, count, nranks, esz, int(p2p_ok))


def auto_bulk() -> int:
    """lfa_coll_auto_bulk: AUTO's choice above the one-shot bounds
    (ALGO_P2P by default, ALGO_TREE with LFA_AUTO_BULK=tree)."""
    return lib().lfa_coll_auto_bulk()


def group_chunk(setting: int, nranks: int, nbytes: int) -> int:
    """lfa_coll_group_chunk: the group chunk an operation of `nbytes` runs
    with under `setting` (GROUP_CHUNK_AUTO, 0 or a size)."""
    return lib().lfa_coll_group_chunk(setting, nranks, nbytes)


def sig_area_bytes() -> int:
    """LFA_SIG_AREA_BYTES: the flag area that ends every P2P workspace (flag
    rows, LL one-shot words, identity word) — for a workspace built by hand."""
    from ._native import lib as native
    f = native("lfa").lfa__sig_area_bytes
    f.restype = ctypes.c_size_t
    return f()


def ws_cached_bytes() -> int:
    """lfa_coll_ws_cached_bytes: released P2P workspaces kept for reuse."""
    return lib().lfa_coll_ws_cached_bytes()


def ws_quarantined_bytes() -> int:
    """lfa_coll_ws_quarantined_bytes: released P2P workspaces held, never reused."""
    return lib().lfa_coll_ws_quarantined_bytes()


def member_chunk(nranks: int, host: bool, group_chunk: int, local_chunk: int) -> int:
    """lfa_coll_member_chunk: the chunk a member stages an operation with."""
    return lib().lfa_coll_member_chunk(nranks, int(host), group_chunk, local_chunk)


def host_chunks(coll: int, count: int, nranks: int, esz: int,
                chunk_bytes: int) -> list[HostChunk]:
    """lfa_coll_host_chunk for every chunk: the staging geometry the provider
    uses for host-memory buffers."""
    out, idx = [], 0
    while True:
        c = HostChunk()
        rc = lib().lfa_coll_host_chunk(coll, count, nranks, esz, chunk_bytes, idx,
                                       ctypes.byref(c))
        if rc < 0:
            raise CollError(rc, "lfa_coll_host_chunk")
        if rc == 0:
            return out
        out.append(c)
        idx += 1


def block(count: int, nranks: int, r: int) -> tuple[int, int]:
    off, ln = c_size_t(0), c_size_t(0)
    lib().lfa_coll_block(count, nranks, r, ctypes.byref(off), ctypes.byref(ln))
    return off.value, ln.value


def loopback(coll: int, algo: int, nranks: int, root: int, dt: int, op: int,
             count: int, sends: list[torch.Tensor], results: list[torch.Tensor],
             stream=None) -> None:
    """Run all ranks' schedules on the current GPU (device tensors)."""
    sp = (c_void_p * nranks)(*[t.data_ptr() if t is not None else None for t in sends])
    rp = (c_void_p * nranks)(*[t.data_ptr() if t is not None else None for t in results])
    h = (stream or torch.cuda.current_stream()).cuda_stream
    _chk(lib().lfa_coll_loopback(coll, algo, nranks, root, dt, op, count, sp, rp, h),
         "lfa_coll_loopback")


# -------------------------------------------------------------- endpoint --

def _ptr(x) -> int | None:
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        if x.nbytes and x.flags.writeable and x.flags.c_contiguous:
            # ~1 us against ~3 us for x.ctypes.data (numpy builds a helper
            # object per access): this runs twice per submitted collective
            return ctypes.addressof(ctypes.c_char.from_buffer(x))
        return x.ctypes.data
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return int(x)


class McCounters(ctypes.Structure):
    """struct lfa_mc_counters (include/lfa_coll.h)."""
    _fields_ = [("p2p_ops", ctypes.c_uint64), ("oneshot", ctypes.c_uint64),
                ("flag_barriers", ctypes.c_uint64), ("timed_out", ctypes.c_int)]


class WsInfo(ctypes.Structure):
    """struct lfa_ws_info (include/lfa_coll.h)."""
    _fields_ = [("mem", ctypes.c_int), ("mapped", ctypes.c_int),
                ("region", ctypes.c_size_t), ("alloc_flags", ctypes.c_uint * 32)]


WS_MEM = {0: "coarse", 1: "fine", 3: "uncached"}   # hipDeviceMalloc* flags


def ws_mem() -> str:
    """lfa_coll_ws_mem: the kind P2P workspaces are allocated as (LFA_WS_MEM)."""
    return WS_MEM.get(lib().lfa_coll_ws_mem(), "other")


class OneShot(ctypes.Structure):
    """struct lfa_oneshot (libfabric_amd/csrc/lfa_signal.h): one rank's
    one-shot reduction over the members' symmetric workspaces."""
    _fields_ = [("send", ctypes.c_void_p), ("result", ctypes.c_void_p),
                ("count", ctypes.c_size_t), ("mode", ctypes.c_int),
                ("sym", ctypes.c_void_p), ("slot_bytes", ctypes.c_size_t),
                ("parity_off", ctypes.c_size_t), ("flag_off", ctypes.c_size_t), ("n", ctypes.c_int), ("rank", ctypes.c_int),
                ("epoch", ctypes.c_uint32), ("status", ctypes.c_void_p),
                ("ticket", ctypes.c_uint64), ("timeout_us", ctypes.c_uint64),
                ("done_ctr", ctypes.c_void_p), ("done_word", ctypes.c_void_p),
                ("done_val", ctypes.c_uint64)]


SIG_NONE = 0xFFFFFFFFFFFFFFFF   # lfa_signal.h LFA_SIG_NONE: no wait of the group timed out


def oneshot_reduce(op: int, dt: int, a: OneShot, stream) -> None:
    """lfa_oneshot_reduce_async (liblfa.so): the LFA_STEP_ONESHOT kernel
    launched directly, for probes and benches that lay out the workspaces
    themselves (the provider does this inside its executor)."""
    L = _lib()
    if not getattr(L, "_oneshot_bound", False):
        L.lfa_oneshot_reduce_async.restype = ctypes.c_int
        L.lfa_oneshot_reduce_async.argtypes = [ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(OneShot), ctypes.c_void_p]
        L._oneshot_bound = True
    h = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    _chk(L.lfa_oneshot_reduce_async(op, dt, ctypes.byref(a), ctypes.c_void_p(h)),
         "lfa_oneshot_reduce_async")


class Endpoint:
    """One rank's domain + endpoint.  Buffers: torch tensors (device or host)
    or numpy arrays (host).  Calls return after enqueueing; completions come
    from cq_read()/wait() with the context value passed in."""

    def __init__(self, rank: int, nranks: int, device: int, uid: bytes):
        L = lib()
        self.rank, self.nranks, self.device = rank, nranks, device
        self.dom, self.ep = c_void_p(), c_void_p()
        buf = ctypes.create_string_buffer(uid, UNIQUE_ID_BYTES)
        _chk(L.lfa_coll_domain_open(device, rank, nranks, buf, UNIQUE_ID_BYTES,
                                    ctypes.byref(self.dom)), "domain_open")
        _chk(L.lfa_coll_ep_open(self.dom, ctypes.byref(self.ep)), "ep_open")
        self.world = L.lfa_coll_world_addr(self.ep)
        self._ctx = 0
        self._fast_init()

    def _fast_init(self) -> None:
        # the per-call path (submit, cq_read, wait) without re-resolving the
        # library or allocating a completion array per poll: the C calls
        # cost ~0.7 us per operation, the Python around them dominated
        self._L = lib()
        self._ents = (CqEntry * 16)()

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        _chk(lib().lfa_coll_get_unique_id(buf, UNIQUE_ID_BYTES), "get_unique_id")
        return buf.raw

    @classmethod
    def from_torch_dist(cls, device: int | None = None) -> "Endpoint":
        """Bootstrap over an initialised torch.distributed group."""
        import torch.distributed as dist
        if not dist.is_initialized():
            return cls(0, 1, device or 0, cls.unique_id())
        rank, world = dist.get_rank(), dist.get_world_size()
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(rank, world, torch.cuda.current_device() if device is None
                   else device, obj[0])

    def group_id(self, mc: int) -> int:
        return lib().lfa_mc_group_id(mc)

    def counters(self, coll_addr: int | None = None) -> dict:
        """lfa_mc_counters: which P2P paths the group's operations took."""
        c = McCounters()
        _chk(lib().lfa_mc_counters(self.ep, coll_addr or self.world, ctypes.byref(c)),
             "lfa_mc_counters")
        return {k: getattr(c, k) for k, _ in McCounters._fields_}

    def flush(self) -> None:
        """lfa_coll_ep_flush: every queued operation completed (peer domains:
        idle staging buffers freed)."""
        _chk(lib().lfa_coll_ep_flush(self.ep), "lfa_coll_ep_flush")

    def stage_bytes(self) -> int:
        """lfa_coll_ep_stage_bytes: device bytes in the staging pool."""
        return lib().lfa_coll_ep_stage_bytes(self.ep)

    def ws_info(self, coll_addr: int | None = None) -> dict:
        """lfa_mc_ws_info: the group's P2P workspaces as mapped here."""
        w = WsInfo()
        _chk(lib().lfa_mc_ws_info(self.ep, coll_addr or self.world, ctypes.byref(w)),
             "lfa_mc_ws_info")
        return {"mem": WS_MEM.get(w.mem, "other"), "mapped": w.mapped, "region": w.region,
                "alloc_flags": list(w.alloc_flags[:max(w.mapped, 0)])}

    def test_solo(self, max_bytes: int) -> None:
        """lfa_coll_ep_test_solo (test entry): one-member reducing collectives
        above max_bytes leave the solo copy for the algorithm's schedule."""
        _chk(lib().lfa_coll_ep_test_solo(self.ep, max_bytes), "lfa_coll_ep_test_solo")

    def seed_ticket(self, ticket: int, coll_addr: int | None = None) -> None:
        """lfa_mc_seed_ticket (test entry): the group's P2P tickets continue
        from `ticket`; every member seeds the same value."""
        _chk(lib().lfa_mc_seed_ticket(self.ep, coll_addr or self.world, ticket),
             "lfa_mc_seed_ticket")

    def test_word(self, drop_next: int = 0, timeout_ms: int = 0,
                  fail_direct: bool = False) -> None:
        """lfa_coll_ep_test_word (test entry): the next `drop_next` word
        operations wait for a value their word never reaches; timeout_ms > 0
        bounds this endpoint's word waits; fail_direct marks its direct queue
        failed."""
        _chk(lib().lfa_coll_ep_test_word(self.ep, drop_next, timeout_ms, int(fail_direct)),
             "lfa_coll_ep_test_word")

    def uses_direct(self) -> int:
        """lfa_coll_ep_uses_direct: 1 direct queue in use, 2 failed, 0 none."""
        return _chk(lib().lfa_coll_ep_uses_direct(self.ep), "lfa_coll_ep_uses_direct")

    def rccl_nranks(self) -> int:
        """lfa_coll_domain_comm_count: ranks in the domain's RCCL communicator
        (ncclCommCount); raises CollError on a peer-transfer domain."""
        n = c_int(0)
        _chk(lib().lfa_coll_domain_comm_count(self.dom, ctypes.byref(n)),
             "lfa_coll_domain_comm_count")
        return n.value

    def word_ops(self) -> int:
        """lfa_coll_ep_word_ops: operations reaped through a completion word."""
        return lib().lfa_coll_ep_word_ops(self.ep)

    def cq_readerr(self):
        """lfa_cq_readerr: (err, prov_errno, op_context) of the pending error
        entry, or None."""
        e = CqErrEntry()
        n = lib().lfa_cq_readerr(self.ep, ctypes.byref(e))
        if n == -EAGAIN:
            return None
        _chk(n, "lfa_cq_readerr")
        return e.err, e.prov_errno, e.op_context

    def close(self) -> None:
        L = lib()
        if self.ep:
            L.lfa_coll_ep_close(self.ep)
            self.ep = c_void_p()
        if self.dom:
            L.lfa_coll_domain_close(self.dom)
            self.dom = c_void_p()

    # configuration
    def set_algo(self, algo: int) -> None:
        _chk(lib().lfa_coll_ep_set_algo(self.ep, algo), "set_algo")

    def set_chunk(self, nbytes: int) -> None:
        _chk(lib().lfa_coll_ep_set_chunk(self.ep, nbytes), "set_chunk")

    def set_group_chunk(self, nbytes: int) -> None:
        """lfa_coll_ep_set_group_chunk: the same value on every member."""
        _chk(lib().lfa_coll_ep_set_group_chunk(self.ep, nbytes), "set_group_chunk")

    @property
    def stream_handle(self) -> int:
        return lib().lfa_coll_ep_stream(self.ep)

    def _next_ctx(self) -> int:
        self._ctx += 1
        return self._ctx

    # fi_ops_collective
    def allreduce(self, buf, result, count: int, dt: int, op: int,
                  coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_allreduce(self.ep, _ptr(buf), count, None, _ptr(result),
                                 None, coll_addr or self.world, dt, op, 0, ctx),
             "lfa_allreduce")
        return ctx

    def reduce_scatter(self, buf, result, count: int, dt: int, op: int,
                       coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_reduce_scatter(self.ep, _ptr(buf), count, None, _ptr(result),
                                      None, coll_addr or self.world, dt, op, 0, ctx),
             "lfa_reduce_scatter")
        return ctx

    def reduce(self, buf, result, count: int, root: int, dt: int, op: int,
               coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_reduce(self.ep, _ptr(buf), count, None, _ptr(result), None,
                              coll_addr or self.world, root, dt, op, 0, ctx),
             "lfa_reduce")
        return ctx

    def allgather(self, buf, result, count: int, dt: int,
                  coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_allgather(self.ep, _ptr(buf), count, None, _ptr(result),
                                 None, coll_addr or self.world, dt, 0, ctx),
             "lfa_allgather")
        return ctx

    def scatter(self, buf, result, count: int, root: int, dt: int,
                coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_scatter(self.ep, _ptr(buf), count, None, _ptr(result), None,
                               coll_addr or self.world, root, dt, 0, ctx),
             "lfa_scatter")
        return ctx

    def broadcast(self, buf, count: int, root: int, dt: int,
                  coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_broadcast(self.ep, _ptr(buf), count, None,
                                 coll_addr or self.world, root, dt, 0, ctx),
             "lfa_broadcast")
        return ctx

    def barrier(self, coll_addr: int | None = None, context: int | None = None) -> int:
        ctx = context or self._next_ctx()
        _chk(self._L.lfa_barrier(self.ep, coll_addr or self.world, ctx), "lfa_barrier")
        return ctx

    def query(self, coll: int, op: int = OP.SUM, dt: int = DT.FLOAT,
              flags: int = 0, mode: int = 0) -> tuple[int, CollectiveAttr]:
        a = CollectiveAttr(op=op, datatype=dt, mode=mode)
        rc = lib().lfa_query_collective(self.dom, coll, ctypes.byref(a), flags)
        return rc, a

    def join(self, ranks: list[int] | None = None, context: int | None = None,
             coll_addr: int | None = None):
        mc = c_void_p()
        arr = (c_int * len(ranks))(*ranks) if ranks is not None else None
        ctx = context or self._next_ctx()
        _chk(lib().lfa_join_collective(self.ep, coll_addr or ADDR_NOTAVAIL, arr,
                                       len(ranks) if ranks else 0, 0,
                                       ctypes.byref(mc), ctx), "lfa_join_collective")
        return mc.value, ctx

    def join_members(self, ranks: list[int], context: int | None = None,
                     coll_addr: int | None = None):
        """lfa_join_members: the group of `ranks` formed by its members only
        (prov/coll's join over an av_set's own address; the other ranks of
        `coll_addr`'s group call nothing)."""
        mc = c_void_p()
        arr = (c_int * len(ranks))(*ranks)
        ctx = context or self._next_ctx()
        _chk(lib().lfa_join_members(self.ep, coll_addr or ADDR_NOTAVAIL, arr, len(ranks),
                                    0, ctypes.byref(mc), ctx), "lfa_join_members")
        return mc.value, ctx

    def mc_addr(self, mc: int) -> int:
        return lib().lfa_mc_addr(mc)

    def bench_loop(self, coll: int, buf, result, count: int, dt: int, op: int,
                   root: int = 0, reps: int = 200, coll_addr: int | None = None,
                   timeout_ms: int = 20000) -> float:
        """Bench only (liblfa_bench.so): `reps` of submit + poll-to-completion
        of one allreduce / reduce_scatter / reduce, timed in C; returns the
        mean microseconds per operation on this rank."""
        from ._native import lib as native
        us = ctypes.c_double()
        _chk(native("bench").lfa_bench_loop(self.ep, coll, _ptr(buf), _ptr(result), count,
                                            root, dt, op, coll_addr or self.world, reps,
                                            timeout_ms, ctypes.byref(us)), "lfa_bench_loop")
        return us.value

    def bench_samples(self, coll: int, buf, result, count: int, dt: int, op: int,
                      root: int = 0, reps: int = 200, coll_addr: int | None = None,
                      timeout_ms: int = 20000) -> list[float]:
        """Bench only (liblfa_bench.so lfa_bench_samples): the same loop as
        bench_loop, returning every operation's microseconds."""
        from ._native import lib as native
        out = (ctypes.c_double * reps)()
        _chk(native("bench").lfa_bench_samples(self.ep, coll, _ptr(buf), _ptr(result), count,
                                               root, dt, op, coll_addr or self.world, reps,
                                               timeout_ms, out), "lfa_bench_samples")
        return list(out)

    # completions
    def cq_read(self, max_entries: int = 16) -> list[int]:
        ents = self._ents if max_entries <= 16 else (CqEntry * max_entries)()
        n = self._L.lfa_cq_read(self.ep, ents, max_entries)
        if n == -EAGAIN:
            return []
        if n == -EIO:
            err = CqErrEntry()
            lib().lfa_cq_readerr(self.ep, ctypes.byref(err))
            raise CollError(-err.err, f"completion error (prov_errno {err.prov_errno})")
        _chk(n, "lfa_cq_read")
        return [ents[i].op_context for i in range(n)]

    def eq_read(self):
        ev, ent = c_uint32(0), EqEntry()
        n = lib().lfa_eq_read(self.ep, ctypes.byref(ev), ctypes.byref(ent))
        if n == -EAGAIN:
            return None
        _chk(n, "lfa_eq_read")
        return ev.value, ent.fid, ent.context

    def wait(self, ctx: int, timeout_s: float = 120.0) -> None:
        """Poll the CQ (the progress call) until `ctx` completes.  Other
        completions read meanwhile are dropped."""
        import time
        read, ep, ents = self._L.lfa_cq_read, self.ep, self._ents
        t0 = time.time()
        while True:
            n = read(ep, ents, 16)
            if n > 0:
                for i in range(n):
                    if ents[i].op_context == ctx:
                        return
            elif n != -EAGAIN:
                self.cq_read()          # the error path: raises CollError
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"collective {ctx} did not complete")

    def wait_join(self, timeout_s: float = 120.0):
        import time
        t0 = time.time()
        while True:
            e = self.eq_read()
            if e is not None:
                return e
            if time.time() - t0 > timeout_s:
                raise TimeoutError("join did not complete")


class TransportAgain(Exception):
    """Raised by a HostEndpoint transport's send/recv when the owner cannot
    take the transfer now (its queue is full): the provider retries the post
    on a later progress call, as prov/coll requeues a SEND that returned
    -FI_EAGAIN (coll_coll.c:845-852)."""


class HostEndpoint(Endpoint):
    """An endpoint of a peer-transfer domain (lfa_coll_domain_open_host):
    host-memory buffers, transfers through `transport` — an object with
    send(peer, ptr, nbytes, tag) -> handle, recv(peer, ptr, nbytes, tag) ->
    handle and test(handle) -> 1 done / 0 pending / <0 error — the way
    prov/coll rides on the owner provider's tagged messages."""

    def __init__(self, rank: int, nranks: int, transport, device: int = -1):
        """device >= 0: lfa_coll_domain_open_peer — device-tensor buffers run
        the same schedule with the gfx950 kernels, transfers staged through
        host memory."""
        L = lib()
        self.rank, self.nranks, self.device = rank, nranks, device
        self.transport = transport

        self.transport_errors = []     # tracebacks of transport exceptions

        def _failed(what):
            # an exception must not cross C: it becomes -EIO for the
            # operation, and its traceback is kept (and shown) for diagnosis
            import traceback
            tb = f"{what}: " + traceback.format_exc()
            self.transport_errors.append(tb)
            sys.stderr.write(f"lfa HostEndpoint rank {rank}: transport {tb}")
            return -EIO

        def _send(ctx, peer, buf, nbytes, tag, req):
            try:
                req[0] = transport.send(peer, buf, nbytes, tag)
                return 0
            except TransportAgain:
                return -EAGAIN
            except Exception:  # noqa: BLE001
                return _failed(f"send(peer={peer}, {nbytes} B, tag={tag:#x})")

        def _recv(ctx, peer, buf, nbytes, tag, req):
            try:
                req[0] = transport.recv(peer, buf, nbytes, tag)
                return 0
            except TransportAgain:
                return -EAGAIN
            except Exception:  # noqa: BLE001
                return _failed(f"recv(peer={peer}, {nbytes} B, tag={tag:#x})")

        def _test(ctx, req):
            try:
                return int(transport.test(req))
            except Exception:  # noqa: BLE001
                return _failed("test")

        # keep the trampolines alive as long as the endpoint
        self._ops = PeerXferOps(XferPost(_send), XferPost(_recv), XferTest(_test))
        self.dom, self.ep = c_void_p(), c_void_p()
        _chk(L.lfa_coll_domain_open_peer(device, rank, nranks, ctypes.byref(self._ops),
                                         None, ctypes.byref(self.dom)), "domain_open_peer")
        _chk(L.lfa_coll_ep_open(self.dom, ctypes.byref(self.ep)), "ep_open")
        self.world = L.lfa_coll_world_addr(self.ep)
        self._ctx = 0
        self._fast_init()


def esz(dt: int) -> int:
    return SIZES[DT(dt)]


__all__ = ["plan", "block", "host_chunks", "group_chunk", "member_chunk", "HostChunk", "loopback", "Endpoint", "Plan", "COLL", "DT", "OP",
           "ALGO_TREE", "ALGO_RD", "ALGO_RCCL", "ALGO_TREE_COLL", "ALGO_P2P", "ALGO_AUTO",
           "auto_algo", "esz",
           "HostEndpoint", "PeerXferOps", "TransportAgain"]
