#!/usr/bin/env python3
"""Small-collective latency, split, timed in C.

1. World 1, RCCL device domain: a 4 KiB float SUM allreduce (the schedule is
   one COPY) through lfa_bench_split — mean per operation, of it the submit
   call and the polling to completion — beside what the same GPU work costs
   without the provider (lfa_bench_raw: the copy kernel + event + spin, + a
   stream synchronize; the launch, event record / query, pointer query and
   an empty lfa_cq_read alone).
2. Two processes on the one GPU, GPU peer domains, LFA_ALGO_P2P (one-shot
   kernel): 4 KiB float SUM allreduce and double PROD reduce_scatter, split
   the same way.

Prints one JSON line.   python tools/probe_latency.py [--reps 2000]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def _split(ep, coll_kind, x, r, cnt, dt, op, reps):
    from libfabric_amd._native import lib as native
    from libfabric_amd.coll import _ptr
    out = (ctypes.c_double * 4)()
    L = native("bench")
    L.lfa_bench_split.restype = ctypes.c_int
    rc = L.lfa_bench_split(ctypes.c_void_p(ep.ep.value if hasattr(ep.ep, "value") else ep.ep),
                           coll_kind, ctypes.c_void_p(_ptr(x)), ctypes.c_void_p(_ptr(r)),
                           ctypes.c_size_t(cnt), 0, dt, op, ctypes.c_uint64(ep.world),
                           reps, 20000, out)
    if rc:
        return {"error": rc}
    return {"total_us": round(out[0], 2), "submit_us": round(out[1], 2),
            "poll_us": round(out[2], 2), "cq_reads_per_op": round(out[3], 1)}


def _raw(ep, dst, src, nbytes, reps):
    from libfabric_amd._native import lib as native
    L = native("bench")
    L.lfa_bench_raw.restype = ctypes.c_int
    names = ("kernel_event_spin_us", "kernel_stream_sync_us", "launch_only_us",
             "event_record_only_us", "event_query_done_us", "pointer_attributes_us",
             "cq_read_empty_us")
    res = {}
    for mode, name in enumerate(names):
        us = ctypes.c_double()
        e = ep.ep if ep is not None else None
        rc = L.lfa_bench_raw(ctypes.c_void_p(e.value if hasattr(e, "value") else e),
                             ctypes.c_void_p(dst), ctypes.c_void_p(src),
                             ctypes.c_size_t(nbytes), mode,
                             reps if mode < 2 else 10 * reps, ctypes.byref(us))
        res[name] = round(us.value, 3) if rc == 0 else f"rc {rc}"
    return res


def world1(reps):
    import torch
    from libfabric_amd import coll
    torch.cuda.set_device(0)
    ep = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    out = {}
    try:
        a = torch.rand(1024, device="cuda")
        b = torch.empty_like(a)
        torch.cuda.synchronize()
        for algo, name in ((coll.ALGO_AUTO, "auto"), (coll.ALGO_TREE, "tree")):
            ep.set_algo(algo)
            ep.wait(ep.allreduce(a, b, 1024, 8, 2))
            _split(ep, 3, a, b, 1024, 8, 2, 200)
            out[f"allreduce_4kib_{name}"] = _split(ep, 3, a, b, 1024, 8, 2, reps)
        assert torch.equal(a, b)
        out["raw"] = _raw(ep, b.data_ptr(), a.data_ptr(), 4096, reps)
    finally:
        ep.close()
    return out


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, reps, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        out = {}
        try:
            ep.set_algo(coll.ALGO_P2P)
            x = torch.rand(1024, device="cuda")
            r = torch.empty_like(x)
            xd = torch.rand(512, device="cuda", dtype=torch.float64) * 0.2 + 0.9
            rd = torch.empty(256, device="cuda", dtype=torch.float64)
            torch.cuda.synchronize()
            for _ in range(50):
                ep.wait(ep.allreduce(x, r, 1024, 8, 2))
            rf = torch.empty(512, device="cuda")
            rdd = torch.empty(512, device="cuda", dtype=torch.float64)
            for name, args in (("p2p_allreduce_4kib", (3, x, r, 1024, 8, 2)),
                               ("p2p_reduce_scatter_4kib_double_prod", (5, xd, rd, 512, 9, 3)),
                               ("p2p_reduce_scatter_4kib_float_sum", (5, x, rf, 1024, 8, 2)),
                               ("p2p_allreduce_4kib_double_prod", (3, xd, rdd, 512, 9, 3))):
                # each kernel's first launch (code object load, milliseconds)
                # outside the timed loop
                dist.barrier()
                _split(ep, *args, 100)
                dist.barrier()
                out[name] = _split(ep, *args, reps)
            out["counters"] = ep.counters()
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def two_process(reps, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    return {f"rank{r}": res[r] for r in sorted(res)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--skip-world1", action="store_true")
    a = ap.parse_args()
    out = {"reps": a.reps}
    if not a.skip_world1:
        out["world1_rccl_domain"] = world1(a.reps)
        print(json.dumps(out), flush=True)
    out["two_process_p2p"] = two_process(a.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
