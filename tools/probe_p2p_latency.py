"""Small-bucket latency of LFA_ALGO_P2P across PROCESSES on one MI355X.

N processes (default 2) share device 0 through GPU peer domains
(lfa_coll_domain_open_peer, the gloo owner transport of the tests): with
LFA_ALGO_P2P every operation runs on the GPU alone — staging copy, flag
barrier (lfa_signal.hip), the system-scope tree kernel over the peers'
IPC-mapped workspaces, closing flag barrier — so this times that path's
kernels and its host submit/complete cost.  Beside it, the TREE schedule on
the same domain, whose transfers go through the owner's (gloo) transport.
Not xGMI: the peers' workspaces are this GPU's own HBM.

  python tools/probe_p2p_latency.py [--world 2] [--reps 300] [--quick] [--parent-gpu]
--quick: the 4 KiB P2P allreduce only.  --parent-gpu: this (parent) process
holds a GPU context of its own while the workers run, as pytest's process
does after the in-process GPU tests — one more process on the GPU.
prints one JSON line (median / p10 / p90 us per allreduce, per size, Python-timed;
c_loop_mean_us: the same operations submitted and reaped in C).
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _kfd_queues(pid=None):
    """Hardware queues the process holds (KFD sysfs), None if unreadable."""
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid or os.getpid()}/queues"))
    except OSError:
        return None


def _worker(rank, world, port, reps, quick, q, only=None):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if world > 4 and "GPU_MAX_HW_QUEUES" not in os.environ:
            os.environ["GPU_MAX_HW_QUEUES"] = "2"   # queue slots
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        out = {}
        try:
            plan = (("p2p", coll.ALGO_P2P, (4096, 65536, 1 << 20), reps),
                    ("p2p_host", coll.ALGO_P2P, (4096, 65536, 1 << 20), reps),
                    ("p2p_pageable", coll.ALGO_P2P, (4096, 65536, 1 << 20), reps),
                    ("p2p_rs", coll.ALGO_P2P, (4096, 65536, 1 << 20), reps),
                    ("tree", coll.ALGO_TREE, (4096,), max(reps // 10, 10)))
            if quick:
                plan = (("p2p", coll.ALGO_P2P, (4096,), reps),
                        ("p2p_host", coll.ALGO_P2P, (4096,), reps))
            if only:
                # --only name:size[,size...]
                name, sizes = only.split(":")
                plan = tuple((nm, al, tuple(int(x) for x in sizes.split(",")), reps)
                             for nm, al, _s, _n in plan if nm == name)
            for name, algo, sizes, n in plan:
                ep.set_algo(algo)
                for nbytes in sizes:
                    if name == "p2p_rs":   # double PROD reduce_scatter (config 5's op)
                        cnt = nbytes // 8
                        x = torch.rand(cnt, device="cuda", dtype=torch.float64) * 0.2 + 0.9
                        r = torch.empty(max(coll.block(cnt, world, rank)[1], 1),
                                        device="cuda", dtype=torch.float64)

                        def op():
                            return ep.reduce_scatter(x, r, cnt, 9, 3)
                    elif name == "p2p_pageable":   # pageable HOST buffers (malloc)
                        cnt = nbytes // 4
                        x = torch.rand(cnt)
                        r = torch.empty_like(x)

                        def op():
                            return ep.allreduce(x, r, cnt, 8, 2)
                    elif name == "p2p_host":   # pinned HOST buffers
                        cnt = nbytes // 4
                        x = torch.rand(cnt).pin_memory()
                        r = torch.empty_like(x).pin_memory()

                        def op():
                            return ep.allreduce(x, r, cnt, 8, 2)
                    else:
                        cnt = nbytes // 4
                        x = torch.rand(cnt, device="cuda")
                        r = torch.empty_like(x)

                        def op():
                            return ep.allreduce(x, r, cnt, 8, 2)
                    torch.cuda.synchronize()
                    for _ in range(20):
                        ep.wait(op())
                    dist.barrier()
                    ts = []
                    for _ in range(n):
                        t0 = time.perf_counter()
                        ep.wait(op())
                        ts.append(time.perf_counter() - t0)
                    ts.sort()
                    out[f"{name}_{nbytes}"] = {
                        "median_us": round(statistics.median(ts) * 1e6, 1),
                        "p10_us": round(ts[len(ts) // 10] * 1e6, 1),
                        "p90_us": round(ts[9 * len(ts) // 10] * 1e6, 1), "reps": n}
                    # the same operation submitted and reaped in C
                    # (liblfa_bench.so): the provider path without Python
                    dist.barrier()
                    kind = 5 if name == "p2p_rs" else 3
                    dt_, op_ = (9, 3) if name == "p2p_rs" else (8, 2)
                    out[f"{name}_{nbytes}"]["c_loop_mean_us"] = round(
                        ep.bench_loop(kind, x, r, cnt, dt_, op_, reps=n), 1)
                    if name in ("p2p", "p2p_host", "p2p_pageable") and world == 2:
                        # the result bit for bit: prov/coll's two-rank tree
                        # is x1 + x0 (coll_coll.c:409-430), one fp32 add
                        torch.cuda.synchronize()
                        xs = [torch.empty(cnt) for _ in range(world)]
                        dist.all_gather(xs, x.cpu())
                        out[f"{name}_{nbytes}"]["exact"] = bool(torch.equal(r.cpu(), xs[1] + xs[0]))
            out["kfd_queues"] = _kfd_queues()
            out["ws_mem"] = coll.ws_mem()
            out["ws_info"] = ep.ws_info()
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--parent-gpu", action="store_true")
    ap.add_argument("--only", default="", help="one row kind and its sizes, e.g. p2p:1048576")
    ap.add_argument("--worker-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES of the workers only (0: inherit); "
                         "the parent keeps the environment's")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    parent_queues = os.environ.get("GPU_MAX_HW_QUEUES", "default")
    if a.parent_gpu:
        import torch
        torch.cuda.set_device(0)
        hold = torch.ones(1 << 20, device="cuda")
        # as pytest's process after GPU tests: work on several streams
        for _ in range(4):
            with torch.cuda.stream(torch.cuda.Stream()):
                hold.add_(1)
        torch.cuda.synchronize()
    if a.worker_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.worker_queues)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, a.world, port, a.reps, a.quick, q,
                                                    a.only or None))
             for r in range(a.world)]
    for p in procs:
        p.start()
    res = {}
    t0 = time.time()
    try:
        for _ in range(a.world):
            r, v = q.get(timeout=120)
            res[r] = v
    except Exception:  # noqa: BLE001  (queue.Empty: a rank did not finish)
        res["timeout"] = f"no result within 120 s; {len(res)} ranks reported"
    wall = round(time.time() - t0, 1)
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    print(json.dumps({"world": a.world, "device": "one MI355X shared by all ranks",
                      "parent_gpu": a.parent_gpu,
                      "parent_hw_queues": parent_queues if a.parent_gpu else None,
                      "parent_kfd_queues": _kfd_queues(),
                      "worker_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"),
                      "wall_s": wall, "timeout": res.get("timeout"),
                      "rank0": res.get(0), "rank1": res.get(1)}), flush=True)
    if not all(isinstance(v, dict) for v in res.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
