#!/usr/bin/env python3
"""2-process allreduce of 256 MiB float SUM on HOST buffers, with and without
a group chunk, on the box's one MI355X.

Two processes open peer domains on device 0 (as tests/test_coll_peer_gpu.py
does) and run LFA_ALGO_P2P: the data moves through the IPC-mapped symmetric
workspaces and the flag barrier, the owner's (gloo) transport carries only
the workspace handshake.  Each process hands in pinned host buffers:

  group chunk 0        every member stages the whole 256 MiB (H2D, collective,
                       D2H one after the other: round 2's rule at N > 1)
  group chunk 32/64 MiB every member splits into the same chunks, H2D of chunk
                       c+1 and D2H of chunk c-1 overlap chunk c's collective

and, for scale, the same collective on device buffers.  Median of `--reps`
wall times (max over the two ranks, barrier before each), results checked
bitwise against the whole-buffer device result.  Both processes share one
GPU's HBM and one PCIe link, so this is the mechanism's relative gain, not an
8-GPU figure.  Prints one JSON line from rank 0.

    python3 tools/probe_host_group_chunk.py [--reps 5]
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

COUNT = 64 << 20          # 256 MiB of float


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
        try:
            ep.set_algo(coll.ALGO_P2P)
            g = torch.Generator().manual_seed(10 + rank)
            hx = (torch.rand(COUNT, generator=g) * 2 - 1).pin_memory()
            hy = torch.empty(COUNT).pin_memory()
            dx, dy = hx.to("cuda"), torch.empty(COUNT, device="cuda")
            torch.cuda.synchronize()

            def timed(x, y):
                ep.wait(ep.allreduce(x, y, COUNT, 8, 2))
                ts = []
                for _ in range(reps):
                    dist.barrier()
                    t0 = time.perf_counter()
                    ep.wait(ep.allreduce(x, y, COUNT, 8, 2))
                    t = torch.tensor([time.perf_counter() - t0])
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                    ts.append(t.item())
                return round(statistics.median(ts) * 1e3, 2)

            # the link itself: both ranks copy 256 MiB H2D then D2H at once
            # (torch copies on torch's stream), the serial staging floor
            tl = []
            for _ in range(reps):
                dist.barrier()
                t0 = time.perf_counter()
                dy.copy_(hx, non_blocking=True)
                hy.copy_(dy, non_blocking=True)
                torch.cuda.synchronize()
                t = torch.tensor([time.perf_counter() - t0])
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                tl.append(t.item())
            row = {"torch_h2d_then_d2h_ms": round(statistics.median(tl) * 1e3, 2)}
            # no setter call: the default group chunk (LFA_GROUP_CHUNK_AUTO,
            # 32 MiB chunks from 64 MiB on)
            row["device_default_ms"] = timed(dx, dy)
            want = dy.cpu()
            row["host_default_ms"] = timed(hx, hy)
            ok = torch.equal(hy, want)
            ep.set_group_chunk(0)
            row["device_whole_ms"] = timed(dx, dy)
            ok = ok and torch.equal(dy.cpu(), want)
            row["host_whole_ms"] = timed(hx, hy)
            ok = ok and torch.equal(hy, want)
            for mib in (64, 32, 16, 8):
                ep.set_group_chunk(mib << 20)
                row[f"host_group_chunk_{mib}mib_ms"] = timed(hx, hy)
                ok = ok and torch.equal(hy, want)
                row[f"device_group_chunk_{mib}mib_ms"] = timed(dx, dy)
                ok = ok and torch.equal(dy.cpu(), want)
            ep.set_group_chunk(0)
            row["host_whole_again_ms"] = timed(hx, hy)     # order / warm-up check
            ep.set_group_chunk(coll.GROUP_CHUNK_AUTO)
            row["host_default_again_ms"] = timed(hx, hy)
            row["bitwise_equal"] = bool(ok)
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, row))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def main():
    import torch.multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, args.reps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    if any(not isinstance(v, dict) for v in res.values()):
        print(json.dumps({"error": {str(k): v for k, v in res.items()}}))
        sys.exit(1)
    out = {"host_allreduce_2proc_256mib_float_sum": res[0],
           "note": "2 processes on one MI355X (peer domains, LFA_ALGO_P2P), pinned host "
                   "in/out; median of %d, max over ranks; both ranks share one GPU's HBM "
                   "and PCIe link" % args.reps}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
