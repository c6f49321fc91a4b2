#!/usr/bin/env python3
"""The P2P workspace export path under repetition, GPU box.

Round 3 saw hipIpcGetMemHandle return "invalid argument" twice, each time on
one member of a 5- or 8-process group at the workspace's SECOND growth (the
8 MiB region to 16 MiB, exported while the old workspace and the peers'
mappings were still held).  This probe drives exactly that path — the
provider's own sym_prepare / sym_open / sym_free through LFA_ALGO_P2P
allreduces on GPU peer domains — many times: every cycle opens an endpoint,
grows its workspace four times (regions 8, 16, 32, 64 MiB) with torch
allocations churning between the steps, checks every result, and closes it.
With LFA_DEBUG every failed export prints the failing pointer, what HIP says
about it and every earlier workspace event of the process overlapping it
(lfa_coll.c va_explain); the worker counts those lines.

    python tools/probe_ipc_growth.py [--world 8] [--cycles 12]
prints one JSON line: exports attempted, failures, and the diagnostics.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

SIZES = (1 << 20, 12 << 20, 24 << 20, 48 << 20)   # bytes: workspace regions 8, 16, 32, 64 MiB


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cycles, logdir, trace, cache, anchor, q):
    try:
        log = open(os.path.join(logdir, f"r{rank}.log"), "w", buffering=1)
        os.dup2(log.fileno(), 2)
        # AMD_LOG_LEVEL=1: the HIP runtime names a failing export's cause
        # (its hsa_status) on stderr too
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1",
                          AMD_LOG_LEVEL="1")
        if trace:
            os.environ["LFA_TRACE"] = "1"     # one stderr line per operation state
        if cache is not None:
            os.environ["LFA_WS_CACHE_BYTES"] = str(cache)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        bad = 0
        failed = []
        churn = []
        # --anchor: a second GPU domain open across the cycles, so released
        # workspaces stay cached between them (the cache is freed when the
        # process's last GPU domain closes, i.e. every cycle without it)
        keep = coll.HostEndpoint(rank, world, GlooXfer(), device=0) if anchor else None
        for c in range(cycles):
            ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
            try:
                ep.set_algo(coll.ALGO_P2P)
                ep.set_group_chunk(0)
                for k, nbytes in enumerate(SIZES):
                    n = nbytes // 4
                    x = torch.full((n,), float(rank + 1), device="cuda")
                    r = torch.empty_like(x)
                    # allocator churn between the growths, as a caller's
                    # tensors come and go
                    churn.append(torch.empty((1 + (c + k) % 5) << 20, dtype=torch.uint8,
                                             device="cuda"))
                    if len(churn) > 6:
                        churn.pop(0)
                    torch.cuda.synchronize()
                    try:
                        ep.wait(ep.allreduce(x, r, n, 8, 2))
                    except coll.CollError as e:
                        # a failed handshake fails on every member at once
                        # (the agreement); a timed-out wait on one member
                        # only, so that one ends the probe
                        if "prov_errno 110" in str(e):
                            raise
                        failed.append((c, k, str(e)))
                        break
                    want = world * (world + 1) / 2
                    if not bool((r == want).all()):
                        bad += 1
            finally:
                ep.close()
            dist.barrier()
        if keep is not None:
            keep.close()
        dist.destroy_process_group()
        log.flush()
        q.put((rank, {"wrong_results": bad, "failed_growths": failed,
                      "ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "unset")}))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--cycles", type=int, default=24)
    ap.add_argument("--trace", action="store_true", help="LFA_TRACE=1 in every rank")
    ap.add_argument("--anchor", action="store_true",
                    help="keep a second GPU domain open across the cycles")
    ap.add_argument("--cache-bytes", type=int, default=None,
                    help="LFA_WS_CACHE_BYTES in every rank (0: workspaces freed)")
    a = ap.parse_args()
    # the IPC mode of every multi-process GPU run (bench.py, tests/conftest.py)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.multiprocessing as mp
    logdir = os.path.join(ROOT, "gpurun_out",
                          "ipc_growth_logs" + ("" if a.cache_bytes is None else f"_c{a.cache_bytes}")
                          + ("_anchor" if a.anchor else ""))
    os.makedirs(logdir, exist_ok=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, a.world, port, a.cycles, logdir, a.trace,
                                                 a.cache_bytes, a.anchor, q))
             for r in range(a.world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(a.world):
            r, v = q.get(timeout=600)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    fails, ids, notes = 0, 0, []
    for r in range(a.world):
        with open(os.path.join(logdir, f"r{r}.log")) as f:
            lines = [ln.rstrip() for ln in f
                     if ln.startswith("lfa:") or ("IPC" in ln or "ipc" in ln)]
        fails += sum("export failed" in ln for ln in lines)
        ids += sum("mapped onto other memory" in ln for ln in lines)
        notes += [f"r{r}: {ln}" for ln in lines if "overlaps event" not in ln][:40]
    out = {"world": a.world, "cycles": a.cycles, "ws_cache_bytes": a.cache_bytes,
           "anchor_domain": a.anchor,
           "hsa_enable_ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
           "identity_mismatches_logged": ids,
           "exports": a.world * a.cycles * 4, "export_failures": fails,
           "per_rank": res, "diagnostics": notes[:200]}
    print(json.dumps({"probe_ipc_growth": out}), flush=True)
    if not all(isinstance(v, dict) for v in res.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
