"""N>1 path on CPU: world_size 2 and 3 `gloo` processes.

Each process asks the C provider (liblfa_coll.so, lfa_coll_plan) for ITS
rank's schedule and executes it with real inter-process point-to-point
transfers (torch.distributed gloo isend/irecv, one RCCL-group equivalent per
GROUP_END) and the oracle as the combine.  Results must match the oracle's
prov/coll allreduce bit for bit — i.e. the distributed schedules interlock
across processes and reproduce the reference association order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exec_plan(pl, bufs, op, dt, esz, nd, seq):
    """seq: per-(direction, peer) message counters — messages between a pair
    match FIFO, as RCCL's do, whatever group structure each rank has."""
    import oracle
    from tests._plansim import lower
    st = lower(pl.steps, dist.get_rank(), dist.get_world_size())
    i = 0
    while i < len(st):
        s = st[i]
        if s["type"] in (0, 1):
            reqs, recvs = [], []
            while i < len(st) and st[i]["type"] != 2:
                x = st[i]
                b, off = x["src"] if x["type"] == 0 else x["dst"]
                key = (x["type"], x["peer"])
                tag = seq.get(key, 0)
                seq[key] = tag + 1
                if x["type"] == 0:
                    t = torch.from_numpy(bufs[b][off:off + x["count"]].copy())
                    reqs.append(dist.isend(t, x["peer"], tag=tag))
                else:
                    t = torch.empty(x["count"], dtype=torch.uint8)
                    reqs.append(dist.irecv(t, x["peer"], tag=tag))
                    recvs.append((t, b, off, x["count"]))
                i += 1
            for q in reqs:
                q.wait()
            for t, b, off, n in recvs:
                bufs[b][off:off + n] = t.numpy()
            i += 1  # GROUP_END
            continue
        if s["type"] == 3:
            b, off = s["dst"]
            d = bufs[b][off:off + s["count"] * esz].view(nd)
            sb, so = s["src"]
            oracle.write(op, dt, d, bufs[sb][so:so + s["count"] * esz].copy().view(nd))
        elif s["type"] == 5:
            sb, so = s["src"]
            b, off = s["dst"]
            bufs[b][off:off + s["count"]] = bufs[sb][so:so + s["count"]].copy()
        elif s["type"] == 4:
            ins = []
            for k in range(s["nsrc"]):
                rb, ro = pl.refs[s["first"] + k]
                ins.append(bufs[rb][ro:ro + s["count"] * esz].copy().view(nd))
            out = oracle.allreduce(op, dt, ins)[0]
            b, off = s["dst"]
            bufs[b][off:off + s["count"] * esz] = out.view(np.uint8)
        i += 1


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from libfabric_amd import coll
        seq = {}
        for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL):
            for dt, op, count in ((8, 2, 70_001), (8, 2, 1000), (6, 0, 5), (1, 7, 3),
                                  (9, 3, 4099), (8, 2, 6 * 20_000)):
                nd = oracle.DT_NP[dt]
                esz = nd.itemsize
                rng = np.random.default_rng(1234)
                allsends = [(rng.uniform(0.9, 1.1, count) if nd.kind == "f" else
                             rng.integers(0, 255, count)).astype(nd) for _ in range(world)]
                want = oracle.allreduce(op, dt, allsends)[0]
                # allreduce
                pl = coll.plan(3, algo, rank, world, -1, count, esz)
                bufs = {0: allsends[rank].view(np.uint8).copy(),
                        1: np.zeros(count * esz, np.uint8),
                        2: np.zeros(pl.tmp_bytes, np.uint8)}
                _exec_plan(pl, bufs, op, dt, esz, nd, seq)
                assert bufs[1].tobytes() == want.view(np.uint8).tobytes(), \
                    f"allreduce algo={algo} dt={dt} count={count}"
                # reduce_scatter
                off, ln = coll.block(count, world, rank)
                pl = coll.plan(5, algo, rank, world, -1, count, esz)
                bufs = {0: allsends[rank].view(np.uint8).copy(),
                        1: np.zeros(ln * esz, np.uint8),
                        2: np.zeros(pl.tmp_bytes, np.uint8)}
                _exec_plan(pl, bufs, op, dt, esz, nd, seq)
                assert bufs[1].tobytes() == want[off:off + ln].view(np.uint8).tobytes()
                # reduce to the last rank
                root = world - 1
                pl = coll.plan(6, algo, rank, world, root, count, esz)
                bufs = {0: allsends[rank].view(np.uint8).copy(),
                        1: np.zeros(count * esz, np.uint8),
                        2: np.zeros(pl.tmp_bytes, np.uint8)}
                _exec_plan(pl, bufs, op, dt, esz, nd, seq)
                if rank == root:
                    assert bufs[1].tobytes() == want.view(np.uint8).tobytes()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_schedules_across_gloo_processes(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, msg = q.get(timeout=150)
        results[r] = msg
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert results[r] == "ok", results[r]
