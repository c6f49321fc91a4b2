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


def _view(bufs, ref, nbytes):
    """(buf, off) into this rank's buffers, or (SYM_IN|SYM_OUT, off, owner)
    into group rank `owner`'s symmetric workspace — a shared-memory mapping
    here, as the provider maps peers' HBM over IPC."""
    if len(ref) == 3:
        b, off, k = ref
        sym, region = bufs["sym"]
        off += region if b == 4 else 0
        return sym[k][off:off + nbytes]
    b, off = ref
    return bufs[b][off:off + nbytes]


def _exec_plan(pl, bufs, op, dt, esz, nd, seq, jitter=None):
    """seq: per-(direction, peer) message counters — messages between a pair
    match FIFO, as RCCL's do, whatever group structure each rank has.
    BARRIER = dist.barrier(); `jitter` (rng) delays this rank at random
    points, so a missing barrier shows up as a data race."""
    import time
    import oracle
    from tests._plansim import lower
    pl.refs = list(pl.refs)
    st = lower(pl.steps, dist.get_rank(), dist.get_world_size(), pl.refs, esz)
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
        if jitter is not None and jitter.random() < 0.3:
            time.sleep(jitter.random() * 0.02)
        if s["type"] == 8:
            dist.barrier()
        elif s["type"] == 3:
            b, off = s["dst"]
            d = bufs[b][off:off + s["count"] * esz].view(nd)
            sb, so = s["src"]
            oracle.write(op, dt, d, bufs[sb][so:so + s["count"] * esz].copy().view(nd))
        elif s["type"] == 5:
            _view(bufs, s["dst"], s["count"])[:] = _view(bufs, s["src"], s["count"]).copy()
        elif s["type"] in (4, 9):
            nb = s["count"] * esz
            ins = [_view(bufs, pl.refs[s["first"] + k], nb).copy().view(nd)
                   for k in range(s["nsrc"])]
            out = oracle.allreduce(op, dt, ins)[0].view(np.uint8)
            dsts = [s["dst"]]
            if s["type"] == 9:
                base = s["first"] + s["nsrc"]
                dsts += [pl.refs[base + j] for j in range(s["peer"])]
            for d in dsts:
                _view(bufs, d, nb)[:] = out
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


SYM_BYTES = 4 << 20


def _p2p_worker(rank, world, port, q, shm):
    """LFA_ALGO_P2P schedules across processes: every rank's symmetric
    workspace is a shared-memory file all ranks map; BARRIER is a gloo
    barrier; ranks are delayed at random points and run many operations
    back to back, so a schedule whose barriers did not fence the workspace
    (a rank restaging while a peer still reads) would corrupt results."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from libfabric_amd import coll
        sym = [np.memmap(f"{shm}.{k}", dtype=np.uint8, mode="r+", shape=(SYM_BYTES,))
               for k in range(world)]
        jitter = np.random.default_rng(rank + 17)
        seq = {}
        for rep in range(3):
            for dt, op, count in ((8, 2, 70_001), (8, 2, 1000), (6, 0, 5), (1, 7, 3),
                                  (9, 3, 4099), (8, 2, 6 * 20_000), (6, 6, 100_000)):
                nd = oracle.DT_NP[dt]
                esz = nd.itemsize
                region = (count * esz + 255) // 256 * 256
                assert 2 * region <= SYM_BYTES
                for coll_op, root in ((3, -1), (5, -1), (6, (rep + count) % world)):
                    # fresh inputs per operation: a rank restaging early
                    # would change bytes a peer is still reading
                    rng = np.random.default_rng(1234 + rep * 7 + count + coll_op)
                    allsends = [(rng.uniform(0.9, 1.1, count) if nd.kind == "f" else
                                 rng.integers(0, 255, count)).astype(nd)
                                for _ in range(world)]
                    want = oracle.allreduce(op, dt, allsends)[0]
                    off, ln = coll.block(count, world, rank)
                    pl = coll.plan(coll_op, coll.ALGO_P2P, rank, world, root, count, esz)
                    nres = ln if coll_op == 5 else count
                    bufs = {0: allsends[rank].view(np.uint8).copy(),
                            1: np.zeros(nres * esz, np.uint8),
                            2: np.zeros(pl.tmp_bytes, np.uint8), "sym": (sym, region)}
                    _exec_plan(pl, bufs, op, dt, esz, nd, seq, jitter)
                    if coll_op == 3 or (coll_op == 6 and rank == root):
                        assert bufs[1].tobytes() == want.view(np.uint8).tobytes(), \
                            f"p2p coll={coll_op} dt={dt} count={count} rep={rep}"
                    elif coll_op == 5:
                        assert bufs[1].tobytes() == want[off:off + ln].view(np.uint8).tobytes()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_schedules_across_gloo_processes(world, tmp_path):
    shm = str(tmp_path / "sym")
    for k in range(world):
        with open(f"{shm}.{k}", "wb") as f:
            f.truncate(SYM_BYTES)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, world, port, q, shm))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, msg = q.get(timeout=240)
        results[r] = msg
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert results[r] == "ok", results[r]
