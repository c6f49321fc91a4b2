"""bench.py's N > 1 parity check, on CPU with gloo.

The 8-GPU leg gathers fixed slices of every rank's input and output to rank 0
and compares the outputs bit for bit with the oracle's prov/coll allreduce
of the gathered inputs (bench.oracle_check).  Here world-2 and world-3 gloo
processes hand it correct results (computed by the oracle from every rank's
seeded input) and corrupted ones: a correct result must pass, one flipped
bit inside a checked slice, a block swapped between ranks, or a
reduce_scatter written with the wrong partition must each be caught.
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


def _inputs(world, count, nd, seed):
    rng = np.random.default_rng(seed)
    if nd == np.float32:
        return [rng.uniform(-1, 1, count).astype(nd) for _ in range(world)]
    return [rng.uniform(0.9, 1.1, count).astype(nd) for _ in range(world)]


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        import oracle
        res = {}
        m = 1000                                 # slice length (small, fast)
        # allreduce, float SUM: 3 slices of m in a 10_001-element vector
        count = 10_001
        xs = _inputs(world, count, np.float32, 11)
        full = oracle.allreduce(2, 8, xs)[0]
        x, y = torch.from_numpy(xs[rank]), torch.from_numpy(full.copy())
        res["ar_ok"] = bench.oracle_check(x, y, count, rank, world, 8, 2, "allreduce", m)
        bad = y.clone()
        if rank == world - 1:                    # one bit, in the middle slice
            bad.view(torch.int32)[count // 2] ^= 1
        res["ar_bit"] = bench.oracle_check(x, bad, count, rank, world, 8, 2, "allreduce", m)
        off = y.clone()
        if rank == 0:                            # outside every checked slice
            off[m + 7] += 1.0
        res["ar_outside"] = bench.oracle_check(x, off, count, rank, world, 8, 2,
                                               "allreduce", m)
        # reduce_scatter, double PROD, ragged blocks (count % world != 0)
        count = 7 * world + (world - 1)
        xs = _inputs(world, count, np.float64, 12)
        full = oracle.allreduce(3, 9, xs)[0]
        bounds = oracle.slice_bounds(count, world)
        lo, hi = bounds[rank]
        x = torch.from_numpy(xs[rank])
        res["rs_ok"] = bench.oracle_check(x, torch.from_numpy(full[lo:hi].copy()), count,
                                          rank, world, 9, 3, "reduce_scatter", 4)
        # every rank writes the NEXT rank's block: a partition / routing bug
        nlo, nhi = bounds[(rank + 1) % world]
        wrong = full[nlo:nhi].copy()
        wrong = np.resize(wrong, hi - lo)
        res["rs_swapped"] = bench.oracle_check(x, torch.from_numpy(wrong), count, rank,
                                               world, 9, 3, "reduce_scatter", 4)
        # an even split instead of the reference's (first count % N ranks
        # hold one element more)
        per = count // world
        elo = rank * per
        even = full[elo:elo + (hi - lo)].copy()
        res["rs_even_split"] = bench.oracle_check(x, torch.from_numpy(even), count, rank,
                                                  world, 9, 3, "reduce_scatter", 4)
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_oracle_check_across_processes(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=120)
            out[r] = v
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        assert isinstance(v, dict), f"rank {r}: {v}"
        if r:
            assert all(x == {} for x in v.values()), v      # rank 0 reports
    res = out[0]
    assert res["ar_ok"] == {"oracle_exact": True, "elements": 3000, "mismatches": 0}
    assert res["ar_bit"]["oracle_exact"] is False and res["ar_bit"]["mismatches"] == 1
    assert res["ar_outside"]["oracle_exact"] is True        # not a checked element
    assert res["rs_ok"]["oracle_exact"] is True
    assert res["rs_ok"]["elements"] > 0
    assert res["rs_swapped"]["oracle_exact"] is False
    assert res["rs_even_split"]["oracle_exact"] is False


def test_oracle_ranges():
    import bench
    # allreduce: start, middle, end; merged when they touch
    assert bench.oracle_ranges(10_000, 8, "allreduce", 1000) == [(0, 1000), (4500, 5500),
                                                                   (9000, 10_000)]
    assert bench.oracle_ranges(1500, 8, "allreduce", 1000) == [(0, 1500)]
    # reduce_scatter: first and last m of every block (reference partition)
    r = bench.oracle_ranges(803, 8, "reduce_scatter", 10)
    assert r[0] == (0, 10) and r[-1] == (793, 803)
    assert sum(b - a for a, b in r) == 8 * 20
    # tiny blocks: the whole vector, once
    assert bench.oracle_ranges(12, 8, "reduce_scatter", 10) == [(0, 12)]


def test_oracle_check_world_one():
    import bench
    import oracle
    x = np.random.default_rng(3).uniform(-1, 1, 5000).astype(np.float32)
    y = oracle.allreduce(2, 8, [x])[0]
    got = bench.oracle_check(torch.from_numpy(x), torch.from_numpy(y), 5000, 0, 1, 8, 2,
                             "allreduce", 100)
    assert got == {"oracle_exact": True, "elements": 300, "mismatches": 0}
