"""The C executor and the C join at N > 1, on CPU: 1, 2 and 3 processes.

Every process opens a peer-transfer domain (lfa_coll_domain_open_host): the
collective provider (liblfa_coll.so) builds its schedules, posts their
SEND/RECV items through the transport callbacks — here torch.distributed
gloo isend/irecv, standing in for the owner provider's FI_PEER_TRANSFER
tagged messages (coll_coll.c:770-814) — and runs REDUCE / TREE items with the
product's host combine (lfa_host_write / lfa_host_reduce_tree).  Progress is
lfa_cq_read, as in prov/coll.  Results must match the oracle bit for bit.
The oracle is only the checker here.
"""
import ctypes
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


from gloo_xfer import GlooXfer  # noqa: E402  (the owner transport over gloo)


def _inputs(oracle, dt, count, world, seed):
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    if nd.kind == "f":
        return [rng.uniform(0.9, 1.1, count).astype(nd) for _ in range(world)]
    return [rng.integers(0, 255, count).astype(nd) for _ in range(world)]


def _collectives(ep, rank, world, oracle, coll):
    """Every fi_ops_collective slot, every algorithm, ragged counts."""
    for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P,
                 coll.ALGO_RCCL):
        ep.set_algo(algo)
        for dt, op, count in ((8, 2, 70_001), (8, 2, 1000), (6, 0, 5), (1, 7, 3),
                              (9, 3, 4099), (6, 6, 6 * 1000), (10, 3, 33)):
            sends = _inputs(oracle, dt, count, world, 1234 + count + algo)
            want = oracle.allreduce(op, dt, sends)[0]
            nd = sends[0].dtype
            # allreduce
            res = np.zeros(count, nd)
            ep.wait(ep.allreduce(sends[rank], res, count, dt, op))
            assert res.tobytes() == want.tobytes(), f"allreduce algo={algo} dt={dt} n={count}"
            # reduce_scatter (block r of the allreduce)
            off, ln = coll.block(count, world, rank)
            res = np.zeros(max(ln, 1), nd)
            ep.wait(ep.reduce_scatter(sends[rank], res, count, dt, op))
            assert res[:ln].tobytes() == want[off:off + ln].tobytes(), "reduce_scatter"
            # reduce to every root
            for root in range(world):
                res = np.zeros(count, nd)
                ep.wait(ep.reduce(sends[rank], res, count, root, dt, op))
                if rank == root:
                    assert res.tobytes() == want.tobytes(), f"reduce root={root}"
        # data movement
        x = np.arange(10, dtype=np.int32) + 100 * rank
        res = np.zeros(10 * world, np.int32)
        ep.wait(ep.allgather(x, res, 10, 4))
        assert np.array_equal(res, np.concatenate([np.arange(10) + 100 * k
                                                   for k in range(world)]))
        for root in range(world):
            b = np.arange(7, dtype=np.float64) * (root + 1) if rank == root else np.zeros(7)
            ep.wait(ep.broadcast(b, 7, root, 9))
            assert np.array_equal(b, np.arange(7) * (root + 1))
            src = (np.arange(5 * world, dtype=np.int64) if rank == root
                   else np.zeros(5 * world, np.int64))
            res = np.zeros(5, np.int64)
            ep.wait(ep.scatter(src, res, 5, root, 6))
            assert np.array_equal(res, np.arange(5) + 5 * rank)
        ep.wait(ep.barrier())
    ep.set_algo(coll.ALGO_TREE)


def _overlap(ep, rank, world, oracle):
    """Several operations in flight at once: each progresses on its own tag
    (cid = group_id << 16 | seq) and completes in issue order."""
    outs, wants, ctxs = [], [], []
    for k in range(5):
        sends = _inputs(oracle, 8, 3000 + k, world, 77 + k)
        want = oracle.allreduce(2, 8, sends)[0]
        res = np.zeros_like(want)
        ctxs.append(ep.allreduce(sends[rank], res, res.size, 8, 2))
        outs.append((res, sends))
        wants.append(want)
    done = []
    while len(done) < len(ctxs):
        done += ep.cq_read()
    assert done == ctxs, "completion order"
    for (res, _), want in zip(outs, wants):
        assert res.tobytes() == want.tobytes()


def _joins(ep, rank, world, oracle):
    """fi_join_collective: the cid-mask BAND allreduce over the parent, the
    lowest common free id, subset membership (coll_coll.c:912-995)."""
    assert ep.group_id(ep.world) == 0
    # world join
    mc, ctx = ep.join()
    ev = ep.wait_join()
    assert ev[0] == 6 and ev[2] == ctx
    gid_world = ep.group_id(mc)
    assert gid_world == 1            # id 0 is the world group
    # subset: the first and the last rank
    members = sorted({0, world - 1})
    sub, ctx2 = ep.join(members)
    ev = ep.wait_join()
    assert ev[2] == ctx2
    assert ep.group_id(sub) == 2
    addr = ep.mc_addr(sub)
    if rank in members:
        pos = members.index(rank)
        sends = _inputs(oracle, 9, 2001, world, 5)
        mine = [sends[m] for m in members]
        want = oracle.allreduce(3, 9, mine)[0]
        res = np.zeros(2001)
        ep.wait(ep.allreduce(mine[pos], res, 2001, 9, 3, coll_addr=addr))
        assert res.tobytes() == want.tobytes()
        # reduce to the last group rank of the subset
        root = len(members) - 1
        res = np.zeros(2001)
        ep.wait(ep.reduce(mine[pos], res, 2001, root, 9, 3, coll_addr=addr))
        if pos == root:
            assert res.tobytes() == want.tobytes()
        ep.wait(ep.barrier(coll_addr=addr))
    else:
        from libfabric_amd.coll import CollError
        with pytest.raises(CollError):
            ep.allreduce(np.zeros(4), np.zeros(4), 4, 9, 2, coll_addr=addr)
    # a join on the subgroup (parent = subset): members only
    if rank in members:
        sub2, _ = ep.join(None, coll_addr=addr)
        ep.wait_join()
        assert ep.group_id(sub2) == 3
        x = np.array([rank + 1], np.uint64)
        res = np.zeros(1, np.uint64)
        ep.wait(ep.allreduce(x, res, 1, 7, 2, coll_addr=ep.mc_addr(sub2)))
        assert int(res[0]) == sum(m + 1 for m in members)
        from libfabric_amd import coll
        coll.lib().lfa_mc_close(sub2)
    # closing frees the id: the next world join reuses 1
    from libfabric_amd import coll
    assert coll.lib().lfa_mc_close(mc) == 0
    mc3, _ = ep.join()
    ep.wait_join()
    assert ep.group_id(mc3) == 1
    coll.lib().lfa_mc_close(mc3)
    coll.lib().lfa_mc_close(sub)
    # the known answer of fabtests/multinode/src/core_coll.c:230-277
    x = np.array([1234 + rank], np.uint64)
    res = np.zeros(1, np.uint64)
    ep.wait(ep.allreduce(x, res, 1, 7, 2))
    assert int(res[0]) == sum(1234 + k for k in range(world))


def _joins_members(ep, rank, world):
    """lfa_join_members — prov/coll's join with coll_addr = the av_set's own
    address (coll_coll.c:939-941): the stride set of fabtests core_coll.c
    (start 1, stride 2, :175-178) forms its group while the other ranks call
    nothing and run a world collective meanwhile; the group gets the lowest
    id its members have free, and core_coll.c's expected sum."""
    from libfabric_amd import coll
    from libfabric_amd.coll import CollError
    members = list(range(1, world, 2))
    if rank in members:
        mc, ctx = ep.join_members(members)
        ev = ep.wait_join()
        assert ev[0] == 6 and ev[2] == ctx
        assert ep.group_id(mc) == 1
        x = np.array([1234 + rank], np.uint64)
        res = np.zeros(1, np.uint64)
        ep.wait(ep.allreduce(x, res, 1, 7, 2, coll_addr=ep.mc_addr(mc)))
        assert int(res[0]) == sum(1234 + m for m in members)
        assert coll.lib().lfa_mc_close(mc) == 0
    else:
        with pytest.raises(CollError):        # only members call this form
            ep.join_members(members or [world])
    # every rank: the whole group through the same form, then the world
    mc, _ = ep.join_members(list(range(world)))
    ep.wait_join()
    assert ep.group_id(mc) == 1
    x = np.array([rank + 1], np.uint64)
    res = np.zeros(1, np.uint64)
    ep.wait(ep.allreduce(x, res, 1, 7, 2, coll_addr=ep.mc_addr(mc)))
    assert int(res[0]) == world * (world + 1) // 2
    assert coll.lib().lfa_mc_close(mc) == 0
    ep.wait(ep.barrier())


def _set_order(world):
    """An av_set's address order as prov/coll leaves it (coll_av_set.c:
    insert appends, remove moves the last address into the hole): stride
    {0, 2, ..} + insert 1 (+ insert 3, remove 2 from N = 4) — N = 3 gives
    [0, 2, 1], N = 5 [0, 3, 4, 1]."""
    a = list(range(0, world, 2))
    if world > 1:
        a.append(1)
    if world > 3:
        a.append(3)
        i = a.index(2)
        a[i] = a[-1]
        a.pop()
    return a


def _joins_set_order(ep, rank, world, oracle, coll):
    """group rank r = the r-th address of the joined set
    (coll_find_local_rank, coll_coll.c:669-689), not the r-th smallest, for
    every algorithm; through lfa_join_collective (every rank calls) and
    lfa_join_members (members only)."""
    order = _set_order(world)
    sends = _inputs(oracle, 8, 4099, world, 99)      # float, indexed by parent rank
    mine = [sends[m] for m in order]
    want = oracle.allreduce(2, 8, mine)[0]
    if order != sorted(order) and len(order) > 2:
        srt = oracle.allreduce(2, 8, [sends[m] for m in sorted(order)])[0]
        assert srt.tobytes() != want.tobytes()        # the order is observable
    for members_only in (False, True):
        if members_only and rank not in order:
            continue
        mc, _ = (ep.join_members(order) if members_only else ep.join(order))
        ep.wait_join()
        addr = ep.mc_addr(mc)
        if rank in order:
            pos = order.index(rank)
            for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P):
                ep.set_algo(algo)
                res = np.zeros(4099, np.float32)
                ep.wait(ep.allreduce(sends[rank], res, 4099, 8, 2, coll_addr=addr))
                assert res.tobytes() == want.tobytes(), (algo, members_only)
                off, ln = coll.block(4099, len(order), pos)
                res = np.zeros(max(ln, 1), np.float32)
                ep.wait(ep.reduce_scatter(sends[rank], res, 4099, 8, 2, coll_addr=addr))
                assert res[:ln].tobytes() == want[off:off + ln].tobytes(), ("rs", algo)
                root = len(order) - 1               # a group rank
                res = np.zeros(4099, np.float32)
                ep.wait(ep.reduce(sends[rank], res, 4099, root, 8, 2, coll_addr=addr))
                if pos == root:
                    assert res.tobytes() == want.tobytes(), ("reduce", algo)
            ep.set_algo(coll.ALGO_TREE)
            x = np.array([rank, 7 * rank], np.int64)
            res = np.zeros(2 * len(order), np.int64)
            ep.wait(ep.allgather(x, res, 2, 6, coll_addr=addr))
            assert res.tolist() == [v for m in order for v in (m, 7 * m)]
            b = (np.arange(3, dtype=np.float64) + rank if pos == 0 else np.zeros(3))
            ep.wait(ep.broadcast(b, 3, 0, 9, coll_addr=addr))
            assert b.tolist() == (np.arange(3) + order[0]).tolist()
        assert coll.lib().lfa_mc_close(mc) == 0
    ep.wait(ep.barrier())


def _reference_known_answers(ep, rank, world, coll):
    """The reference's own acceptance checks for fi_allreduce / fi_broadcast /
    fi_barrier, from prov/cxi/test/multinode/test_coll.c (a provider's test of
    the same fi_collective API): int64 SUM of data[4r+v] = 4r+v, exact
    (:722-792); double SUM of (4r+v)/1000 within 1e-8 (:795-865); a 4-word
    uint64 broadcast from every root (:656-717); barrier (:608-654)."""
    for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P):
        ep.set_algo(algo)
        data = np.array([4 * rank + v for v in range(4)], np.int64)
        res = np.zeros(4, np.int64)
        ep.wait(ep.allreduce(data, res, 4, 6, 2))
        comp = [sum(4 * r + v for r in range(world)) for v in range(4)]
        assert res.tolist() == comp, ("isum", algo)
        data = np.array([(4 * rank + v) / 1000.0 for v in range(4)])
        res = np.zeros(4)
        ep.wait(ep.allreduce(data, res, 4, 9, 2))
        comp = [sum((4 * r + v) / 1000.0 for r in range(world)) for v in range(4)]
        assert all(abs(a - b) <= 1e-8 for a, b in zip(res, comp)), ("dsum", algo)
        for i in range(2):
            for root in range(world):
                want = np.array([i, root, 0x13579bdf, 0x10101010], np.uint64)
                buf = want.copy() if rank == root else np.zeros(4, np.uint64)
                ep.wait(ep.broadcast(buf, 4, root, 7))
                assert np.array_equal(buf, want), ("broadcast", algo, root)
        ep.wait(ep.barrier())
    ep.set_algo(coll.ALGO_TREE)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from libfabric_amd import coll
        xfer = GlooXfer()
        ep = coll.HostEndpoint(rank, world, xfer)
        try:
            _collectives(ep, rank, world, oracle, coll)
            _reference_known_answers(ep, rank, world, coll)
            _overlap(ep, rank, world, oracle)
            _joins(ep, rank, world, oracle)
            _joins_members(ep, rank, world)
            _joins_set_order(ep, rank, world, oracle, coll)
            if world > 1:
                assert xfer.sent > 0 and xfer.received > 0
            assert not xfer.reqs, "transfers left behind"
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


class FlakyXfer(GlooXfer):
    """The owner pushing back: every `every`-th post is refused with
    TransportAgain (-EAGAIN, the provider must retry it later), and a chosen
    receive can be made to complete with an error."""

    def __init__(self, every=3):
        super().__init__()
        self.every, self.n, self.refused = every, 0, 0
        self.fail_recv = False
        self.failing = set()

    def _gate(self):
        from libfabric_amd.coll import TransportAgain
        self.n += 1
        if self.n % self.every == 0:
            self.refused += 1
            raise TransportAgain()

    def send(self, peer, ptr, nbytes, tag):
        self._gate()
        return super().send(peer, ptr, nbytes, tag)

    def recv(self, peer, ptr, nbytes, tag):
        self._gate()
        h = super().recv(peer, ptr, nbytes, tag)
        if self.fail_recv:
            self.failing.add(h)
        return h

    def test(self, h):
        bad = h in self.failing
        r = super().test(h)
        if bad:
            self.failing.discard(h)
            return -5                         # the transfer failed: -EIO
        return r


def _flaky_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from libfabric_amd import coll
        xfer = FlakyXfer()
        ep = coll.HostEndpoint(rank, world, xfer)
        try:
            for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL):
                ep.set_algo(algo)
                sends = _inputs(oracle, 8, 5000, world, 31 + algo)
                want = oracle.allreduce(2, 8, sends)[0]
                res = np.zeros(5000, np.float32)
                ep.wait(ep.allreduce(sends[rank], res, 5000, 8, 2))
                assert res.tobytes() == want.tobytes(), algo
            assert xfer.refused > 0, "no post was refused"
            # a failed transfer fails its operation, on that rank only
            xfer.every = 10 ** 9
            xfer.fail_recv = rank == 1
            x = np.ones(64, np.float32)
            res = np.zeros(64, np.float32)
            ctx = ep.allreduce(x, res, 64, 8, 2)
            if rank == 1:
                with pytest.raises(coll.CollError):
                    ep.wait(ctx)
            else:
                ep.wait(ctx)
                assert np.all(res == world)
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_transport_pushback_and_failure():
    """prov/coll's requeue of a SEND the owner refused with -FI_EAGAIN
    (coll_coll.c:845-852) — here every third post, sends and receives, over
    three algorithms, results still exact — and a transfer that completes in
    error failing its operation through lfa_cq_readerr."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flaky_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=120)
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert results.get(r) == "ok", results.get(r)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5])
def test_c_executor_across_processes(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=150)
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert results.get(r) == "ok", results.get(r)


def test_host_domain_errors():
    from libfabric_amd import coll
    L = coll.lib()
    d = ctypes.c_void_p()
    ops = coll.PeerXferOps()
    assert L.lfa_coll_domain_open_host(0, 1, None, None, ctypes.byref(d)) == -22
    assert L.lfa_coll_domain_open_host(2, 2, ctypes.byref(ops), None, ctypes.byref(d)) == -22
