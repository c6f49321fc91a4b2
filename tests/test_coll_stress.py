"""Random programs of collectives across processes (CPU, the C executor over
an owner's tagged transport).

Every rank draws the same program from one seed: three groups (the world and
two joined over random subsets in random set order, so group ranks are set
positions — coll_coll.c:669-689), then a few hundred operations, each naming
a group, a collective, an algorithm, a datatype / op, a count (ragged, empty,
fewer elements than members) and a root.  A rank issues the operations of
the groups it belongs to, in program order, with up to DEPTH of them in
flight at once, so operations of different groups interleave differently on
different ranks while every group's members agree on its sequence — the tag
(group_id << 16 | seq, coll_coll.c:37-52) is what keeps them apart.  Each
result is checked against the oracle fed in the group's set order.

The transport is MpXfer below: non-blocking tagged messages over one inbound
queue per process, matched per (sender, tag) in post order with an
unexpected-message list — the way rxm's tagged receive queue serves
prov/coll (coll_coll.c:770-814).  (tests/gloo_xfer.py's transfers complete
only in a blocking wait, which is fine for one operation at a time but not
for several groups' operations in flight.)
"""
import collections
import ctypes
import os
import queue as queue_mod
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER, BROADCAST, SCATTER, BARRIER = \
    3, 5, 6, 4, 1, 7, 0
PAIRS = [(2, 8), (3, 9), (0, 6), (1, 8), (6, 7), (7, 1), (9, 4), (4, 8), (3, 10), (5, 2)]
DEPTH = 6


class MpXfer:
    """Tagged send / recv / test over multiprocessing queues (host bytes).
    refuse_every = k: every k-th post is refused with TransportAgain (the
    owner's queue full, -FI_EAGAIN), which the provider must retry later
    (coll_coll.c:845-852)."""

    def __init__(self, rank, queues, refuse_every=0):
        self.rank, self.queues = rank, queues
        self.unexpected = collections.defaultdict(collections.deque)
        self.posted = collections.defaultdict(collections.deque)
        self.reqs, self.next = {}, 1
        self.refuse_every, self.posts, self.refused = refuse_every, 0, 0

    def _gate(self):
        if self.refuse_every:
            self.posts += 1
            if self.posts % self.refuse_every == 0:
                from libfabric_amd.coll import TransportAgain
                self.refused += 1
                raise TransportAgain()

    def _new(self, state):
        h = self.next
        self.next += 1
        self.reqs[h] = state
        return h

    def send(self, peer, ptr, nbytes, tag):
        self._gate()
        self.queues[peer].put((self.rank, tag, ctypes.string_at(ptr, nbytes) if nbytes else b""))
        return self._new({"done": True})

    def _deliver(self, st, data):
        assert len(data) == st["n"], (len(data), st["n"])
        if st["n"]:
            ctypes.memmove(st["ptr"], data, st["n"])
        st["done"] = True

    def recv(self, peer, ptr, nbytes, tag):
        self._gate()
        st = {"done": False, "ptr": ptr, "n": nbytes}
        key = (peer, tag)
        if self.unexpected[key]:
            self._deliver(st, self.unexpected[key].popleft())
        else:
            self.posted[key].append(st)
        return self._new(st)

    def _pump(self):
        while True:
            try:
                src, tag, data = self.queues[self.rank].get_nowait()
            except queue_mod.Empty:
                return
            key = (src, tag)
            if self.posted[key]:
                self._deliver(self.posted[key].popleft(), data)
            else:
                self.unexpected[key].append(data)

    def pump(self):
        self._pump()

    def waiting(self):
        return {(p, hex(t)): len(v) for (p, t), v in self.posted.items() if v}

    def stray(self):
        return {(p, hex(t)): len(v) for (p, t), v in self.unexpected.items() if v}

    def test(self, h):
        if not self.reqs[h]["done"]:
            self._pump()
        if self.reqs[h]["done"]:
            del self.reqs[h]
            return 1
        return 0


def _program(world, seed, nops):
    rng = np.random.default_rng(seed)
    groups = [list(range(world))]
    for _ in range(2):
        k = int(rng.integers(1, world + 1))
        groups.append([int(x) for x in rng.permutation(world)[:k]])
    ops = []
    for i in range(nops):
        g = int(rng.integers(0, len(groups)))
        coll = int(rng.choice([ALLREDUCE, ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER,
                               BROADCAST, SCATTER, BARRIER]))
        op, dt = PAIRS[int(rng.integers(0, len(PAIRS)))]
        count = int(rng.choice([0, 1, 2, 3, 7, int(rng.integers(1, 3000))]))
        ops.append(dict(i=i, g=g, coll=coll, op=op, dt=dt, count=count,
                        root=int(rng.integers(0, len(groups[g]))),
                        algo=int(rng.choice([0, 1, 3, 4, 5])), seed=seed * 1000 + i))
    return groups, ops


def _data(oracle, o, members):
    """Every member's input for operation o, in group-rank order."""
    nd = oracle.DT_NP[o["dt"]]
    rng = np.random.default_rng(o["seed"])
    n = len(members)
    cnt = o["count"] * (n if o["coll"] == SCATTER else 1)
    if nd.kind == "f":
        return [rng.uniform(0.9, 1.1, cnt).astype(nd) for _ in range(n)]
    if nd.kind == "c":
        return [rng.uniform(0.9, 1.1, 2 * cnt).astype(np.float32).view(nd) for _ in range(n)]
    ii = np.iinfo(nd)
    return [rng.integers(ii.min, ii.max, cnt, dtype=nd, endpoint=True) for _ in range(n)]


class HostMem:
    """Buffers in host memory (numpy)."""

    @staticmethod
    def put(a):
        return np.ascontiguousarray(a).copy()

    @staticmethod
    def zeros(n, nd):
        return np.zeros(max(n, 1), nd)

    @staticmethod
    def get(b, nd):
        return b


class DevMem:
    """Buffers in HBM (torch byte tensors on cuda:0): the kernels' path."""

    @staticmethod
    def put(a):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to("cuda")
        torch.cuda.synchronize()        # ready before the provider's stream reads it
        return t

    @staticmethod
    def zeros(n, nd):
        import torch
        t = torch.zeros(max(n, 1) * nd.itemsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        return t

    @staticmethod
    def get(b, nd):
        return b.cpu().numpy().view(nd)


def _submit(ep, coll, oracle, o, members, addr, pos, mem=HostMem):
    """Issue operation o on this rank; returns (ctx, check) where check()
    verifies the result once the operation has completed.  The buffers stay
    referenced by check until then: the caller owns them until completion
    (fi_collective.3; prov/coll reads and writes them during progress)."""
    ctx, check, bufs = _issue(ep, coll, oracle, o, members, addr, pos, mem)
    return ctx, lambda: (check(), bufs)


def _issue(ep, coll, oracle, o, members, addr, pos, mem):
    ep.set_algo(o["algo"])
    n, c, root = len(members), o["count"], o["root"]
    nd = oracle.DT_NP[o["dt"]]
    ins = _data(oracle, o, members)
    mine = mem.put(ins[pos])
    kind = o["coll"]
    if kind == BARRIER:
        return ep.barrier(coll_addr=addr), lambda: None, ()
    if kind in (ALLREDUCE, REDUCE_SCATTER, REDUCE):
        want = oracle.allreduce(o["op"], o["dt"], ins)[0] if c else np.zeros(0, nd)
        if kind == REDUCE_SCATTER:
            off, ln = coll.block(c, n, pos)
            res = mem.zeros(ln, nd)
            ctx = ep.reduce_scatter(mine, res, c, o["dt"], o["op"], coll_addr=addr)
            return ctx, lambda: _eq(mem.get(res, nd)[:ln], want[off:off + ln], o), (mine, res)
        res = mem.zeros(c, nd)
        if kind == ALLREDUCE:
            ctx = ep.allreduce(mine, res, c, o["dt"], o["op"], coll_addr=addr)
            return ctx, lambda: _eq(mem.get(res, nd)[:c], want, o), (mine, res)
        ctx = ep.reduce(mine, res, c, root, o["dt"], o["op"], coll_addr=addr)
        return ctx, (lambda: _eq(mem.get(res, nd)[:c], want, o)) if pos == root else \
            (lambda: None), (mine, res)
    if kind == ALLGATHER:
        res = mem.zeros(n * c, nd)
        ctx = ep.allgather(mine, res, c, o["dt"], coll_addr=addr)
        return ctx, lambda: _eq(mem.get(res, nd)[:n * c],
                                np.concatenate(ins) if c else np.zeros(0, nd), o), (mine, res)
    if kind == BROADCAST:
        buf = mine if pos == root else mem.zeros(c, nd)
        ctx = ep.broadcast(buf, c, root, o["dt"], coll_addr=addr)
        return ctx, lambda: _eq(mem.get(buf, nd)[:c], ins[root][:c], o), (buf,)
    # SCATTER: the root's buffer holds n blocks of c elements
    res = mem.zeros(c, nd)
    src = mine if pos == root else None
    ctx = ep.scatter(src, res, c, root, o["dt"], coll_addr=addr)
    return ctx, lambda: _eq(mem.get(res, nd)[:c], ins[root][pos * c:(pos + 1) * c], o), \
        (src, res)


def _eq(got, want, o):
    assert got.tobytes() == np.ascontiguousarray(want).tobytes(), f"operation {o}"


def _worker(rank, world, queues, seed, nops, q, dev=False, host_rank=-1, gchunk=0,
            refuse_every=0):
    try:
        import oracle
        from libfabric_amd import coll
        mem = HostMem
        if dev:
            import torch
            if world > 4:
                # past the scheduler's queue slots the GPU time-slices the
                # processes' queues (tests/test_coll_peer_gpu.py::_share_gpu)
                os.environ["GPU_MAX_HW_QUEUES"] = "1" if world > 5 else "2"
            torch.cuda.set_device(0)
            # host_rank: that member hands in host buffers on its GPU peer
            # domain (staged), the others device buffers — one schedule
            mem = HostMem if rank == host_rank else DevMem
        xf = MpXfer(rank, queues, refuse_every)
        stall_s = float(os.environ.get("STRESS_STALL_S", "60"))
        logdir = os.environ.get("STRESS_LOG_DIR")
        logf = open(os.path.join(logdir, f"{'dev' if dev else 'host'}_w{world}_s{seed}_r{rank}.log"),
                    "w", buffering=1) if logdir else None
        if logf:
            # the provider's LFA_TRACE lines (stderr) into the same file
            os.dup2(logf.fileno(), 2)

        def trace(*a):
            if logf:
                logf.write(f"{time.time():.3f} " + " ".join(str(x) for x in a) + "\n")
        ep = coll.HostEndpoint(rank, world, xf, device=0 if dev else -1)
        if gchunk:
            ep.set_group_chunk(gchunk)      # the same value on every member
        try:
            groups, ops = _program(world, seed, nops)
            addrs = [ep.world]
            handles = []
            for members in groups[1:]:
                mc, _ = ep.join(members)
                ep.wait_join()
                handles.append(mc)
                addrs.append(ep.mc_addr(mc))
            inflight, done = [], set()

            def reap(ctx):
                t0 = time.time()
                trace("reap", ctx)
                while ctx not in done:
                    try:
                        got = ep.cq_read()
                    except Exception as e:  # noqa: BLE001
                        trace("cq error", e)
                        raise
                    if got:
                        trace("done", got)
                    done.update(got)
                    if time.time() - t0 > stall_s:
                        xf.pump()
                        if dev:
                            trace("counters", [ep.counters(a) for a in addrs])
                        raise TimeoutError(
                            f"rank {rank}: op {ids[ctx]} stalled; in flight "
                            f"{[ids[c] for c, _ in inflight]}; waiting recvs "
                            f"{xf.waiting()}; unexpected {xf.stray()}")

            ids = {}
            for o in ops:
                members = groups[o["g"]]
                if rank not in members:
                    continue
                pos = members.index(rank)
                ctx, check = _submit(ep, coll, oracle, o, members, addrs[o["g"]], pos, mem)
                ids[ctx] = (o["i"], o["g"], o["coll"], o["algo"], o["count"])
                trace("submit", ctx, ids[ctx])
                inflight.append((ctx, check))
                while len(inflight) > DEPTH or (inflight and inflight[0][0] in done):
                    ctx, check = inflight[0]
                    reap(ctx)
                    check()
                    inflight.pop(0)
            while inflight:
                ctx, check = inflight[0]
                reap(ctx)
                check()
                inflight.pop(0)
            if refuse_every and world > 1:
                assert xf.refused > 0, "no post was refused"
            for mc in handles:
                coll.lib().lfa_mc_close(mc)
            # the algorithm is endpoint state that every member must agree
            # on; each rank's last set_algo was its own last operation's
            ep.set_algo(coll.ALGO_TREE)
            ep.wait(ep.barrier())
        finally:
            ep.close()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def _run(world, seed, nops, dev=False, timeout=200, host_rank=-1, gchunk=0,
         refuse_every=0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    queues = [ctx.Queue() for _ in range(world)]
    procs = [ctx.Process(target=_worker,
                         args=(r, world, queues, seed, nops, q, dev, host_rank, gchunk,
                               refuse_every))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=timeout)
            except Exception:  # noqa: BLE001 — a rank hung: report the others
                break
            results[r] = msg
    finally:
        t_end = time.time() + 20
        for p in procs:
            p.join(timeout=max(0.1, t_end - time.time()))
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


@pytest.mark.parametrize("world,seed", [(2, 11), (3, 12), (4, 13), (5, 14), (6, 15), (3, 16)])
def test_random_programs_across_processes(world, seed):
    _run(world, seed, 400)


@pytest.mark.parametrize("world,seed,every", [(3, 41, 3), (4, 42, 7)])
def test_random_programs_with_transport_pushback(world, seed, every):
    """The same programs while the owner refuses every k-th send / receive
    post with -FI_EAGAIN: the provider re-posts it on a later progress call
    (coll_coll.c:845-852) and every result stays exact."""
    _run(world, seed, 300, refuse_every=every)


@pytest.mark.gpu
@pytest.mark.parametrize("world,seed", [(2, 21), (3, 22), (4, 23), (5, 24)])
def test_random_programs_gpu_peer_domains(world, seed):
    """The same programs with DEVICE buffers on GPU peer domains (processes
    sharing the GPU): every algorithm's kernels, transfers staged through
    the owner's transport, and under P2P / AUTO the IPC workspaces, flag
    barriers and one-shot kernels of three groups at once."""
    _run(world, seed, 160, dev=True, timeout=100)


@pytest.mark.gpu
@pytest.mark.parametrize("world,seed,gchunk", [(3, 31, 0), (4, 32, 4000)])
def test_random_programs_gpu_mixed_members(world, seed, gchunk):
    """The same with rank 0 handing in HOST buffers on its GPU peer domain
    while the others hand in device buffers (staged through device copies
    under P2P, the host form of the schedule otherwise), and with a group
    chunk on every member (P2P allreduce / reduce split into the same chunks
    everywhere)."""
    _run(world, seed, 160, dev=True, timeout=100, host_rank=0, gchunk=gchunk)


@pytest.mark.gpu
def test_random_programs_gpu_with_transport_pushback():
    """GPU peer domains (device buffers, staged transfers, P2P workspaces)
    while the owner refuses every 5th post with -FI_EAGAIN."""
    _run(3, 51, 160, dev=True, timeout=100, refuse_every=5)


def _join_worker(rank, world, queues, q):
    try:
        import oracle
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, MpXfer(rank, queues))
        try:
            # every member a different algorithm at join time: the join's own
            # agreement (a BAND allreduce over the parent) must not follow it
            ep.set_algo([coll.ALGO_RD, coll.ALGO_TREE, coll.ALGO_TREE_COLL][rank % 3])
            members = [world - 1] + list(range(world - 1))
            mc, _ = ep.join(members)
            ep.wait_join()
            ep.set_algo(coll.ALGO_RD)
            rng = np.random.default_rng(3)
            ins = [rng.uniform(0.9, 1.1, 1001).astype(np.float32) for _ in range(world)]
            res = np.zeros(1001, np.float32)
            pos = members.index(rank)
            ep.wait(ep.allreduce(ins[pos], res, 1001, 8, 2, coll_addr=ep.mc_addr(mc)))
            want = oracle.allreduce(2, 8, ins)[0]
            assert res.tobytes() == want.tobytes()
            coll.lib().lfa_mc_close(mc)
        finally:
            ep.close()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [3, 5])
def test_join_agreement_ignores_selected_algorithm(world):
    """The join's group-id agreement runs one fixed schedule (TREE) whatever
    algorithm each member has selected for its own collectives; round 3 found
    internal collectives — the join agreement and the P2P workspace
    handshake, which starts from progress at a different point of each
    member's calls — following the endpoint's current setting, which members
    may hold differently at that moment (a hang when the schedules differ)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    queues = [ctx.Queue() for _ in range(world)]
    procs = [ctx.Process(target=_join_worker, args=(r, world, queues, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=60)
            except Exception:  # noqa: BLE001
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _bench_loop_worker(rank, world, queues, q):
    try:
        import oracle
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, MpXfer(rank, queues))
        try:
            rng = np.random.default_rng(9)
            ins = [rng.uniform(0.9, 1.1, 1024).astype(np.float32) for _ in range(world)]
            want = oracle.allreduce(2, 8, ins)[0]
            res = np.zeros(1024, np.float32)
            for algo in (coll.ALGO_TREE, coll.ALGO_RD):
                ep.set_algo(algo)
                us = ep.bench_loop(3, ins[rank], res, 1024, 8, 2, reps=50)
                assert us > 0 and res.tobytes() == want.tobytes(), (algo, us)
                off, ln = coll.block(1024, world, rank)
                rs = np.zeros(ln, np.float32)
                ep.bench_loop(5, ins[rank], rs, 1024, 8, 2, reps=20)
                assert rs.tobytes() == want[off:off + ln].tobytes()
                rr = np.zeros(1024, np.float32)
                ep.bench_loop(6, ins[rank], rr, 1024, 8, 2, root=world - 1, reps=20)
                if rank == world - 1:
                    assert rr.tobytes() == want.tobytes()
        finally:
            ep.close()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_bench_c_loop_across_processes():
    """bench.py's C-timed latency loop (liblfa_bench.so lfa_bench_loop):
    allreduce / reduce_scatter / reduce submitted and reaped in C across 3
    processes, results equal to the oracle."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    queues = [ctx.Queue() for _ in range(world)]
    procs = [ctx.Process(target=_bench_loop_worker, args=(r, world, queues, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=60)
            except Exception:  # noqa: BLE001
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))
