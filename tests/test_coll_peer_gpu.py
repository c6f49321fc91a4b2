"""The C executor with the gfx950 kernels across PROCESSES, on the GPU.

Two and three processes share the box's one MI355X.  Each opens a
peer-transfer domain on device 0 (lfa_coll_domain_open_peer): the collective
provider builds the same schedules as on every other path, the owner's
transport (gloo, tests/gloo_xfer.py) carries every SEND/RECV as host bytes
(staged device <-> host by the provider), and every REDUCE / TREE / COPY item
runs as the product kernels on the endpoint's stream.  With LFA_ALGO_P2P the
members exchange IPC handles of their symmetric workspaces (the handshake as
host collectives, from progress), and the system-scope tree_put kernel reads
the other processes' inputs and writes their outputs through the IPC
mappings — the P2P path's mechanics, on one device.  Results must equal
prov/coll's (the oracle) bit for bit, including when one member hands in
host buffers and the others device buffers.  The oracle is only the checker.
"""
import os
import sys
import queue
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(oracle, dt, count, world, seed):
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    if nd.kind == "f":
        return [rng.uniform(0.9, 1.1, count).astype(nd) for _ in range(world)]
    return [rng.integers(0, 255, count).astype(nd) for _ in range(world)]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _ready(*_):
    """fi_allreduce takes buffers that are ready when it is called (there is
    no stream in libfabric's API): torch's copies and fills, on torch's
    stream, must have finished before the provider's stream touches them."""
    torch.cuda.synchronize()


def _body(ep, rank, world, oracle, coll):
    torch.cuda.synchronize()
    for algo in (coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P):
        ep.set_algo(algo)
        for dt, op, count in ((8, 2, 70_001), (9, 3, 4099), (6, 6, 6000), (1, 7, 33),
                              (8, 0, 1000)):
            sends = _inputs(oracle, dt, count, world, 4321 + count + algo)
            want = oracle.allreduce(op, dt, sends)[0]
            nd = sends[0].dtype
            # rank 0 hands in host buffers, the others device buffers: one
            # schedule either way
            # (under P2P the host member's buffers are staged through the
            # device so it follows the P2P schedule too)
            host = rank == 0 and algo in (coll.ALGO_TREE, coll.ALGO_P2P)
            x = sends[rank] if host else _dev(sends[rank])
            res = np.zeros(count, nd) if host else torch.zeros(count, dtype=x.dtype,
                                                                device="cuda")
            _ready()
            ep.wait(ep.allreduce(x, res, count, dt, op))
            got = res if host else res.cpu().numpy()
            assert got.tobytes() == want.tobytes(), f"allreduce algo={algo} dt={dt} n={count}"
            off, ln = coll.block(count, world, rank)
            xs = _dev(sends[rank])
            rs = torch.zeros(max(ln, 1), dtype=xs.dtype, device="cuda")
            _ready()
            ep.wait(ep.reduce_scatter(xs, rs, count, dt, op))
            assert rs[:ln].cpu().numpy().tobytes() == want[off:off + ln].tobytes()
            for root in range(world):
                r = torch.zeros(count, dtype=rs.dtype, device="cuda")
                _ready()
                ep.wait(ep.reduce(xs, r, count, root, dt, op))
                if rank == root:
                    assert r.cpu().numpy().tobytes() == want.tobytes(), f"reduce {root}"
    ep.set_algo(coll.ALGO_TREE)
    x = torch.arange(10, dtype=torch.int32, device="cuda") + 100 * rank
    res = torch.zeros(10 * world, dtype=torch.int32, device="cuda")
    _ready()
    ep.wait(ep.allgather(x, res, 10, 4))
    assert torch.equal(res.cpu(), torch.cat([torch.arange(10, dtype=torch.int32) + 100 * k
                                             for k in range(world)]))
    for root in range(world):
        b = (torch.arange(7, dtype=torch.float64, device="cuda") * (root + 1) if rank == root
             else torch.zeros(7, dtype=torch.float64, device="cuda"))
        _ready()
        ep.wait(ep.broadcast(b, 7, root, 9))
        assert torch.equal(b.cpu(), torch.arange(7, dtype=torch.float64) * (root + 1))
        src = (torch.arange(5 * world, dtype=torch.int64, device="cuda") if rank == root
               else None)
        out = torch.zeros(5, dtype=torch.int64, device="cuda")
        _ready()
        ep.wait(ep.scatter(src, out, 5, root, 6))
        assert torch.equal(out.cpu(), torch.arange(5) + 5 * rank)
    ep.wait(ep.barrier())
    # several in flight: completions in issue order, each result exact
    outs, ctxs = [], []
    for k in range(4):
        sends = _inputs(oracle, 8, 5000 + k, world, 99 + k)
        want = oracle.allreduce(2, 8, sends)[0]
        r = torch.zeros(want.size, dtype=torch.float32, device="cuda")
        xs = _dev(sends[rank])
        _ready()
        ctxs.append(ep.allreduce(xs, r, want.size, 8, 2))
        outs.append((r, want, xs))
    done = []
    while len(done) < len(ctxs):
        done += ep.cq_read()
    assert done == ctxs
    for r, want, _ in outs:
        assert r.cpu().numpy().tobytes() == want.tobytes()
    # P2P with operations in flight: each waits for the one before it (they
    # share the symmetric workspace), the middle one grows the workspace
    # (12 MiB > the 8 MiB first size) through the asynchronous handshake
    ep.set_algo(coll.ALGO_P2P)
    outs, ctxs = [], []
    for k, n in enumerate((5000, 3 << 20, 777)):
        sends = _inputs(oracle, 8, n, world, 7 + k)
        want = oracle.allreduce(2, 8, sends)[0]
        r = torch.zeros(n, dtype=torch.float32, device="cuda")
        xs = _dev(sends[rank])
        _ready()
        ctxs.append(ep.allreduce(xs, r, n, 8, 2))
        outs.append((r, want, xs))
    done = []
    while len(done) < len(ctxs):
        done += ep.cq_read()
    assert done == ctxs
    for r, want, _ in outs:
        assert r.cpu().numpy().tobytes() == want.tobytes(), "P2P in flight"
    _group_chunk(ep, rank, world, oracle, coll)
    ep.set_algo(coll.ALGO_TREE)
    _set_order(ep, rank, world, oracle, coll)
    # a mixed pair on one member is refused
    from libfabric_amd.coll import CollError
    with pytest.raises(CollError):
        ep.allreduce(torch.zeros(4, device="cuda"), np.zeros(4, np.float32), 4, 8, 2)


def _group_chunk(ep, rank, world, oracle, coll):
    """VERDICT r2 #4 across processes: under one group chunk (the same value
    on every member, lfa_coll_ep_set_group_chunk) rank 0 hands in HOST
    buffers and pipelines them chunk by chunk while the device members split
    the same operation into the same chunks; TREE and P2P, allreduce and
    reduce_scatter, odd chunk sizes and a ragged last chunk, all bit-exact
    against the oracle.  A member that chunked alone would issue a different
    schedule and the group would hang or mismatch."""
    count = 300_001
    try:
        for algo in (coll.ALGO_TREE, coll.ALGO_P2P):
            ep.set_algo(algo)
            for group in (1 << 16, 3 * 4 * 1000 + 4):
                ep.set_group_chunk(group)
                sends = _inputs(oracle, 8, count, world, 77 + group + algo)
                want = oracle.allreduce(2, 8, sends)[0]
                host = rank == 0
                x = sends[rank] if host else _dev(sends[rank])
                r = (np.zeros(count, np.float32) if host
                     else torch.zeros(count, dtype=torch.float32, device="cuda"))
                _ready()
                ep.wait(ep.allreduce(x, r, count, 8, 2))
                got = r if host else r.cpu().numpy()
                assert got.tobytes() == want.tobytes(), ("group chunk allreduce", algo, group)
                off, ln = coll.block(count, world, rank)
                rs = (np.zeros(ln, np.float32) if host
                      else torch.zeros(ln, dtype=torch.float32, device="cuda"))
                _ready()
                ep.wait(ep.reduce_scatter(x, rs, count, 8, 2))
                got = rs if host else rs.cpu().numpy()
                assert got.tobytes() == want[off:off + ln].tobytes(), (
                    "group chunk reduce_scatter", algo, group)
                root = world - 1             # a device member, or the host one
                for rt in sorted({0, root}):
                    rr = (np.zeros(count, np.float32) if host
                          else torch.zeros(count, dtype=torch.float32, device="cuda"))
                    _ready()
                    ep.wait(ep.reduce(x, rr, count, rt, 8, 2))
                    if rank == rt:
                        got = rr if host else rr.cpu().numpy()
                        assert got.tobytes() == want.tobytes(), ("group chunk reduce", algo,
                                                                 group, rt)
    finally:
        ep.set_group_chunk(coll.GROUP_CHUNK_AUTO)   # the default


def _set_order(ep, rank, world, oracle, coll):
    """VERDICT r2 #1 on the GPU: a group over a set whose order is not
    ascending (prov/coll's av_set after stride + insert (+ remove): N = 3
    gives [0, 2, 1], N = 5 [0, 3, 4, 1]) numbers its members by set position:
    device-buffer allgather blocks in set order, a float SUM allreduce equal
    to the oracle fed in set order (TREE on the kernels, and P2P's one-shot
    and two-barrier paths), reduce and broadcast roots as group ranks."""
    from test_coll_host import _set_order as order_of   # the reference's order rules
    order = order_of(world)
    mc, _ = ep.join(order)
    ep.wait_join()
    addr = ep.mc_addr(mc)
    if rank in order:
        pos = order.index(rank)
        for algo in (coll.ALGO_TREE, coll.ALGO_P2P):
            ep.set_algo(algo)
            for count in (4099, 300_001):          # one-shot / copy + barriers + tree
                sends = _inputs(oracle, 8, count, world, 555 + count)
                want = oracle.allreduce(2, 8, [sends[m] for m in order])[0]
                x = _dev(sends[rank])
                r = torch.zeros(count, dtype=torch.float32, device="cuda")
                _ready()
                ep.wait(ep.allreduce(x, r, count, 8, 2, coll_addr=addr))
                assert r.cpu().numpy().tobytes() == want.tobytes(), ("set order", algo, count)
                root = len(order) - 1
                r.zero_()
                _ready()
                ep.wait(ep.reduce(x, r, count, root, 8, 2, coll_addr=addr))
                if pos == root:
                    assert r.cpu().numpy().tobytes() == want.tobytes(), ("reduce", algo)
        ep.set_algo(coll.ALGO_TREE)
        g = torch.tensor([rank, 3 * rank], dtype=torch.int64, device="cuda")
        out = torch.zeros(2 * len(order), dtype=torch.int64, device="cuda")
        _ready()
        ep.wait(ep.allgather(g, out, 2, 6, coll_addr=addr))
        assert out.cpu().tolist() == [v for m in order for v in (m, 3 * m)]
        b = (torch.arange(5, dtype=torch.float64, device="cuda") + rank if pos == 1
             else torch.zeros(5, dtype=torch.float64, device="cuda"))
        _ready()
        ep.wait(ep.broadcast(b, 5, 1 if len(order) > 1 else 0, 9, coll_addr=addr))
        src = order[1] if len(order) > 1 else order[0]
        if len(order) > 1:
            assert b.cpu().tolist() == (np.arange(5) + src).tolist()
    coll.lib().lfa_mc_close(mc)
    ep.wait(ep.barrier())




def _share_gpu(world):
    """Before this process's first HIP call: with more than 4 processes on
    the one GPU, 2 hardware queues each instead of the default 4.  Past the
    scheduler's queue slots the GPU time-slices the processes' queues, and a
    one-shot kernel waiting for a peer whose queue is not mapped waits out a
    quantum: 8 processes took 10-26 ms per 4 KiB allreduce with 4 queues each
    and 0.1-0.2 ms with 2 (tools/probe_p2p_latency.py) —
    slow enough to time tests out.  One process per GPU (the product's
    layout) never meets this."""
    if world > 4:
        # the test process itself holds queues too (every GPU test before this
        # one ran in it): 8 workers at 2 queues each beside it crossed the
        # limit in one round-4 suite run (the 8-process test timed out there
        # and passed alone), so 6+ workers take 1 queue each — 47 us per
        # 4 KiB one-shot at 8 processes against 31 us at 2 queues and 10.6 ms
        # at 3 (tools/gpu.sh procs, profiles/r04_procs_queues.jsonl)
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("LFA_TEST_HW_QUEUES",
                                                         "1" if world > 5 else "2")


def _kfd_queues(pid=None):
    """Hardware queues the process holds on the GPU (KFD's sysfs view), or
    None where that is not readable."""
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid or os.getpid()}/queues"))
    except OSError:
        return None

def _log_stderr(tag, rank, world):
    """PEER_LOG_DIR set: this rank's stderr (LFA_DEBUG / LFA_TRACE lines) goes
    to a file there, so a hung multi-process test leaves per-rank traces."""
    d = os.environ.get("PEER_LOG_DIR")
    if d:
        f = open(os.path.join(d, f"{tag}_w{world}_r{rank}.log"), "w", buffering=1)
        os.dup2(f.fileno(), 2)

def _worker(rank, world, port, q):
    _log_stderr("exec", rank, world)
    try:
        # LFA_DEBUG: a failing HIP call is named on stderr (and its code is
        # the completion's prov_errno)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        xfer = GlooXfer()
        ep = coll.HostEndpoint(rank, world, xfer, device=0)
        try:
            _body(ep, rank, world, oracle, coll)
            if world > 1:
                assert xfer.sent > 0 and xfer.received > 0
        finally:
            if os.environ.get("PEER_LOG_DIR"):
                sys.stderr.write(f"open fds before close: {len(os.listdir('/proc/self/fd'))}\n")
            ep.close()
            if os.environ.get("PEER_LOG_DIR"):
                sys.stderr.write(f"open fds after close: {len(os.listdir('/proc/self/fd'))}\n")
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_c_executor_gpu_kernels_across_processes(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=100)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, (f"test process holds {_kfd_queues()} GPU queues; " +
                     "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items())))


def _growth_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            # sizes that grow the symmetric workspace again and again, with
            # small operations between them, all in flight at once
            sizes = (1000, 3 << 20, 777, 6 << 20, 5, 11 << 20, 4096, 23 << 20, 3 << 20)
            for rep in range(2):
                outs, ctxs = [], []
                for k, n in enumerate(sizes):
                    sends = _inputs(oracle, 8, n, world, 1000 * rep + k)
                    want = oracle.allreduce(2, 8, sends)[0]
                    r = torch.zeros(n, dtype=torch.float32, device="cuda")
                    xs = _dev(sends[rank])
                    _ready()
                    ctxs.append(ep.allreduce(xs, r, n, 8, 2))
                    outs.append((r, want, xs))
                done = []
                while len(done) < len(ctxs):
                    done += ep.cq_read()
                assert done == ctxs
                for (r, want, _), n in zip(outs, sizes):
                    assert r.cpu().numpy().tobytes() == want.tobytes(), f"P2P n={n} rep={rep}"
            assert not ep.transport_errors, ep.transport_errors
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_p2p_workspace_growth_in_flight():
    """LFA_ALGO_P2P across two processes: nine allreduces queued at once, four
    of which grow the IPC-shared symmetric workspace (the asynchronous
    handshake from progress, each after the operations before it), twice
    over; every result bit-exact."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_growth_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=110)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _spawn(target, world, timeout=110, args=()):
    """Run `target(rank, world, port, q, *args)` in `world` spawned processes
    and fail with every rank's message unless all put "ok"."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *args))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=timeout)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _ticket_wrap_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            base = (1 << 32) - 3
            ep.seed_ticket(base)
            # one-shot buckets and two-barrier ones, in flight together,
            # with tickets 2^32-2 ... 2^32+5: 0xffffffff is one of them
            sizes = (1000, 3 << 18, 5, 4096, 70_001, 1 << 20, 33, 2048)
            outs, ctxs = [], []
            for k, n in enumerate(sizes):
                sends = _inputs(oracle, 8, n, world, 500 + k)
                want = oracle.allreduce(2, 8, sends)[0]
                r = torch.zeros(n, dtype=torch.float32, device="cuda")
                xs = _dev(sends[rank])
                _ready()
                ctxs.append(ep.allreduce(xs, r, n, 8, 2))
                outs.append((r, want, xs))
            done = []
            while len(done) < len(ctxs):
                done += ep.cq_read()
            assert done == ctxs
            for (r, want, _), n in zip(outs, sizes):
                assert r.cpu().numpy().tobytes() == want.tobytes(), f"P2P n={n}"
            c = ep.counters()
            assert c["p2p_ops"] == base + len(sizes) and c["timed_out"] == 0, c
            assert c["oneshot"] > 0 and c["flag_barriers"] > 0, c
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_p2p_tickets_cross_2_pow_32():
    """the per-group P2P ticket and the timed-out status word are
    64-bit.  With 32-bit ones, ticket 0xffffffff equalled the 'no timeout'
    value, so that operation failed with ETIMEDOUT and the group refused P2P
    from then on.  Tickets seeded just below 2^32 on both members, eight
    one-shot and two-barrier allreduces in flight across the boundary: all
    complete, bit-exact, with no timeout recorded."""
    _spawn(_ticket_wrap_worker, 2)


def _stage_pool_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1",
                          LFA_STAGE_POOL_BYTES=str(8 << 20))
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        try:
            ep.set_algo(coll.ALGO_P2P)
            ep.set_group_chunk(0)
            # rank 0 on host buffers: every operation stages its input and
            # output through the pool; a sweep of sizes, each larger than the
            # last, would have kept every one of them
            for k, mib in enumerate((1, 2, 3, 5, 6)):
                n = (mib << 20) // 4
                sends = _inputs(oracle, 8, n, world, 900 + k)
                want = oracle.allreduce(2, 8, sends)[0]
                x = sends[rank] if rank == 0 else _dev(sends[rank])
                r = np.zeros(n, np.float32) if rank == 0 else torch.zeros(n, device="cuda")
                _ready()
                ep.wait(ep.allreduce(x, r, n, 8, 2))
                got = r if rank == 0 else r.cpu().numpy()
                if got.tobytes() != want.tobytes():
                    msg = f"allreduce of {mib} MiB wrong"
            held = ep.stage_bytes()
            if held > (8 << 20):
                msg = f"idle staging {held} B after the sweep, cap 8 MiB"
            ep.flush()
            if ep.stage_bytes():
                msg = f"{ep.stage_bytes()} B still staged after flush"
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_staging_pool_is_bounded():
    """the peer domain's staging pool keeps at most its cap of
    idle bytes (LFA_STAGE_POOL_BYTES, 1 GiB by default; 8 MiB here) across
    a sweep of sizes with a host-buffer member, results exact, and
    lfa_coll_ep_flush frees every idle buffer."""
    _spawn(_stage_pool_worker, 2)


def _ws_cycle_worker(rank, world, port, q, cap):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        if cap is not None:
            os.environ["LFA_WS_CACHE_BYTES"] = str(cap)
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        msg = "ok"
        held = []
        # a second GPU domain open throughout: the cache lives while any GPU
        # domain of the process is open and is freed at the last close
        anchor = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        for c in range(6):
            # every cycle: a new endpoint whose workspace grows three times,
            # then closes — the address pattern of round 4's stale exports
            ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
            try:
                ep.set_algo(coll.ALGO_P2P)
                ep.set_group_chunk(0)
                for mib in (1, 6, 12):
                    n = (mib << 20) // 4
                    x = torch.full((n,), float(rank + 1 + c), device="cuda")
                    r = torch.empty_like(x)
                    torch.cuda.synchronize()
                    ep.wait(ep.allreduce(x, r, n, 8, 2))
                    want = world * (world + 1) / 2 + world * c
                    if not bool((r == want).all()):
                        msg = f"cycle {c}: {mib} MiB allreduce wrong"
            finally:
                ep.close()
            held.append(coll.ws_cached_bytes())
            dist.barrier()
        if cap is None:
            # every size released in cycle 0 is taken back by cycle 1 and
            # released again: the cache holds the same bytes every cycle
            if not held[0] or len(set(held)) != 1:
                msg = f"kept workspace bytes per cycle {held}"
        elif max(held) > cap:
            msg = f"kept {max(held)} B over the {cap} B cap"
        anchor.close()
        if msg == "ok" and (coll.ws_cached_bytes() or coll.ws_quarantined_bytes()):
            msg = (f"after the last domain closed: {coll.ws_cached_bytes()} B cached, "
                   f"{coll.ws_quarantined_bytes()} B quarantined")
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [None, 40 << 20], ids=["default", "cap40mib"])
def test_released_workspaces_are_reused(cap):
    """Round 4: an exported workspace freed and a new one
    allocated at its address was refused an export, or exported as the OLD
    memory, so its owner waited for posts that landed elsewhere.  Released
    workspaces are now kept and taken back by the next growth of that size;
    every peer also checks the owner's identity word through its mapping.
    Four processes, six endpoint cycles, three growths each, beside a
    second GPU domain that stays open; once that one closes too (the last
    GPU domain of the process), nothing is kept."""
    _spawn(_ws_cycle_worker, 4, args=(cap,))


def _ws_mem_worker(rank, world, port, q, kind):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        if kind is not None:
            os.environ["LFA_WS_MEM"] = kind
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        want_kind = kind or "uncached"
        assert coll.ws_mem() == want_kind, (coll.ws_mem(), want_kind)
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            ep.set_group_chunk(0)
            # one-shot (flags + slots), then the two-barrier form (staging
            # copy, flag barriers, system-scope tree_put over the peers'
            # workspaces, unstage) and a growth, then one-shots again on the
            # grown workspace: every word a peer writes lives in the kind
            for k, (dt, op, n) in enumerate(((8, 2, 1024), (9, 3, 5000), (8, 2, 3 << 20),
                                             (6, 6, 700_001), (8, 2, 4097), (1, 7, 33))):
                sends = _inputs(oracle, dt, n, world, 31 + k)
                want = oracle.allreduce(op, dt, sends)[0]
                xs = _dev(sends[rank])
                r = torch.zeros_like(xs)
                _ready()
                ep.wait(ep.allreduce(xs, r, n, dt, op))
                assert r.cpu().numpy().tobytes() == want.tobytes(), f"allreduce {k}"
                off, ln = coll.block(n, world, rank)
                rs = torch.zeros(max(ln, 1), dtype=xs.dtype, device="cuda")
                _ready()
                ep.wait(ep.reduce_scatter(xs, rs, n, dt, op))
                assert rs[:ln].cpu().numpy().tobytes() == want[off:off + ln].tobytes(), \
                    f"reduce_scatter {k}"
            c = ep.counters()
            assert c["oneshot"] >= 6 and c["flag_barriers"] >= 4, c
            info = ep.ws_info()
            assert info["mem"] == want_kind and info["mapped"] == world, info
            assert info["region"] >= (3 << 20) * 4, info
            assert not ep.transport_errors, ep.transport_errors
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,kind", [(2, None), (3, None), (8, None), (2, "fine"),
                                        (2, "coarse")],
                         ids=["2-uncached-default", "3-uncached-default", "8-uncached-default",
                              "2-fine", "2-coarse"])
def test_p2p_workspace_memory_kind(world, kind):
    """peers post epochs, push one-shot slots and write
    blocks into a member's workspace while its kernels run, so on the 8-GPU
    node those writes cross xGMI into the owner's HBM.  The workspace is
    allocated uncached by default (hipDeviceMallocUncached: no GPU's L2 holds
    its lines), exported and mapped over IPC like before; the one-shot and
    two-barrier P2P paths and a growth run on it bit-exact, and every member
    maps every peer's workspace.  fine / coarse (LFA_WS_MEM) are the A/B."""
    _spawn(_ws_mem_worker, world, args=(kind,))


def _pinned_member_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        tdt = {8: torch.float32, 9: torch.float64}

        def buf(a, off=0):
            # rank 0: pinned host; rank 1: device; rank 2: pinned host at an
            # offset that is not 16-B aligned (the byte-wise bodies)
            t = torch.from_numpy(np.ascontiguousarray(a))
            if rank == 1:
                return t.to("cuda")
            raw = torch.zeros(t.numel() * t.element_size() + 64, dtype=torch.uint8).pin_memory()
            o = 8 if rank == 2 else 0
            v = raw[o:o + t.numel() * t.element_size()].view(t.dtype)
            v.copy_(t)
            return v

        try:
            ep.set_algo(coll.ALGO_P2P)
            ep.set_group_chunk(0)
            for k, nbytes in enumerate((4096, 1 << 20, (3 << 20) + 8)):
                n = nbytes // 4
                sends = _inputs(oracle, 8, n, world, 1200 + k)
                want = oracle.allreduce(2, 8, sends)[0]
                x, r = buf(sends[rank]), buf(np.zeros(n, np.float32))
                _ready()
                ep.wait(ep.allreduce(x, r, n, 8, 2))
                if r.cpu().numpy().tobytes() != want.tobytes():
                    msg = f"allreduce {nbytes} B wrong"
                # double PROD reduce_scatter, ragged blocks
                m = nbytes // 8 + 1
                sd = _inputs(oracle, 9, m, world, 1300 + k)
                wantd = oracle.allreduce(3, 9, sd)[0]
                off, ln = coll.block(m, world, rank)
                xd, rd = buf(sd[rank]), buf(np.zeros(max(ln, 1), np.float64))
                _ready()
                ep.wait(ep.reduce_scatter(xd, rd, m, 9, 3))
                if rd.cpu().numpy()[:ln].tobytes() != wantd[off:off + ln].tobytes():
                    msg = f"reduce_scatter {nbytes} B wrong"
                for root in (0, 1):
                    rr = buf(np.zeros(n, np.float32))
                    _ready()
                    ep.wait(ep.reduce(x, rr, n, root, 8, 2))
                    if rank == root and rr.cpu().numpy().tobytes() != want.tobytes():
                        msg = f"reduce {nbytes} B to {root} wrong"
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_p2p_pinned_host_members():
    """LFA_ALGO_P2P with PINNED host members (ranks 0 and 2; rank 2's
    buffers 8 bytes off 16-B alignment) and a device member (rank 1): the
    host members run the device schedule on their buffers' mappings with
    nothing staged — the one-shot (4 KiB) and the staged-workspace schedule
    (1 MiB, 3 MiB + 8 B) — allreduce, ragged double PROD reduce_scatter and
    reduce to a host and a device root, bit-exact with the oracle."""
    _spawn(_pinned_member_worker, 3)


def _bounce_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        try:
            ep.set_algo(coll.ALGO_P2P)
            ep.set_group_chunk(0)
            # 20 operations in flight: more than the 8 bounce blocks, so the
            # later ones stage; sizes on both sides of LFA_BOUNCE_BYTES
            ops = []
            for k in range(20):
                nbytes = (4096, 65536 + 4, 1 << 20, (1 << 20) + 8)[k % 4]
                kind = ("allreduce", "reduce_scatter", "reduce")[k % 3]
                n = nbytes // 8
                sends = _inputs(oracle, 9, n, world, 1500 + k)
                want = oracle.allreduce(3, 9, sends)[0]
                # rank 0 pageable numpy, rank 1 device
                x = sends[rank].copy() if rank == 0 else _dev(sends[rank])
                if kind == "reduce_scatter":
                    off, ln = coll.block(n, world, rank)
                    want = want[off:off + ln]
                    cnt_out = max(ln, 1)
                else:
                    cnt_out = n
                # a non-root's result is never written — rank 0's
                # holds a sentinel that must survive
                r = (np.full(cnt_out, -12345.5, np.float64) if rank == 0
                     else torch.zeros(cnt_out * 8, dtype=torch.uint8, device="cuda"))
                _ready()
                if kind == "allreduce":
                    ctx = ep.allreduce(x, r, n, 9, 3)
                elif kind == "reduce_scatter":
                    ctx = ep.reduce_scatter(x, r, n, 9, 3)
                else:
                    ctx = ep.reduce(x, r, n, k % 2, 9, 3)
                check = kind != "reduce" or rank == k % 2
                if not check and rank == 0:
                    want = np.full(cnt_out, -12345.5, np.float64)
                    check = True
                ops.append((ctx, r, want if check else None, f"{kind} {nbytes} B #{k}"))
            # a non-root in-place reduce (buf == result) keeps its input
            n = 4096 // 8
            sends = _inputs(oracle, 9, n, world, 1777)
            x = sends[rank].copy() if rank == 0 else _dev(sends[rank])
            _ready()
            ops.append((ep.reduce(x, x, n, 1, 9, 3), x,
                        sends[0] if rank == 0 else None, "in-place non-root reduce"))
            ep.wait(ops[-1][0], timeout_s=60)
            for ctx, r, want, what in ops:
                if want is None:
                    continue
                got = r if rank == 0 else r.cpu().numpy().view(np.float64)
                if got[:want.size].tobytes() != want.tobytes():
                    msg = f"{what} wrong"
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_p2p_pageable_member_bounce_blocks():
    """A PAGEABLE host member (numpy) under LFA_ALGO_P2P: operations of at
    most LFA_BOUNCE_BYTES go through a pinned bounce block (input copied in
    on the CPU at submit, the schedule on the block's mapping, the result
    copied out at completion); 20 in flight, more than the pool's 8 blocks,
    so later ones and the larger ones stage through HBM as before.
    allreduce, ragged reduce_scatter, reduce to either root, double PROD,
    bit-exact with the oracle."""
    _spawn(_bounce_worker, 2)


def _chunk_error_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          LFA_SIG_TIMEOUT_MS="300")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import ctypes
        import time
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        try:
            ep.set_algo(coll.ALGO_P2P)
            # members disagree on the group chunk (a caller error): rank 0
            # splits 8 MiB into 4 chunks, rank 1 into 2, so rank 0's third
            # chunk waits for a peer that never arrives and fails — a middle
            # chunk — and its fourth fails behind it.  Chunks of 2 and 4 MiB
            # both take the staged P2P schedule (above the one-shot's 2 MiB
            # over the members), whose barriers pair whatever the sizes
            ep.set_group_chunk((2 << 20) * (rank + 1))
            n = 2 << 20
            xs = torch.ones(n, dtype=torch.float32, device="cuda")
            rs = torch.zeros(n, dtype=torch.float32, device="cuda")
            _ready()
            ctx = ep.allreduce(xs, rs, n, 8, 2)
            L = coll.lib()
            ok, errs = [], []
            t0 = time.time()
            while time.time() - t0 < 3.0:
                got = L.lfa_cq_read(ep.ep, ep._ents, 16)
                if got > 0:
                    ok += [ep._ents[i].op_context for i in range(got)]
                elif got == -coll.EIO:
                    e = coll.CqErrEntry()
                    assert L.lfa_cq_readerr(ep.ep, ctypes.byref(e)) == 1
                    errs.append((e.op_context, e.prov_errno))
            if rank == 0 and (ok or [c for c, _ in errs] != [ctx] or errs[0][1] != 110):
                msg = f"rank 0: successes {ok}, errors {errs} (ctx {ctx}): want one ETIMEDOUT"
            if rank == 1 and (ok != [ctx] or errs):
                msg = f"rank 1: successes {ok}, errors {errs} (ctx {ctx}): want one success"
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_chunked_operation_posts_one_completion():
    """a group-chunked operation is ONE operation to the caller.
    Before, every chunk that failed posted its own error entry under the
    caller's context (and the last chunk a further one), so one fi_allreduce
    produced several completions.  Now the first failing chunk's error is the
    operation's only entry; a member whose chunks all succeed posts one
    success."""
    _spawn(_chunk_error_worker, 2)


def _timeout_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          LFA_SIG_TIMEOUT_MS="300")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            sends = _inputs(oracle, 8, 4096, world, 5)
            want = oracle.allreduce(2, 8, sends)[0]
            r = torch.zeros(4096, dtype=torch.float32, device="cuda")
            xs = _dev(sends[rank])
            _ready()
            ep.wait(ep.allreduce(xs, r, 4096, 8, 2))
            assert r.cpu().numpy().tobytes() == want.tobytes()
            msg = "ok"
            if rank == 1:
                # rank 0 skips this collective: the flag barrier gives up
                # after LFA_SIG_TIMEOUT_MS and the operation completes in
                # error (prov_errno ETIMEDOUT) instead of spinning forever
                import time
                t0 = time.time()
                try:
                    ep.wait(ep.allreduce(xs, r, 4096, 8, 2), timeout_s=30)
                    msg = "no error"
                except coll.CollError as e:
                    msg = "ok" if "prov_errno 110" in str(e) else f"wrong error {e}"
                if time.time() - t0 > 10:
                    msg = f"took {time.time() - t0:.1f} s"
                # the members' flag epochs now disagree: further P2P
                # operations on this endpoint are refused at submit
                if msg == "ok":
                    try:
                        ep.allreduce(xs, r, 4096, 8, 2)
                        msg = "P2P accepted after a timeout"
                    except coll.CollError:
                        pass
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_flag_barrier_timeout_is_an_error_completion():
    """LFA_ALGO_P2P's device-side flag barrier (lfa_signal.hip) is bounded:
    when a member never joins the collective, the waiting rank's operation
    completes with an error after LFA_SIG_TIMEOUT_MS, and the kernel retires;
    the endpoint then refuses further P2P operations (the members' flag
    epochs no longer agree)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=100)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _timeout_queue_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          LFA_SIG_TIMEOUT_MS="300")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        try:
            ep.set_algo(coll.ALGO_P2P)
            sends = _inputs(oracle, 8, 4096, world, 6)
            want = oracle.allreduce(2, 8, sends)[0]
            ra = torch.zeros(4096, dtype=torch.float32, device="cuda")
            rb = torch.zeros(4096, dtype=torch.float32, device="cuda")
            xs = _dev(sends[rank])
            _ready()
            ctx_a = ep.allreduce(xs, ra, 4096, 8, 2)      # every member
            if rank == 0:
                ep.wait(ctx_a)
            else:
                # B: rank 0 never calls it.  Both are queued before either
                # is reaped; A must complete normally and only B fail.
                ctx_b = ep.allreduce(xs, rb, 4096, 8, 2)
                import time
                time.sleep(1.0)                         # B's wait has timed out by now
                done, err = [], None
                t0 = time.time()
                while err is None and time.time() - t0 < 30:
                    try:
                        done += ep.cq_read()
                    except coll.CollError as e:
                        err = str(e)
                if done != [ctx_a]:
                    msg = f"completions {done} (A={ctx_a}, B={ctx_b})"
                elif err is None or "prov_errno 110" not in err:
                    msg = f"B: {err}"
                elif ra.cpu().numpy().tobytes() != want.tobytes():
                    msg = "A's result is wrong"
                else:
                    try:                                # the group refuses P2P now
                        ep.allreduce(xs, rb, 4096, 8, 2)
                        msg = "P2P accepted on the timed-out group"
                    except coll.CollError:
                        pass
            dist.barrier()
            # another group of the same endpoint is unaffected (ADVICE r2:
            # the timeout state is per group).  Formed by its members alone:
            # the world group's tag sequence now differs between the ranks
            # (rank 1 issued B), as it would under prov/coll
            mc, _ = ep.join_members(list(range(world)))
            ep.wait_join()
            rc = torch.zeros(4096, dtype=torch.float32, device="cuda")
            _ready()
            ep.wait(ep.allreduce(xs, rc, 4096, 8, 2, coll_addr=ep.mc_addr(mc)))
            if msg == "ok" and rc.cpu().numpy().tobytes() != want.tobytes():
                msg = "new group's P2P result is wrong"
            coll.lib().lfa_mc_close(mc)
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_timeout_fails_that_operation_not_the_one_before():
    """two P2P operations queued, the second one's wait times out
    (a member skips it), both reaped only afterwards: the first completes
    normally with its result, the second fails with ETIMEDOUT — the kernel
    records WHICH operation timed out (its ticket), not a bare flag — and the
    timed-out group refuses P2P operations while a new group of the same
    endpoint runs them."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_queue_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=100)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _oneshot_stream_worker(rank, world, port, q, seed=77, nops=48):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            seed = int(os.environ.get("ONESHOT_SEED", seed))
            rng = np.random.default_rng(seed)       # the same sequence on every rank
            ops, ctxs, n_os = [], [], 0
            # ONESHOT_MIX (diagnosis): "small" = one-shot kinds only
            kinds = (["allreduce", "reduce_scatter", "reduce"]
                     if os.environ.get("ONESHOT_MIX") == "small" else
                     ["allreduce", "reduce_scatter", "reduce", "big"])
            nops = int(os.environ.get("ONESHOT_NOPS", nops))
            meta = []
            for i in range(nops):
                kind = rng.choice(kinds)
                dt, op = [(8, 2), (9, 3), (6, 1), (2, 0), (4, 7), (1, 9)][rng.integers(6)]
                count = int(rng.integers(1, 3000)) if kind != "big" else 300_001
                sends = _inputs(oracle, dt, count, world, 1000 * seed + i)
                want = oracle.allreduce(op, dt, sends)[0]
                xs = _dev(sends[rank])
                if kind in ("allreduce", "big"):
                    r = torch.zeros(count, dtype=xs.dtype, device="cuda")
                    exp = want
                    _ready()
                    ctxs.append(ep.allreduce(xs, r, count, dt, op))
                elif kind == "reduce_scatter":
                    off, ln = coll.block(count, world, rank)
                    r = torch.zeros(max(ln, 1), dtype=xs.dtype, device="cuda")
                    exp = want[off:off + ln]
                    _ready()
                    ctxs.append(ep.reduce_scatter(xs, r, count, dt, op))
                else:
                    root = int(rng.integers(world))
                    r = torch.zeros(count, dtype=xs.dtype, device="cuda")
                    exp = want if rank == root else None
                    _ready()
                    ctxs.append(ep.reduce(xs, r, count, root, dt, op))
                ops.append((kind, r, exp, xs))
                # the planner's one-shot rule (lfa_coll_plan.c plan_p2p)
                nb = count * oracle.datatype_size(dt)
                is_os = (nb <= (4 << 20) if kind == "reduce_scatter"   # LFA_OS_RS_BYTES
                         else nb * world <= (2 << 20))     # LFA_OS_AG_BYTES_DEFAULT
                meta.append((dt, op, count, n_os if is_os else None))
                n_os += is_os
            done = []
            while len(done) < len(ctxs):
                done += ep.cq_read()
            assert done == ctxs
            # the one-shot kernel ran (not the four items it replaces)
            c = ep.counters()
            assert n_os > 0 and c["oneshot"] == n_os and not c["timed_out"], (c, n_os)
            bad = []
            for i, (kind, r, exp, _) in enumerate(ops):
                if exp is not None:
                    got = r[:exp.size].cpu().numpy()
                    if got.tobytes() != exp.tobytes():
                        w = np.nonzero(got.view(np.uint8) != exp.view(np.uint8))[0]
                        dt, op, count, os_i = meta[i]
                        bad.append(f"op {i} {kind} dt={dt} op={op} count={count} "
                                   f"oneshot#={os_i} wrong_bytes={w.size} "
                                   f"first={w[:4].tolist()} last={w[-2:].tolist()}")
            assert not bad, "; ".join(bad)
            assert not ep.transport_errors, ep.transport_errors
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,seed,nops", [(2, 77, 48), (3, 77, 48), (4, 77, 48),
                                             (5, 77, 48), (8, 77, 48), (4, 78, 160),
                                             (8, 79, 160)])
def test_oneshot_ops_in_flight_mixed(world, seed, nops):
    """LFA_ALGO_P2P operations queued at once across processes: one-shot
    allreduce / reduce_scatter / reduce (every root) of ragged small counts
    over six (datatype, op) pairs, with large two-barrier allreduces between
    them — so consecutive one-shots alternate slot parity, with slot sizes
    that change from one operation to the next, while a member may still be
    reducing the previous one — every result bit-exact.  Round 3's first
    runs failed here (parity regions that moved with the slot size, §6b)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oneshot_stream_worker, args=(r, world, port, q, seed, nops))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=110)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if results.get(r) != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _every_entry_worker(rank, world, port, q, ll="0"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1",
                          LFA_OS_LL=ll)
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import json as _json
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        from tests._cmp import assert_parity
        gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
        with open(os.path.join(gdir, "manifest.json")) as f:
            cases = [c for c in _json.load(f)["combine"] if c["op"] <= 9]   # reducing ops
        if world > 5:
            # 8 processes time-share the one GPU: every
            # datatype and op still runs, a third of the (op, type) pairs
            cases = cases[::3]
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            for c in cases:
                z = np.load(os.path.join(gdir, c["file"]))
                esz = oracle.datatype_size(c["dt"])
                # the fixture's edge-lane operands as the ranks' inputs
                pool = [np.ascontiguousarray(z[k]).view(np.uint8) for k in ("dst", "src", "out")]
                sends = [pool[k % 3].copy() for k in range(world)]
                n = sends[0].nbytes // esz
                want = oracle.allreduce(c["op"], c["dt"], [s.view(oracle.DT_NP[c["dt"]])
                                                          for s in sends])[0].view(np.uint8)
                x = torch.from_numpy(sends[rank]).cuda()
                r = torch.zeros_like(x)
                _ready()
                ep.wait(ep.allreduce(x, r, n, c["dt"], c["op"]))
                assert_parity(c["dt"], r.cpu().numpy(), want, f"allreduce {c['file']}")
                off, ln = coll.block(n, world, rank)
                rs = torch.zeros(max(ln, 1) * esz, dtype=torch.uint8, device="cuda")
                _ready()
                ep.wait(ep.reduce_scatter(x, rs, n, c["dt"], c["op"]))
                assert_parity(c["dt"], rs[:ln * esz].cpu().numpy(),
                              want[off * esz:(off + ln) * esz], f"reduce_scatter {c['file']}")
                root = cases.index(c) % world
                rr = torch.zeros_like(x)
                _ready()
                ep.wait(ep.reduce(x, rr if rank == root else None, n, root, c["dt"], c["op"]))
                if rank == root:
                    assert_parity(c["dt"], rr.cpu().numpy(), want, f"reduce {c['file']}")
            # every one of them ran as the one-shot kernel (world <= 8 and
            # <= 4 KiB per input: under the planner's thresholds)
            cnt = ep.counters()
            assert cnt["oneshot"] == 3 * len(cases) and not cnt["timed_out"], cnt
        finally:
            ep.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, f"ok {len(cases)}"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,ll", [(2, "0"), (3, "0"), (4, "0"), (5, "0"), (8, "0"),
                                      (2, "1"), (5, "1"), (8, "1")])
def test_oneshot_every_reducing_entry(world, ll):
    """Every (op, datatype) of the write table with a reducing op (MIN..BXOR,
    int8..uint64, float, double, float complex, int128) through LFA_ALGO_P2P's
    one-shot allreduce, reduce_scatter and reduce (roots in turn, non-roots
    passing no result buffer) across processes, on the golden
    fixtures' operands with their edge lanes (±0, ±inf, NaN, extremes):
    equal to prov/coll's recursive-doubling result (the oracle), bit for bit
    (NaN lanes: NaN on both sides).  ll "0": the flagged kernel (the
    default); "1" (LFA_OS_LL=1 on every member): allreduce and reduce_scatter
    parts of these sizes take the LL kernel, reduce keeps the flagged one."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_every_entry_worker, args=(r, world, port, q, ll))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            try:
                r, msg = q.get(timeout=140)
            except queue.Empty:         # a rank hung: report the others
                break
            results[r] = msg
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    bad = {r: results.get(r) for r in range(world) if not str(results.get(r)).startswith("ok")}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in sorted(bad.items()))


def _word_drop_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import time
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        # a second GPU domain keeps the workspace cache and quarantine alive
        # across the re-join
        anchor = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        msg = "ok"
        try:
            ep.set_algo(coll.ALGO_P2P)
            sends = [_inputs(oracle, 8, 4096, world, 40 + k) for k in range(3)]
            wants = [oracle.allreduce(2, 8, s)[0] for s in sends]
            xs = [_dev(s[rank]) for s in sends]
            rs = [torch.zeros(4096, dtype=torch.float32, device="cuda") for _ in range(3)]
            _ready()
            ep.wait(ep.allreduce(xs[0], rs[0], 4096, 8, 2))
            before = ep.word_ops()
            if rank == 0:
                # this member's next one-shot waits for a word value its
                # kernel never stores
                ep.test_word(drop_next=1, timeout_ms=300)
            c1 = ep.allreduce(xs[1], rs[1], 4096, 8, 2)
            c2 = ep.allreduce(xs[2], rs[2], 4096, 8, 2)
            ok, errs = [], []
            t0 = time.time()
            while len(ok) < (1 if rank == 0 else 2) and time.time() - t0 < 10:
                n = ep._L.lfa_cq_read(ep.ep, ep._ents, 16)
                if n > 0:
                    ok += [ep._ents[i].op_context for i in range(n)]
                elif n == -coll.EIO:
                    errs.append(ep.cq_readerr())
            time.sleep(0.05)
            if ep.cq_readerr() is not None or ep.cq_read():
                msg = "a second entry"
            if rank == 0 and (ok != [c2] or [(e[0], e[2]) for e in errs] != [(110, c1)]):
                msg = f"rank 0: successes {ok}, errors {errs} (c1 {c1}, c2 {c2})"
            if rank == 1 and (ok != [c1, c2] or errs):
                msg = f"rank 1: successes {ok}, errors {errs}"
            torch.cuda.synchronize()
            for k in (1, 2):
                if rs[k].cpu().numpy().tobytes() != wants[k].tobytes():
                    msg = f"allreduce {k} wrong"
            want_words = 1 if rank == 0 else 2      # the lost word is not one
            if msg == "ok" and ep.word_ops() - before != want_words:
                msg = f"word operations {ep.word_ops() - before}, want {want_words}"
            # the member whose operation failed cannot know its
            # kernel finished, so its group refuses further P2P operations
            # and its workspace goes to the quarantine at close, as after a
            # timed-out wait; the members close and re-join
            quar0 = coll.ws_quarantined_bytes()
            if rank == 0:
                try:
                    ep.allreduce(xs[0], rs[0], 4096, 8, 2)
                    msg = msg if msg != "ok" else "a P2P submit on the failed group"
                except coll.CollError as e:
                    if e.rc != -coll.EIO and msg == "ok":
                        msg = f"refused with {e.rc}"
            ep.close()
            if msg == "ok" and rank == 0 and not coll.ws_quarantined_bytes() > quar0:
                msg = "the failed group's workspace was not quarantined"
            ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
            ep.set_algo(coll.ALGO_P2P)
            rs[0].zero_()
            _ready()
            ep.wait(ep.allreduce(xs[0], rs[0], 4096, 8, 2))
            if msg == "ok" and rs[0].cpu().numpy().tobytes() != wants[0].tobytes():
                msg = "allreduce after the re-join wrong"
        finally:
            ep.close()
            anchor.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_lost_one_shot_word_fails_that_operation_once():
    """VERDICT r4 #1 on the P2P one-shot (2 processes, peer domains): one
    member's one-shot waits for a completion-word value its kernel never
    stores.  That operation is reaped once, as an ETIMEDOUT error entry,
    after the bound; the one queued behind it completes normally on both
    members and every result is exact.  That member's group then refuses
    P2P operations (EIO) and its workspace is quarantined at close (ADVICE
    r5: the failed operation's kernel may still post into it); the re-made
    group is exact."""
    _spawn(_word_drop_worker, 2)


def _late_member_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          LFA_SIG_TIMEOUT_MS="300")
        _share_gpu(world)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import time
        import oracle
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        msg = "ok"
        n = 4096
        sends = [_inputs(oracle, 8, n, world, 70 + k) for k in range(3)]
        wants = [oracle.allreduce(2, 8, s)[0] for s in sends]
        xs = [_dev(s[rank]) for s in sends]
        anchor = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        ep.set_algo(coll.ALGO_P2P)
        r = torch.zeros(n, dtype=torch.float32, device="cuda")
        _ready()
        ep.wait(ep.allreduce(xs[0], r, n, 8, 2))                  # A, both
        if r.cpu().numpy().tobytes() != wants[0].tobytes():
            msg = "A wrong"
        cached0, quar0 = coll.ws_cached_bytes(), coll.ws_quarantined_bytes()
        rb = torch.zeros(n, dtype=torch.float32, device="cuda")
        _ready()
        if rank == 1:
            # B: rank 0 is late; this member's one-shot gives up after 300 ms
            try:
                ep.wait(ep.allreduce(xs[1], rb, n, 8, 2), timeout_s=30)
                msg = "B did not time out"
            except coll.CollError as e:
                if "prov_errno 110" not in str(e):
                    msg = f"B: {e}"
            ep.close()                   # the timed-out group's workspace
            if msg == "ok" and not (coll.ws_quarantined_bytes() > quar0 and
                                    coll.ws_cached_bytes() == cached0):
                msg = (f"after close: cached {cached0} -> {coll.ws_cached_bytes()}, "
                       f"quarantined {quar0} -> {coll.ws_quarantined_bytes()}")
            ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
            ep.set_algo(coll.ALGO_P2P)
            rc = torch.zeros(n, dtype=torch.float32, device="cuda")
            _ready()
            ctx_c = ep.allreduce(xs[2], rc, n, 8, 2)   # new group: workspace reset now
            dist.barrier()                              # 1: rank 0 may run its late B
            ep.wait(ctx_c)
        else:
            dist.barrier()                              # 1
            # the late member: its B kernel pushes into rank 1's OLD
            # workspace and posts B's epoch there through its old mapping
            ep.wait(ep.allreduce(xs[1], rb, n, 8, 2), timeout_s=30)
            ep.close()
            ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
            ep.set_algo(coll.ALGO_P2P)
            rc = torch.zeros(n, dtype=torch.float32, device="cuda")
            _ready()
            ep.wait(ep.allreduce(xs[2], rc, n, 8, 2))
        # C on the re-made group: rank 1's new workspace is not the one the
        # late kernel wrote into, so C's wait cannot pass on B's stale post
        if msg == "ok" and rc.cpu().numpy().tobytes() != wants[2].tobytes():
            msg = "C after the re-join wrong (stale post or slot data)"
        for _ in range(3):
            rc.zero_()
            _ready()
            ep.wait(ep.allreduce(xs[2], rc, n, 8, 2))
            if msg == "ok" and rc.cpu().numpy().tobytes() != wants[2].tobytes():
                msg = "a later C wrong"
        ep.close()
        anchor.close()
        if msg == "ok" and (coll.ws_cached_bytes() or coll.ws_quarantined_bytes()):
            msg = "workspaces kept after the last GPU domain closed"
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, msg))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_rejoin_after_timeout_does_not_reuse_the_timed_out_workspace():
    """after a P2P timeout the fix is to close and re-join
    the group.  The re-join used to take the SAME workspace back from the
    cache while the late member's kernel could still push data and post its
    old epoch through its old mapping — satisfying the new group's first wait
    with stale slots.  A timed-out group's workspace is now quarantined (held,
    never reused): the member that timed out keeps it out of the cache, the
    late member runs its old operation into it, and the re-made group's
    operations are exact.  Every kept workspace is freed with the last GPU
    domain."""
    _spawn(_late_member_worker, 2)


def _world1_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LFA_DEBUG="1")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gloo_xfer import GlooXfer
        from libfabric_amd import coll
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=0)
        try:
            ep.set_algo(coll.ALGO_P2P)
            # a one-member GPU peer domain under P2P: one-shot-sized buckets
            # plan the n = 1 one-shot (round 6), larger ones the two-barrier
            # schedule; each is a copy of the input
            for n in (1, 1000, 70_001, (3 << 20) + 5):
                x = torch.rand(n, device="cuda")
                for kind in ("allreduce", "reduce_scatter", "reduce"):
                    y = torch.full_like(x, -1.0)
                    _ready()
                    if kind == "allreduce":
                        ep.wait(ep.allreduce(x, y, n, 8, 2))
                    elif kind == "reduce_scatter":
                        ep.wait(ep.reduce_scatter(x, y, n, 8, 2))
                    else:
                        ep.wait(ep.reduce(x, y, n, 0, 8, 2))
                    assert torch.equal(x, y), f"{kind} n={n}"
            c = ep.counters()
            assert c["oneshot"] >= 9 and not c["timed_out"], c
        finally:
            ep.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_p2p_one_member_peer_domain():
    """LFA_ALGO_P2P on a one-member GPU peer domain: the n = 1 one-shot the
    planner emits for one-shot-sized buckets since round 6 (the workspace
    handshake of a group of one, the kernel's degenerate copy, the
    completion word) and the two-barrier schedule above; allreduce,
    reduce_scatter and reduce give the input back."""
    _spawn(_world1_worker, 1)
