"""GPU tests of the collective provider (liblfa_coll.so).

* loopback: the schedules of N = 2..16 ranks run on ONE MI355X with the real
  combine kernels (lfa_coll_loopback), compared with the oracle's prov/coll
  recursive-doubling results — bit-exact;
* a real RCCL domain + endpoint at world size 1 (the box has one GPU):
  every fi_ops_collective call on device and host buffers, completions,
  join, query and error codes through the C ABI.
The N>1 RCCL transport runs in the driver's 8-GPU bench; its schedules are
covered across processes by tests/test_coll_gloo.py.
"""
import numpy as np
import pytest
import torch

import oracle
from tests._cmp import assert_parity

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ALLREDUCE, BROADCAST, ALLGATHER, REDUCE_SCATTER, REDUCE, SCATTER = 3, 1, 4, 5, 6, 7


@pytest.fixture(scope="module")
def coll():
    from libfabric_amd import coll as c
    c.lib()
    return c


def _inputs(dt, n, count, seed, lo=-1.0, hi=1.0):
    rng = np.random.default_rng(seed)
    nd = oracle.DT_NP[dt]
    if nd.kind == "f":
        return [rng.uniform(lo, hi, count).astype(nd) for _ in range(n)]
    info = np.iinfo(nd)
    return [rng.integers(info.min, info.max, count, dtype=nd, endpoint=True)
            for _ in range(n)]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


CASES = [(8, 2), (9, 3), (6, 0), (6, 6), (1, 7), (4, 9), (8, 1)]


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
def test_loopback_allreduce(coll, algo, n):
    for dt, op in CASES:
        for count in (1, 777, 100_003, 120_000):
            sends = _inputs(dt, n, count, n + count + op,
                            *((0.9, 1.1) if op == 3 else (-1, 1)))
            want = oracle.allreduce(op, dt, sends)[0]
            sd = [_dev(s) for s in sends]
            rd = [torch.zeros_like(x) for x in sd]
            coll.loopback(ALLREDUCE, algo, n, -1, dt, op, count, sd, rd)
            torch.cuda.synchronize()
            for r in range(n):
                assert_parity(dt, rd[r].cpu().numpy(), want, f"n={n} dt={dt} op={op} r={r}")


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("count", [50_001, 48_000])
def test_loopback_reduce_scatter_and_reduce(coll, algo, n, count):
    dt, op = 9, 3
    sends = _inputs(dt, n, count, 99 + n, 0.9, 1.1)
    want = oracle.allreduce(op, dt, sends)[0]
    sd = [_dev(s) for s in sends]
    rd = []
    for r in range(n):
        off, ln = coll.block(count, n, r)
        rd.append(torch.zeros(ln * 8, dtype=torch.uint8, device=DEV))
    coll.loopback(REDUCE_SCATTER, algo, n, -1, dt, op, count, sd, rd)
    torch.cuda.synchronize()
    for r in range(n):
        off, ln = coll.block(count, n, r)
        assert_parity(dt, rd[r].cpu().numpy(), want[off:off + ln], f"rs r={r}")
    root = n - 1
    rd = [torch.zeros(count * 8, dtype=torch.uint8, device=DEV) for _ in range(n)]
    coll.loopback(REDUCE, algo, n, root, dt, op, count, sd, rd)
    torch.cuda.synchronize()
    assert_parity(dt, rd[root].cpu().numpy(), want, "reduce root")


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
def test_loopback_skewed_blocks(coll, algo):
    """Blocks >= 1 MiB: TMP holds them 6 KiB-skewed; results
    stay bit-exact with prov/coll (ragged count, so TREE_COLL falls back)."""
    n, dt, op = 4, 9, 3
    for count in (n * 300_001 + 3, n * 300_000):
        sends = _inputs(dt, n, count, count, 0.9, 1.1)
        want = oracle.allreduce(op, dt, sends)[0]
        sd = [_dev(s) for s in sends]
        rd = [torch.zeros_like(x) for x in sd]
        coll.loopback(ALLREDUCE, algo, n, -1, dt, op, count, sd, rd)
        torch.cuda.synchronize()
        for r in range(n):
            assert_parity(dt, rd[r].cpu().numpy(), want, f"count={count} r={r}")


def test_loopback_moves(coll):
    n, count = 5, 12_345
    sends = _inputs(6, n, count, 5)
    sd = [_dev(s) for s in sends]
    rd = [torch.zeros(n * count * 8, dtype=torch.uint8, device=DEV) for _ in range(n)]
    coll.loopback(ALLGATHER, 0, n, -1, 6, 2, count, sd, rd)
    torch.cuda.synchronize()
    want = np.concatenate(sends).view(np.uint8)
    for r in range(n):
        assert np.array_equal(rd[r].cpu().numpy(), want)
    bufs = [x.clone() for x in sd]
    coll.loopback(BROADCAST, 0, n, 2, 6, 2, count, [None] * n, bufs)
    torch.cuda.synchronize()
    for r in range(n):
        assert np.array_equal(bufs[r].cpu().numpy(), sends[2].view(np.uint8))


def test_loopback_16_ranks_int_bitwise(coll):
    n, count = 16, 4099
    for dt, op in ((7, 6), (7, 9), (2, 2)):
        sends = _inputs(dt, n, count, op)
        want = oracle.allreduce(op, dt, sends)[0]
        sd = [_dev(s) for s in sends]
        rd = [torch.zeros_like(x) for x in sd]
        coll.loopback(ALLREDUCE, 0, n, -1, dt, op, count, sd, rd)
        torch.cuda.synchronize()
        for r in range(n):
            assert np.array_equal(rd[r].cpu().numpy(), want.view(np.uint8))


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
def test_loopback_reference_known_answers(coll, algo):
    """prov/cxi/test/multinode/test_coll.c's fi_allreduce checks, every rank
    count 2..8 on the kernels: int64 SUM of 4r+v exact (:722-792), double SUM
    of (4r+v)/1000 within 1e-8 (:795-865)."""
    for n in range(2, 9):
        sd = [_dev(np.array([4 * r + v for v in range(4)], np.int64)) for r in range(n)]
        rd = [torch.zeros_like(x) for x in sd]
        coll.loopback(ALLREDUCE, algo, n, -1, 6, 2, 4, sd, rd)
        torch.cuda.synchronize()
        comp = [sum(4 * r + v for r in range(n)) for v in range(4)]
        for r in range(n):
            assert rd[r].cpu().numpy().view(np.int64).tolist() == comp, (n, r)
        sd = [_dev(np.array([(4 * r + v) / 1000.0 for v in range(4)])) for r in range(n)]
        rd = [torch.zeros_like(x) for x in sd]
        coll.loopback(ALLREDUCE, algo, n, -1, 9, 2, 4, sd, rd)
        torch.cuda.synchronize()
        comp = [sum((4 * r + v) / 1000.0 for r in range(n)) for v in range(4)]
        for r in range(n):
            got = rd[r].cpu().numpy().view(np.float64)
            assert all(abs(a - b) <= 1e-8 for a, b in zip(got, comp)), (n, r)


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_loopback_ragged_counts_every_root(coll, algo, n):
    """Counts of 0, 1, n-1 and 7n+3 (empty, fewer elements than ranks,
    ragged blocks) through allreduce, reduce_scatter and reduce to EVERY
    root, bit-exact with the oracle; int64 SUM and double PROD."""
    for dt, op in ((6, 2), (9, 3)):
        esz = 8
        for count in (0, 1, n - 1, 7 * n + 3):
            sends = _inputs(dt, n, count, 17 * n + count + op,
                            *((0.9, 1.1) if op == 3 else (-1, 1)))
            want = oracle.allreduce(op, dt, sends)[0] if count else np.zeros(0)
            sd = [_dev(s) if count else torch.zeros(8, dtype=torch.uint8, device=DEV)
                  for s in sends]
            rd = [torch.zeros(max(count, 1) * esz, dtype=torch.uint8, device=DEV)
                  for _ in range(n)]
            coll.loopback(ALLREDUCE, algo, n, -1, dt, op, count, sd, rd)
            torch.cuda.synchronize()
            for r in range(n):
                assert_parity(dt, rd[r].cpu().numpy()[:count * esz], want,
                              f"allreduce n={n} count={count} r={r}")
            rd = [torch.zeros(max(coll.block(count, n, r)[1], 1) * esz, dtype=torch.uint8,
                              device=DEV) for r in range(n)]
            coll.loopback(REDUCE_SCATTER, algo, n, -1, dt, op, count, sd, rd)
            torch.cuda.synchronize()
            for r in range(n):
                off, ln = coll.block(count, n, r)
                assert_parity(dt, rd[r].cpu().numpy()[:ln * esz], want[off:off + ln],
                              f"reduce_scatter n={n} count={count} r={r}")
            for root in range(n):
                rd = [torch.zeros(max(count, 1) * esz, dtype=torch.uint8, device=DEV)
                      for _ in range(n)]
                coll.loopback(REDUCE, algo, n, root, dt, op, count, sd, rd)
                torch.cuda.synchronize()
                assert_parity(dt, rd[root].cpu().numpy()[:count * esz], want,
                              f"reduce n={n} count={count} root={root}")


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
def test_loopback_edge_values_minmax(coll, algo):
    """NaN, +-inf and +-0 lanes in some ranks' inputs through float and
    double MIN / MAX / SUM allreduces: the dst-biased compare of the
    reference (util_atomic.c:291-316: a NaN partial on the hi side stays, one
    on the lo side is ignored; ties keep hi) at every level of the tree."""
    edge = [np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, -1.0]
    for n in (2, 3, 5, 8):
        for dt in (8, 9):
            nd = oracle.DT_NP[dt]
            rng = np.random.default_rng(n * 10 + dt)
            count = 4099
            sends = []
            for _ in range(n):
                x = rng.uniform(-1, 1, count).astype(nd)
                lanes = rng.random(count) < 0.3
                x[lanes] = rng.choice(np.array(edge, nd), int(lanes.sum()))
                sends.append(x)
            for op in (0, 1, 2):
                want = oracle.allreduce(op, dt, sends)[0]
                sd = [_dev(x) for x in sends]
                rd = [torch.zeros_like(x) for x in sd]
                coll.loopback(ALLREDUCE, algo, n, -1, dt, op, count, sd, rd)
                torch.cuda.synchronize()
                for r in range(n):
                    assert_parity(dt, rd[r].cpu().numpy(), want,
                                  f"n={n} dt={dt} op={op} r={r}")


@pytest.fixture(scope="module")
def full_size_sum():
    """BASELINE.json configs[3]'s shape on loopback: 8 ranks, 256 MiB of
    float32 per rank, FI_SUM. The C oracle (oracle_allreduce, the
    coll_coll.c:364-420 schedule) finishes this in seconds."""
    n, count = 8, (256 << 20) // 4
    sends = _inputs(8, n, count, 2026)
    return n, count, sends, oracle.allreduce(2, 8, sends)


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
def test_loopback_allreduce_full_size(coll, full_size_sum, algo):
    """Full-size parity: every algorithm (TREE, RD, TREE_COLL, P2P) returns
    the oracle's bits on every rank at 256 MiB per rank, so the per-size
    choices bench.py measures (sweep rows) never change a result."""
    n, count, sends, want = full_size_sum
    sd = [_dev(s) for s in sends]
    rd = [torch.empty_like(x) for x in sd]
    coll.loopback(ALLREDUCE, algo, n, -1, 8, 2, count, sd, rd)
    torch.cuda.synchronize()
    del sd
    for r in range(n):
        assert_parity(8, rd[r].cpu().numpy(), want[r], f"algo={algo} r={r}")


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
def test_loopback_prod_reduce_scatter_full_size(coll, algo):
    """BASELINE.json configs[4]'s largest bucket: double FI_PROD
    reduce_scatter, 256 MiB per rank, 8 ranks, bit-exact per block."""
    n, dt, op = 8, 9, 3
    count = (256 << 20) // 8
    sends = _inputs(dt, n, count, 4242, 0.999, 1.001)
    want = oracle.reduce_scatter(op, dt, sends)
    sd = [_dev(s) for s in sends]
    rd = [torch.empty(coll.block(count, n, r)[1] * 8, dtype=torch.uint8,
                      device=DEV) for r in range(n)]
    coll.loopback(REDUCE_SCATTER, algo, n, -1, dt, op, count, sd, rd)
    torch.cuda.synchronize()
    for r in range(n):
        assert_parity(dt, rd[r].cpu().numpy(), want[r], f"algo={algo} rs r={r}")


def test_loopback_int64_min_bor_64mib(coll):
    """BASELINE.json configs[2]'s dtype/ops and size through the 8-rank
    allreduce: int64 FI_MIN and FI_BOR over 64 MiB, bit-exact."""
    n, dt, count = 8, 6, (64 << 20) // 8
    for op in (0, 6):
        sends = _inputs(dt, n, count, 7 + op)
        want = oracle.allreduce(op, dt, sends)[0]
        sd = [_dev(s) for s in sends]
        rd = [torch.empty_like(x) for x in sd]
        coll.loopback(ALLREDUCE, 0, n, -1, dt, op, count, sd, rd)
        torch.cuda.synchronize()
        for r in range(n):
            assert np.array_equal(rd[r].cpu().numpy(), want.view(np.uint8)), (op, r)


# ------------------------------------------------ RCCL domain, world = 1 ----

class _ReadyBuffers:
    """fi_allreduce & co. take buffers that are ready when called: libfabric
    carries no stream, and the endpoint's stream does not wait for torch's.
    This wrapper synchronises the device before each collective call, as a
    caller that filled its buffers with kernels must."""

    _CALLS = {"allreduce", "reduce_scatter", "reduce", "allgather", "scatter",
              "broadcast", "barrier"}

    def __init__(self, ep):
        self._ep = ep

    def __getattr__(self, name):
        a = getattr(self._ep, name)
        if name not in self._CALLS:
            return a

        def call(*args, **kw):
            torch.cuda.synchronize()
            return a(*args, **kw)
        return call


@pytest.fixture(scope="module")
def ep(coll):
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    yield _ReadyBuffers(e)
    e.close()


def test_rccl_allreduce_device_and_host(coll, ep):
    count = 1 << 20
    x = torch.rand(count, device=DEV)
    y = torch.empty_like(x)
    ctx = ep.allreduce(x, y, count, 8, 2)
    ep.wait(ctx)
    assert torch.equal(x, y)
    # host buffers, chunked through HBM (small chunks: several pipeline steps)
    ep.set_chunk(1 << 18)
    hx = np.random.default_rng(1).uniform(-1, 1, count).astype(np.float32)
    hy = np.zeros_like(hx)
    ctx = ep.allreduce(hx, hy, count, 8, 2)
    ep.wait(ctx)
    assert np.array_equal(hx, hy)
    # mixed: device buf, host result (and the reverse), both staging forms
    hy[:] = 0
    ep.wait(ep.allreduce(x, hy, count, 8, 2))
    assert np.array_equal(x.cpu().numpy(), hy)
    y.zero_()
    ep.wait(ep.allreduce(hx, y, count, 8, 2))
    assert np.array_equal(hx, y.cpu().numpy())
    hy[:] = 0
    ep.wait(ep.reduce_scatter(x, hy, count, 8, 2))
    assert np.array_equal(x.cpu().numpy(), hy)
    ep.set_chunk(0)


def test_completion_word_interleaved_with_events(coll, ep):
    """a one-member group runs small reducing collectives as
    a copy kernel dispatched on liblfa's own HSA queue, which completes
    through that queue's completion word (no event); larger ones, allgather,
    broadcast and the barrier stay on the endpoint's stream with events.
    Sixty operations of both kinds in flight at once,
    every op and datatype class, unaligned buffers among them: completions
    in issue order, every result the copy the reference defines."""
    rng = np.random.default_rng(11)
    cases = []
    for k in range(60):
        dt, op = CASES[k % len(CASES)]
        nd = oracle.DT_NP[dt]
        count = int(rng.choice([1, 33, 1024, 65_536 // nd.itemsize,
                                (256 << 10) // nd.itemsize, (300 << 10) // nd.itemsize]))
        off = int(rng.integers(0, 3)) * nd.itemsize if k % 5 == 0 else 0
        src = _inputs(dt, 1, count, 1000 + k)[0]
        buf = torch.zeros(off + count * nd.itemsize + 64, dtype=torch.uint8, device=DEV)
        buf[off:off + count * nd.itemsize] = torch.from_numpy(src.view(np.uint8).copy())
        res = torch.zeros_like(buf)
        cases.append((dt, op, count, off, src, buf, res, k % 3))
    torch.cuda.synchronize()
    e = ep._ep          # buffers are ready: submit without a sync in between
    ctxs = []
    for dt, op, count, off, src, buf, res, kind in cases:
        x, y = buf[off:], res[off:]
        if kind == 0:
            ctxs.append(e.allreduce(x, y, count, dt, op))
        elif kind == 1:
            ctxs.append(e.reduce_scatter(x, y, count, dt, op))
        else:
            ctxs.append(e.reduce(x, y, count, 0, dt, op))
        if len(ctxs) % 7 == 0:
            ctxs.append(e.barrier())
    done = []
    while len(done) < len(ctxs):
        done += e.cq_read()
    assert done == ctxs
    for dt, op, count, off, src, buf, res, kind in cases:
        nb = count * oracle.DT_NP[dt].itemsize
        got = res[off:off + nb].cpu().numpy().view(oracle.DT_NP[dt])
        assert got.tobytes() == src.tobytes(), (dt, op, count, off, kind)
        assert not res[:off].any() and not res[off + nb:].any(), "wrote outside"


@pytest.mark.parametrize("direct", ["1", "0"])
def test_small_ops_past_the_direct_queue_ring(coll, direct, monkeypatch):
    """700 small allreduces in flight at once on a one-member group, more
    than the direct queue's 256 packets and kernarg slots (lfa_direct.cpp):
    the submitter waits for the ring, every completion comes back in issue
    order and every result is its own input.  direct "0" (LFA_DIRECT=0): the
    same through the HIP launch on the endpoint's stream."""
    monkeypatch.setenv("LFA_DIRECT", direct)
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        n = 700
        srcs = torch.arange(n * 257, dtype=torch.float32, device=DEV).view(n, 257)
        outs = torch.zeros_like(srcs)
        torch.cuda.synchronize()
        ctxs = [e.allreduce(srcs[i], outs[i], 257, 8, 2) for i in range(n)]
        done = []
        while len(done) < n:
            done += e.cq_read()
        assert done == ctxs
        torch.cuda.synchronize()
        assert torch.equal(srcs, outs)
    finally:
        e.close()


def test_two_endpoints_share_the_direct_queue(coll):
    """Endpoints of one process share one direct queue per device, each with
    its own counter and completion word: small operations of two one-member
    endpoints interleaved, 300 in flight on each, every completion back on
    its own endpoint in issue order and every result its own input; closing
    one endpoint leaves the other's queue working."""
    e1 = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    e2 = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        n = 300
        srcs = torch.arange(2 * n * 129, dtype=torch.float32, device=DEV).view(2, n, 129)
        outs = torch.zeros_like(srcs)
        torch.cuda.synchronize()
        c1, c2 = [], []
        for i in range(n):
            c1.append(e1.allreduce(srcs[0, i], outs[0, i], 129, 8, 2))
            c2.append(e2.allreduce(srcs[1, i], outs[1, i], 129, 8, 2))
        d1, d2 = [], []
        while len(d1) < n or len(d2) < n:
            d1 += e1.cq_read()
            d2 += e2.cq_read()
        assert d1 == c1 and d2 == c2
        torch.cuda.synchronize()
        assert torch.equal(srcs, outs)
        e1.close()
        e1 = None
        outs.zero_()
        torch.cuda.synchronize()
        c2 = [e2.allreduce(srcs[1, i], outs[1, i], 129, 8, 2) for i in range(20)]
        d2 = []
        while len(d2) < 20:
            d2 += e2.cq_read()
        assert d2 == c2
        torch.cuda.synchronize()
        assert torch.equal(srcs[1, :20], outs[1, :20])
    finally:
        if e1 is not None:
            e1.close()
        e2.close()


@pytest.mark.parametrize("zero_copy", ["1", "0"])
def test_one_member_pinned_host_buffers(coll, ep, zero_copy, monkeypatch):
    """A one-member group's reducing collectives on PINNED host buffers run
    zero-copy: the copy kernel reads and writes their device mappings over
    PCIe — the solo copy ending in the completion word up to 4 MiB, the
    ATOMIC_WRITE body above — and LFA_HOST_ZERO_COPY=0 restores the staged
    pipeline.  Sizes on both sides of the bound, an odd byte count at an
    odd offset (the byte-wise bodies), a device buf with a pinned result
    and the reverse; several in flight before one wait; every result the
    copy the reference defines."""
    monkeypatch.setenv("LFA_HOST_ZERO_COPY", zero_copy)
    rng = np.random.default_rng(31)
    cases = []
    for nbytes, off, dt, nd in ((4096, 0, 8, np.float32), ((1 << 20) + 3, 1, 0, np.int8),
                                (6 << 20, 0, 9, np.float64), (40 << 10, 8, 6, np.int64)):
        count = nbytes // nd().itemsize
        raw = torch.from_numpy(rng.integers(0, 256, nbytes + 64, dtype=np.uint8)).pin_memory()
        src = raw[off:off + count * nd().itemsize].view(
            {np.float32: torch.float32, np.int8: torch.int8, np.float64: torch.float64,
             np.int64: torch.int64}[nd])
        for coll_name in ("allreduce", "reduce", "reduce_scatter"):
            dst = torch.zeros(count * nd().itemsize + off, dtype=torch.uint8).pin_memory()
            out = dst[off:].view(src.dtype)
            op = 6 if nd in (np.int8, np.int64) else 2     # BOR / SUM
            if coll_name == "allreduce":
                ctx = ep.allreduce(src, out, count, dt, op)
            elif coll_name == "reduce":
                ctx = ep.reduce(src, out, count, 0, dt, op)
            else:
                ctx = ep.reduce_scatter(src, out, count, dt, op)
            cases.append((ctx, src, out, f"{coll_name} {nbytes} B +{off}"))
    ep.wait(cases[-1][0], timeout_s=20)   # completions come in issue order
    for ctx, src, out, what in cases:
        assert torch.equal(src.view(torch.uint8), out.view(torch.uint8)), what
    # mixed: device buf with a pinned result, pinned buf with a device result
    x = torch.rand(3 << 20, device=DEV)
    hy = torch.zeros(3 << 20).pin_memory()
    ep.wait(ep.allreduce(x, hy, x.numel(), 8, 2))
    assert torch.equal(x.cpu(), hy)
    y = torch.zeros_like(x)
    ep.wait(ep.allreduce(hy, y, x.numel(), 8, 2))
    assert torch.equal(y, x)


def test_one_member_pageable_bounce_blocks(coll, ep):
    """A one-member group's reducing collectives on PAGEABLE (numpy) buffers
    of at most LFA_BOUNCE_BYTES go through a pinned bounce block: input
    copied in at submit, the solo copy on the block's mapping, the result
    copied out when reaped.  20 in flight (more than the 8 blocks: the rest
    stage), odd sizes at odd offsets, sizes past the bound, a device buf
    with a pageable result (staged); every result the copy."""
    rng = np.random.default_rng(41)
    cases = []
    for k in range(20):
        nbytes = (4096, 65536 + 3, 1 << 20, (1 << 20) + 5)[k % 4]
        raw = rng.integers(0, 256, nbytes + 8, dtype=np.uint8)
        src = raw[k % 3:k % 3 + nbytes]
        out = np.zeros(nbytes + 8, np.uint8)
        dst = out[(k + 1) % 5:(k + 1) % 5 + nbytes]
        name = ("allreduce", "reduce", "reduce_scatter")[k % 3]
        if name == "allreduce":
            ctx = ep.allreduce(src, dst, nbytes, 0, 6)      # int8 BOR
        elif name == "reduce":
            ctx = ep.reduce(src, dst, nbytes, 0, 0, 6)
        else:
            ctx = ep.reduce_scatter(src, dst, nbytes, 0, 6)
        cases.append((src, dst, f"{name} {nbytes} B #{k}"))
    ep.wait(ctx, timeout_s=30)
    for src, dst, what in cases:
        assert np.array_equal(src, dst), what
    x = torch.randint(0, 256, (4096,), dtype=torch.uint8, device=DEV)
    hy = np.zeros(4096, np.uint8)
    ep.wait(ep.allreduce(x, hy, 4096, 0, 6), timeout_s=30)
    assert np.array_equal(x.cpu().numpy(), hy)


def test_rccl_host_reduce_and_reduce_scatter_chunked(coll, ep):
    """reduce and reduce_scatter on host buffers go through the chunked
    H2D / collective / D2H pipeline (reduce_scatter: one 2-D H2D per chunk);
    ragged last chunks, an odd chunk size and mixed host/device operands."""
    count = (1 << 20) + 37
    rng = np.random.default_rng(7)
    hx = rng.uniform(0.9, 1.1, count)
    for chunk in (1 << 16, 3 * 8 * 1000 + 8, 0):
        ep.set_chunk(chunk)
        ho = np.zeros_like(hx)
        ep.wait(ep.reduce_scatter(hx, ho, count, 9, 3))
        assert np.array_equal(ho, hx)
        ho[:] = 0
        ep.wait(ep.reduce(hx, ho, count, 0, 9, 3))
        assert np.array_equal(ho, hx)
        d = torch.zeros(count, device=DEV, dtype=torch.float64)
        ep.wait(ep.reduce_scatter(hx, d, count, 9, 3))
        assert np.array_equal(d.cpu().numpy(), hx)
        ho[:] = 0
        ep.wait(ep.reduce_scatter(torch.from_numpy(hx).to(DEV), ho, count, 9, 3))
        assert np.array_equal(ho, hx)
    ep.set_chunk(0)


def test_group_chunk_device_and_host_members(coll, ep):
    """under a group chunk a device-buffer member splits large
    operations into the chunks the host members stage (lfa_coll_member_chunk)
    — contiguous chunks run in place on its buffers, reduce_scatter's 2-D
    chunks through device-to-device staging — and host members pipeline
    with the group chunk instead of their local one.  At world size 1 every
    chunk's collective is a copy, so the output must be the input at every
    offset: odd chunk sizes, a ragged last chunk, mixed operands."""
    count = (1 << 20) + 37
    rng = np.random.default_rng(17)
    hx = rng.uniform(0.9, 1.1, count)
    dx = torch.from_numpy(hx).to(DEV)
    try:
        for group in (1 << 16, 3 * 8 * 1000 + 8, 1 << 30):
            ep.set_group_chunk(group)
            ep.set_chunk(1 << 12)          # a local chunk the group rule overrides
            for fn, args in ((ep.allreduce, (9, 2)), (ep.reduce_scatter, (9, 3))):
                d = torch.zeros_like(dx)
                ep.wait(fn(dx, d, count, *args))
                assert torch.equal(d, dx), (fn.__name__, group, "device")
                h = np.zeros_like(hx)
                ep.wait(fn(hx, h, count, *args))
                assert np.array_equal(h, hx), (fn.__name__, group, "host")
                h[:] = 0
                ep.wait(fn(dx, h, count, *args))
                assert np.array_equal(h, hx), (fn.__name__, group, "mixed")
            d = torch.zeros_like(dx)
            ep.wait(ep.reduce(dx, d, count, 0, 9, 1))
            assert torch.equal(d, dx), ("reduce", group)
            b = dx.clone()
            ep.wait(ep.broadcast(b, count, 0, 9))
            assert torch.equal(b, dx), ("broadcast", group)
    finally:
        ep.set_group_chunk(coll.GROUP_CHUNK_AUTO)   # the default
        ep.set_chunk(0)


def test_rccl_other_collectives(coll, ep):
    count = 10_000
    x = torch.arange(count, dtype=torch.int64, device=DEV)
    out = torch.zeros_like(x)
    ep.wait(ep.reduce_scatter(x, out, count, 6, 2))
    assert torch.equal(out, x)
    out.zero_()
    ep.wait(ep.reduce(x, out, count, 0, 6, 0))
    assert torch.equal(out, x)
    out.zero_()
    ep.wait(ep.allgather(x, out, count, 6))
    assert torch.equal(out, x)
    out.zero_()
    ep.wait(ep.scatter(x, out, count, 0, 6))
    assert torch.equal(out, x)
    b = x.clone()
    ep.wait(ep.broadcast(b, count, 0, 6))
    assert torch.equal(b, x)
    ep.wait(ep.barrier())
    # host-buffer reduce_scatter (whole-buffer staging)
    hx = np.arange(count, dtype=np.int64)
    ho = np.zeros_like(hx)
    ep.wait(ep.reduce_scatter(hx, ho, count, 6, 2))
    assert np.array_equal(ho, hx)


def test_rccl_algorithms_selectable(coll, ep):
    count = 4096
    x = torch.rand(count, device=DEV, dtype=torch.float64)
    for algo in (coll.ALGO_RD, coll.ALGO_RCCL, coll.ALGO_TREE_COLL, coll.ALGO_TREE):
        ep.set_algo(algo)
        y = torch.zeros_like(x)
        ep.wait(ep.allreduce(x, y, count, 9, 3))
        assert torch.equal(x, y)
    ep.set_algo(coll.ALGO_TREE)


def test_join_world_and_completion_order(coll, ep):
    mc, ctx = ep.join(None)
    ev, fid, context = ep.wait_join()
    assert ev == coll.JOIN_COMPLETE and fid == mc and context == ctx
    addr = ep.mc_addr(mc)
    x = torch.ones(1000, device=DEV)
    y = torch.zeros_like(x)
    c1 = ep.allreduce(x, y, 1000, 8, 2, coll_addr=addr)
    c2 = ep.barrier(coll_addr=addr)
    got = []
    import time
    t0 = time.time()
    while len(got) < 2 and time.time() - t0 < 60:
        got += ep.cq_read()
    assert got == [c1, c2]            # completions in issue order
    assert ep.cq_read() == []         # -EAGAIN when nothing is pending
    assert torch.equal(x, y)


def test_join_subset_via_comm_split(coll, ep):
    """fi_join_collective with an explicit member list: ncclCommSplit over
    the parent, group id from the BAND of free-id masks."""
    mc, ctx = ep.join([0])
    ev, fid, context = ep.wait_join()
    assert ev == coll.JOIN_COMPLETE and fid == mc and context == ctx
    addr = ep.mc_addr(mc)
    x = torch.arange(4096, dtype=torch.int32, device=DEV)
    y = torch.zeros_like(x)
    ep.wait(ep.allreduce(x, y, 4096, 4, 9, coll_addr=addr))   # BXOR, 1 member
    assert torch.equal(x, y)
    assert coll.lib().lfa_mc_close(mc) == 0


def test_close_mc_with_join_in_flight(coll, ep):
    """Closing a multicast handle before its join completed: the queued join
    is dropped (no EQ event for the freed handle), later work is unaffected."""
    mc, _ = ep.join([0])
    assert coll.lib().lfa_mc_close(mc) == 0
    assert ep.cq_read() == []
    assert ep.eq_read() is None
    x = torch.ones(256, device=DEV)
    y = torch.zeros_like(x)
    ep.wait(ep.allreduce(x, y, 256, 8, 2))
    assert torch.equal(x, y)


def test_errors_and_query(coll, ep):
    x = torch.ones(16, device=DEV)
    with pytest.raises(coll.CollError) as e:
        ep.allreduce(x, x, 16, 8, 6)                # float BOR
    assert e.value.rc == -95
    with pytest.raises(coll.CollError) as e:
        ep.allreduce(x, x, 16, 8, 11)               # ATOMIC_WRITE: not a reduce op
    assert e.value.rc == -38
    with pytest.raises(coll.CollError) as e:
        ep.reduce(x, x, 16, 3, 8, 2)                # root outside the group
    assert e.value.rc == -22
    rc, a = ep.query(3, 2, 8)
    assert rc == 0 and a.max_members == 0x7fffffff and a.datatype_attr.size == 4
    assert ep.query(3, 6, 8)[0] == -95              # BOR on float
    assert ep.query(3, 12, 8)[0] == -38             # CSWAP: not a reduction
    assert ep.query(3, 2, 8, mode=1)[0] == -22      # mode must be 0
    assert ep.query(2, 2, 8)[0] == -38              # ALLTOALL
    assert ep.query(8, 2, 8)[0] == -38              # GATHER
    assert ep.query(0, 256, 256)[0] == 0            # BARRIER
    assert ep.query(5, 2, 8)[0] == 0                # REDUCE_SCATTER (new here)


def test_p2p_kernel_on_ipc_mapped_memory(coll):
    """LFA_ALGO_P2P's data path across processes: a child process maps this
    process's hipMalloc'd buffer with hipIpcOpenMemHandle and runs the P2P
    kernel on it — N inputs read from and N-1 outputs written into the
    mapping (on one GPU the mapping is same-device; on the 8-GPU node the
    provider maps peers over xGMI the same way).  Outputs == prov/coll's
    tree, bit-exact."""
    import ctypes
    import os
    import subprocess
    import sys
    from libfabric_amd import _native
    L = _native.lib()
    nsrc, ndst, count, dt, op = 8, 7, 300_007, 8, 2
    stride = (count * 4 + 4095) // 4096 * 4096
    out_off = nsrc * stride
    total = out_off + ndst * stride
    sends = _inputs(dt, nsrc, count, 4242)
    want = oracle.allreduce(op, dt, sends)[0]

    class IpcHandle(ctypes.Structure):
        _fields_ = [("reserved", ctypes.c_char * 64)]

    base = ctypes.c_void_p()
    assert L.hipMalloc(ctypes.byref(base), ctypes.c_size_t(total)) == 0
    try:
        L.hipMemset(base, 0, ctypes.c_size_t(total))
        for k, x in enumerate(sends):
            assert L.hipMemcpy(ctypes.c_void_p(base.value + k * stride),
                               x.ctypes.data_as(ctypes.c_void_p),
                               ctypes.c_size_t(count * 4), 1) == 0   # H2D
        assert L.hipDeviceSynchronize() == 0
        h = IpcHandle()
        L.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(IpcHandle), ctypes.c_void_p]
        assert L.hipIpcGetMemHandle(ctypes.byref(h), base) == 0
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        r = subprocess.run([sys.executable, os.path.join(root, "tests", "_ipc_child.py"),
                            bytes(h).hex(), str(nsrc), str(ndst), str(count), str(dt),
                            str(op), str(stride), str(out_off)],
                           cwd=root, capture_output=True, text=True, timeout=180,
                           env=dict(os.environ, PYTHONPATH=root))
        assert r.returncode == 0, r.stdout + r.stderr
        out = np.zeros(count, np.float32)
        for j in range(ndst):
            assert L.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p),
                               ctypes.c_void_p(base.value + out_off + j * stride),
                               ctypes.c_size_t(count * 4), 2) == 0   # D2H
            assert_parity(dt, out, want, f"ipc out{j}")
    finally:
        L.hipFree(base)


@pytest.mark.parametrize("algo", [0, 1, 3, 4])
@pytest.mark.parametrize("n", [33, 64])
def test_loopback_groups_above_32_ranks(coll, algo, n):
    """Groups larger than one tree kernel's 32 inputs: the TREE is split into
    whole subtrees of the reference tree (TMP partials), P2P / TREE_COLL run
    as TREE; the bits stay prov/coll's."""
    for dt, op, count in ((8, 2, 1000), (5, 9, 4 * n + 3), (9, 3, 20_001)):
        sends = _inputs(dt, n, count, n + op, *((0.9, 1.1) if op == 3 else (-1, 1)))
        want = oracle.allreduce(op, dt, sends)[0]
        sd = [_dev(s) for s in sends]
        rd = [torch.zeros_like(x) for x in sd]
        coll.loopback(ALLREDUCE, algo, n, -1, dt, op, count, sd, rd)
        torch.cuda.synchronize()
        for r in (0, n // 2, n - 1):
            assert_parity(dt, rd[r].cpu().numpy(), want, f"n={n} algo={algo} r={r}")


def test_progress_continues_during_subset_join(coll, ep):
    """The subset join's communicator split runs outside ep->lock: a thread
    polling the CQ (off_lfa's progress thread does this) is never held up
    behind it."""
    import threading
    import time
    stamps, stop = [], threading.Event()

    def poll():
        while not stop.is_set():
            ep.cq_read()
            stamps.append(time.perf_counter())
            time.sleep(0.001)

    t = threading.Thread(target=poll)
    t.start()
    try:
        time.sleep(0.05)
        t0 = time.perf_counter()
        mc, _ = ep.join([0])
        ev = ep.wait_join()
        t1 = time.perf_counter()
    finally:
        stop.set()
        t.join(timeout=30)
    assert ev[1] == mc
    inside = [s for s in stamps if t0 <= s <= t1]
    gaps = np.diff([t0] + inside + [t1])
    assert gaps.max() < 0.5, f"poller stalled {gaps.max():.3f} s during the join"
    assert coll.lib().lfa_mc_close(mc) == 0
