"""The C schedule builder (lfa_coll_plan) executed on the host for N ranks.

Every collective × algorithm × rank count × ragged count: the schedules the
GPU executor runs must produce the reference results — allreduce bit-exact
with prov/coll's recursive doubling (coll_coll.c:349-449), reduce_scatter
slice r of it, reduce at root, allgather / broadcast / scatter moves.
"""
import numpy as np
import pytest

import oracle
from libfabric_amd import coll
from tests import _plansim

# P2P one-shot bounds (lfa_coll_plan.h): allreduce / reduce over all members
# (LFA_OS_AG_BYTES_DEFAULT; 256 KiB before round 5), reduce_scatter input per
# member (LFA_OS_RS_BYTES; 1 MiB before round 5)
OS_AG_BYTES = 2 << 20
OS_RS_BYTES = 4 << 20

ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER, BROADCAST, SCATTER = 3, 5, 6, 4, 1, 7
F32, I64, U8, F64 = 8, 6, 1, 9
SUM, MIN, BOR, BAND, PROD = 2, 0, 6, 7, 3


def _inputs(dt, n, count, seed):
    rng = np.random.default_rng(seed)
    nd = oracle.DT_NP[dt]
    if nd.kind == "f":
        return [rng.uniform(-1, 1, count).astype(nd) for _ in range(n)]
    info = np.iinfo(nd)
    return [rng.integers(info.min, info.max, count, dtype=nd, endpoint=True)
            for _ in range(n)]


NS = [1, 2, 3, 4, 5, 7, 8]
COUNTS = [0, 1, 5, 1000, 70_001]


ALGOS = [coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("count", COUNTS + [8 * 9000])
def test_allreduce_schedule(algo, n, count):
    for dt, op in ((F32, SUM), (I64, MIN)):
        sends = _inputs(dt, n, count, n * 1000 + count)
        want = oracle.allreduce(op, dt, sends)[0] if count else sends[0]
        res = [np.zeros(count * sends[0].itemsize, np.uint8) for _ in range(n)]
        _plansim.run(ALLREDUCE, algo, n, -1, dt, op, count,
                     [s.view(np.uint8) for s in sends], res)
        for r in range(n):
            assert res[r].tobytes() == want.view(np.uint8).tobytes(), (r, dt)


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("count", COUNTS + [8 * 9000])
def test_reduce_scatter_schedule(algo, n, count):
    dt, op = F64, PROD
    sends = _inputs(dt, n, count, 7 + n + count)
    full = oracle.allreduce(op, dt, sends)[0] if count else np.zeros(0)
    res = []
    for r in range(n):
        off, ln = coll.block(count, n, r)
        res.append(np.zeros(ln * 8, np.uint8))
    _plansim.run(REDUCE_SCATTER, algo, n, -1, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    for r in range(n):
        off, ln = coll.block(count, n, r)
        assert res[r].tobytes() == full[off:off + ln].tobytes()


@pytest.mark.parametrize("algo", [coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_P2P])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
def test_reduce_schedule(algo, n):
    dt, op, count = U8, BAND, 4099
    for root in sorted({0, n - 1, n // 2}):
        sends = _inputs(dt, n, count, root + 31 * n)
        want = oracle.allreduce(op, dt, sends)[0]
        res = [np.zeros(count, np.uint8) for _ in range(n)]
        _plansim.run(REDUCE, algo, n, root, dt, op, count,
                     [s.view(np.uint8) for s in sends], res)
        assert res[root].tobytes() == want.tobytes()


@pytest.mark.parametrize("n", [1, 2, 3, 6])
def test_allgather_broadcast_scatter_schedules(n):
    count = 333
    sends = _inputs(I64, n, count, n)
    res = [np.zeros(n * count * 8, np.uint8) for _ in range(n)]
    _plansim.run(ALLGATHER, 0, n, -1, I64, SUM, count,
                 [s.view(np.uint8) for s in sends], res)
    want = np.concatenate(sends).view(np.uint8)
    for r in range(n):
        assert res[r].tobytes() == want.tobytes()
    root = n - 1
    bufs = [s.view(np.uint8).copy() for s in sends]
    _plansim.run(BROADCAST, 0, n, root, I64, SUM, count, [None] * n, bufs)
    for r in range(n):
        assert bufs[r].tobytes() == sends[root].view(np.uint8).tobytes()
    big = np.concatenate(sends).view(np.uint8)
    res = [np.zeros(count * 8, np.uint8) for _ in range(n)]
    _plansim.run(SCATTER, 0, n, 0, I64, SUM, count,
                 [big if r == 0 else np.zeros(0, np.uint8) for r in range(n)], res)
    for r in range(n):
        assert res[r].tobytes() == sends[r].view(np.uint8).tobytes()


def test_tree_schedule_traffic_is_bandwidth_optimal():
    """Per rank: (N-1)/N·S out in each of the two exchange phases."""
    n, count, esz = 8, 8 * 1_000_000, 4
    p = coll.plan(ALLREDUCE, coll.ALGO_TREE, 3, n, -1, count, esz)
    sent = sum(s["count"] for s in p.steps if s["type"] == 0)
    assert sent == 2 * (n - 1) * count * esz // n
    trees = [s for s in p.steps if s["type"] == 4]
    assert len(trees) == 1 and trees[0]["nsrc"] == n


def test_tree_coll_uses_rccl_collectives_when_even():
    p = coll.plan(ALLREDUCE, coll.ALGO_TREE_COLL, 2, 8, -1, 8 * 1_000_000, 4)
    kinds = [s["type"] for s in p.steps]
    assert kinds == [6, 4, 7]          # ALLTOALL, TREE, ALLGATHER
    p = coll.plan(ALLREDUCE, coll.ALGO_TREE_COLL, 2, 8, -1, 8 * 1_000_000 + 1, 4)
    assert 6 not in [s["type"] for s in p.steps]   # ragged: grouped p2p


def test_p2p_schedule_shape():
    """LFA_ALGO_P2P allreduce, big path: stage the input (one copy),
    barrier, ONE tree over every rank's SYM_IN pushing its result into all
    N-1 peers' SYM_OUT, barrier, copy the gathered blocks out.  Bytes staged
    in S (own block included: one launch), out (N-1)/N·S; no RCCL data
    transfers at all."""
    n, count, esz, r = 8, 8 * 1_000_000, 4, 3
    p = coll.plan(ALLREDUCE, coll.ALGO_P2P, r, n, -1, count, esz)
    kinds = [s["type"] for s in p.steps]
    assert kinds == [coll.STEP_COPY, coll.STEP_BARRIER,
                     coll.STEP_TREE_PUT, coll.STEP_BARRIER, coll.STEP_COPY]
    assert p.tmp_bytes == 0
    copies = [s for s in p.steps if s["type"] == coll.STEP_COPY]
    assert copies[0]["count"] == count * esz and copies[1]["count"] == count * esz
    assert copies[1]["src"] == (coll.BUF_SYM_OUT, 0, r)
    t = p.steps[2]
    assert t["nsrc"] == n and t["peer"] == n - 1
    off, ln = coll.block(count, n, r)
    ins = p.refs[t["first"]:t["first"] + n]
    outs = p.refs[t["first"] + n:t["first"] + n + n - 1]
    assert ins[r] == (coll.BUF_SEND, off * esz)            # own block in place
    assert all(ins[k] == (coll.BUF_SYM_IN, off * esz, k) for k in range(n) if k != r)
    assert sorted(o[2] for o in outs) == [k for k in range(n) if k != r]
    assert all(o[:2] == (coll.BUF_SYM_OUT, off * esz) for o in outs)
    assert t["dst"] == (coll.BUF_SYM_OUT, off * esz, r)     # own block too
    # reduce_scatter: one tree into the result, closing barrier, no pushes
    p = coll.plan(REDUCE_SCATTER, coll.ALGO_P2P, r, n, -1, count, esz)
    assert [s["type"] for s in p.steps][-2:] == [coll.STEP_TREE_PUT, coll.STEP_BARRIER]
    assert p.steps[-2]["peer"] == 0
    # transport-only collectives keep the RCCL schedules
    p = coll.plan(ALLGATHER, coll.ALGO_P2P, r, n, -1, 100, 8)
    assert coll.STEP_BARRIER not in [s["type"] for s in p.steps]


def test_p2p_small_allreduce_is_one_phase():
    """Small P2P allreduces of 2..8 members are ONE step (the one-shot
    kernel: push into the peers' slots, flags, tree); above 8 members the
    one-phase copy / barrier / tree / barrier form."""
    n, count = 4, 1000
    p = coll.plan(ALLREDUCE, coll.ALGO_P2P, 1, n, -1, count, 4)
    assert [s["type"] for s in p.steps] == [coll.STEP_ONESHOT]
    s = p.steps[0]
    assert s["count"] == count and s["nsrc"] == n
    assert s["src"] == (coll.BUF_SEND, 0) and s["dst"] == (coll.BUF_RESULT, 0)
    # the largest bucket that still fits OS_AG_BYTES (2 MiB) over all members
    p = coll.plan(ALLREDUCE, coll.ALGO_P2P, 0, 8, -1, OS_AG_BYTES // 32, 4)
    assert [s["type"] for s in p.steps] == [coll.STEP_ONESHOT]
    p = coll.plan(ALLREDUCE, coll.ALGO_P2P, 0, 8, -1, OS_AG_BYTES // 32 + 1, 4)
    assert coll.STEP_ONESHOT not in [s["type"] for s in p.steps]
    # reduce_scatter up to OS_RS_BYTES, reduce up to OS_AG_BYTES over all members:
    # one step too, `peer` naming what this rank keeps
    p = coll.plan(REDUCE_SCATTER, coll.ALGO_P2P, 2, 8, -1, OS_RS_BYTES // 8, 8)
    assert [(s["type"], s["peer"]) for s in p.steps] == [(coll.STEP_ONESHOT, -2)]
    p = coll.plan(REDUCE_SCATTER, coll.ALGO_P2P, 2, 8, -1, OS_RS_BYTES // 8 + 1, 8)
    assert coll.STEP_ONESHOT not in [s["type"] for s in p.steps]
    p = coll.plan(REDUCE, coll.ALGO_P2P, 2, 4, 3, 1000, 8)       # root 3
    assert [(s["type"], s["peer"]) for s in p.steps] == [(coll.STEP_ONESHOT, 3)]
    n = 9
    p = coll.plan(ALLREDUCE, coll.ALGO_P2P, 1, n, -1, count, 4)
    assert [s["type"] for s in p.steps] == [coll.STEP_COPY, coll.STEP_BARRIER,
                                            coll.STEP_TREE_PUT, coll.STEP_BARRIER]
    assert p.steps[2]["count"] == count and p.steps[2]["peer"] == 0


def test_plan_errors():
    with pytest.raises(coll.CollError) as e:
        coll.plan(8, 0, 0, 2, -1, 10, 4)         # FI_GATHER: not planned
    assert e.value.rc == -38
    with pytest.raises(coll.CollError):
        coll.plan(ALLREDUCE, 0, 2, 2, -1, 10, 4)  # rank out of range
    with pytest.raises(coll.CollError):
        coll.plan(REDUCE, 0, 0, 2, 5, 10, 4)      # root out of range


def test_block_split():
    for count in (0, 1, 7, 8, 1001):
        for n in (1, 3, 8):
            offs = [coll.block(count, n, r) for r in range(n)]
            assert [o for o, _ in offs] == list(np.cumsum([0] + [ln for _, ln in offs])[:-1])
            assert sum(ln for _, ln in offs) == count
            assert [(a, b - a) for a, b in oracle.slice_bounds(count, n)] == offs


@pytest.mark.parametrize("n", [2, 3])
def test_tree_blocks_skewed_in_tmp(n):
    """Blocks of >= 1 MiB sit round_up(B, 256) + 6 KiB apart in TMP (HBM
    channel skew for the tree kernel's N concurrent streams); results stay
    bit-exact with prov/coll for allreduce, reduce_scatter and reduce."""
    dt, op, count = F64, PROD, n * 140_001 + 1
    off, mlen = coll.block(count, n, 0)
    stride = ((mlen * 8 + 255) // 256) * 256 + 6144
    p = coll.plan(ALLREDUCE, coll.ALGO_TREE, 0, n, -1, count, 8)
    assert p.tmp_bytes == n * stride
    rng = np.random.default_rng(n)
    sends = [rng.uniform(0.9, 1.1, count) for _ in range(n)]
    want = oracle.allreduce(op, dt, sends)[0]
    res = [np.zeros(count * 8, np.uint8) for _ in range(n)]
    _plansim.run(ALLREDUCE, coll.ALGO_TREE, n, -1, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    for r in range(n):
        assert np.array_equal(res[r].view(np.float64), want)
    res = [np.zeros(coll.block(count, n, r)[1] * 8, np.uint8) for r in range(n)]
    _plansim.run(REDUCE_SCATTER, coll.ALGO_TREE, n, -1, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    for r in range(n):
        o, ln = coll.block(count, n, r)
        assert np.array_equal(res[r].view(np.float64), want[o:o + ln])
    res = [np.zeros(count * 8, np.uint8) for _ in range(n)]
    _plansim.run(REDUCE, coll.ALGO_TREE, n, n - 1, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    assert np.array_equal(res[n - 1].view(np.float64), want)


# ---- host-buffer staging geometry (lfa_coll_host_chunk) -------------------

def _stage_and_run(kind, bufs, count, n, esz, chunk, root=0):
    """Replay the provider's host pipeline on numpy: per chunk, the 2-D H2D
    gather, the device collective on dev_count elements (integer SUM, so
    order-free) and the D2H; returns every rank's result."""
    chunks = coll.host_chunks(kind, count, n, esz, chunk)
    res = [np.zeros(count // n if kind == REDUCE_SCATTER else count, np.int64)
           for _ in range(n)]
    covered = 0
    for c in chunks:
        w = c.width // esz
        assert c.dev_count == c.height * w
        staged = []
        for b in bufs:
            rows = [b[(c.src_off + h * c.src_pitch) // esz:][:w] for h in range(c.height)]
            staged.append(np.concatenate(rows))
        total = np.sum(staged, axis=0)
        for r in range(n):
            if kind == REDUCE_SCATTER:
                off, ln = coll.block(c.dev_count, n, r)
                assert ln == w
                part = total[off:off + ln]
            else:
                part = total
            if kind != REDUCE or r == root:
                res[r][c.dst_off // esz:][:w] = part
        covered += w
    return res, covered


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("count_per", [1, 7, 1000, 4097])
@pytest.mark.parametrize("chunk", [8, 24, 1000, 4096, 1 << 20])
def test_host_chunked_reduce_scatter_geometry(n, count_per, chunk):
    """Chunked host reduce_scatter hands rank r exactly block r of the sum:
    every chunk gathers elements [j, j+w) of all N blocks with one 2-D copy."""
    esz, count = 8, n * count_per
    rng = np.random.default_rng(count + n)
    bufs = [rng.integers(-2**40, 2**40, count) for _ in range(n)]
    res, covered = _stage_and_run(REDUCE_SCATTER, bufs, count, n, esz, chunk)
    assert covered == count_per
    total = np.sum(bufs, axis=0)
    for r in range(n):
        off, ln = coll.block(count, n, r)
        assert np.array_equal(res[r], total[off:off + ln])


@pytest.mark.parametrize("kind", [ALLREDUCE, REDUCE])
@pytest.mark.parametrize("count", [1, 5, 1000, 70_001])
@pytest.mark.parametrize("chunk", [8, 24, 4096, 1 << 20])
def test_host_chunked_elementwise_geometry(kind, count, chunk):
    n, esz = 3, 8
    rng = np.random.default_rng(count)
    bufs = [rng.integers(-2**40, 2**40, count) for _ in range(n)]
    res, covered = _stage_and_run(kind, bufs, count, n, esz, chunk, root=1)
    assert covered == count
    total = np.sum(bufs, axis=0)
    for r in range(n):
        if kind == ALLREDUCE or r == 1:
            assert np.array_equal(res[r], total)
        else:
            assert not res[r].any()


def _member_schedule(kind, count, n, esz, host, group_chunk, local_chunk):
    """The device collectives a member issues for one operation: the
    dev_count of each chunk (the shape of each device collective)."""
    chunk = coll.member_chunk(n, host, group_chunk, local_chunk)
    try:
        cs = coll.host_chunks(kind, count, n, esz, chunk)
    except coll.CollError:          # not chunkable: staged / run whole
        return [count]
    if not host and chunk and count * esz <= chunk:
        return [count]              # a device member runs it in one piece
    return [c.dev_count for c in cs]


@pytest.mark.parametrize("n", range(2, 9))
@pytest.mark.parametrize("local", [8, 4096, 1 << 20, 32 << 20])
def test_host_staging_is_one_chunk_in_groups(n, local):
    """a member's LOCAL chunk is a choice its peers cannot
    see, so without a group chunk a group of N > 1 stages host buffers
    whole: one device collective of the full shape, the one a device-buffer
    member issues, whatever the local chunk size."""
    for kind, count in ((ALLREDUCE, 70_001), (REDUCE, 70_001), (BROADCAST, 513),
                        (REDUCE_SCATTER, n * 9001)):
        assert coll.member_chunk(n, True, 0, local) == 0
        cs = coll.host_chunks(kind, count, n, 8, coll.member_chunk(n, True, 0, local))
        assert len(cs) == 1, (kind, n, local)
        assert cs[0].dev_count == count and cs[0].src_off == 0 and cs[0].dst_off == 0
        assert _member_schedule(kind, count, n, 8, False, 0, local) == [count]
    # a one-member group still pipelines with its local chunk
    assert len(coll.host_chunks(ALLREDUCE, 70_001, 1, 8,
                                coll.member_chunk(1, True, 0, 4096))) > 1


@pytest.mark.parametrize("n", range(2, 9))
@pytest.mark.parametrize("group", [8, 4096, 100_000, 1 << 20])
def test_group_chunk_same_schedule_for_every_member(n, group):
    """with a GROUP chunk (the same value on every member)
    host and device members of N = 2..8 issue the identical sequence of
    device collectives — whatever their local chunk — so mixed groups
    stay matched; and the chunks still cover every element exactly once
    (the staged replay below sums them)."""
    for kind, count in ((ALLREDUCE, 70_001), (REDUCE, 70_001), (BROADCAST, 5_130),
                        (REDUCE_SCATTER, n * 9001), (REDUCE_SCATTER, n * 9001 + 1),
                        (ALLGATHER, 777), (ALLREDUCE, 3)):
        scheds = {_member_schedule(kind, count, n, 8, host, group, local).__repr__()
                  for host in (False, True) for local in (4096, 32 << 20)}
        assert len(scheds) == 1, (kind, count, n, group, scheds)
    # and the chunks are real when the buffer exceeds the chunk
    assert len(_member_schedule(ALLREDUCE, 70_001, n, 8, False, group, 0)) == \
        max(1, -(-70_001 * 8 // max(group, 8)))


@pytest.mark.parametrize("n", range(1, 9))
def test_default_group_chunk_same_schedule_for_every_member(n):
    """the group chunk is ON by default (GROUP_CHUNK_AUTO).
    Its size is a function of the operation's byte count (and N) alone —
    32 MiB chunks from 64 MiB on in groups of N > 1, none below — so host
    and device members of N = 2..8, whatever their local chunk, issue the
    identical sequence of device collectives without any setter call; a
    one-member group keeps its local chunk."""
    auto, ch = coll.GROUP_CHUNK_AUTO, coll.AUTO_CHUNK_BYTES
    for nbytes in (4096, ch, 2 * ch - 8, 2 * ch, 256 << 20, (256 << 20) + 24, 1 << 30):
        g = coll.group_chunk(auto, n, nbytes)
        assert g == (ch if n > 1 and nbytes >= 2 * ch else 0), (n, nbytes, g)
        for kind, esz in ((ALLREDUCE, 4), (REDUCE, 8), (BROADCAST, 4), (REDUCE_SCATTER, 8)):
            count = nbytes // esz
            if kind == REDUCE_SCATTER:
                count -= count % n
            g = coll.group_chunk(auto, n, count * esz)
            scheds = {repr(_member_schedule(kind, count, n, esz, host, g, local))
                      for host in (False, True) for local in (4096, 32 << 20)}
            if n > 1:
                assert len(scheds) == 1, (kind, count, n, scheds)
            sched = _member_schedule(kind, count, n, esz, False, g, 0)
            assert sum(sched) == count
            if g:                       # chunked: at least two device collectives
                assert len(sched) >= count * esz // g, (kind, count, n, sched)
    # explicit settings are used as they are, AUTO never reaches a one-member group
    assert coll.group_chunk(0, 8, 1 << 30) == 0
    assert coll.group_chunk(1 << 20, 8, 4096) == 1 << 20
    assert coll.group_chunk(auto, 1, 1 << 30) == 0


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("group", [4096, 100_000])
def test_group_chunked_results_equal_unchunked(n, group):
    """The group-chunked staging, replayed on numpy for every member, gives
    the unchunked result: allreduce, reduce and equal-block reduce_scatter."""
    rng = np.random.default_rng(n * 13 + group)
    for kind, count in ((ALLREDUCE, 70_001), (REDUCE, 70_001), (REDUCE_SCATTER, n * 9001)):
        bufs = [rng.integers(-2**40, 2**40, count) for _ in range(n)]
        res, covered = _stage_and_run(kind, bufs, count, n, 8,
                                      coll.member_chunk(n, True, group, 0), root=n - 1)
        total = np.sum(bufs, axis=0)
        for r in range(n):
            if kind == REDUCE_SCATTER:
                off, ln = coll.block(count, n, r)
                assert np.array_equal(res[r], total[off:off + ln])
            elif kind == ALLREDUCE or r == n - 1:
                assert np.array_equal(res[r], total)


def test_host_chunk_rejects_unchunked_collectives():
    with pytest.raises(coll.CollError):
        coll.host_chunks(REDUCE_SCATTER, 10, 3, 8, 1 << 20)   # ragged blocks
    with pytest.raises(coll.CollError):
        coll.host_chunks(ALLGATHER, 10, 2, 8, 1 << 20)
    assert coll.host_chunks(ALLREDUCE, 0, 2, 8, 1 << 20) == []


# ------------------------------------------------ groups above 32 ranks --
# (one TREE item per group capped groups at LFA_TREE_MAX = 32.)

def _rd_tree(xs):
    """prov/coll's recursive-doubling association as a nested tuple: leaf
    pairs (x[2v+1], x[2v]) for v < rem, then hi-over-lo merges."""
    n = len(xs)
    if n == 1:
        return xs[0]
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    level = [(xs[2 * v + 1], xs[2 * v]) if v < rem else xs[v + rem] for v in range(pof2)]
    while len(level) > 1:
        level = [(level[i + 1], level[i]) for i in range(0, len(level), 2)]
    return level[0]


def _symbolic_tree_result(n, r, count=3):
    """Execute rank r's TREE items of the allreduce schedule symbolically:
    TMP slot k (block exchange) holds x_k, SEND holds x_r; TREE items are
    _rd_tree of their inputs.  Returns the expression left in RESULT."""
    pl = coll.plan(ALLREDUCE, coll.ALGO_TREE, r, n, -1, count * 1000, 4)
    moff, mlen = coll.block(count * 1000, n, r)
    stride = mlen * 4          # < 1 MiB blocks: dense slots
    mem = {("S", moff * 4): f"x{r}"}
    for k in range(n):
        if k != r:
            mem[("T", k * stride)] = f"x{k}"
    out = None
    for s in pl.steps:
        if s["type"] != _plansim.TREE:
            continue
        ins = []
        for k in range(s["nsrc"]):
            b, off = pl.refs[s["first"] + k][:2]
            ins.append(mem[("S" if b == 0 else "T", off)])
        e = _rd_tree(ins)
        b, off = s["dst"][:2]
        if b == 2:
            mem[("T", off)] = e
        else:
            out = e
    assert pl.tmp_bytes >= max(off for (b, off) in mem if b == "T") + mlen * 4
    return out


@pytest.mark.parametrize("n", [32, 33, 47, 48, 64, 100, 511, 512, 513, 1024, 1100])
def test_large_group_tree_is_the_reference_tree(n):
    want = _rd_tree([f"x{k}" for k in range(n)])
    for r in sorted({0, n // 2, n - 1}):
        assert _symbolic_tree_result(n, r) == want, (n, r)


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", [33, 40, 64])
def test_large_group_schedules_execute(algo, n):
    """> 32 ranks, every algorithm (P2P / TREE_COLL fall back to TREE):
    executed across all ranks, bit-exact with the oracle."""
    count = 3 * n + 5
    for dt, op in ((F32, SUM), (I64, BXOR_ := 9)):
        sends = _inputs(dt, n, count, n + 99)
        want = oracle.allreduce(op, dt, sends)[0]
        res = [np.zeros(count * sends[0].itemsize, np.uint8) for _ in range(n)]
        _plansim.run(ALLREDUCE, algo, n, -1, dt, op, count,
                     [s.view(np.uint8) for s in sends], res)
        for r in range(n):
            assert res[r].tobytes() == want.view(np.uint8).tobytes(), (r, dt)
    # reduce_scatter and reduce at n > 32 too
    dt, op = F64, PROD
    sends = _inputs(dt, n, count, 5)
    full = oracle.allreduce(op, dt, sends)[0]
    res = [np.zeros(coll.block(count, n, r)[1] * 8, np.uint8) for r in range(n)]
    _plansim.run(REDUCE_SCATTER, algo, n, -1, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    for r in range(n):
        off, ln = coll.block(count, n, r)
        assert res[r].tobytes() == full[off:off + ln].tobytes()


# ----------------------------------- LFA_ALGO_AUTO --------

@pytest.mark.parametrize("n", range(1, 11))
def test_auto_algo_same_choice_on_every_member(n):
    """LFA_ALGO_AUTO picks per operation from (collective, count, members,
    datatype size) and the group's agreed P2P state only — no rank-local
    input — so every member of N = 1..10 selects the same algorithm; and the
    algorithm it picks for a small bucket is exactly the one-kernel path:
    every member's P2P schedule is ONE one-shot step.  Above the thresholds
    (round 6, LFA_AUTO_BULK's default): P2P's two-barrier schedule for 2..32
    members, with no one-shot step in it.  Allgather, one member, or once the
    P2P agreement failed: the tree."""
    for kind, esz in ((ALLREDUCE, 4), (REDUCE, 8), (REDUCE_SCATTER, 8), (ALLGATHER, 4)):
        for count in (1, 1000, OS_AG_BYTES // (4 * max(n, 1)), OS_AG_BYTES // (4 * max(n, 1)) + 1,
                      OS_RS_BYTES // 8, OS_RS_BYTES // 8 + 1, 1 << 24):
            a = coll.auto_algo(kind, count, n, esz)
            nb = count * esz
            small = (nb * n <= OS_AG_BYTES if kind in (ALLREDUCE, REDUCE) else
                     nb <= OS_RS_BYTES if kind == REDUCE_SCATTER else False)
            reducing = kind in (ALLREDUCE, REDUCE, REDUCE_SCATTER)
            one_shot = 2 <= n <= 8 and small
            want = coll.ALGO_P2P if (reducing and 2 <= n <= 32) else coll.ALGO_TREE
            assert a == want, (kind, count, n, esz)
            assert coll.auto_algo(kind, count, n, esz, p2p_ok=False) == coll.ALGO_TREE
            if a == coll.ALGO_P2P:
                for r in range(n):
                    p = coll.plan(kind, a, r, n, n - 1 if kind == REDUCE else -1, count, esz)
                    types = [s["type"] for s in p.steps]
                    if one_shot:
                        assert types == [coll.STEP_ONESHOT], (kind, n, r)
                    else:
                        assert coll.STEP_ONESHOT not in types and coll.STEP_BARRIER in types, \
                            (kind, count, n, r, types)


def test_auto_bulk_knob():
    """LFA_AUTO_BULK (FI_OFF_LFA_AUTO_BULK): AUTO above the one-shot bounds
    takes P2P's two-barrier schedule by default and the tree with "tree";
    the one-shot-sized buckets stay P2P either way.  Read once per process,
    so each setting runs in its own interpreter."""
    import json
    import os
    import subprocess
    import sys
    code = (
        "import json\n"
        "from libfabric_amd import coll\n"
        "print(json.dumps([coll.auto_algo(3, c, 8, 4) for c in (1024, 1 << 22, 1 << 26)]"
        " + [coll.auto_algo(5, c, 8, 8) for c in (1024, 1 << 22)]))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(val):
        e = {k: v for k, v in os.environ.items() if k != "LFA_AUTO_BULK"}
        if val is not None:
            e["LFA_AUTO_BULK"] = val
        out = subprocess.run([sys.executable, "-c", code], cwd=root, env=e, check=True,
                             capture_output=True, text=True).stdout
        return json.loads(out.strip().splitlines()[-1])

    P2P, TREE = coll.ALGO_P2P, coll.ALGO_TREE
    assert run(None) == [P2P, P2P, P2P, P2P, P2P]
    assert run("p2p") == [P2P, P2P, P2P, P2P, P2P]
    assert run("tree") == [P2P, TREE, TREE, P2P, TREE]


def test_one_shot_bounds_follow_their_knobs():
    """LFA_OS_AG_BYTES / LFA_OS_RS_BYTES (lfa_coll_plan.h) move the P2P
    one-shot bounds, the same for the planner and LFA_ALGO_AUTO; read once per
    process, so each setting runs in its own interpreter."""
    import json
    import os
    import subprocess
    import sys
    code = (
        "import json\n"
        "from libfabric_amd import coll\n"
        "ar = [coll.auto_algo(3, c, 4, 4) for c in (16384, 16385, 131072, 131073)]\n"
        "rs = [coll.auto_algo(5, c, 4, 8) for c in (65536, 65537, 524288, 524289)]\n"
        "p = coll.plan(3, coll.ALGO_P2P, 0, 4, -1, 131072, 4)\n"
        "print(json.dumps([ar, rs, [s['type'] for s in p.steps]]))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(env):
        e = {k: v for k, v in os.environ.items()
             if k not in ("LFA_OS_AG_BYTES", "LFA_OS_RS_BYTES")}
        # the bounds alone: above them the tree (test_auto_bulk_knob covers
        # AUTO's bulk default)
        e["LFA_AUTO_BULK"] = "tree"
        e.update(env)
        out = subprocess.run([sys.executable, "-c", code], cwd=root, env=e, check=True,
                             capture_output=True, text=True).stdout
        return json.loads(out.strip().splitlines()[-1])

    P2P, TREE = coll.ALGO_P2P, coll.ALGO_TREE
    # defaults: allreduce 2 MiB over 4 members = 131072 floats each;
    # reduce_scatter 4 MiB per member = 524288 doubles
    ar, rs, steps = run({})
    assert ar == [P2P, P2P, P2P, TREE] and rs == [P2P, P2P, P2P, TREE]
    assert steps == [coll.STEP_ONESHOT]
    # the pre-round-5 bounds: 256 KiB over the members, 512 KiB per member
    ar, rs, steps = run({"LFA_OS_AG_BYTES": str(256 << 10), "LFA_OS_RS_BYTES": str(512 << 10)})
    assert ar == [P2P, TREE, TREE, TREE] and rs == [P2P, TREE, TREE, TREE]
    assert coll.STEP_ONESHOT not in steps
