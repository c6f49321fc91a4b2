"""Property-based parity (hypothesis): random shapes against the oracle.

The fixture and grid tests pin chosen points; these draw the cross product —
every table entry, any length, any byte offset of either operand, edge lanes
(±0, ±inf, NaN, denormals, type extremes) at a drawn density, any fan-in, any
group size, root and algorithm — and hold the product to the same bar:
bit-exact for integer / bitwise results, bit-exact on every non-NaN lane of
float results (tests/_cmp.py).  `derandomize=True` makes every run draw the
same examples, so a failure reproduces.

CPU: the host combine (lfa_host_write / lfa_host_reduce_tree, the kernels'
functors compiled for the host), the synchronous fetch and compare tables on
host pointers, and the collective schedules (lfa_coll_plan) executed by
tests/_plansim.py.  GPU (``-m gpu``): the same draws through the gfx950
kernels — lfa_atomic_write_async, lfa_atomic_readwrite_async /
lfa_atomic_swap_async and lfa_reduce_tree_async.
"""
import ctypes

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle
from libfabric_amd import coll
from tests import _plansim
from tests._cmp import assert_parity

WRITE_PAIRS = [(op, dt) for op in range(12) for dt in oracle.DT_NP
               if op != 10 and oracle.has_handler(op, dt)]
REDUCE_PAIRS = [(op, dt) for op, dt in WRITE_PAIRS if op <= 9]
RW_PAIRS = [(op, dt) for op in range(12) for dt in oracle.DT_NP
            if oracle.has_readwrite(op, dt)]
SWAP_PAIRS = [(op, dt) for op in range(12, 19) for dt in oracle.DT_NP
              if oracle.has_swap(op, dt)]

CPU_SETTINGS = settings(max_examples=400, deadline=None, derandomize=True,
                        suppress_health_check=[HealthCheck.too_slow])
GPU_SETTINGS = settings(max_examples=120, deadline=None, derandomize=True,
                        suppress_health_check=[HealthCheck.too_slow,
                                               HealthCheck.function_scoped_fixture])


def _edge_values(nd):
    if nd.kind == "f":
        fi = np.finfo(nd)
        return np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan, fi.tiny,
                         fi.smallest_subnormal, -fi.smallest_subnormal, fi.max,
                         -fi.max, 1.0, -1.0], dtype=nd)
    if nd.kind == "c":
        f = _edge_values(np.dtype(np.float32))
        c = np.empty(f.size * f.size, nd)
        c.real = np.repeat(f, f.size)
        c.imag = np.tile(f[::-1], f.size)
        return c
    if nd.kind == "V":
        return None
    ii = np.iinfo(nd)
    return np.array([ii.min, ii.max, 0, 1, ii.max - 1] + ([-1] if ii.min < 0 else []),
                    dtype=nd)


def _operand(dt, n, rng, edge_frac):
    """n elements of dt as bytes: random lanes with a fraction of edge lanes."""
    nd = oracle.DT_NP[dt]
    if nd.kind == "V":
        return rng.integers(0, 256, size=n * 16, dtype=np.uint8)
    if nd.kind == "c":
        x = rng.uniform(-2, 2, size=2 * n).astype(np.float32).view(np.complex64)
    elif nd.kind == "f":
        x = rng.uniform(-2, 2, size=n).astype(nd)
    else:
        ii = np.iinfo(nd)
        x = rng.integers(ii.min, ii.max, size=n, dtype=nd, endpoint=True)
    ev = _edge_values(nd)
    if n and ev is not None and edge_frac:
        m = rng.random(n) < edge_frac
        x[m] = ev[rng.integers(0, ev.size, size=int(m.sum()))]
    return x.view(np.uint8).copy()


def _at(buf, off, nbytes):
    """A view of nbytes starting `off` bytes into a fresh padded buffer (so
    the pointer carries the drawn misalignment)."""
    raw = np.zeros(nbytes + 64, np.uint8)
    base = (-raw.ctypes.data) % 64          # 64-B aligned origin, then `off`
    v = raw[base + off: base + off + nbytes]
    v[:] = buf
    return v


# ---------------------------------------------------------------- CPU ----

@pytest.fixture(scope="module")
def L():
    from libfabric_amd import lib
    return lib()


@CPU_SETTINGS
@given(pair=st.sampled_from(WRITE_PAIRS), n=st.integers(0, 700),
       doff=st.integers(0, 15), soff=st.integers(0, 15),
       edge=st.sampled_from([0.0, 0.05, 0.5]), seed=st.integers(0, 2**31))
def test_host_write_any_shape(L, pair, n, doff, soff, edge, seed):
    op, dt = pair
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(seed)
    d0, s0 = _operand(dt, n, rng, edge), _operand(dt, n, rng, edge)
    want = d0.copy()
    if n:
        oracle.write(op, dt, want.view(oracle.DT_NP[dt]), s0.copy().view(oracle.DT_NP[dt]))
    d, s = _at(d0, doff, n * esz), _at(s0, soff, n * esz)
    assert L.lfa_host_write(op, dt, d.ctypes.data, s.ctypes.data, n) == 0
    assert_parity(dt, d, want, f"op={op} dt={dt} n={n} offs={doff},{soff}")
    assert np.array_equal(s, s0)            # src is read-only


@CPU_SETTINGS
@given(pair=st.sampled_from(REDUCE_PAIRS), nsrc=st.integers(1, 32), n=st.integers(0, 300),
       edge=st.sampled_from([0.0, 0.1]), seed=st.integers(0, 2**31))
def test_host_tree_any_fan_in(L, pair, nsrc, n, edge, seed):
    from libfabric_amd import atomic
    op, dt = pair
    rng = np.random.default_rng(seed)
    nd = oracle.DT_NP[dt]
    sends = [_operand(dt, n, rng, edge).view(nd) for _ in range(nsrc)]
    out = np.zeros(n * oracle.datatype_size(dt), np.uint8).view(nd)
    atomic.host_reduce_tree(op, dt, out, sends, n)
    if n:
        want = oracle.allreduce(op, dt, sends)[0]
        assert_parity(dt, out.view(np.uint8), want.view(np.uint8),
                      f"op={op} dt={dt} nsrc={nsrc} n={n}")


_RW = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_size_t)
_SW = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_void_p, ctypes.c_size_t)


@CPU_SETTINGS
@given(pair=st.sampled_from(RW_PAIRS + SWAP_PAIRS), n=st.integers(0, 500),
       edge=st.sampled_from([0.0, 0.3]), seed=st.integers(0, 2**31))
def test_host_fetch_and_compare_tables(L, pair, n, edge, seed):
    """The synchronous readwrite / swap tables on host pointers (the host
    loop below lfa_host_small_bytes) against the oracle."""
    op, dt = pair
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    d0, s0 = _operand(dt, n, rng, edge), _operand(dt, n, rng, edge)
    # compare operands: half the lanes equal to dst so every CSWAP form fires
    c0 = _operand(dt, n, rng, edge)
    if n:
        eq = np.repeat(rng.random(n) < 0.5, oracle.datatype_size(dt))
        c0[eq] = d0[eq]
    want_d, want_r = d0.copy(), np.zeros_like(d0)
    d, r = d0.copy(), np.zeros_like(d0)
    if op < 12:
        if n:
            oracle.readwrite(op, dt, want_d.view(nd), s0.copy().view(nd), want_r.view(nd))
        fn = _RW((ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_readwrite_handlers")
                 [op * 16 + dt])
        fn(d.ctypes.data, s0.ctypes.data, r.ctypes.data, n)
        assert_parity(dt, d, want_d, f"readwrite op={op} dt={dt} n={n}")
        assert_parity(dt, r, want_r, f"readwrite res op={op} dt={dt} n={n}")
    else:
        if n:
            oracle.swap(op, dt, want_d.view(nd), s0.copy().view(nd), c0.copy().view(nd),
                        want_r.view(nd), oracle.CAS)
        fn = _SW((ctypes.c_void_p * (7 * 16)).in_dll(L, "lfa_atomic_swap_handlers")
                 [(op - 12) * 16 + dt])
        fn(d.ctypes.data, s0.ctypes.data, c0.ctypes.data, r.ctypes.data, n)
        # compare semantics follow the shipping build's bit compare: exact bytes
        assert np.array_equal(d, want_d), f"swap op={op} dt={dt} n={n}"
        assert np.array_equal(r, want_r), f"swap res op={op} dt={dt} n={n}"
    assert L.lfa_atomic_last_error() == 0


def test_zero_count_table_calls_are_no_ops(L):
    """A zero-element call of any synchronous table entry does nothing and
    reports nothing (the reference's loops run zero times), even where no GPU
    is present: the fetch and compare entries once sent it to the device
    launcher and a stream synchronize (-FI_EIO without a GPU)."""
    w = (ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_write_handlers")
    rw = (ctypes.c_void_p * (12 * 16)).in_dll(L, "lfa_atomic_readwrite_handlers")
    sw = (ctypes.c_void_p * (7 * 16)).in_dll(L, "lfa_atomic_swap_handlers")
    W = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
    buf = np.zeros(64, np.uint8)
    p = buf.ctypes.data
    assert L.lfa_atomic_last_error() == 0
    for op, dt in WRITE_PAIRS:
        W(w[op * 16 + dt])(p, p, 0)
        W(w[op * 16 + dt])(None, None, 0)
    for op, dt in RW_PAIRS:
        _RW(rw[op * 16 + dt])(p, p, p, 0)
        _RW(rw[op * 16 + dt])(None, None, None, 0)
    for op, dt in SWAP_PAIRS:
        _SW(sw[(op - 12) * 16 + dt])(p, p, p, p, 0)
        _SW(sw[(op - 12) * 16 + dt])(None, None, None, None, 0)
    assert L.lfa_atomic_last_error() == 0
    assert not buf.any()


ALLREDUCE, REDUCE_SCATTER, REDUCE = 3, 5, 6
SCHED_PAIRS = [(2, 8), (3, 9), (0, 6), (1, 8), (6, 7), (7, 1), (9, 4), (4, 8), (3, 10)]
ALGOS = [coll.ALGO_TREE, coll.ALGO_RD, coll.ALGO_TREE_COLL, coll.ALGO_P2P]


@settings(max_examples=300, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow])
@given(coll_op=st.sampled_from([ALLREDUCE, REDUCE_SCATTER, REDUCE]),
       algo=st.sampled_from(ALGOS), n=st.integers(1, 9), count=st.integers(0, 400),
       root_pick=st.integers(0, 1 << 16), pair=st.sampled_from(SCHED_PAIRS),
       seed=st.integers(0, 2**31))
def test_schedule_any_group(coll_op, algo, n, count, root_pick, pair, seed):
    """Every rank's schedule for a drawn (collective, algorithm, group size,
    count, root, op, datatype), run by the host simulator: allreduce equals
    prov/coll's tree on every rank, reduce_scatter block r of it, reduce the
    whole of it at the root only."""
    if coll_op == REDUCE and algo == coll.ALGO_TREE_COLL:
        algo = coll.ALGO_TREE            # reduce has no ALLTOALL form
    op, dt = pair
    nd = oracle.DT_NP[dt]
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(seed)
    sends = [_operand(dt, count, rng, 0.05).view(nd) for _ in range(n)]
    root = root_pick % n if coll_op == REDUCE else -1
    full = oracle.allreduce(op, dt, sends)[0] if count else np.zeros(0, nd)
    res = []
    for r in range(n):
        if coll_op == REDUCE_SCATTER:
            ln = coll.block(count, n, r)[1]
        else:
            ln = count
        res.append(np.zeros(ln * esz, np.uint8))
    _plansim.run(coll_op, algo, n, root, dt, op, count,
                 [s.view(np.uint8) for s in sends], res)
    for r in range(n):
        if coll_op == REDUCE_SCATTER:
            off, ln = coll.block(count, n, r)
            want = full[off:off + ln]
        elif coll_op == REDUCE and r != root:
            continue
        else:
            want = full
        assert_parity(dt, res[r], want.view(np.uint8),
                      f"coll={coll_op} algo={algo} n={n} count={count} rank={r}")


ALLGATHER, BROADCAST, SCATTER = 4, 1, 7


@settings(max_examples=200, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow])
@given(coll_op=st.sampled_from([ALLGATHER, BROADCAST, SCATTER]), n=st.integers(1, 9),
       count=st.integers(0, 300), esz=st.sampled_from([1, 2, 4, 8, 16]),
       root_pick=st.integers(0, 1 << 16), seed=st.integers(0, 2**31))
def test_data_movement_schedules_any_group(coll_op, n, count, esz, root_pick, seed):
    """allgather (rank blocks in group-rank order), broadcast (the root's
    buffer everywhere) and scatter (block r of the root's buffer to rank r)
    at drawn group sizes, counts, element sizes and roots, every rank's
    schedule run by the host simulator (coll_do_allgather coll_coll.c:452,
    coll_do_scatter :510, coll_ep_broadcast :1158)."""
    dt = {1: 1, 2: 3, 4: 5, 8: 7, 16: 15}[esz]
    rng = np.random.default_rng(seed)
    root = root_pick % n
    nb = count * esz
    if coll_op == ALLGATHER:
        sends = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(n)]
        res = [np.zeros(n * nb, np.uint8) for _ in range(n)]
        _plansim.run(coll_op, 0, n, -1, dt, 2, count, sends, res)
        want = np.concatenate(sends) if nb else np.zeros(0, np.uint8)
        for r in range(n):
            assert res[r].tobytes() == want.tobytes(), (n, count, esz, r)
    elif coll_op == BROADCAST:
        bufs = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(n)]
        want = bufs[root].copy()
        _plansim.run(coll_op, 0, n, root, dt, 2, count, [None] * n, bufs)
        for r in range(n):
            assert bufs[r].tobytes() == want.tobytes(), (n, count, esz, r, root)
    else:
        big = rng.integers(0, 256, n * nb, dtype=np.uint8)
        res = [np.zeros(nb, np.uint8) for _ in range(n)]
        _plansim.run(coll_op, 0, n, root, dt, 2, count,
                     [big if r == root else np.zeros(0, np.uint8) for r in range(n)], res)
        for r in range(n):
            assert res[r].tobytes() == big[r * nb:(r + 1) * nb].tobytes(), (n, count, r, root)


# ---------------------------------------------------------------- GPU ----

def _dev(buf, off, nbytes, torch):
    """Device bytes at a drawn byte offset inside a fresh allocation."""
    t = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    v = t[off: off + nbytes]
    if nbytes:
        v.copy_(torch.from_numpy(np.ascontiguousarray(buf)))
    return v


@pytest.mark.gpu
@GPU_SETTINGS
@given(pair=st.sampled_from(WRITE_PAIRS),
       n=st.one_of(st.integers(0, 5000), st.integers(5000, 1 << 20)),
       doff=st.integers(0, 15), soff=st.integers(0, 15),
       edge=st.sampled_from([0.0, 0.05, 0.5]), seed=st.integers(0, 2**31))
def test_gpu_write_any_shape(pair, n, doff, soff, edge, seed):
    """lfa_atomic_write_async at any length and byte offset of either operand
    (co-aligned vector body + element head/tail, the element kernel, the
    byte-gather kernel) against the oracle."""
    import torch
    from libfabric_amd import atomic
    op, dt = pair
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(seed)
    d0, s0 = _operand(dt, n, rng, edge), _operand(dt, n, rng, edge)
    want = d0.copy()
    if n:
        oracle.write(op, dt, want.view(oracle.DT_NP[dt]), s0.copy().view(oracle.DT_NP[dt]))
    d, s = _dev(d0, doff, n * esz, torch), _dev(s0, soff, n * esz, torch)
    atomic.write(op, dt, d, s, n)
    torch.cuda.synchronize()
    assert_parity(dt, d.cpu().numpy(), want, f"op={op} dt={dt} n={n} offs={doff},{soff}")
    assert np.array_equal(s.cpu().numpy(), s0)


@pytest.mark.gpu
@GPU_SETTINGS
@given(pair=st.sampled_from(REDUCE_PAIRS), nsrc=st.integers(1, 32),
       n=st.one_of(st.integers(0, 3000), st.integers(3000, 1 << 18)),
       off=st.sampled_from([0, 16, 4, 1]), edge=st.sampled_from([0.0, 0.1]),
       seed=st.integers(0, 2**31))
def test_gpu_tree_any_fan_in(pair, nsrc, n, off, edge, seed):
    """lfa_reduce_tree_async: any fan-in (the 2/4/8/16/32-leaf bodies and
    their pair leaves), any length, inputs at a drawn common offset."""
    import torch
    from libfabric_amd import atomic
    op, dt = pair
    esz = oracle.datatype_size(dt)
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    sends = [_operand(dt, n, rng, edge) for _ in range(nsrc)]
    srcs = [_dev(x, off, n * esz, torch) for x in sends]
    out = _dev(np.zeros(n * esz, np.uint8), off, n * esz, torch)
    atomic.reduce_tree(op, dt, out, srcs, n)
    torch.cuda.synchronize()
    if n:
        want = oracle.allreduce(op, dt, [x.view(nd) for x in sends])[0]
        assert_parity(dt, out.cpu().numpy(), want.view(np.uint8),
                      f"op={op} dt={dt} nsrc={nsrc} n={n} off={off}")


@pytest.mark.gpu
@GPU_SETTINGS
@given(pair=st.sampled_from(RW_PAIRS + SWAP_PAIRS),
       n=st.one_of(st.integers(0, 4000), st.integers(4000, 1 << 19)),
       off=st.sampled_from([0, 16, 8, 3]), edge=st.sampled_from([0.0, 0.3]),
       seed=st.integers(0, 2**31))
def test_gpu_fetch_and_compare_any_shape(pair, n, off, edge, seed):
    """lfa_atomic_readwrite_async / lfa_atomic_swap_async against the oracle
    (dst, src, cmp and res at one drawn byte offset)."""
    import torch
    from libfabric_amd import atomic
    op, dt = pair
    esz = oracle.datatype_size(dt)
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    d0, s0, c0 = (_operand(dt, n, rng, edge) for _ in range(3))
    if n:
        eq = np.repeat(rng.random(n) < 0.5, esz)
        c0[eq] = d0[eq]
    want_d, want_r = d0.copy(), np.zeros_like(d0)
    d, s, c = (_dev(x, off, n * esz, torch) for x in (d0, s0, c0))
    r = _dev(np.zeros(n * esz, np.uint8), off, n * esz, torch)
    if op < 12:
        if n:
            oracle.readwrite(op, dt, want_d.view(nd), s0.copy().view(nd), want_r.view(nd))
        atomic.readwrite(op, dt, d, s, r, n)
        torch.cuda.synchronize()
        assert_parity(dt, d.cpu().numpy(), want_d, f"readwrite op={op} dt={dt} n={n}")
        assert_parity(dt, r.cpu().numpy(), want_r, f"readwrite res op={op} dt={dt} n={n}")
    else:
        if n:
            oracle.swap(op, dt, want_d.view(nd), s0.copy().view(nd), c0.copy().view(nd),
                        want_r.view(nd), oracle.CAS)
        atomic.swap(op, dt, d, s, c, r, n)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), want_d), f"swap op={op} dt={dt} n={n}"
        assert np.array_equal(r.cpu().numpy(), want_r), f"swap res op={op} dt={dt} n={n}"


@pytest.mark.gpu
@GPU_SETTINGS
@given(pair=st.sampled_from(REDUCE_PAIRS), nsrc=st.integers(1, 16), ndst=st.integers(1, 4),
       n=st.one_of(st.integers(0, 3000), st.integers(3000, 1 << 17)),
       offs=st.lists(st.sampled_from([0, 0, 16, 1, 2, 3, 5, 8]), min_size=20, max_size=20),
       seed=st.integers(0, 2**31))
def test_gpu_tree_put_any_offsets(pair, nsrc, ndst, n, offs, seed):
    """lfa_reduce_tree_put_async (the P2P kernel) with every operand at its
    own drawn byte offset: co-aligned vector body, element path, and the
    byte-wise path for operands not aligned to the element (a caller's own
    block read or result written in place)."""
    import torch
    from libfabric_amd import atomic
    op, dt = pair
    esz = oracle.datatype_size(dt)
    nd = oracle.DT_NP[dt]
    rng = np.random.default_rng(seed)
    sends = [_operand(dt, n, rng, 0.05) for _ in range(nsrc)]
    srcs = [_dev(x, offs[k], n * esz, torch) for k, x in enumerate(sends)]
    outs = [_dev(np.zeros(n * esz, np.uint8), offs[16 + j], n * esz, torch)
            for j in range(ndst)]
    atomic.reduce_tree_put(op, dt, outs, srcs, n)
    torch.cuda.synchronize()
    if n:
        want = oracle.allreduce(op, dt, [x.view(nd) for x in sends])[0].view(np.uint8)
        for j, o in enumerate(outs):
            assert_parity(dt, o.cpu().numpy(), want,
                          f"op={op} dt={dt} nsrc={nsrc} out={j} n={n} offs={offs}")


@pytest.mark.gpu
@GPU_SETTINGS
@given(coll_op=st.sampled_from([ALLREDUCE, REDUCE_SCATTER, REDUCE]),
       algo=st.sampled_from(ALGOS), n=st.integers(1, 8),
       count=st.one_of(st.integers(0, 700), st.integers(700, 200_000)),
       pair=st.sampled_from(SCHED_PAIRS), soff=st.integers(0, 15), roff=st.integers(0, 15),
       root_pick=st.integers(0, 1 << 16), seed=st.integers(0, 2**31))
def test_gpu_collectives_any_buffer_offset(coll_op, algo, n, count, pair, soff, roff,
                                           root_pick, seed):
    """Every rank's schedule on the GPU (lfa_coll_loopback: the executor, its
    kernels and a device-copy transport) with the send and result buffers at
    drawn byte offsets — including offsets that are not a multiple of the
    element, which prov/coll's host loops accept as well."""
    import torch
    if coll_op == REDUCE and algo == coll.ALGO_TREE_COLL:
        algo = coll.ALGO_TREE
    op, dt = pair
    nd = oracle.DT_NP[dt]
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(seed)
    sends = [_operand(dt, count, rng, 0.05) for _ in range(n)]
    root = root_pick % n if coll_op == REDUCE else -1
    full = oracle.allreduce(op, dt, [x.view(nd) for x in sends])[0] if count else \
        np.zeros(0, nd)
    lens = [coll.block(count, n, r)[1] if coll_op == REDUCE_SCATTER else count
            for r in range(n)]
    sd = [_dev(x, soff, count * esz, torch) for x in sends]
    rd = [_dev(np.zeros(lens[r] * esz, np.uint8), roff, lens[r] * esz, torch)
          for r in range(n)]
    coll.loopback(coll_op, algo, n, root, dt, op, count, sd, rd)
    torch.cuda.synchronize()
    for r in range(n):
        if coll_op == REDUCE and r != root:
            continue
        off = coll.block(count, n, r)[0] if coll_op == REDUCE_SCATTER else 0
        assert_parity(dt, rd[r].cpu().numpy(), full[off:off + lens[r]].view(np.uint8),
                      f"coll={coll_op} algo={algo} n={n} count={count} rank={r} "
                      f"offs={soff},{roff}")
    for x, d in zip(sends, sd):
        assert np.array_equal(d.cpu().numpy(), x)      # inputs untouched


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [8, 2, 9, 6])
@pytest.mark.parametrize("mode", [-1, -2, 0, 1])
@pytest.mark.parametrize("offs", [(0, 0), (1, 3), (2, 0), (0, 5)])
def test_gpu_oneshot_misaligned_buffers(dt, mode, offs):
    """The one-shot kernel (LFA_STEP_ONESHOT) with the caller's send and
    result at byte offsets that are not a multiple of the element: two ranks
    on two streams of this process, each with its own workspace; every mode
    (allreduce, reduce_scatter, reduce to either root) bit-exact against the
    oracle, no wait timed out."""
    import torch
    op = 2 if dt in (8, 9) else 0                     # float/double SUM, ints MIN
    esz = oracle.datatype_size(dt)
    nd = oracle.DT_NP[dt]
    count = 4000 // esz
    rng = np.random.default_rng(dt * 100 + mode)
    sends = [_operand(dt, count, rng, 0.05) for _ in range(2)]
    full = oracle.allreduce(op, dt, [x.view(nd) for x in sends])[0].view(np.uint8)
    region, flag_off = 1 << 20, 2 << 20
    from libfabric_amd.coll import sig_area_bytes
    ws = [torch.zeros(flag_off + sig_area_bytes(), dtype=torch.uint8, device="cuda")
          for _ in range(2)]
    sym = (ctypes.c_void_p * 2)(*[w.data_ptr() for w in ws])
    status = torch.full((1,), -1, dtype=torch.int64).pin_memory()
    sd = [_dev(x, offs[0], count * esz, torch) for x in sends]
    want, rd = [], []
    for r in range(2):
        off, ln = coll.block(count, 2, r) if mode == -2 else (0, count)
        want.append(full[off * esz:(off + ln) * esz] if mode < 0 or mode == r else None)
        rd.append(_dev(np.zeros(ln * esz, np.uint8), offs[1], ln * esz, torch))
    torch.cuda.synchronize()
    # two priorities: HIP keeps a hardware-queue pool per priority, so the
    # ranks' kernels cannot land in one queue, where rank 0's wait would hold
    # rank 1's launch behind it until the timeout
    streams = [torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)]
    for r in range(2):
        coll.oneshot_reduce(op, dt, coll.OneShot(
            sd[r].data_ptr(), rd[r].data_ptr(), count, mode,
            ctypes.cast(sym, ctypes.c_void_p), 4096, region // 2, flag_off, 2, r, 1,
            status.data_ptr(), 1, 5_000_000), streams[r])
    for s in streams:
        s.synchronize()
    assert int(status.item()) == -1, "a one-shot wait timed out"
    for r in range(2):
        if want[r] is not None:
            assert_parity(dt, rd[r].cpu().numpy(), want[r], f"rank {r} mode {mode} offs {offs}")


@pytest.mark.gpu
@GPU_SETTINGS
@given(coll_op=st.sampled_from([ALLGATHER, BROADCAST, SCATTER]), n=st.integers(1, 8),
       count=st.one_of(st.integers(0, 500), st.integers(500, 100_000)),
       esz=st.sampled_from([1, 2, 4, 8, 16]), soff=st.integers(0, 15), roff=st.integers(0, 15),
       root_pick=st.integers(0, 1 << 16), seed=st.integers(0, 2**31))
def test_gpu_data_movement_any_buffer_offset(coll_op, n, count, esz, soff, roff, root_pick,
                                             seed):
    """allgather / broadcast / scatter through the executor on the GPU
    (lfa_coll_loopback) with the buffers at drawn byte offsets."""
    import torch
    dt = {1: 1, 2: 3, 4: 5, 8: 7, 16: 15}[esz]
    rng = np.random.default_rng(seed)
    root = root_pick % n
    nb = count * esz
    if coll_op == ALLGATHER:
        sends = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(n)]
        sd = [_dev(x, soff, nb, torch) for x in sends]
        rd = [_dev(np.zeros(n * nb, np.uint8), roff, n * nb, torch) for _ in range(n)]
        coll.loopback(coll_op, 0, n, -1, dt, 2, count, sd, rd)
        torch.cuda.synchronize()
        want = np.concatenate(sends) if nb else np.zeros(0, np.uint8)
        for r in range(n):
            assert np.array_equal(rd[r].cpu().numpy(), want), (n, count, esz, r)
    elif coll_op == BROADCAST:
        bufs = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(n)]
        want = bufs[root].copy()
        bd = [_dev(x, roff, nb, torch) for x in bufs]
        coll.loopback(coll_op, 0, n, root, dt, 2, count, [None] * n, bd)
        torch.cuda.synchronize()
        for r in range(n):
            assert np.array_equal(bd[r].cpu().numpy(), want), (n, count, esz, r, root)
    else:
        big = rng.integers(0, 256, n * nb, dtype=np.uint8)
        sd = [_dev(big if r == root else np.zeros(0, np.uint8), soff,
                   n * nb if r == root else 0, torch) for r in range(n)]
        rd = [_dev(np.zeros(nb, np.uint8), roff, nb, torch) for _ in range(n)]
        coll.loopback(coll_op, 0, n, root, dt, 2, count, sd, rd)
        torch.cuda.synchronize()
        for r in range(n):
            assert np.array_equal(rd[r].cpu().numpy(), big[r * nb:(r + 1) * nb]), (n, count, r)


@settings(max_examples=300, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow])
@given(kind=st.sampled_from([ALLREDUCE, REDUCE, REDUCE_SCATTER]), n=st.integers(1, 9),
       per=st.integers(1, 3000), chunk=st.integers(8, 1 << 16), root_pick=st.integers(0, 99),
       seed=st.integers(0, 2**31))
def test_host_chunk_geometry_any_shape(kind, n, per, chunk, root_pick, seed):
    """lfa_coll_host_chunk's staging geometry (the host-buffer pipeline and
    the group chunk) at drawn collective, group size, count and chunk bytes:
    replayed on numpy (tests/test_coll_plan.py::_stage_and_run) every element
    is covered once and every rank ends with exactly its part of the sum."""
    from tests.test_coll_plan import _stage_and_run
    esz = 8
    count = n * per if kind == REDUCE_SCATTER else per
    root = root_pick % n
    rng = np.random.default_rng(seed)
    bufs = [rng.integers(-2**40, 2**40, count) for _ in range(n)]
    res, covered = _stage_and_run(kind, bufs, count, n, esz, chunk, root=root)
    total = np.sum(bufs, axis=0)
    if kind == REDUCE_SCATTER:
        assert covered == per
        for r in range(n):
            off, ln = coll.block(count, n, r)
            assert np.array_equal(res[r], total[off:off + ln])
    else:
        assert covered == count
        for r in range(n):
            if kind == ALLREDUCE or r == root:
                assert np.array_equal(res[r], total)


@pytest.mark.gpu
@GPU_SETTINGS
@given(kind=st.sampled_from([ALLREDUCE, REDUCE_SCATTER, REDUCE, ALLGATHER, BROADCAST, SCATTER]),
       algo=st.sampled_from([0, 1, 2, 3, 4, 5]), pair=st.sampled_from(SCHED_PAIRS),
       count=st.one_of(st.integers(0, 3000), st.integers(3000, 300_000)),
       host=st.booleans(), gchunk=st.sampled_from([0, 0, 4096, 1 << 20]),
       off=st.sampled_from([0, 0, 16, 4, 1]), seed=st.integers(0, 2**31))
def test_gpu_rccl_domain_world1_any_call(ep1, kind, algo, pair, count, host, gchunk, off,
                                         seed):
    """The RCCL device domain at world size 1 (every collective is a copy of
    the caller's data): each submit path — device buffers in place, host
    buffers staged whole or in chunks, a group chunk, every algorithm, byte
    offsets — returns the input where the reference's one-rank collective
    does."""
    import torch
    ep = ep1
    op, dt = pair
    esz = oracle.datatype_size(dt)
    rng = np.random.default_rng(seed)
    nb = count * esz
    data = _operand(dt, count * (1 if kind != SCATTER else 1), rng, 0.05)
    ep.set_algo(algo)
    ep.set_group_chunk(gchunk)
    try:
        if host:
            src = _at(data, off, nb)
            dst = _at(np.zeros(nb, np.uint8), (off + 3) % 16, nb)
            get = lambda b: b.copy()                                     # noqa: E731
        else:
            src = _dev(data, off, nb, torch)
            dst = _dev(np.zeros(nb, np.uint8), (off + 3) % 16, nb, torch)
            get = lambda b: b.cpu().numpy()                              # noqa: E731
            torch.cuda.synchronize()
        if kind == ALLREDUCE:
            ctx = ep.allreduce(src, dst, count, dt, op)
        elif kind == REDUCE_SCATTER:
            ctx = ep.reduce_scatter(src, dst, count, dt, op)
        elif kind == REDUCE:
            ctx = ep.reduce(src, dst, count, 0, dt, op)
        elif kind == ALLGATHER:
            ctx = ep.allgather(src, dst, count, dt)
        elif kind == SCATTER:
            ctx = ep.scatter(src, dst, count, 0, dt)
        else:
            ctx = ep.broadcast(src, count, 0, dt)
            dst = src
        ep.wait(ctx, timeout_s=60)
        got = get(dst)
        assert got.tobytes() == data.tobytes(), (kind, algo, count, host, gchunk, off)
    finally:
        ep.set_group_chunk(coll.GROUP_CHUNK_AUTO)   # the default


@pytest.fixture(scope="module")
def ep1():
    """One RCCL device-domain endpoint at world size 1 for the module."""
    from libfabric_amd import coll as c
    ep = c.Endpoint(0, 1, 0, c.Endpoint.unique_id())
    yield ep
    ep.close()
