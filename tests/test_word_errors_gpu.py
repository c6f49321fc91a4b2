"""The error path of operations completed by a host-mapped word.

A one-member group's small reducing collectives, and the one-shot P2P kernel
of larger groups, complete through a word the last workgroup stores into
pinned host memory instead of an event.  A word that never comes must not
hold the endpoint: the operation completes ONCE, in error, through
lfa_cq_readerr (ETIMEDOUT past LFA_SIG_TIMEOUT_MS, EIO when the direct queue
owing it has failed), the operations behind it complete normally, and the
endpoint — and a fresh one — keep working.  lfa_coll_ep_test_word is the
test knob: it makes the next word wait for a value the kernel never stores,
shortens the bound, or marks the direct queue failed.

The reference's error path here is a TODO (prov/coll/src/coll_coll.c:1243-1265);
its completion path is coll_coll.c:722-756.
"""
import errno
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FLOAT, SUM = 8, 2


@pytest.fixture(scope="module")
def coll():
    from libfabric_amd import coll as c
    c.lib()
    return c


def _drain(e, want_ok, timeout_s=10.0):
    """Poll until `want_ok` completions have come; return (ok contexts,
    error entries) in the order they were reaped."""
    ok, errs = [], []
    t0 = time.monotonic()
    while len(ok) < want_ok:
        n = e._L.lfa_cq_read(e.ep, e._ents, 16)
        if n > 0:
            ok += [e._ents[i].op_context for i in range(n)]
        elif n == -errno.EIO:
            ent = e.cq_readerr()
            assert ent is not None
            errs.append(ent)
        else:
            assert n == -errno.EAGAIN, n
        assert time.monotonic() - t0 < timeout_s, (ok, errs)
    return ok, errs


@pytest.mark.parametrize("direct", ["1", "0"])
def test_lost_word_fails_once_then_endpoint_continues(coll, direct, monkeypatch):
    """The second of four small allreduces waits for a word value its kernel
    never stores: it is reaped as exactly one ETIMEDOUT error entry after the
    bound (300 ms here), the other three complete normally in issue order
    with their results, and the next operations on the same and on a fresh
    endpoint succeed.  direct "1": the direct HSA queue's word; "0": the
    endpoint stream's word (LFA_DIRECT=0)."""
    monkeypatch.setenv("LFA_DIRECT", direct)
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        src = torch.arange(4 * 1024, dtype=torch.float32, device=DEV).view(4, 1024)
        out = torch.zeros_like(src)
        torch.cuda.synchronize()
        e.wait(e.allreduce(src[0], out[0], 1024, FLOAT, SUM))
        assert e.uses_direct() == (1 if direct == "1" else 0)
        out.zero_()
        torch.cuda.synchronize()
        words = e.word_ops()
        assert words == 1
        c0 = e.allreduce(src[0], out[0], 1024, FLOAT, SUM)
        e.test_word(drop_next=1, timeout_ms=300)
        c1 = e.allreduce(src[1], out[1], 1024, FLOAT, SUM)
        c2 = e.allreduce(src[2], out[2], 1024, FLOAT, SUM)
        c3 = e.allreduce(src[3], out[3], 1024, FLOAT, SUM)
        t0 = time.monotonic()
        ok, errs = _drain(e, 3)
        took = time.monotonic() - t0
        assert ok == [c0, c2, c3]
        assert len(errs) == 1, errs
        err, prov, ctx = errs[0]
        assert (err, prov, ctx) == (errno.ETIMEDOUT, errno.ETIMEDOUT, c1)
        assert 0.25 < took < 5.0, took
        # nothing more: the failure was reported once
        assert e.cq_readerr() is None
        assert e.cq_read() == []
        assert e.word_ops() == words + 3
        torch.cuda.synchronize()
        # the kernel itself ran: every result is its input
        assert torch.equal(out, src)
        # the endpoint goes on
        out.zero_()
        torch.cuda.synchronize()
        e.wait(e.allreduce(src[1], out[1], 1024, FLOAT, SUM))
        torch.cuda.synchronize()
        assert torch.equal(out[1], src[1])
    finally:
        e.close()
    e2 = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        y = torch.zeros(1024, device=DEV)
        torch.cuda.synchronize()
        e2.wait(e2.allreduce(src[2], y, 1024, FLOAT, SUM))
        torch.cuda.synchronize()
        assert torch.equal(y, src[2])
    finally:
        e2.close()


def test_failed_direct_queue_fails_its_word_with_eio(coll, monkeypatch):
    """An operation whose word the direct queue still owes when the queue is
    found failed (as the runtime's queue-error callback reports it) completes
    in error with EIO within the check interval — long before the bound —
    and later small operations take the HIP launch and complete."""
    monkeypatch.setenv("LFA_DIRECT", "1")
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        src = torch.arange(3 * 512, dtype=torch.float32, device=DEV).view(3, 512)
        out = torch.zeros_like(src)
        torch.cuda.synchronize()
        e.wait(e.allreduce(src[0], out[0], 512, FLOAT, SUM))
        assert e.uses_direct() == 1
        e.test_word(drop_next=1, timeout_ms=20000)
        c1 = e.allreduce(src[1], out[1], 512, FLOAT, SUM)
        e.test_word(fail_direct=True)
        assert e.uses_direct() == 2
        c2 = e.allreduce(src[2], out[2], 512, FLOAT, SUM)
        t0 = time.monotonic()
        ok, errs = _drain(e, 1)
        assert time.monotonic() - t0 < 2.0
        assert ok == [c2]
        assert [(x[0], x[2]) for x in errs] == [(errno.EIO, c1)]
        assert e.cq_readerr() is None
        torch.cuda.synchronize()
        assert torch.equal(out[2], src[2])
        y = torch.zeros(512, device=DEV)
        torch.cuda.synchronize()
        e.wait(e.allreduce(src[0], y, 512, FLOAT, SUM))
        torch.cuda.synchronize()
        assert torch.equal(y, src[0])
    finally:
        e.close()


def test_direct_queue_reopens_after_failed_one_is_released(coll, monkeypatch):
    """Once every endpoint holding a failed direct queue has closed, the next
    endpoint opens a fresh queue and uses it."""
    monkeypatch.setenv("LFA_DIRECT", "1")
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        x = torch.rand(256, device=DEV)
        y = torch.zeros_like(x)
        torch.cuda.synchronize()
        e.wait(e.allreduce(x, y, 256, FLOAT, SUM))
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        assert e.uses_direct() == 1
    finally:
        e.close()

