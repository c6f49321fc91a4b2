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



def test_device_domain_one_shot_reaps_through_the_word(coll):
    """exec_plan hands the one-shot launch's word
    value back to the submit, so a device domain's one-shot operations
    complete through the completion word, not an event.  The one-shot plan
    needs a group of 2..8 on device domains, i.e. two GPUs; lfa_coll_ep_test_solo
    sends a one-member group's small reducing collectives through the
    schedule of the endpoint's algorithm instead of the solo copy, so under
    LFA_ALGO_P2P they run the n = 1 one-shot kernel through the same
    run_device / exec_plan path.  Each of allreduce, reduce and reduce_scatter
    must be reaped through the word (lfa_coll_ep_word_ops), counted as a
    one-shot (lfa_mc_counters) and give its input back; a dropped word then
    fails that one operation once, with ETIMEDOUT."""
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        e.test_solo(0)
        e.set_algo(coll.ALGO_P2P)
        src = torch.arange(3 * 1024, dtype=torch.float32, device=DEV).view(3, 1024) - 7.5
        out = torch.zeros_like(src)
        torch.cuda.synchronize()
        w0, c0 = e.word_ops(), e.counters()
        e.wait(e.allreduce(src[0], out[0], 1024, FLOAT, SUM))
        e.wait(e.reduce(src[1], out[1], 1024, 0, FLOAT, SUM))
        e.wait(e.reduce_scatter(src[2], out[2], 1024, FLOAT, SUM))
        torch.cuda.synchronize()
        assert torch.equal(out, src)
        c1 = e.counters()
        assert c1["oneshot"] - c0["oneshot"] == 3, (c0, c1)
        assert e.word_ops() - w0 == 3, (w0, e.word_ops())
        # the word's error path on this form: one dropped word, one entry
        out.zero_()
        torch.cuda.synchronize()
        e.test_word(drop_next=1, timeout_ms=300)
        k0 = e.allreduce(src[0], out[0], 1024, FLOAT, SUM)
        k1 = e.allreduce(src[1], out[1], 1024, FLOAT, SUM)
        ok, errs = _drain(e, 1)
        assert ok == [k1]
        assert [(x[0], x[2]) for x in errs] == [(errno.ETIMEDOUT, k0)]
        assert e.cq_readerr() is None
        torch.cuda.synchronize()
        assert torch.equal(out[:2], src[:2])
        # a P2P operation reaped as failed leaves the group
        # refusing P2P operations (its kernel may still post into the
        # workspace), as after a timed-out wait: close and re-join
        with pytest.raises(coll.CollError) as ei:
            e.allreduce(src[2], out[2], 1024, FLOAT, SUM)
        assert ei.value.rc == -coll.EIO
    finally:
        e.close()


def test_word_bound_starts_at_the_head_of_the_queue(coll, monkeypatch):
    """a word operation's bound runs from when it reaches the head
    of the endpoint's in-order queue, not from its submit.  The endpoint's
    stream is held ~1 s by a spin kernel, a large allreduce (event-completed)
    is queued on it, then a small one completed by the word with a 300 ms
    bound.  The small one's kernel runs ~1 s after its submit, so a bound
    counted from the submit failed it with ETIMEDOUT; from the head it
    completes normally."""
    monkeypatch.setenv("LFA_DIRECT", "0")
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        big = torch.rand(8 << 20 >> 2, device=DEV)
        big_out = torch.zeros_like(big)
        x = torch.rand(1024, device=DEV)
        y = torch.zeros_like(x)
        torch.cuda.synchronize()
        e.wait(e.allreduce(x, y, 1024, FLOAT, SUM))     # warm: solo path, word
        # calibrate the spin kernel's cycles per second
        t0 = time.monotonic()
        torch.cuda._sleep(50_000_000)
        torch.cuda.synchronize()
        per_s = 50_000_000 / max(time.monotonic() - t0, 1e-4)
        e.test_word(timeout_ms=300)
        s = torch.cuda.ExternalStream(e.stream_handle, device=torch.device(DEV))
        w0 = e.word_ops()
        t0 = time.monotonic()
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(per_s * 1.0))
        k0 = e.allreduce(big, big_out, big.numel(), FLOAT, SUM)
        k1 = e.allreduce(x, y, 1024, FLOAT, SUM)
        ok, errs = _drain(e, 2, timeout_s=20.0)
        took = time.monotonic() - t0
        assert errs == [] and ok == [k0, k1], (ok, errs)
        assert took > 0.6, took     # the stream was held: the bound was tested
        assert e.word_ops() - w0 == 1
        torch.cuda.synchronize()
        assert torch.equal(big_out, big) and torch.equal(y, x)
    finally:
        e.close()


def test_lost_word_on_a_bounced_operation(coll, monkeypatch):
    """a one-member group's small operation on PAGEABLE host
    buffers runs through a pinned bounce block and completes through the
    word.  When that word is lost the operation fails once (ETIMEDOUT) and
    its block leaves the pool — its kernel may still run — so the operations
    after it, which take other blocks, keep their own results."""
    import numpy as np
    monkeypatch.setenv("LFA_DIRECT", "0")
    e = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        xs = [np.arange(1024, dtype=np.float32) + 1000 * k for k in range(12)]
        ys = [np.zeros(1024, np.float32) for _ in range(12)]
        e.wait(e.allreduce(xs[0], ys[0], 1024, FLOAT, SUM))
        assert np.array_equal(ys[0], xs[0])
        e.test_word(drop_next=1, timeout_ms=300)
        ctxs = [e.allreduce(xs[k], ys[k], 1024, FLOAT, SUM) for k in range(1, 12)]
        ok, errs = _drain(e, 10, timeout_s=10.0)
        assert ok == ctxs[1:]
        assert [(x[0], x[2]) for x in errs] == [(errno.ETIMEDOUT, ctxs[0])]
        for k in range(2, 12):
            assert np.array_equal(ys[k], xs[k]), k
        # the pool goes on with the blocks it has left
        for k in range(12):
            ys[k][:] = 0
            e.wait(e.allreduce(xs[k], ys[k], 1024, FLOAT, SUM))
            assert np.array_equal(ys[k], xs[k]), k
    finally:
        e.close()
