"""Host simulation of lfa_coll_plan schedules (test infrastructure).

Executes every rank's schedule — built by the C provider, liblfa_coll.so —
with numpy byte buffers: SEND/RECV groups matched FIFO per (src, dst) pair
exactly as the GPU loopback executor and RCCL groups match them; REDUCE via
the oracle's combine; TREE via the oracle's recursive-doubling allreduce of
the listed inputs (which IS the tree association order).
"""
import numpy as np

import oracle
from libfabric_amd import coll

SEND, RECV, GEND, REDUCE, TREE, COPY, ALLTOALL, ALLGATHER, BARRIER, TREE_PUT, ONESHOT = \
    range(11)
SYM_IN, SYM_OUT = 3, 4


def lower(steps, r, n, refs=None, esz=None):
    """ALLTOALL / ALLGATHER -> grouped SEND/RECV + COPY, and ONESHOT -> the
    COPY / BARRIER / TREE / BARRIER it is defined by (as lfa_coll_plan.c's
    lower_plan does for its loopback executor); ONESHOT's tree inputs are
    appended to `refs`."""
    out = []
    for s in steps:
        if s["type"] == ONESHOT:
            # this rank's part: the whole vector (peer -1), block r (-2), or
            # the whole vector on the root `peer` only
            moff, mlen = 0, s["count"]
            if s["peer"] == -2:
                moff, mlen = coll.block(s["count"], n, r)
            elif s["peer"] >= 0 and s["peer"] != r:
                mlen = 0
            out.append({"type": COPY, "count": s["count"] * esz, "src": s["src"],
                        "dst": (SYM_IN, 0, r), "peer": 0})
            out.append({"type": BARRIER, "count": 0, "src": (0, 0), "dst": (0, 0), "peer": 0})
            if mlen:
                first = len(refs)
                sb, so = s["src"]
                refs.extend((sb, so + moff * esz) if k == r else (SYM_IN, moff * esz, k)
                            for k in range(s["nsrc"]))
                out.append({"type": TREE, "count": mlen, "dst": s["dst"], "first": first,
                            "nsrc": s["nsrc"], "src": (0, 0), "peer": 0})
            out.append({"type": BARRIER, "count": 0, "src": (0, 0), "dst": (0, 0), "peer": 0})
            continue
        if s["type"] not in (ALLTOALL, ALLGATHER):
            out.append(s)
            continue
        a2a = s["type"] == ALLTOALL
        c = s["count"]
        for k in range(1, n):
            to, frm = (r + k) % n, (r - k) % n
            sb, so = s["src"]
            out.append({"type": SEND, "peer": to, "count": c,
                        "src": (sb, so + (to * c if a2a else 0)), "dst": (0, 0)})
            db, do = s["dst"]
            out.append({"type": RECV, "peer": frm, "count": c, "src": (0, 0),
                        "dst": (db, do + frm * c)})
        if n > 1:
            out.append({"type": GEND, "peer": 0, "count": 0, "src": (0, 0), "dst": (0, 0)})
        sb, so = s["src"]
        db, do = s["dst"]
        src = (sb, so + (r * c if a2a else 0))
        dst = (db, do + r * c)
        if src != dst:
            out.append({"type": COPY, "count": c, "src": src, "dst": dst, "peer": 0})
    return out


def _view(bufs, ref, nbytes):
    """ref = (buf, off) into this rank's buffers, or (SYM_IN|SYM_OUT, off,
    owner) into group rank `owner`'s symmetric workspace (bufs["sym"])."""
    if len(ref) == 3:
        b, off, k = ref
        sym, region = bufs["sym"]
        if b == SYM_OUT:
            off += region
        return sym[k][off:off + nbytes]
    b, off = ref
    return bufs[b][off:off + nbytes]


def run(coll_op, algo, n, root, dt, op, count, sends, results):
    """sends/results: per-rank uint8 arrays (results modified in place)."""
    esz = oracle.datatype_size(dt)
    nd = oracle.DT_NP[dt]
    plans = [coll.plan(coll_op, algo, r, n, root, count, esz) for r in range(n)]
    for r in range(n):
        plans[r].refs = list(plans[r].refs)
        plans[r].steps = lower(plans[r].steps, r, n, plans[r].refs, esz)
    region = (count * esz + 255) // 256 * 256
    # symmetric workspaces (LFA_ALGO_P2P), poisoned so stale reads show
    sym = [np.full(2 * region, 0xA5, np.uint8) for _ in range(n)]
    bufs = []
    for r in range(n):
        tmp = np.zeros(plans[r].tmp_bytes, np.uint8)
        send = sends[r] if coll_op != 1 else results[r]   # broadcast: in/out
        bufs.append({0: send, 1: results[r], 2: tmp, "sym": (sym, region)})
    pc = [0] * n
    arrived = [0] * n          # barriers reached
    waiting = [False] * n
    box = {}
    posted = [set() for _ in range(n)]
    while True:
        progressed, done = False, True
        for r in range(n):
            st = plans[r].steps
            while pc[r] < len(st):
                s = st[pc[r]]
                if s["type"] == BARRIER:
                    if not waiting[r]:
                        waiting[r] = True
                        arrived[r] += 1
                        progressed = True
                    if min(arrived) < arrived[r]:
                        break
                    waiting[r] = False
                    pc[r] += 1
                    progressed = True
                    continue
                if s["type"] not in (SEND, RECV, GEND):
                    if s["type"] == REDUCE:
                        d = _view(bufs[r], s["dst"], s["count"] * esz).view(nd)
                        x = _view(bufs[r], s["src"], s["count"] * esz).view(nd).copy()
                        oracle.write(op, dt, d, x)
                    elif s["type"] == COPY:
                        src = _view(bufs[r], s["src"], s["count"]).copy()
                        _view(bufs[r], s["dst"], s["count"])[:] = src
                    else:
                        nb = s["count"] * esz
                        refs = plans[r].refs
                        ins = [_view(bufs[r], refs[s["first"] + k], nb).view(nd).copy()
                               for k in range(s["nsrc"])]
                        out = oracle.allreduce(op, dt, ins)[0].view(np.uint8)
                        dsts = [s["dst"]]
                        if s["type"] == TREE_PUT:
                            base = s["first"] + s["nsrc"]
                            dsts += [refs[base + j] for j in range(s["peer"])]
                        for d in dsts:
                            _view(bufs[r], d, nb)[:] = out
                    pc[r] += 1
                    progressed = True
                    continue
                end = pc[r]
                while end < len(st) and st[end]["type"] != GEND:
                    end += 1
                for i in range(pc[r], end):
                    x = st[i]
                    if x["type"] == SEND and i not in posted[r]:
                        box.setdefault((r, x["peer"]), []).append(
                            _view(bufs[r], x["src"], x["count"]).copy())
                        posted[r].add(i)
                        progressed = True
                need = {}
                for i in range(pc[r], end):
                    if st[i]["type"] == RECV:
                        need[st[i]["peer"]] = need.get(st[i]["peer"], 0) + 1
                if any(len(box.get((p, r), [])) < k for p, k in need.items()):
                    break
                for i in range(pc[r], end):
                    x = st[i]
                    if x["type"] == RECV:
                        m = box[(x["peer"], r)].pop(0)
                        assert m.nbytes == x["count"]
                        _view(bufs[r], x["dst"], x["count"])[:] = m
                pc[r] = min(end + 1, len(st))
                posted[r].clear()
                progressed = True
            if pc[r] < len(st):
                done = False
        if done:
            break
        if not progressed:
            raise RuntimeError("schedule deadlock")
    assert all(not v for v in box.values()), "unmatched sends"
    return results
