"""The off_lfa offload-collective provider (libfabric_amd/csrc/off_lfa.c)
driven the way rxm drives an offload provider, by examples/off_lfa_host.c:
a minimal owner (peer AV / CQ / EQ / endpoint) built from libfabric's public
headers, loading liboff_lfa-fi.so through fi_prov_ini.

* CPU: discovery (FI_PEER_TRANSFER required, "off_" prefix), fi_domain2 with
  FI_PEER, rxm's capability probe (rxm_domain.c:878-893) giving the mask
  BARRIER|BROADCAST|ALLREDUCE|ALLGATHER|REDUCE_SCATTER|REDUCE|SCATTER, peer
  AV/CQ/EQ/endpoint contexts, options, av_set algebra, errors before join.
* GPU: world join through the peer EQ, every collective on device and host
  buffers with completions delivered through the owner's peer CQ (carrying
  the owner's context), av_set address, subset join — with the progress
  thread and with owner-driven progress through the util_ep slot.

Both binaries are compiled in the build container against libfabric's public
headers; the GPU box runs the prebuilt files.
"""
import os
import subprocess

import pytest

from libfabric_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binaries():
    if build.have_fabric_headers():
        build.build_all()
    lib, exe = build.LIB_OFF, build.OFF_HOST
    if not (os.path.exists(lib) and os.path.exists(exe)):
        pytest.fail("off_lfa provider / host driver not built (needs libfabric's "
                    "public headers at build time)")
    return lib, exe


def _run(*args, timeout=300):
    lib, exe = _binaries()
    env = dict(os.environ)
    env.pop("OFF_LFA_PROGRESS", None)
    r = subprocess.run([exe, lib, *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.strip().splitlines()[-1]    # RCCL prints a banner first


def test_provider_exports():
    lib, _ = _binaries()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert "fi_prov_ini" in syms
    assert os.path.basename(lib) == "liboff_lfa-fi.so"     # lib<name>-fi.so


def _params(env_extra, knobs):
    lib, exe = _binaries()
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("FI_OFF_LFA_", "OFF_LFA_", "LFA_"))}
    env.update(env_extra)
    r = subprocess.run([exe, lib, "params", *knobs], capture_output=True, text=True,
                       timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    params = {}
    seen = {}
    for line in r.stdout.splitlines():
        if line.startswith("PARAM "):
            name, rest = line[6:].split(" ", 1)
            params[name] = rest
        elif line.startswith("LFA "):
            k, v = line[4:].split("=", 1)
            seen[k] = v
    return params, seen


def test_provider_parameters_through_fi_param():
    """the provider registers its knobs with libfabric's
    parameter system (fi_param_define at fi_prov_ini, src/var.c:188-231, as
    rxm does, prov/rxm/src/rxm_init.c:633-671) — FI_OFF_LFA_<NAME>, listed
    with type and help like `fi_info -e` — and what fi_param_get returns for
    the executor's and kernels' knobs reaches liblfa (lfa_param).  The raw
    names still work when FI_OFF_LFA_* is unset; FI_OFF_LFA_* wins over them.
    The owner stands in for libfabric's core (examples/fi_param_stub.h)."""
    want = {"FI_OFF_LFA_TRANSPORT", "FI_OFF_LFA_PROGRESS", "FI_OFF_LFA_ALGO",
            "FI_OFF_LFA_DEVICE", "FI_OFF_LFA_SIG_TIMEOUT_MS",
            "FI_OFF_LFA_ONESHOT_ALLREDUCE_BYTES", "FI_OFF_LFA_ONESHOT_RS_BYTES",
            "FI_OFF_LFA_GROUP_CHUNK_BYTES", "FI_OFF_LFA_WS_MEM", "FI_OFF_LFA_HOST_ZERO_COPY",
            "FI_OFF_LFA_DIRECT", "FI_OFF_LFA_STAGE_POOL_BYTES"}
    knobs = ["LFA_SIG_TIMEOUT_MS", "LFA_OS_AG_BYTES", "LFA_OS_RS_BYTES", "LFA_DIRECT",
             "LFA_WS_MEM", "LFA_HOST_SMALL_BYTES"]
    params, seen = _params({}, knobs)
    assert want <= set(params), sorted(want - set(params))
    assert params["FI_OFF_LFA_ONESHOT_ALLREDUCE_BYTES"].startswith("size_t:")
    assert "provisional" in params["FI_OFF_LFA_ONESHOT_ALLREDUCE_BYTES"]
    assert params["FI_OFF_LFA_DIRECT"].startswith("Boolean")
    assert all(v == "(unset)" for v in seen.values()), seen
    params, seen = _params({"FI_OFF_LFA_SIG_TIMEOUT_MS": "1234",
                            "FI_OFF_LFA_ONESHOT_RS_BYTES": "0x10000",
                            "FI_OFF_LFA_DIRECT": "off", "FI_OFF_LFA_WS_MEM": "fine",
                            "LFA_OS_AG_BYTES": "777",              # raw name, no FI_ one
                            "LFA_HOST_SMALL_BYTES": "5",
                            "FI_OFF_LFA_HOST_SMALL_BYTES": "4096"}, knobs)
    assert seen == {"LFA_SIG_TIMEOUT_MS": "1234", "LFA_OS_AG_BYTES": "777",
                    "LFA_OS_RS_BYTES": "65536", "LFA_DIRECT": "0", "LFA_WS_MEM": "fine",
                    "LFA_HOST_SMALL_BYTES": "4096"}, seen


@pytest.mark.parametrize("mode", [[], ["manual"]])
def test_host_driver_cpu(mode):
    assert _run("cpu", *mode).startswith("OK cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [[], ["manual"]])
def test_host_driver_gpu(mode):
    assert _run("gpu", *mode).startswith("OK gpu")


# ------------------------------------------ peer transport, N processes ----
# off_lfa had only ever run at world size 1, where every
# collective is an identity copy.  examples/off_lfa_peer forks N ranks, each
# an owner with its own tagged transport (socket pairs); the provider moves
# every transfer through it with FI_PEER_TRANSFER, as prov/coll does through
# rxm.  The outputs must be prov/coll's results bit for bit.

def _peer_run(n, tmp_path, mode):
    if build.have_fabric_headers():
        build.build_all()
    lib, exe = build.LIB_OFF, build.OFF_PEER
    if not (os.path.exists(lib) and os.path.exists(exe)):
        pytest.fail("off_lfa provider / peer driver not built")
    env = dict(os.environ)
    env.pop("OFF_LFA_PROGRESS", None)
    r = subprocess.run([exe, lib, str(n), str(tmp_path), *mode], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1].startswith("OK peer")


def _load(tmp_path, r, name, io, dt):
    import numpy as np
    return np.fromfile(tmp_path / f"r{r}_{name}_{io}.bin", dtype=dt)


@pytest.mark.parametrize("n,mode", [(2, []), (2, ["manual"]), (3, []), (3, ["manual"]),
                                    (4, []), (5, ["manual"])])
def test_peer_transport_collectives(tmp_path, n, mode):
    _peer_run(n, tmp_path, mode)
    _check_peer_outputs(tmp_path, n, ("", "_rd"))   # TREE and the reference's RD
    _check_ordered_sets(tmp_path, n)


def ref_union(dst, src):
    """coll_av_set_union, coll_av_set.c:35-69, loop for loop."""
    d = list(dst)
    for x in src:
        if x not in d:
            d.append(x)
    return d


def ref_intersect(dst, src):
    """coll_av_set_intersect, coll_av_set.c:71-96, loop for loop: walk src,
    search dst from the moving front `temp`, and on a match OVERWRITE
    dst[temp] with the match."""
    d = list(dst)
    temp = 0
    for x in src:
        for j in range(temp, len(d)):
            if d[j] == x:
                d[temp] = d[j]
                temp += 1
                break
    return d[:temp]


def ref_diff(dst, src):
    """coll_av_set_diff, coll_av_set.c:98-125, loop for loop: on a match at
    j, dst[--temp] = dst[j] (the found address is written over the last)."""
    d = list(dst)
    temp = len(d)
    for x in src:
        for j in range(temp):
            if d[j] == x:
                temp -= 1
                d[temp] = d[j]
                break
    return d[:temp]


def build_intersect(dst, src):
    """off_lfa's intersect: the reference's walk over src with a moving
    front, the front entry SWAPPED with the match instead of overwritten."""
    d = list(dst)
    front = 0
    for x in src:
        if x in d[front:]:
            j = d.index(x, front)
            d[front], d[j] = d[j], d[front]
            front += 1
    return d[:front]


def build_diff(dst, src):
    """off_lfa's diff: src's addresses removed in src's order, as remove
    does (the last address moves into the hole, coll_av_set.c:149-164)."""
    d = list(dst)
    for x in src:
        if x in d:
            i = d.index(x)
            d[i] = d[-1]
            d.pop()
    return d


class RefAvSet:
    """The address order prov/coll's av_set calls leave (coll_av_set.c):
    insert appends (:127-147), remove moves the last address into the hole
    (:149-164), intersect puts the common addresses in src's order
    (:71-96), diff removes src's addresses in src's order the way remove
    does — the reference's own diff overwrites the last address instead,
    and its intersect can lose a member; the build keeps every member and
    equals the reference wherever the reference does
    (test_av_set_algebra_against_reference_loops)."""

    def __init__(self, start, end, stride):
        self.a = list(range(start, end + 1, stride))

    @classmethod
    def of(cls, addrs):
        s = cls(0, -1, 1)
        for x in addrs:
            s.insert(x)
        return s

    def insert(self, x):
        assert x not in self.a
        self.a.append(x)

    def remove(self, x):
        i = self.a.index(x)
        self.a[i] = self.a[-1]
        self.a.pop()

    def intersect(self, other):
        self.a = build_intersect(self.a, other.a)

    def diff(self, other):
        self.a = build_diff(self.a, other.a)


def _ordered_subsets(universe, kmax):
    import itertools
    for k in range(kmax + 1):
        yield from itertools.permutations(universe, k)


def test_av_set_algebra_against_reference_loops():
    """the member order union / intersect / diff leave decides
    group ranks, so it is checked exhaustively — every ordered dst and src
    drawn from 5 addresses with up to 4 members (206 x 206 pairs per op) —
    through the provider (examples/off_lfa_host avset) against the
    reference's loops restated above:
      * union: identical to coll_av_set.c:35-69 everywhere;
      * intersect: identical to :71-96 wherever that loop keeps every common
        address; elsewhere every common address in src's order, of which the
        reference's result is a subsequence;
      * diff: identical to :98-125 wherever that loop drops exactly src's
        addresses; elsewhere the exact set difference in remove's order."""
    lib, exe = _binaries()
    sets = list(_ordered_subsets(range(5), 4))
    lines, want = [], []
    for d in sets:
        for s in sets:
            for op in "uid":
                lines.append(f"{op} {len(d)} {' '.join(map(str, d))} "
                             f"{len(s)} {' '.join(map(str, s))}")
                want.append((op, d, s))
    r = subprocess.run([exe, lib, "avset"], input="\n".join(lines) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.strip().splitlines()
    out = out[len(out) - len(want):]            # RCCL may print a banner first
    assert len(out) == len(want)
    seen = {"i_equal": 0, "i_ref_loses": 0, "d_equal": 0, "d_ref_wrong": 0}
    for (op, d, s), line in zip(want, out):
        rc, n, *got = map(int, line.split())
        assert rc == 0 and n == len(got), (op, d, s, line)
        common = [x for x in s if x in d]
        if op == "u":
            assert got == ref_union(d, s), (d, s, got)
        elif op == "i":
            ref = ref_intersect(d, s)
            assert got == build_intersect(d, s) == common, (d, s, got)
            if sorted(ref) == sorted(common):
                assert got == ref, (d, s, got, ref)
                seen["i_equal"] += 1
            else:
                it = iter(got)                  # ref is a subsequence of got
                assert all(x in it for x in ref), (d, s, got, ref)
                seen["i_ref_loses"] += 1
        else:
            ref = ref_diff(d, s)
            assert got == build_diff(d, s), (d, s, got)
            assert sorted(got) == sorted(set(d) - set(s)), (d, s, got)
            if sorted(ref) == sorted(set(d) - set(s)):
                assert got == ref, (d, s, got, ref)
                seen["d_equal"] += 1
            else:
                seen["d_ref_wrong"] += 1
    # the verdict's case, and both regimes of both loops were exercised
    assert ref_intersect([3, 2, 1, 0], [0, 1]) == build_intersect([3, 2, 1, 0], [0, 1]) == [0, 1]
    assert ref_intersect(list("abcd"), list("ca")) == ["c"]
    assert ref_diff(list("abcd"), ["b"]) == list("abc")
    assert all(v > 100 for v in seen.values()), seen


def _check_ordered_sets(tmp_path, n):
    """a group's rank r is the r-th address of the joined
    set, not the r-th smallest.  Set A = stride {0,2,..} + insert 1 (+3,
    -2 from N = 4), joined over the world; set B = all diff {0}, joined over
    its own address.  The allgather blocks come in set order, the float SUM
    allreduce equals the oracle fed in set order (its association order is
    the set's), and the reduce root / broadcast root are group ranks."""
    import numpy as np
    import oracle
    a = RefAvSet(0, n - 1, 2)
    if n > 1:
        a.insert(1)
    if n > 3:
        a.insert(3)
        a.remove(2)
    b = RefAvSet(0, n - 1, 1)
    b.diff(RefAvSet(0, 0, 1))
    # set C: the world in descending order intersected with [0, 2, 1]
    # (N >= 5), [0, 1] (N = 3, 4) or [0]: src's order, which the reference's
    # own loop keeps for these (at N = 2 it would drop a member of [0, 1])
    c_src = [0, 2, 1] if n >= 5 else ([0, 1] if n >= 3 else [0])
    c = RefAvSet.of(range(n - 1, -1, -1))
    c.intersect(RefAvSet.of(c_src))
    assert c.a == ref_intersect(list(range(n - 1, -1, -1)), c_src) == c_src
    for tag, ref in (("setA", a.a), ("setB", b.a), ("setC", c.a)):
        order = _load(tmp_path, 0, tag, "order", np.uint64).tolist()
        assert order == ref, (tag, order, ref)
        if not order:
            continue
        for r in order:
            ag = _load(tmp_path, r, tag + "_allgather", "out", np.int32).reshape(-1, 3)
            assert ag.tolist() == [[m, 10 * m, k] for k, m in enumerate(order)], (tag, r)
        ins = [_load(tmp_path, r, tag + "_sum_f32", "in", np.float32) for r in order]
        want = oracle.allreduce(2, 8, ins)[0]
        for r in order:
            got = _load(tmp_path, r, tag + "_sum_f32", "out", np.float32)
            assert got.tobytes() == want.tobytes(), (tag, r)
        if order != sorted(order) and len(order) > 2:
            # the association order is visible: ascending numbering differs
            srt = oracle.allreduce(2, 8, [ins[order.index(r)] for r in sorted(order)])[0]
            assert srt.tobytes() != want.tobytes()
        root = order[1] if len(order) > 1 else order[0]
        ins = [_load(tmp_path, r, tag + "_reduce_f64", "in", np.float64) for r in order]
        got = _load(tmp_path, root, tag + "_reduce_f64", "out", np.float64)
        assert got.tobytes() == oracle.allreduce(2, 9, ins)[0].tobytes(), tag


@pytest.mark.gpu
@pytest.mark.parametrize("n,mode", [(2, []), (3, ["manual"])])
def test_peer_transport_device_buffers(tmp_path, n, mode):
    """The provider with DEVICE buffers over the owner's transport, N
    processes on the one GPU: the reducing collectives (TREE, RD and P2P —
    the IPC workspace handshake and the system-scope kernel across the
    processes) run the gfx950 kernels, every transfer staged through host
    memory for an owner that moves host bytes only."""
    _peer_run(n, tmp_path, mode + ["device"])
    _check_peer_outputs(tmp_path, n, ("", "_rd", "_p2p"))


def _check_peer_outputs(tmp_path, n, sfxs):
    import numpy as np
    import oracle
    for name, op, dt, nd in (("sum_f32", 2, 8, np.float32), ("prod_f64", 3, 9, np.float64),
                             ("bxor_i64", 9, 6, np.int64)):
        ins = [_load(tmp_path, r, name, "in", nd) for r in range(n)]
        want = oracle.allreduce(op, dt, ins)[0]
        assert ins[0].size and not all(np.array_equal(ins[0], x) for x in ins[1:])
        for sfx in sfxs:
            for r in range(n):
                got = _load(tmp_path, r, name + sfx, "out", nd)
                assert got.tobytes() == want.tobytes(), (name + sfx, r)
    ins = [_load(tmp_path, r, "rs_f32", "in", np.float32) for r in range(n)]
    full = oracle.allreduce(2, 8, ins)[0]
    for r, (a, b) in enumerate(oracle.slice_bounds(full.size, n)):
        assert _load(tmp_path, r, "rs_f32", "out", np.float32).tobytes() == full[a:b].tobytes()
    ins = [_load(tmp_path, r, "reduce_f64", "in", np.float64) for r in range(n)]
    assert (_load(tmp_path, n - 1, "reduce_f64", "out", np.float64).tobytes() ==
            oracle.allreduce(2, 9, ins)[0].tobytes())
    members = sorted({0, n - 1})
    ins = [_load(tmp_path, r, "sub_f32", "in", np.float32) for r in members]
    want = oracle.allreduce(2, 8, ins)[0]
    for r in members:
        assert _load(tmp_path, r, "sub_f32", "out", np.float32).tobytes() == want.tobytes()


def test_peer_transport_latency_mode(tmp_path):
    """The config-1 shape (2 ranks, 4 KiB float SUM fi_allreduce) timed
    through the provider's peer transport: what bench.py reports as the
    host-path figure."""
    if build.have_fabric_headers():
        build.build_all()
    r = subprocess.run([build.OFF_PEER, build.LIB_OFF, "2", str(tmp_path), "manual",
                        "latency"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("LATENCY_US")]
    assert line and 0 < float(line[0].split()[1]) < 10_000


CORE_TESTS = ("join_test", "barrier_test", "sum_all_reduce_test",
              "sum_all_reduce_w_stride_test", "all_gather_test", "scatter_test",
              "broadcast_test")


@pytest.mark.parametrize("n,mode", [(1, "thread"), (2, "thread"), (3, "manual"),
                                    (4, "thread"), (4, "manual"), (5, "thread")])
def test_reference_multinode_suite(tmp_path, n, mode):
    """The reference's own collective suite, fabtests/multinode/src/
    core_coll.c:453-521, in its setup / run / pm_barrier / teardown cycle
    (:607-648): each test joins with coll_addr = fi_av_set_addr of its own
    set, on the set's ranks only — at N >= 4 the stride test's {1, 3, ..}
    forms its group while the other ranks call nothing (the members-only
    join, lfa_join_members) — and checks core_coll.c's expected values."""
    if build.have_fabric_headers():
        build.build_all()
    args = [build.OFF_PEER, build.LIB_OFF, str(n), str(tmp_path), "core"]
    if mode == "manual":
        args.append("manual")
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    passed = [x.split()[1] for x in r.stdout.splitlines() if x.startswith("CORE ")]
    assert tuple(passed) == CORE_TESTS, r.stdout + r.stderr


@pytest.mark.parametrize("n", [1, 2])
def test_join_event_waits_for_its_group(tmp_path, n):
    """A join that completes inside its lfa_join_* call (a one-member group)
    posts its event before off_lfa has registered the group.  The progress
    thread used to hand it to the owner's EQ with no fid, so the owner never
    matched it and the join timed out (seen once in the serial CPU suite:
    test_reference_multinode_suite[1-thread]).  LFA_TEST_JOIN_DELAY_US holds
    every join 20 ms between the call and the registration, so the thread
    always drains the event inside that window: the event must still reach
    the owner with its group's fid (olfa_post_join holds it until then)."""
    if build.have_fabric_headers():
        build.build_all()
    env = dict(os.environ, LFA_TEST_JOIN_DELAY_US="20000")
    r = subprocess.run([build.OFF_PEER, build.LIB_OFF, str(n), str(tmp_path), "core"],
                       capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    passed = [x.split()[1] for x in r.stdout.splitlines() if x.startswith("CORE ")]
    assert tuple(passed) == CORE_TESTS, r.stdout + r.stderr
