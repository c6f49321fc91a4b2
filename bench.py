#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X.

metric : device-resident GiB/s, float32 FI_SUM reduce, 256 MiB buffers
step   : one pass of the hot path — ofi_atomic_write_handler(FI_SUM, FI_FLOAT,
         dst, src, 67,108,864) (prov/coll/src/coll_coll.c:763) — over one
         256 MiB (dst, src) pair already resident in HBM, launched through the
         C ABI (lfa_atomic_write_async, liblfa.so).
value  : whole-job traffic rate, 3·S bytes per step (read dst, read src,
         write dst) × steps ÷ the max-over-ranks wall time, in GiB/s.
         The buffer rate S/t is reported beside it.
N > 1  : one process per GPU.  The headline is WEAK-scaled (the tier's rule
         for a path that partitions: independent objects sharded across ranks
         with no data-path collective): every rank combines its own 256 MiB
         pair per step, so a step is N independent 256 MiB combines and value =
         3·S·N·steps ÷ the max-over-ranks wall time.  The strong-scaled figure
         (one 256 MiB pair split into N contiguous 4 KiB-aligned shards, GPU g
         combining shard g — SURVEY §8(e), BASELINE configs[3]'s "8 GPUs each
         combine S/8") sits beside it in extras.  `python bench.py --gpus N`
         without RANK in the environment starts the N rank processes itself
         (before any GPU call); under torch.distributed.run it is one of them.
         A world size that differs from --gpus is an error (exit 2).  The N > 1
         provider extras (allreduce / reduce_scatter over RCCL, xGMI P2P) run as
         a child job of the ranks (run_isolated), so a fault there cannot lose
         the line.

Extra objects on the JSON line:
  roofline      dominant kernel (combine_lds<SUM,float>): algorithmic bytes per
                launch (3·S) ÷ its average duration from HIP events on the
                launch stream; peak 8.0 TB/s (MI355X HBM3E spec); ``traffic``
                from the committed rocprofv3 PMC pass (profiles/) when present.
  cpu_baseline  rank 0, N=1 only: the reference combine on 1 pinned host core,
                same shape (256 MiB float SUM), median of a bounded sample;
                beside it configs[2] (int64 BOR/MIN 64 MiB), configs[0] (2-rank
                4 KiB allreduce through the provider's host path) and
                configs[4]'s per-bucket double PROD combine.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu]
       python bench.py --tune      # kernel-variant sweep (dev tool)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

S_BYTES = 256 * 1024 * 1024            # BASELINE config 2: 256 MiB buffers
COUNT = S_BYTES // 4                   # 67,108,864 float
BUFFER_SETS = 4                        # rotate: 2 GiB of inputs >> 256 MiB MALL
PEAK_GBPS = 8000.0                     # MI355X HBM3E peak (MI355X_MICROARCH.md)
ACCESS_MIX_CEILING_GBPS = 6756.0       # 2 reads + 1 write, tools/probe_hbm.py
FI_SUM, FI_FLOAT = 2, 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, cmd: list[str], timeout_s: float | None = None) -> int:
    """Start `cmd` as N rank processes (one per GPU) with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as torch.distributed.run
    would, and return the worst exit code.  Runs before anything in this
    process touches the GPU (children are started with Popen, never exec).
    If a rank fails, the others are stopped by PID so none is left waiting in
    a collective."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen(cmd, env=env))
    t0 = time.time()
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or code
                for q in pending:       # a failed rank: stop its peers
                    q.kill()
        if timeout_s is not None and time.time() - t0 > timeout_s:
            for q in pending:
                q.kill()
            rc = rc or 124
            break
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


_CHILD = None                          # the running isolated child (watchdog kills it)
_ISO_SEQ = [0]


def run_isolated(cmd: list[str], rank: int, world: int, budget_s: float,
                 env_extra: dict | None = None) -> dict:
    """Run `cmd` as this rank's member of a NEW N-rank job (fresh rendezvous
    port, same RANK / LOCAL_RANK / WORLD_SIZE) in a child process, and return
    rank 0's last JSON line from it.

    The N > 1 provider extras run this way: they are the first run of the
    RCCL / xGMI / IPC transports on N GPUs, and a GPU fault or crash there
    aborts its process — here the child, not the rank that holds the headline,
    so the one JSON line is still printed.  The ranks coordinate through the
    job's store only (no GPU collective): rank 0 publishes the port, and a
    rank whose child fails or overruns posts it, so every rank stops its child
    (by PID) instead of leaving it waiting in a collective.  Each rank returns
    only after its own child has exited."""
    import subprocess
    import tempfile
    global _CHILD
    store = dist.distributed_c10d._get_default_store()
    _ISO_SEQ[0] += 1
    key = f"lfa_iso{_ISO_SEQ[0]}"
    if rank == 0:
        store.set(key + "_port", str(_free_port()))
    port = store.get(key + "_port").decode()
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=port, LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(env_extra or {})
    status = "ok"
    with tempfile.TemporaryFile("w+") as out:
        p = _CHILD = subprocess.Popen(cmd, env=env, stdout=out)
        t_start = time.time()
        deadline = t_start + budget_s
        beat = t_start
        while True:
            if rank == 0 and time.time() - beat > 20.0:
                # a heartbeat on stderr: a runner that takes a silent job for
                # a hung one sees the extras are still going
                beat = time.time()
                log(f"bench.py: provider extras running, {beat - t_start:.0f} s")
            rc = p.poll()
            if rc is not None:
                if rc != 0:
                    status = f"rank {rank}: child exited with code {rc}"
                    store.set(key + "_fail", status)
                break
            if store.check([key + "_fail"]):
                status = "stopped: " + store.get(key + "_fail").decode()
                p.kill()
                p.wait()
                break
            if time.time() > deadline:
                status = f"rank {rank}: child overran {budget_s:.0f} s"
                store.set(key + "_fail", status)
                p.kill()
                p.wait()
                break
            time.sleep(0.1)
        _CHILD = None
        # rank 0 hosts the store: it leaves last, after every peer's final
        # store call (this add) has been answered, so no peer still polling
        # the fail key sees the store torn down under it
        n_done = store.add(key + "_done", 1)
        while rank == 0 and n_done < world:
            time.sleep(0.05)
            n_done = store.add(key + "_done", 0)
        out.seek(0)
        lines = [x for x in out.read().splitlines() if x.startswith("{")]
    res = {}
    if lines:
        try:
            res = json.loads(lines[-1])
        except ValueError:
            status += "; last line unparsable"
    if status != "ok":
        res["isolated_status"] = status
    return res


def check_world(expected: int, world: int) -> None:
    if world != expected:
        log(f"bench.py: --gpus {expected} but the job has WORLD_SIZE={world}")
        sys.exit(2)


# LFA_BENCH_REHEARSE=1: a dry run of the N-rank flow on fewer GPUs than ranks
# (ranks share devices round-robin, torch.distributed over gloo).  RCCL
# refuses two ranks on one GPU, so the provider's collectives report errors
# there; the launch, the sharded headline, the timing and the JSON line are
# what it exercises.  Never used for a reported number.
REHEARSE = os.environ.get("LFA_BENCH_REHEARSE") == "1"


def init_dist(n_gpus: int):
    if n_gpus > 1 or "RANK" in os.environ:
        rank = int(os.environ.get("RANK", 0))
        world = int(os.environ.get("WORLD_SIZE", 1))
        local = int(os.environ.get("LOCAL_RANK", rank))
        check_world(n_gpus, world)
        if REHEARSE:
            local %= torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
        check_world(n_gpus, dist.get_world_size())
        return rank, world, local
    torch.cuda.set_device(0)
    return 0, 1, 0


def shard_of(count: int, world: int, rank: int, align_elems: int = 1024):
    """Rank `rank`'s contiguous shard [off, off + len) of a `count`-element
    buffer split over `world` GPUs, shard starts 4 KiB-aligned (1024 float)."""
    per = -(-count // world)
    per = -(-per // align_elems) * align_elems
    off = min(rank * per, count)
    return off, min(per, count - off)


def barrier(world: int) -> None:
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if REHEARSE else "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


ROTATE_BYTES = 1 << 30                 # >= 1 GiB of operands per GPU rotated


def n_sets(count: int) -> int:
    """Buffer pairs to rotate so the 256 MiB MALL cannot serve repeats."""
    return max(BUFFER_SETS, -(-ROTATE_BYTES // max(1, 2 * 4 * count)))


def make_buffers(dev, seed: int, count: int = COUNT, nsets: int | None = None):
    g = torch.Generator(device=dev).manual_seed(seed)
    sets = []
    for _ in range(nsets or n_sets(count)):
        src = torch.rand(count, device=dev, generator=g) * 2 - 1
        dst = torch.rand(count, device=dev, generator=g) * 2 - 1
        sets.append((dst, src))
    return sets


def prewarm(step, min_s: float) -> int:
    """Untimed launches of the step until `min_s` seconds have passed, so the
    timed region starts at steady-state GPU clocks (a short run otherwise
    measures the ramp: 129 us/launch after 10 launches vs 121 us at steady
    state).  Returns the number of launches."""
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min_s:
        for _ in range(20):
            step(n)
            n += 1
        torch.cuda.synchronize()
    return n


def read_traffic():
    """Per-launch HBM bytes of the headline kernel from the committed PMC pass."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), d.get("source")


def read_traffic_shard(shard_bytes: int):
    """Per-launch HBM bytes of the same kernel at the shard's operand size,
    from the committed PMC passes over `--only-extra sizes`
    (profiles/r03_pmc_traffic_sizes.json, tools/pmc_sizes.py)."""
    path = os.path.join(ROOT, "profiles", "r03_pmc_traffic_sizes.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    for row in d.get("by_operand_mib", {}).values():
        if row["operand_bytes"] == shard_bytes:
            return row["hbm_bytes_per_launch"], (
                f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of the same kernel at a "
                f"{shard_bytes >> 20} MiB operand on one GPU ({path[len(ROOT) + 1:]})")
    return None, None


def cpu_baseline(sample_reps: int = 5):
    """The reference combine timed on ONE pinned host core (rank 0, N=1).

    Primary: our restatement of the shipping HAVE_BUILTIN_MM_ATOMICS handler
    (per-element seq_cst CAS, util_atomic.c:266-289) — kind "port".  Beside
    it: the open-coded variant (util_atomic.c:119-153) and the reference's own
    fabtests restatement compiled from /root/reference (oracle/_ref).
    """
    import numpy as np
    import oracle

    rng = np.random.default_rng(1)
    src = rng.uniform(-1, 1, COUNT).astype(np.float32)
    dst0 = rng.uniform(-1, 1, COUNT).astype(np.float32)
    dst = dst0.copy()
    try:
        prev = os.sched_getaffinity(0)
        core = sorted(prev)[-1]
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        prev, core = None, None

    def timeit(fn):
        ts = []
        for _ in range(sample_reps):
            dst[:] = dst0
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    res = {}
    try:
        res["cas"] = timeit(lambda: oracle.write(FI_SUM, FI_FLOAT, dst, src, oracle.CAS))
        res["plain"] = timeit(lambda: oracle.write(FI_SUM, FI_FLOAT, dst, src, oracle.PLAIN))
        if oracle.ref_available():
            res["ref"] = timeit(lambda: oracle.ref_write(FI_SUM, FI_FLOAT, dst, src))
    finally:
        if prev is not None:
            os.sched_setaffinity(0, prev)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass

    def gib(t):
        return round(3 * S_BYTES / t / 2**30, 3)

    out = {
        "value": gib(res["cas"]), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": (f"256 MiB float FI_SUM combine (67,108,864 elements), median of "
                   f"{sample_reps} runs, 1 pinned core (cpu {core}) of {os.cpu_count()} "
                   f"({cpu}); shipping CAS handler restated in oracle/"),
        "ms_per_combine": round(res["cas"] * 1e3, 2),
        "plain_loop": {"value": gib(res["plain"]), "kind": "port",
                       "ms_per_combine": round(res["plain"] * 1e3, 2)},
    }
    if "ref" in res:
        out["reference_fabtests"] = {
            "value": gib(res["ref"]), "kind": "reference",
            "ms_per_combine": round(res["ref"] * 1e3, 2),
            "what": "fabtests/common/ofi_atomic.c plain loop, built from /root/reference"}
    return out


def cpu_config1_peer(timeout_s: float = 90.0):
    """BASELINE configs[0]'s shape on the host: a 2-rank 4 KiB float FI_SUM
    fi_allreduce through the off_lfa provider's PEER transport (the
    transfers ride on an rxm-like owner's tagged messaging over AF_UNIX
    sockets, the reductions in liblfa's host combine) — the build's own
    prov/coll-shaped host path; examples/off_lfa_peer, median of 1000 after
    100 warm-up, owner-driven progress."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "examples", "off_lfa_peer")
    lib = os.path.join(ROOT, "libfabric_amd", "liboff_lfa-fi.so")
    if not (os.path.exists(exe) and os.path.exists(lib)):
        return {"error": "examples/off_lfa_peer not built"}
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for mode in ("manual", "thread"):
            args = [exe, lib, "2", td, "latency"] + (["manual"] if mode == "manual" else [])
            # host buffers only: OFF_LFA_DEVICE=-1 keeps the GPU out of it
            r = subprocess.run(args, capture_output=True, text=True, timeout=timeout_s,
                               env=dict(os.environ, OFF_LFA_DEVICE="-1"))
            line = [x for x in r.stdout.splitlines() if x.startswith("LATENCY_US")]
            if r.returncode or not line:
                out[mode] = {"error": (r.stdout + r.stderr)[-200:]}
                continue
            med, p10, p90 = (float(v) for v in line[0].split()[1:4])
            out[mode] = {"us_median": med, "us_p10": p10, "us_p90": p90}
    out.update({"kind": "port", "cores": 2,
                "what": "2 processes, fi_allreduce 1024 float FI_SUM through liboff_lfa-fi.so's "
                        "peer transport (owner tagged messages over AF_UNIX socket pairs, "
                        "host combine); 'manual' = owner-driven progress, 'thread' = the "
                        "provider's FI_PROGRESS_AUTO thread"})
    return out


def splitmix64(seed: int, n: int):
    """SURVEY §8(d) config 3 data: full-range splitmix64 stream."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + np.uint64(seed))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z.view(np.int64)


def config3_data(seed: int, n: int):
    """splitmix64 int64 lanes with ~1 % forced to INT64_MIN/MAX/0/-1."""
    import numpy as np
    x = splitmix64(seed, n)
    rng = np.random.default_rng(seed)
    idx = rng.choice(n, n // 100, replace=False)
    x[idx] = rng.choice(np.array([np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1],
                                 dtype=np.int64), idx.size)
    return x


def cpu_baseline_config3(sample_reps: int = 5):
    """BASELINE configs[2] on ONE pinned host core: int64 FI_BOR (`lock or`,
    util_atomic.c:78-79) and FI_MIN (CAS-if-smaller, util_atomic.c:71,
    291-316), 64 MiB, the SURVEY §8(d) data distribution; shipping atomic
    handler restated in oracle/ ("port") and the plain loop beside it.
    GiB/s of traffic (3 x 64 MiB per combine)."""
    import oracle
    n = 64 * 1024 * 1024 // 8
    src, dst0 = config3_data(4, n), config3_data(3, n)
    dst = dst0.copy()
    try:
        prev = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(prev)[-1]})
    except (AttributeError, OSError):
        prev = None
    out = {}
    try:
        for name, op in (("bor", 6), ("min", 0)):
            row = {}
            for var, vname in ((oracle.CAS, "atomic"), (oracle.PLAIN, "plain")):
                ts = []
                for _ in range(sample_reps):
                    dst[:] = dst0
                    t0 = time.perf_counter()
                    oracle.write(op, 6, dst, src, var)
                    ts.append(time.perf_counter() - t0)
                t = statistics.median(ts)
                row[vname] = {"ms": round(t * 1e3, 2),
                              "gib_s": round(3 * n * 8 / t / 2**30, 3)}
            out[name] = row
    finally:
        if prev is not None:
            os.sched_setaffinity(0, prev)
    out.update({"cores": 1, "kind": "port",
                "sample": f"64 MiB int64 (8,388,608 lanes) splitmix64 seeds 3/4 with 1 % "
                          f"INT64_MIN/MAX/0/-1 lanes, median of {sample_reps}, 1 pinned core"})
    return out


def cpu_baseline_config5(budget_s: float = 1.0):
    """BASELINE configs[4]'s CPU column: the reference's per-bucket combine,
    double FI_PROD (CAS loop, util_atomic.c:266-289 via the PROD row
    :898/:913), one pinned core, for each bucket of the 4 KiB .. 256 MiB
    sweep.  prov/coll has no reduce_scatter (coll_ep.c:75-76); an allreduce
    of the bucket costs log2(N) such combines per rank (coll_coll.c:409-430),
    so the N-rank compute is this figure x log2(N).  Data uniform[0.9,1.1)
    (SURVEY §8(d)); median over repetitions bounded by `budget_s` per size."""
    import numpy as np
    import oracle
    try:
        prev = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(prev)[-1]})
    except (AttributeError, OSError):
        prev = None
    rng = np.random.default_rng(200)
    top = 256 * 1024 * 1024 // 8
    src_all = rng.uniform(0.9, 1.1, top)
    dst_all = rng.uniform(0.9, 1.1, top)
    sweep = {}
    try:
        for nbytes in [4096 * 4 ** k for k in range(9)]:
            n = nbytes // 8
            src, dst0 = src_all[:n], dst_all[:n]
            dst = dst0.copy()
            ts, t_end = [], time.perf_counter() + budget_s
            while len(ts) < 3 or (len(ts) < 200 and time.perf_counter() < t_end):
                dst[:] = dst0
                t0 = time.perf_counter()
                oracle.write(3, 9, dst, src, oracle.CAS)   # FI_PROD, FI_DOUBLE
                ts.append(time.perf_counter() - t0)
            t = statistics.median(ts)
            sweep[str(nbytes)] = {"us": round(t * 1e6, 1),
                                  "gib_s": round(3 * nbytes / t / 2**30, 3)}
    finally:
        if prev is not None:
            os.sched_setaffinity(0, prev)
    return {"per_bucket_combine": sweep, "cores": 1, "kind": "port",
            "sample": "double FI_PROD CAS combine of one bucket (dst *= src), 4 KiB .. "
                      "256 MiB x4 steps, uniform[0.9,1.1), 1 pinned core; an N-rank "
                      "allreduce of the bucket is log2(N) of these per rank"}



# ------------------------------------------------------------------ extras --

def _kernel_events(fn, reps, stream):
    """Mean per-launch duration (ms) of fn(i): one HIP event pair on `stream`
    around `reps` back-to-back launches, as for the headline (an event pair
    per launch adds its own gap: +2.5 us on a 31 us kernel)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for i in range(reps):
        fn(i)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def _two_streams_s(launch, k: int = 100) -> float:
    """Per-launch wall time of K independent launches round-robin over two
    streams (buckets in flight, as a provider progressing several operations
    at once), between device synchronizes; median of 5.  One stream makes
    every launch pay its own ramp and drain; two let the next
    launch's waves fill the CUs the previous one's are leaving
    (tools/probe_streams.py: a win up to 64 MiB per operand, a loss at
    256 MiB, where two concurrent streams contend)."""
    ss = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i in range(10):
        launch(i, ss[i % 2])
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            launch(i, ss[i % 2])
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / k)
    return statistics.median(ts)


def extra_two_streams(dev, counts) -> dict:
    """The headline combine (float SUM) at the given operand counts, K
    independent launches over two streams vs one (beside the single-stream
    headline, never instead of it)."""
    from libfabric_amd import atomic
    out = {}
    for count in counts:
        sets = make_buffers(dev, 3000, count)
        nsets = len(sets)

        def launch(i, st):
            d, s_ = sets[i % nsets]
            atomic.write(FI_SUM, FI_FLOAT, d, s_, count, st)
        one = torch.cuda.Stream()
        prewarm(lambda i: launch(i, one), 0.1)
        t1 = _two_streams_s(lambda i, st: launch(i, one))
        t2 = _two_streams_s(launch)
        nb = 3 * count * 4
        out[f"{count * 4 >> 20}mib"] = {
            "one_stream_us": round(t1 * 1e6, 2), "two_streams_us": round(t2 * 1e6, 2),
            "one_stream_frac": round(nb / t1 / 1e9 / PEAK_GBPS, 4),
            "two_streams_frac": round(nb / t2 / 1e9 / PEAK_GBPS, 4)}
        del sets
        torch.cuda.empty_cache()
    return out


def extra_config3(dev, stream):
    """BASELINE configs[2]: int64 FI_BOR and FI_MIN, 64 MiB, bit-exact path.
    8 rotating buffer pairs (1 GiB) so the 256 MiB MALL cannot serve reruns."""
    from libfabric_amd import atomic
    n = 64 * 1024 * 1024 // 8
    g = torch.Generator(device=dev).manual_seed(3)
    sets = []
    for _ in range(8):
        a = torch.randint(-2**63, 2**63 - 1, (n,), device=dev, dtype=torch.int64, generator=g)
        b = torch.randint(-2**63, 2**63 - 1, (n,), device=dev, dtype=torch.int64, generator=g)
        sets.append((a, b))
    out = {}
    for name, op in (("bor", 6), ("min", 0)):
        def fn(i, op=op):
            d, s = sets[i % 8]
            atomic.write(op, 6, d, s, n, stream)
        prewarm(fn, 0.1)            # steady clocks, as for the headline
        torch.cuda.synchronize()
        ms = _kernel_events(fn, 100, stream)
        gbps = 3 * n * 8 / (ms * 1e-3) / 1e9
        out[name] = {"kernel_us": round(ms * 1e3, 2), "achieved_gbs": round(gbps, 1),
                     "frac": round(gbps / PEAK_GBPS, 4),
                     "gib_s": round(3 * n * 8 / (ms * 1e-3) / 2**30, 1)}
        # the same independent buckets two streams at a time
        t2 = _two_streams_s(lambda i, st, op=op: atomic.write(op, 6, sets[i % 8][0],
                                                                sets[i % 8][1], n, st))
        out[name]["two_streams_us"] = round(t2 * 1e6, 2)
        out[name]["two_streams_frac"] = round(3 * n * 8 / t2 / 1e9 / PEAK_GBPS, 4)
    return out


def extra_fetch_tables(dev, stream):
    """§8(f) row 4 on the bench line: the fetch table (float SUM readwrite:
    res = dst, dst += src; 4·S bytes) and the compare table (float CSWAP:
    res = dst, dst = src where cmp == dst; 5·S bytes) at 256 MiB per operand,
    two rotating sets (2 GiB) so the MALL cannot serve repeats."""
    from libfabric_amd import atomic
    g = torch.Generator(device=dev).manual_seed(5)
    sets = [[torch.rand(COUNT, device=dev, generator=g) for _ in range(4)] for _ in range(2)]
    out = {}
    for name, nb, fn in (
            ("readwrite_float_sum", 4 * S_BYTES,
             lambda i: atomic.readwrite(FI_SUM, FI_FLOAT, sets[i % 2][0], sets[i % 2][1],
                                        sets[i % 2][2], COUNT, stream)),
            ("swap_float_cswap", 5 * S_BYTES,
             lambda i: atomic.swap(12, FI_FLOAT, sets[i % 2][0], sets[i % 2][1],
                                   sets[i % 2][3], sets[i % 2][2], COUNT, stream))):
        # steady clocks first, as for the headline (round 5 timed 20 launches
        # after 4 and measured the clock ramp with them: 170.2 / 219.3 us
        # against 163-168 / 210 us after a prewarm)
        prewarm(fn, 0.1)
        ms = _kernel_events(fn, 40, stream)
        gbps = nb / (ms * 1e-3) / 1e9
        out[name] = {"kernel_us": round(ms * 1e3, 1), "achieved_gbs": round(gbps, 1),
                     "frac": round(gbps / PEAK_GBPS, 4)}
    del sets
    torch.cuda.empty_cache()
    return out


def extra_sizes(dev, stream, reps: int = 100, prewarm_s: float = 0.1):
    """The product float SUM combine vs size per operand (the shard sizes of
    the strong-scaled extra: 256 MiB / N): average launch duration from an
    event pair around 100 back-to-back launches over >= 1 GiB of rotated
    operands, after a clock prewarm."""
    from libfabric_amd import atomic
    out = {}
    for mib in (8, 16, 32, 64, 128, 256):
        n = mib * 1024 * 1024 // 4
        sets = make_buffers(dev, 5, n)

        def fn(i, sets=sets, n=n):
            d, s = sets[i % len(sets)]
            atomic.write(FI_SUM, FI_FLOAT, d, s, n, stream)
        if prewarm_s > 0:
            prewarm(fn, prewarm_s)
        ms = _kernel_events(fn, reps, stream)
        gbps = 3 * n * 4 / (ms * 1e-3) / 1e9
        out[str(mib)] = {"kernel_us": round(ms * 1e3, 2), "achieved_gbs": round(gbps, 1),
                         "frac": round(gbps / PEAK_GBPS, 4)}
        del sets
        torch.cuda.empty_cache()
    return out


def extra_config1_two_process(timeout_s: float = 120.0) -> dict:
    """BASELINE configs[0]'s shape on the GPU path between PROCESSES: a 2-rank
    float FI_SUM allreduce of 4 KiB, two worker processes sharing this GPU
    through GPU peer domains, LFA_ALGO_P2P's one-shot kernel ending in the
    completion word (tools/probe_p2p_latency.py --quick, its own processes;
    this one only waits).  Median / p10 / p90 over Python-timed operations,
    the mean of a C loop (lfa_bench_loop), and the result checked on both
    ranks against x1 + x0 (prov/coll's two-rank tree, coll_coll.c:409-430)."""
    import subprocess
    try:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_p2p_latency.py"),
                            "--quick", "--reps", "1000"], capture_output=True, text=True,
                           timeout=timeout_s)
        lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
        if p.returncode or not lines:
            return {"error": f"probe exited {p.returncode}: {p.stderr[-200:]}"}
        d = json.loads(lines[-1])
        r = (d.get("rank0") or {}).get("p2p_4096", {})
        h = (d.get("rank0") or {}).get("p2p_host_4096", {})
        return {"us_median": r.get("median_us"), "us_p10": r.get("p10_us"),
                "us_p90": r.get("p90_us"), "n": r.get("reps"),
                "c_loop_mean_us": r.get("c_loop_mean_us"),
                "exact": bool(r.get("exact")) and bool(
                    (d.get("rank1") or {}).get("p2p_4096", {}).get("exact")),
                "pinned_host_buffers": {
                    "us_median": h.get("median_us"), "us_p10": h.get("p10_us"),
                    "us_p90": h.get("p90_us"), "c_loop_mean_us": h.get("c_loop_mean_us"),
                    "exact": bool(h.get("exact")) and bool(
                        (d.get("rank1") or {}).get("p2p_host_4096", {}).get("exact"))},
                "what": "2 processes on this GPU, GPU peer domains, LFA_ALGO_P2P one-shot + "
                        "completion word; Python-timed submit + wait per operation; device "
                        "buffers, and pinned host buffers (the one-shot on their mappings)"}
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"[:200]}


def extra_config1_loopback(dev, stream, reps=1000, warm=100):
    """BASELINE configs[0] at its stated shape on ONE GPU: a 2-rank float
    FI_SUM allreduce of 4 KiB per rank, both ranks' schedules executed by the
    C executor with the real kernels and a device-copy loopback transport
    (lfa_coll_loopback).  Median wall time per collective (launch + sync) of
    `reps` after `warm`; the result is checked against r1 + r0 bitwise.  The
    reference's own figure for this shape is the known answer of
    fabtests/multinode/src/core_coll.c:230-277 over tcp;ofi_rxm."""
    from libfabric_amd import coll
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    sends = [torch.rand(1024, device=dev, generator=g) * 2 - 1 for _ in range(2)]
    results = [torch.empty(1024, device=dev) for _ in range(2)]
    want = sends[1] + sends[0]
    out = {}
    for name, algo in (("tree_us", coll.ALGO_TREE), ("rd_us", coll.ALGO_RD)):
        ts = []
        for i in range(warm + reps):
            t0 = time.perf_counter()
            coll.loopback(3, algo, 2, -1, 8, 2, 1024, sends, results, stream)
            torch.cuda.synchronize()
            if i >= warm:
                ts.append(time.perf_counter() - t0)
        ok = all(torch.equal(r, want) for r in results)
        st = sample_stats([t * 1e6 for t in ts], 1)
        out[name] = st["median_us"]
        out[name.replace("_us", "_stats")] = st
        out[name.replace("_us", "_bitwise_ok")] = bool(ok)
    out["note"] = ("2 ranks on one GPU, loopback transport; median of 1000 after 100 "
                   "warm-up; wall time incl. hipStreamSynchronize")
    # LFA_ALGO_P2P's one-shot kernel (push, flags, tree) for the same shape:
    # the two ranks on two streams of this process, each with its own
    # symmetric workspace (the loopback runs every rank on one stream, where
    # one rank's kernel could not wait for the other's)
    import ctypes
    region, flag_off = 1 << 20, 2 << 20
    from libfabric_amd.coll import sig_area_bytes
    ws = [torch.zeros(flag_off + sig_area_bytes(), dtype=torch.uint8, device=dev)
          for _ in range(2)]
    sym = (ctypes.c_void_p * 2)(*[w.data_ptr() for w in ws])
    status = torch.full((1,), -1, dtype=torch.int64).pin_memory()   # LFA_SIG_NONE
    # two priorities: HIP keeps a hardware-queue pool per priority, so the
    # two ranks' kernels never share a queue (rank 0's wait would hold rank
    # 1's launch behind it until the timeout)
    streams = [torch.cuda.Stream(device=dev, priority=0),
               torch.cuda.Stream(device=dev, priority=-1)]
    for r in results:
        r.zero_()
    torch.cuda.synchronize()
    ts = []
    for i in range(warm + reps):
        t0 = time.perf_counter()
        for r in range(2):
            coll.oneshot_reduce(FI_SUM, FI_FLOAT, coll.OneShot(
                sends[r].data_ptr(), results[r].data_ptr(), 1024, -1,
                ctypes.cast(sym, ctypes.c_void_p), 4096, region // 2, flag_off, 2, r, i + 1,
                status.data_ptr(), i + 1, 2_000_000), streams[r])
        for st in streams:
            st.synchronize()
        if int(status.item()) != -1:
            break            # a wait timed out: the two streams did not run together
        if i >= warm:
            ts.append(time.perf_counter() - t0)
    out["oneshot_kernel_only_us"] = round(statistics.median(ts) * 1e6, 1) if ts else None
    if ts:
        out["oneshot_kernel_only_stats"] = sample_stats([t * 1e6 for t in ts], 1)
    out["oneshot_bitwise_ok"] = bool(all(torch.equal(r, want) for r in results)
                                     and int(status.item()) == -1)
    out["oneshot_note"] = ("KERNEL ONLY: the LFA_ALGO_P2P one-shot kernel launched directly, "
                           "the 2 ranks on two streams of one process with hand-built "
                           "workspaces — no provider submit / completion path (that is "
                           "probe_p2p_latency's figure); wall time of both launches + both "
                           "stream syncs, every iteration's status checked; region %d B"
                           % region)
    return out


def extra_tree(dev, stream, nsrc=8):
    """N-input fused combine (the allreduce's local step): 8 x 32 MiB float
    blocks -> 1, recursive-doubling order.  Traffic (N+1)·B per launch."""
    from libfabric_amd import atomic
    blk = 32 * 1024 * 1024 // 4
    sets = []
    for k in range(2):
        srcs = [torch.rand(blk, device=dev) for _ in range(nsrc)]
        sets.append((srcs, torch.empty(blk, device=dev)))

    def fn(i):
        srcs, out = sets[i % 2]
        atomic.reduce_tree(2, 8, out, srcs, blk, stream)
    for i in range(4):
        fn(i)
    ms = _kernel_events(fn, 30, stream)
    gbps = (nsrc + 1) * blk * 4 / (ms * 1e-3) / 1e9
    out = {"nsrc": nsrc, "block_bytes": blk * 4, "kernel_us": round(ms * 1e3, 2),
           "achieved_gbs": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4),
           "layout": "separate allocations (the caller's buffers)"}
    del sets
    # the collective's own layout: the N slots of one TMP workspace sit
    # round_up(B, 256) + 6 KiB apart (lfa_coll_plan.c blk_stride)
    stride = (blk * 4 + 255) // 256 * 256 + 6 * 1024
    ws = [torch.empty(nsrc * stride, dtype=torch.uint8, device=dev) for _ in range(2)]
    for w in ws:
        w.view(torch.float32)[: w.numel() // 4].uniform_()
    wsets = [([w[k * stride:k * stride + blk * 4].view(torch.float32) for k in range(nsrc)],
              torch.empty(blk, device=dev)) for w in ws]

    def fw(i):
        srcs, o = wsets[i % 2]
        atomic.reduce_tree(2, 8, o, srcs, blk, stream)
    for i in range(4):
        fw(i)
    ms = _kernel_events(fw, 30, stream)
    gbps = (nsrc + 1) * blk * 4 / (ms * 1e-3) / 1e9
    out["collective_workspace_layout"] = {
        "kernel_us": round(ms * 1e3, 2), "achieved_gbs": round(gbps, 1),
        "frac": round(gbps / PEAK_GBPS, 4),
        "layout": "8 slots of one allocation, round_up(B, 256) + 6 KiB apart (TREE's TMP)"}
    return out


def extra_tree_put(dev, stream, nsrc=8, reps=5, nsets=3, launches=30):
    """The LFA_ALGO_P2P kernel on local HBM: 8 x 32 MiB float blocks -> 1
    and -> 8 outputs, system-scope (sc0 sc1) loads and stores.  Traffic
    (nsrc + ndst)·B per launch.  On the 8-GPU node 7 of the inputs and 7 of
    the outputs are peers' HBM over xGMI instead.

    The 8 -> 8 time depends on where the allocator put the 16 blocks (84-98 us
    by buffer set on one box), so one set is not a figure
    that compares across runs: each of `reps` repetitions
    allocates `nsets` FRESH sets (3 x 16 x 32 MiB = 1.5 GiB at 8 -> 8, past the
    256 MB Infinity Cache) and times `launches` launches rotating over them
    with one event pair; the row reports the median over repetitions and the
    range."""
    from libfabric_amd import atomic
    blk = 32 * 1024 * 1024 // 4
    out = {}
    for ndst in (1, 8):
        per = []
        for rep in range(reps):
            sets = []
            for k in range(nsets):
                srcs = [torch.rand(blk, device=dev) for _ in range(nsrc)]
                sets.append((srcs, [torch.empty(blk, device=dev) for _ in range(ndst)]))

            def fn(i, sets=sets):
                srcs, dsts = sets[i % nsets]
                atomic.reduce_tree_put(2, 8, dsts, srcs, blk, stream)
            for i in range(2 * nsets):
                fn(i)
            per.append(_kernel_events(fn, launches, stream))
            del sets, fn
            torch.cuda.empty_cache()
        ms = statistics.median(per)
        nb = (nsrc + ndst) * blk * 4

        def frac(t):
            return round(nb / (t * 1e-3) / 1e9 / PEAK_GBPS, 4)
        out[f"{nsrc}to{ndst}"] = {
            "kernel_us": round(ms * 1e3, 2), "achieved_gbs": round(nb / (ms * 1e-3) / 1e9, 1),
            "frac": frac(ms),
            "kernel_us_range": [round(min(per) * 1e3, 2), round(max(per) * 1e3, 2)],
            "frac_range": [frac(max(per)), frac(min(per))],
            "samples": f"median of {reps} repetitions, each {launches} launches over "
                       f"{nsets} freshly allocated buffer sets"}
    return out


def extra_e2e_host(dev, stream, reps=5):
    """The same 256 MiB float SUM combine when the buffers start and end in
    pinned host memory (what a libfabric caller hands over): H2D dst and src,
    combine, D2H dst — the PCIe-inclusive rate (never the headline value)."""
    from libfabric_amd import atomic
    hd = torch.rand(COUNT).pin_memory()
    hs = torch.rand(COUNT).pin_memory()
    d = torch.empty(COUNT, device=dev)
    s = torch.empty(COUNT, device=dev)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(hd, non_blocking=True)
        s.copy_(hs, non_blocking=True)
        atomic.write(FI_SUM, FI_FLOAT, d, s, COUNT, stream)
        hd.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts[1:])
    return {"ms": round(t * 1e3, 2), "buffer_gib_s": round(S_BYTES / t / 2**30, 2),
            "traffic_gib_s": round(3 * S_BYTES / t / 2**30, 2),
            "note": "pinned host buffers; 2x256 MiB H2D + combine + 256 MiB D2H, serial"}


def extra_host_allreduce(ep, world, reps=3, sweep=False):
    """fi_allreduce on HOST buffers (what a libfabric caller hands over):
    the provider streams 32 MiB chunks H2D -> collective -> D2H on three HIP
    streams (both PCIe directions busy at once).  Rate = buffer bytes / wall time, PCIe-inclusive."""
    from libfabric_amd import coll
    hx = torch.rand(COUNT).pin_memory()
    hy = torch.empty(COUNT).pin_memory()
    ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
    ts = []
    for _ in range(reps):
        barrier(world)
        t0 = time.perf_counter()
        ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
        ts.append(max_over_ranks(time.perf_counter() - t0, world))
    t = statistics.median(ts)
    by_chunk = {}
    if sweep:
        for mib in (8, 16, 32, 64, 128):
            ep.set_chunk(mib << 20)
            ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
            tc = []
            for _ in range(reps):
                barrier(world)
                t0 = time.perf_counter()
                ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
                tc.append(max_over_ranks(time.perf_counter() - t0, world))
            by_chunk[str(mib)] = round(statistics.median(tc) * 1e3, 2)
        ep.set_chunk(0)
    row = {"ms": round(t * 1e3, 2), "buffer_gib_s": round(S_BYTES / t / 2**30, 2),
           "note": "pinned host in/out, default chunks; H2D, collective and D2H on "
                   "three streams"}
    if world == 1:
        # a one-member group's allreduce is a copy, run on the pinned buffers'
        # mappings; the staged pipeline it replaces beside it
        os.environ["LFA_HOST_ZERO_COPY"] = "0"
        try:
            ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                ep.wait(ep.allreduce(hx, hy, COUNT, 8, 2))
                ts.append(time.perf_counter() - t0)
        finally:
            del os.environ["LFA_HOST_ZERO_COPY"]
        row["staged_ms"] = round(statistics.median(ts) * 1e3, 2)
        row["note"] = ("pinned host in/out; one member: the copy on the buffers' mappings "
                       "over PCIe (zero-copy); staged_ms = H2D / copy / D2H on three streams")
    if by_chunk:
        row["ms_by_chunk_mib"] = by_chunk
    if world > 1:
        # a GROUP chunk (every rank sets the same value) lets a
        # group of N > 1 pipeline host buffers; device-buffer members then
        # split into the same chunks — both sides of that trade measured
        def timed(x, y):
            ep.wait(ep.allreduce(x, y, COUNT, 8, 2))
            tt = []
            for _ in range(reps):
                barrier(world)
                t0 = time.perf_counter()
                ep.wait(ep.allreduce(x, y, COUNT, 8, 2))
                tt.append(max_over_ranks(time.perf_counter() - t0, world))
            return round(statistics.median(tt) * 1e3, 3)
        dx, dy = hx.to("cuda"), torch.empty(COUNT, device="cuda")
        torch.cuda.synchronize()
        # the default (LFA_GROUP_CHUNK_AUTO: 32 MiB chunks from 64 MiB on,
        # every member) — row["ms"] above is the host side of it
        row["device_default_ms"] = timed(dx, dy)
        want = dy.cpu()
        ep.set_group_chunk(0)
        row["device_whole_ms"] = timed(dx, dy)
        row["host_whole_ms"] = timed(hx, hy)
        for mib in (32, 64):
            ep.set_group_chunk(mib << 20)
            row[f"group_chunk_{mib}mib_host_ms"] = timed(hx, hy)
            row[f"group_chunk_{mib}mib_device_ms"] = timed(dx, dy)
            row[f"group_chunk_{mib}mib_bitwise_equal"] = bool(torch.equal(hy, want) and
                                                             torch.equal(dy.cpu(), want))
        ep.set_group_chunk(coll.GROUP_CHUNK_AUTO)
        row["group_chunk_note"] = ("lfa_coll_ep_set_group_chunk on every rank: host members "
                                   "pipeline H2D/collective/D2H per chunk, device members "
                                   "run the same chunks in place")
    return row


def extra_host_reduce_scatter(ep, rank, world, reps=3):
    """fi_reduce_scatter on HOST buffers, double PROD, 256 MiB per rank: the
    provider streams 32 MiB chunks (one 2-D H2D gathers chunk j of every
    rank's block) through the device reduce_scatter, H2D/D2H overlapped.
    Checked bitwise against the device-buffer result; the one-chunk
    (serial-staging) time beside it."""
    from libfabric_amd import coll
    cnt = S_BYTES // 8
    cnt -= cnt % world
    off, ln = coll.block(cnt, world, rank)
    g = torch.Generator().manual_seed(200 + rank)
    hx = (torch.rand(cnt, generator=g, dtype=torch.float64) * 0.2 + 0.9).pin_memory()
    hy = torch.zeros(ln, dtype=torch.float64).pin_memory()
    dx = hx.to("cuda")
    dy = torch.empty(ln, device="cuda", dtype=torch.float64)
    torch.cuda.synchronize()     # buffers ready: the provider's stream is its own
    ep.wait(ep.reduce_scatter(dx, dy, cnt, 9, 3))
    ep.wait(ep.reduce_scatter(hx, hy, cnt, 9, 3))
    row = {"bitwise_equal_device": bool(torch.equal(hy, dy.cpu()))}
    # a one-member group copies pinned buffers on their mappings (zero-copy);
    # its staged forms are timed with LFA_HOST_ZERO_COPY=0
    forms = [("ms", 0, "1"), ("one_chunk_ms", 1 << 40, "0" if world == 1 else "1")]
    if world == 1:
        forms.insert(1, ("staged_ms", 0, "0"))
    for name, chunk, zc in forms:
        ep.set_chunk(chunk)
        os.environ["LFA_HOST_ZERO_COPY"] = zc
        try:
            ts = []
            for _ in range(reps):
                barrier(world)
                t0 = time.perf_counter()
                ep.wait(ep.reduce_scatter(hx, hy, cnt, 9, 3))
                ts.append(max_over_ranks(time.perf_counter() - t0, world))
        finally:
            del os.environ["LFA_HOST_ZERO_COPY"]
        row[name] = round(statistics.median(ts) * 1e3, 2)
    ep.set_chunk(0)
    row["buffer_gib_s"] = round(S_BYTES / (row["ms"] * 1e-3) / 2**30, 2)
    row["note"] = ("pinned host in/out; one member: zero-copy on the mappings, staged "
                   "(32 MiB chunks) and one-chunk staging beside it" if world == 1 else
                   "pinned host in/out; default 32 MiB chunks vs one chunk (serial staging)")
    return row


def cpu_model_allreduce(world: int):
    """Modelled reference compute for a 256 MiB float SUM allreduce at N
    ranks: log2(N) x (CAS combine [+ COPY]) — prov/coll's per-rank REDUCE
    items (coll_coll.c:409-430).  The reference itself cannot run this
    (eager-size hang); transport is excluded.  Measured on a 16 MiB
    slice on 1 core and scaled linearly."""
    import numpy as np
    import oracle
    n = 4 * 1024 * 1024
    rng = np.random.default_rng(0)
    d, s = rng.uniform(-1, 1, n).astype(np.float32), rng.uniform(-1, 1, n).astype(np.float32)
    t0 = time.perf_counter()
    oracle.write(FI_SUM, FI_FLOAT, d, s, oracle.CAS)
    t = (time.perf_counter() - t0) * (COUNT / n)
    steps = max(1, (world - 1).bit_length())
    return {"ms": round(t * steps * 1e3, 1), "steps": steps, "kind": "modelled",
            "note": "log2(N) CAS combines of 256 MiB on 1 host core; transport excluded"}


def extra_e2e_staged(reps=3):
    """The same combine with dst/src in pinned HOST memory through the host
    entry point lfa_atomic_write_staged.  Its default on pinned buffers is
    zero-copy: one combine on the mapped buffers, reading and writing host
    memory over PCIe.  Beside it, the staged pipeline it replaces
    (LFA_HOST_ZERO_COPY=0: H2D of chunk c+1 overlapping the combine + D2H of
    chunk c) at three chunk sizes.  The row's ms is the default call's."""
    from libfabric_amd import _native
    L = _native.lib()
    hd = torch.rand(COUNT).pin_memory()
    hs = torch.rand(COUNT).pin_memory()

    def timed(chunk, zero_copy):
        os.environ["LFA_HOST_ZERO_COPY"] = zero_copy
        try:
            assert L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, hd.data_ptr(), hs.data_ptr(),
                                             COUNT, chunk) == 0
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, hd.data_ptr(), hs.data_ptr(),
                                          COUNT, chunk)
                ts.append(time.perf_counter() - t0)
        finally:
            del os.environ["LFA_HOST_ZERO_COPY"]
        return statistics.median(ts)

    t = timed(0, "1")
    by_chunk = {mib: timed(mib << 20, "0") for mib in (16, 32, 64)}
    return {"ms": round(t * 1e3, 2), "buffer_gib_s": round(S_BYTES / t / 2**30, 2),
            "traffic_gib_s": round(3 * S_BYTES / t / 2**30, 2), "form": "zero-copy",
            "staged_ms_by_chunk_mib": {k: round(v * 1e3, 2) for k, v in by_chunk.items()},
            "note": "pinned host dst/src; default = one combine over PCIe on the mapped "
                    "buffers; staged = H2D / combine / D2H on two streams"}


ORACLE_SLICE = 65536                   # elements per checked slice


def oracle_ranges(count: int, world: int, kind: str, m: int = ORACLE_SLICE):
    """Element ranges of a collective's result that the N > 1 leg checks
    against the oracle, merged and sorted: allreduce — three
    fixed m-element slices (start, middle, end); reduce_scatter — the first
    and last m elements of every rank's block, the blocks as the reference
    semantics define them (oracle.slice_bounds: the first count % N ranks one
    element more)."""
    import oracle
    if kind == "allreduce":
        m = min(m, count)
        mid = count // 2 - m // 2
        cand = [(0, m), (mid, mid + m), (count - m, count)]
    else:
        cand = []
        for lo, hi in oracle.slice_bounds(count, world):
            k = min(m, hi - lo)
            cand += [(lo, lo + k), (hi - k, hi)]
    out = []
    for a, b in sorted(cand):
        if a >= b:
            continue
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def oracle_check(x, y, count: int, rank: int, world: int, dt: int, op: int, kind: str,
                 m: int = ORACLE_SLICE) -> dict:
    """The N > 1 leg's parity check.  Every rank's input at
    oracle_ranges and its output there — the whole range for allreduce, the
    part inside its own block for reduce_scatter — are gathered to every rank;
    rank 0 runs the oracle's prov/coll allreduce (recursive doubling,
    coll_coll.c:409-430's `hi OP lo` order) over the gathered inputs and
    compares every rank's output with it bit for bit.  The oracle is only the
    checker, outside any timed region.  Collective over the job (every rank
    calls it); returns {"oracle_exact", "elements", "mismatches"} on rank 0,
    {} elsewhere."""
    import numpy as np
    import oracle
    ranges = oracle_ranges(count, world, kind, m)
    total = sum(b - a for a, b in ranges)
    if kind == "allreduce":
        yout = torch.cat([y[a:b] for a, b in ranges])
        mask = torch.ones(total, dtype=torch.uint8, device=y.device)
    else:
        lo, hi = oracle.slice_bounds(count, world)[rank]
        yout = torch.zeros(total, dtype=y.dtype, device=y.device)
        mask = torch.zeros(total, dtype=torch.uint8, device=y.device)
        pos = 0
        for a, b in ranges:
            c, d = max(a, lo), min(b, hi)
            if c < d:
                yout[pos + c - a:pos + d - a] = y[c - lo:d - lo]
                mask[pos + c - a:pos + d - a] = 1
            pos += b - a
    xin = torch.cat([x[a:b] for a, b in ranges])
    if world > 1:
        gloo = dist.get_backend() == "gloo"
        parts = []
        for t in (xin, yout, mask):
            t = t.cpu() if gloo else t.contiguous()
            lst = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(lst, t)
            parts.append([u.cpu() for u in lst])
        xs, ys, ms = parts
    else:
        xs, ys, ms = [xin.cpu()], [yout.cpu()], [mask.cpu()]
    if rank != 0:
        return {}
    want = oracle.allreduce(op, dt, [t.numpy() for t in xs])[0]
    uint = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[want.dtype.itemsize]
    w = want.view(uint)
    bad, covered = 0, np.zeros(total, dtype=bool)
    for yk, mk in zip(ys, ms):
        sel = mk.numpy().astype(bool)
        covered |= sel
        bad += int((yk.numpy().view(uint)[sel] != w[sel]).sum())
    bad += int((~covered).sum())            # an element no rank holds
    return {"oracle_exact": bad == 0, "elements": total, "mismatches": bad}


def topology() -> dict:
    """What the N-GPU run saw: devices and the hipDeviceCanAccessPeer matrix
    (torch.cuda.can_device_access_peer)."""
    n = torch.cuda.device_count()
    return {"hip_device_count": n,
            "peer_access": [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j))
                             for j in range(n)] for i in range(n)]}


def sample_stats(samples_us, world: int) -> dict:
    """Latency rows as a distribution: the per-sample max
    over ranks (an operation is done when its last member is), then median,
    p10 and p90 over the n samples."""
    t = torch.tensor(samples_us, dtype=torch.float64,
                     device="cpu" if (REHEARSE or world == 1) else "cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = sorted(t.cpu().tolist())

    def q(p):
        return v[min(len(v) - 1, int(round(p * (len(v) - 1))))]
    return {"median_us": round(statistics.median(v), 2), "p10_us": round(q(0.1), 2),
            "p90_us": round(q(0.9), 2), "n": len(v)}


def _py_samples(submit_wait, n: int) -> list[float]:
    """Microseconds of `n` operations one at a time (submit, then wait for
    that one), timed from Python — for buckets whose time dwarfs the
    wrapper's ~10 us per call."""
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        submit_wait()
        out.append((time.perf_counter() - t0) * 1e6)
    return out


def _rs_sweep(ep, rank, world, algo, egress_gbs=None):
    """double PROD reduce_scatter, 4 KiB .. 256 MiB per rank (configs[4]); each
    size's result checked against the oracle on slices (oracle_check).  Per
    size: "us" is the median latency of n operations one at a time (p10 /
    p90 beside it, max over ranks per sample); "pipelined_us" the mean per
    operation with a batch in flight, from which busbw is computed."""
    from libfabric_amd import coll
    ep.set_algo(algo)
    sweep = {}
    for k, nbytes in enumerate([4096 * 4 ** k for k in range(9)]):   # 4 KiB .. 256 MiB
        cnt = nbytes // 8
        g = torch.Generator(device="cuda").manual_seed(5000 + 97 * rank + k)
        a = torch.rand(cnt, device="cuda", dtype=torch.float64, generator=g) * 0.2 + 0.9
        off, ln = coll.block(cnt, world, rank)
        b = torch.empty(max(ln, 1), device="cuda", dtype=torch.float64)
        torch.cuda.synchronize()
        ep.wait(ep.reduce_scatter(a, b, cnt, 9, 3))
        torch.cuda.synchronize()
        chk = oracle_check(a, b, cnt, rank, world, 9, 3, "reduce_scatter")
        # latency, one operation submitted and reaped at a time: n samples,
        # median with p10 / p90.  Up to 1 MiB timed in C
        # (liblfa_bench.so), without the Python wrapper's ~10 us per call
        barrier(world)
        if nbytes <= (1 << 20):
            lat = ep.bench_samples(5, a, b, cnt, 9, 3, reps=200)
            how = "C loop (lfa_bench_samples)"
        else:
            n = 20 if REHEARSE and nbytes >= (16 << 20) else 100
            lat = _py_samples(lambda: ep.wait(ep.reduce_scatter(a, b, cnt, 9, 3)), n)
            how = "Python submit + wait"
        st = sample_stats(lat, world)
        # throughput with operations in flight (the busbw figure)
        barrier(world)
        reps = 20 if nbytes < (16 << 20) else 5
        t0 = time.perf_counter()
        ctxs = [ep.reduce_scatter(a, b, cnt, 9, 3) for _ in range(reps)]
        ep.wait(ctxs[-1])
        t = max_over_ranks(time.perf_counter() - t0, world) / reps
        sweep[str(nbytes)] = {"us": st["median_us"], "p10_us": st["p10_us"],
                              "p90_us": st["p90_us"], "n": st["n"], "timed": how,
                              "pipelined_us": round(t * 1e6, 1),
                              "busbw_gbs": round((world - 1) / world * nbytes / t / 1e9, 2)}
        sweep[str(nbytes)].update(chk)
        if algo == coll.ALGO_AUTO:
            # the per-bucket choice (lfa_coll_auto_algo; the same on every
            # rank) — device domains only: a peer domain runs AUTO as TREE
            chosen = coll.ALGO_TREE if REHEARSE else coll.auto_algo(5, cnt, world, 8)
            sweep[str(nbytes)]["algo"] = {coll.ALGO_P2P: "p2p_oneshot",
                                          coll.ALGO_TREE: "tree"}.get(chosen, str(chosen))
        if egress_gbs and world > 1:
            # reduce_scatter moves (N-1)/N of the bucket out of every GPU
            floor = (world - 1) / world * nbytes / (egress_gbs * 1e9)
            sweep[str(nbytes)]["frac_of_xgmi_bound"] = round(floor / t, 4)
    return sweep


def extra_xgmi(rank, world, device="cuda", nbytes=S_BYTES):
    """SURVEY §8(d) config 4's bound, measured: per-GPU xGMI egress with every
    GPU sending to every other at once (RCCL all-to-all of 256 MiB per rank:
    (N-1)/N·S leaves each GPU), and one link alone (each rank sends 256 MiB
    to its ring neighbour while receiving from the other).  The allreduce
    extras report their time against the all-to-all figure: an allreduce
    moves 2(N-1)/N·S out of every GPU."""
    x = torch.empty(nbytes, dtype=torch.uint8, device=device)
    y = torch.empty_like(x)
    out = {}
    sync = torch.cuda.synchronize if device == "cuda" else (lambda: None)

    def timed(fn, reps):
        fn()
        sync()
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sync()
        return max_over_ranks(time.perf_counter() - t0, world) / reps

    t = timed(lambda: dist.all_to_all_single(y, x), 5)
    out["alltoall_egress_gbs"] = round((world - 1) / world * nbytes / t / 1e9, 1)
    out["alltoall_ms"] = round(t * 1e3, 3)

    def ring():
        reqs = dist.batch_isend_irecv([
            dist.P2POp(dist.isend, x, (rank + 1) % world),
            dist.P2POp(dist.irecv, y, (rank - 1) % world)])
        for r in reqs:
            r.wait()
    t = timed(ring, 5)
    out["one_link_gbs"] = round(nbytes / t / 1e9, 1)
    out["what"] = ("RCCL all_to_all_single and a ring send/recv of 256 MiB per rank "
                   "(torch.distributed over RCCL); GB/s leaving each GPU")
    return out


def _allreduce_sweep(ep, world, algos, out=None):
    """float SUM allreduce time per algorithm at 64 KiB, 1 MiB and 16 MiB per
    rank (N > 1): the data the choice of a default per size needs.  `algos`:
    (name, algo) pairs; rows merge into `out`."""
    from libfabric_amd import coll
    out = {} if out is None else out
    for nbytes, reps in ((64 << 10, 50), (1 << 20, 30), (16 << 20, 10)):
        n = nbytes // 4
        x = torch.rand(n, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        row = out.setdefault(str(nbytes), {})
        for name, algo in algos:
            try:
                ep.set_algo(algo)
                ep.wait(ep.allreduce(x, y, n, 8, 2))
                barrier(world)
                t0 = time.perf_counter()
                ctxs = [ep.allreduce(x, y, n, 8, 2) for _ in range(reps)]
                ep.wait(ctxs[-1])
                t = max_over_ranks(time.perf_counter() - t0, world) / reps
                row[name + "_us"] = round(t * 1e6, 1)
            except Exception as e:  # noqa: BLE001
                row[name + "_error"] = f"{e}"[:120]
    ep.set_algo(coll.ALGO_TREE)
    return out


OS_CROSSOVER_BOUND = 1 << 30     # one-shot bounds in the crossover child


def _provider_ep(rank, world):
    """The endpoint the N > 1 provider extras use: a device domain over RCCL,
    or in a rehearsal (ranks sharing a GPU, which RCCL refuses) a GPU peer
    domain whose transfers gloo carries."""
    from libfabric_amd import coll
    if REHEARSE and world > 1:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from gloo_xfer import GlooXfer
        return coll.HostEndpoint(rank, world, GlooXfer(), device=torch.cuda.current_device())
    return coll.Endpoint.from_torch_dist()


def extra_oneshot_crossover(rank, world, emit=None):
    """where the one-shot kernel stops beating the tree, per
    bucket, on THIS topology — so the first 8-GPU run retunes LFA_OS_AG_BYTES
    / LFA_OS_RS_BYTES (FI_OFF_LFA_ONESHOT_*) from data.  Runs in its own
    child with both bounds at OS_CROSSOVER_BOUND, so LFA_ALGO_P2P plans the
    one-shot at every size here; TREE beside it.  Float SUM allreduce and
    double PROD reduce_scatter, batches in flight, max over ranks.  Reports
    per size both times, and the largest bucket where the one-shot wins —
    the bound to set (allreduce: summed over the members, as the knob is)."""
    from libfabric_amd import coll
    emit = emit or (lambda _o: None)
    out = {"bounds_in_this_child": {"LFA_OS_AG_BYTES": os.environ.get("LFA_OS_AG_BYTES"),
                                    "LFA_OS_RS_BYTES": os.environ.get("LFA_OS_RS_BYTES")},
           "defaults": {"LFA_OS_AG_BYTES": 2 << 20, "LFA_OS_RS_BYTES": 4 << 20},
           "tuned_on": "2-4 processes sharing one MI355X (DESIGN.md §5b)"}
    # the second child of the pair runs with both bounds at 1 byte: there
    # LFA_ALGO_P2P is the two-barrier schedule at every size, AUTO's bulk
    # choice since round 6 (LFA_AUTO_BULK) — timed as "p2p_bulk"
    bulk = os.environ.get("LFA_OS_AG_BYTES") == "1"
    algos = ((("p2p_bulk", coll.ALGO_P2P),) if bulk else
             (("tree", coll.ALGO_TREE), ("oneshot", coll.ALGO_P2P)))
    ep = _provider_ep(rank, world)
    try:
        for coll_name, sizes in (("allreduce", (16 << 10, 64 << 10, 256 << 10, 1 << 20,
                                                4 << 20)),
                                 ("reduce_scatter", (64 << 10, 256 << 10, 1 << 20, 4 << 20,
                                                     16 << 20))):
            rows, win, lost = {}, 0, False
            for nbytes in sizes:
                if coll_name == "allreduce":
                    n = nbytes // 4
                    x = torch.rand(n, device="cuda")
                    y = torch.empty_like(x)

                    def op():
                        return ep.allreduce(x, y, n, 8, 2)
                else:
                    n = nbytes // 8
                    x = torch.rand(n, device="cuda", dtype=torch.float64) * 0.2 + 0.9
                    y = torch.empty(max(coll.block(n, world, rank)[1], 1), device="cuda",
                                    dtype=torch.float64)

                    def op():
                        return ep.reduce_scatter(x, y, n, 9, 3)
                torch.cuda.synchronize()
                row = {}
                reps = 30 if nbytes <= (1 << 20) else 10
                for name, algo in algos:
                    try:
                        ep.set_algo(algo)
                        ep.wait(op())
                        barrier(world)
                        t0 = time.perf_counter()
                        ctxs = [op() for _ in range(reps)]
                        ep.wait(ctxs[-1])
                        row[name + "_us"] = round(
                            max_over_ranks(time.perf_counter() - t0, world) / reps * 1e6, 1)
                    except Exception as e:  # noqa: BLE001
                        row[name + "_error"] = f"{e}"[:120]
                # the bound: the largest bucket up to which the one-shot wins
                # at every size measured
                if not lost and row.get("oneshot_us", 1e30) < row.get("tree_us", 0.0):
                    win = nbytes
                else:
                    lost = True
                rows[str(nbytes)] = row
            ep.set_algo(coll.ALGO_TREE)
            c = ep.counters()
            out[coll_name] = {"by_bucket_bytes_per_rank": rows,
                              "oneshot_wins_up_to_bytes_per_rank": win,
                              "suggested_bound": win * world if coll_name == "allreduce" else win,
                              "knob": ("LFA_OS_AG_BYTES (summed over the members)"
                                       if coll_name == "allreduce" else "LFA_OS_RS_BYTES")}
            out["counters"] = c
            emit(out)
    finally:
        ep.close()
    return out


def merge_crossover(out: dict, bulk: dict, world: int) -> None:
    """Fold the bulk child's P2P two-barrier times into the crossover rows
    and set `suggested_bound` against AUTO's choice above the bounds
    (LFA_AUTO_BULK: p2p by default, so the one-shot is priced against the
    two-barrier schedule; the tree when it is set to "tree")."""
    from libfabric_amd import coll
    if not isinstance(out, dict) or not isinstance(bulk, dict):
        return
    if "isolated_status" in bulk:
        out["bulk_isolated_status"] = bulk["isolated_status"]
    auto = "p2p_bulk" if coll.auto_bulk() == coll.ALGO_P2P else "tree"
    out["auto_above_bound"] = auto
    for name in ("allreduce", "reduce_scatter"):
        rows = (out.get(name) or {}).get("by_bucket_bytes_per_rank")
        brows = (bulk.get(name) or {}).get("by_bucket_bytes_per_rank") or {}
        if not rows:
            continue
        # without the bulk child's times (it failed or ran out of budget)
        # the first child's pricing against the tree stands
        alt = auto if auto == "tree" or any("p2p_bulk_us" in r for r in brows.values()) \
            else "tree"
        win, lost = 0, False
        for size in sorted(rows, key=int):
            if "p2p_bulk_us" in brows.get(size, {}):
                rows[size]["p2p_bulk_us"] = brows[size]["p2p_bulk_us"]
            other = rows[size].get(alt + "_us")
            if not lost and other is not None and rows[size].get("oneshot_us", 1e30) < other:
                win = int(size)
            else:
                lost = True
        out[name]["oneshot_wins_up_to_bytes_per_rank"] = win
        out[name]["suggested_bound"] = win * world if name == "allreduce" else win
        out[name]["priced_against"] = alt


def extra_collectives(rank, world, stream, emit=None):
    """BASELINE configs[3]/[4] at N>1: float SUM allreduce of 256 MiB per rank
    and a double PROD reduce_scatter bucket sweep, through the C provider
    (liblfa_coll.so).  algbw = S/t, busbw = 2(N-1)/N·S/t.  The exact
    algorithms (TREE, TREE_COLL, P2P) must agree bit for bit; the line says
    whether they did on this run.  `emit(out)` is called after each section
    (the isolated child prints the rows collected so far)."""
    from libfabric_amd import coll
    emit = emit or (lambda _o: None)
    xgmi = {}
    if world > 1 and not REHEARSE:
        try:
            xgmi = extra_xgmi(rank, world)
        except Exception as e:  # noqa: BLE001 — a probe must not hide the rest
            xgmi = {"error": f"{type(e).__name__}: {e}"[:200]}
    out = {"xgmi_peer_copy_256mib": xgmi} if xgmi else {}
    out["topology"] = topology()
    emit(out)
    if REHEARSE and world > 1:
        # ranks share a GPU here and RCCL refuses that (its refusal is the
        # rccl_nranks field): the same executor and kernels through a
        # peer-transfer domain (gloo carries the transfers), so the rows and
        # their oracle checks still run
        try:
            probe = coll.Endpoint.from_torch_dist()
            try:
                out["rccl_nranks"] = probe.rccl_nranks()
            finally:
                probe.close()
        except Exception as e:  # noqa: BLE001
            out["rccl_nranks"] = f"error: {type(e).__name__}: {e}"[:160]
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from gloo_xfer import GlooXfer
        ep = coll.HostEndpoint(rank, world, GlooXfer(), device=torch.cuda.current_device())
        out["endpoint"] = "peer-transfer domain over gloo (rehearsal)"
    else:
        ep = coll.Endpoint.from_torch_dist()
        try:
            out["rccl_nranks"] = ep.rccl_nranks()
        except coll.CollError as e:
            out["rccl_nranks"] = f"error: {e}"
    emit(out)
    # TREE unless a row selects another: the P2P forms (and LFA_ALGO_AUTO,
    # the device-domain default, whose small buckets are P2P) run last
    ep.set_algo(coll.ALGO_TREE)
    try:
        g = torch.Generator(device="cuda").manual_seed(7000 + rank)
        x = torch.rand(COUNT, device="cuda", generator=g) * 2 - 1
        y = torch.empty_like(x)
        ref = None
        # P2P (cross-GPU IPC mappings + system-scope kernel) last: the
        # RCCL-only forms are measured even if it were to fail
        for name, algo in (("allreduce_tree_exact", coll.ALGO_TREE),
                           ("allreduce_tree_exact_rccl_xfer", coll.ALGO_TREE_COLL),
                           ("allreduce_rccl", coll.ALGO_RCCL),
                           ("allreduce_p2p_exact", coll.ALGO_P2P)):
            try:
                ep.set_algo(algo)
                y.zero_()
                # fi_allreduce takes ready buffers: torch's fill and the
                # input's generation run on torch's stream, the provider on
                # its own
                torch.cuda.synchronize()
                ep.wait(ep.allreduce(x, y, COUNT, 8, 2))
                torch.cuda.synchronize()
                # every algorithm's bits against the oracle on three slices
                # (RCCL's ring order is not prov/coll's: informational there)
                row = oracle_check(x, y, COUNT, rank, world, 8, 2, "allreduce")
                if algo == coll.ALGO_RCCL and row:
                    row = {"oracle_bitwise_equal": row["oracle_exact"],
                           "oracle_elements": row["elements"],
                           "oracle_mismatches": row["mismatches"],
                           "oracle_note": "RCCL's ring order is not prov/coll's: "
                                          "tolerance, not bits (DESIGN §6)"}
                if algo != coll.ALGO_RCCL:
                    if ref is None:
                        ref = y.clone()
                    else:
                        row["bitwise_equal_tree"] = bool(torch.equal(y, ref))
                elif ref is not None:
                    # RCCL's ring order: within the stated bound of the exact
                    # tree, |got - ref| <= 2(N-1) 2^-24 sum_r |x_r|
                    ep.set_algo(coll.ALGO_TREE)
                    ax, sab = x.abs(), torch.empty_like(x)
                    torch.cuda.synchronize()
                    ep.wait(ep.allreduce(ax, sab, COUNT, 8, 2))
                    bound = 2 * max(world - 1, 1) * 2.0 ** -24 * sab
                    err = (y - ref).abs()
                    row["within_stated_tolerance_of_tree"] = bool((err <= bound).all())
                    row["max_abs_err"] = float(err.max())
                    row["bitwise_equal_tree"] = bool(torch.equal(y, ref))
                    del ax, sab, err, bound
                    ep.set_algo(algo)
                barrier(world)
                reps = 10
                t0 = time.perf_counter()
                ctxs = [ep.allreduce(x, y, COUNT, 8, 2) for _ in range(reps)]
                ep.wait(ctxs[-1])
                t = max_over_ranks(time.perf_counter() - t0, world) / reps
                row.update({"ms": round(t * 1e3, 3),
                            "algbw_gbs": round(S_BYTES / t / 1e9, 1),
                            "busbw_gbs": round(2 * (world - 1) / world * S_BYTES / t / 1e9, 1)})
                if xgmi.get("alltoall_egress_gbs"):
                    # the xGMI floor: 2(N-1)/N·S out of each GPU at the
                    # measured all-to-all egress rate
                    floor = 2 * (world - 1) / world * S_BYTES / (xgmi["alltoall_egress_gbs"] * 1e9)
                    row["frac_of_xgmi_bound"] = round(floor / t, 4)
                out[name] = row
            except Exception as e:  # noqa: BLE001 — one algorithm must not hide the rest
                out[name] = {"error": f"{type(e).__name__}: {e}"[:200]}
            emit(out)
        del ref
        ep.set_algo(coll.ALGO_TREE)
        try:
            out["allreduce_host_buffers_256mib"] = extra_host_allreduce(ep, world)
        except Exception as e:  # noqa: BLE001
            out["allreduce_host_buffers_256mib"] = {"error": f"{e}"[:200]}
        try:
            out["reduce_scatter_host_buffers_256mib"] = extra_host_reduce_scatter(
                ep, rank, world)
        except Exception as e:  # noqa: BLE001
            out["reduce_scatter_host_buffers_256mib"] = {"error": f"{e}"[:200]}
        emit(out)
        egress = xgmi.get("alltoall_egress_gbs")
        # the P2P forms (cross-GPU IPC mappings + system-scope kernels) come
        # last in every group below: if one stalled, the rows before it are out
        sizes = {}
        if world > 1:
            out["allreduce_float_sum_by_size_us"] = _allreduce_sweep(
                ep, world, (("tree", coll.ALGO_TREE), ("tree_coll", coll.ALGO_TREE_COLL),
                            ("rccl", coll.ALGO_RCCL)), sizes)
            emit(out)
        out["reduce_scatter_double_prod_tree"] = _rs_sweep(ep, rank, world, coll.ALGO_TREE,
                                                           egress)
        emit(out)
        if world > 1:
            # the same schedule with the block exchange as one ncclAllToAll
            try:
                out["reduce_scatter_double_prod_tree_coll"] = _rs_sweep(
                    ep, rank, world, coll.ALGO_TREE_COLL, egress)
            except Exception as e:  # noqa: BLE001
                out["reduce_scatter_double_prod_tree_coll"] = {"error": f"{e}"[:200]}
            ep.set_algo(coll.ALGO_TREE)
            emit(out)
        # configs[0] shape on the GPU path: 4 KiB float SUM allreduce latency
        a = torch.rand(1024, device="cuda", generator=g)
        b = torch.empty_like(a)
        torch.cuda.synchronize()
        for name, algo in (("allreduce_4kib_float_sum_us", coll.ALGO_TREE),
                           ("allreduce_4kib_float_sum_tree_coll_us", coll.ALGO_TREE_COLL),
                           ("allreduce_4kib_float_sum_rccl_us", coll.ALGO_RCCL),
                           ("allreduce_4kib_float_sum_p2p_us", coll.ALGO_P2P)):
            if algo != coll.ALGO_TREE and world == 1:
                continue
            try:
                ep.set_algo(algo)
                ep.wait(ep.allreduce(a, b, 1024, 8, 2))
                barrier(world)
                t0 = time.perf_counter()
                for _ in range(200):
                    ep.wait(ep.allreduce(a, b, 1024, 8, 2))
                t = max_over_ranks(time.perf_counter() - t0, world) / 200
                out[name] = round(t * 1e6, 1)
                # the same loop timed in C (liblfa_bench.so): what a C caller
                # of fi_allreduce + fi_cq_read sees, without the Python
                # wrapper's ~10 us per call
                barrier(world)
                ep.bench_loop(3, a, b, 1024, 8, 2, reps=200)        # warm-up
                barrier(world)
                st = sample_stats(ep.bench_samples(3, a, b, 1024, 8, 2, reps=2000), world)
                out[name.replace("_us", "_c_loop_us")] = st["median_us"]
                out[name.replace("_us", "_c_loop_stats")] = st
                torch.cuda.synchronize()
                if algo != coll.ALGO_RCCL:
                    c4 = oracle_check(a, b, 1024, rank, world, 8, 2, "allreduce")
                    if rank == 0:
                        out[name.replace("_us", "_oracle_exact")] = c4["oracle_exact"]
                if algo == coll.ALGO_TREE:
                    ref4k = b.clone()
                elif algo == coll.ALGO_P2P and world > 1:
                    # the one-shot kernel (push, flags, tree) against TREE's bits
                    differ = 0.0 if torch.equal(b, ref4k) else 1.0
                    out["allreduce_4kib_p2p_bitwise_equal_tree"] = \
                        max_over_ranks(differ, world) == 0.0
            except Exception as e:  # noqa: BLE001
                out[name] = {"error": f"{e}"[:120]}
            emit(out)
        ep.set_algo(coll.ALGO_TREE)
        if world > 1:
            _allreduce_sweep(ep, world, (("p2p", coll.ALGO_P2P),), sizes)
            emit(out)
            try:
                out["reduce_scatter_double_prod_p2p"] = _rs_sweep(ep, rank, world,
                                                                  coll.ALGO_P2P, egress)
            except Exception as e:  # noqa: BLE001
                out["reduce_scatter_double_prod_p2p"] = {"error": f"{e}"[:200]}
            ep.set_algo(coll.ALGO_TREE)
            emit(out)
            # the device-domain default (LFA_ALGO_AUTO): one-shot P2P for
            # small buckets, P2P's two-barrier schedule above (LFA_AUTO_BULK;
            # TREE before round 6) — the chosen algorithm per bucket
            try:
                out["reduce_scatter_double_prod_auto"] = _rs_sweep(ep, rank, world,
                                                                   coll.ALGO_AUTO, egress)
                ep.set_algo(coll.ALGO_AUTO)
                ep.wait(ep.allreduce(a, b, 1024, 8, 2))
                barrier(world)
                words0 = ep.word_ops()
                t0 = time.perf_counter()
                for _ in range(200):
                    ep.wait(ep.allreduce(a, b, 1024, 8, 2))
                t = max_over_ranks(time.perf_counter() - t0, world) / 200
                out["allreduce_4kib_float_sum_auto_us"] = round(t * 1e6, 1)
                # AUTO's small bucket is the P2P one-shot: on a device domain
                # it must complete through the completion word, not an event
                # (exec_plan used to drop the word's value)
                words = float(ep.word_ops() - words0)
                lo, hi = -max_over_ranks(-words, world), max_over_ranks(words, world)
                if REHEARSE:
                    # a peer-transfer domain runs AUTO as TREE (lfa_coll.c
                    # host_start): no one-shot, so no word to count
                    out["allreduce_4kib_auto_reaped_by_word"] = "n/a (peer domain: AUTO runs TREE)"
                else:
                    out["allreduce_4kib_auto_reaped_by_word"] = lo == hi == 200.0
                out["allreduce_4kib_auto_word_ops_min_max"] = [int(lo), int(hi)]
                out["allreduce_4kib_auto_bitwise_equal_tree"] = \
                    max_over_ranks(0.0 if torch.equal(b, ref4k) else 1.0, world) == 0.0
                out["auto_counters"] = ep.counters()
            except Exception as e:  # noqa: BLE001
                out["reduce_scatter_double_prod_auto"] = {"error": f"{e}"[:200]}
            ep.set_algo(coll.ALGO_TREE)
            emit(out)
        if rank == 0:
            out["cpu_model_allreduce_256mib"] = cpu_model_allreduce(world)
        emit(out)
    finally:
        ep.close()
    return out


def tune(args) -> None:
    """Interleaved A/B of the combine_vec variants (guide §5.4 rule 24)."""
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    count = args.tune_bytes // 4
    nsets = max(BUFFER_SETS, (2 << 30) // (2 * args.tune_bytes))  # >= 2 GiB rotated
    g = torch.Generator(device="cuda").manual_seed(7)
    sets = [(torch.rand(count, device="cuda", generator=g),
             torch.rand(count, device="cuda", generator=g)) for _ in range(nsets)]
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    nvec = count // 4
    variants = [int(v) for v in args.variants.split(',')] if args.variants else list(range(30))

    def run(v, d, s, n):
        fn = (L.lfa__tune_sum_f32 if v < 12 or v == 30 else
              L.lfa__tune3_sum_f32 if 70 <= v < 80 else L.lfa__tune2_sum_f32)
        return fn(v, d.data_ptr(), s.data_ptr(), n, h)

    # correctness of every variant first (odd size: exercises the tail path)
    nchk = (1 << 20) + 77
    for v in variants:
        a = torch.rand(nchk * 4, device="cuda")
        b = torch.rand(nchk * 4, device="cuda")
        want = a + b
        assert run(v, a, b, nchk) == 0
        torch.cuda.synchronize()
        if not torch.equal(a, want):
            raise SystemExit(f"tune variant {v} is WRONG")
    times = {v: [] for v in variants}
    region = {v: [] for v in variants}
    for _ in range(3):
        for v in variants:
            for i in range(4):
                d, s = sets[i % len(sets)]
                assert run(v, d, s, nvec) == 0
    torch.cuda.synchronize()
    for rnd in range(args.tune_rounds):
        for v in variants:
            evs = [(torch.cuda.Event(enable_timing=True),
                    torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for i, (a, b) in enumerate(evs):
                d, s = sets[i % len(sets)]
                a.record(stream)
                run(v, d, s, nvec)
                b.record(stream)
            torch.cuda.synchronize()
            times[v].extend(a.elapsed_time(b) for a, b in evs)
            region[v].append(evs[0][0].elapsed_time(evs[-1][1]) / len(evs))
    rows = []
    for v in variants:
        ms = statistics.median(times[v])
        nb = args.tune_bytes
        rows.append({"variant": v, "bytes": nb, "median_us": round(ms * 1e3, 2),
                     "min_us": round(min(times[v]) * 1e3, 2),
                     "region_us": round(statistics.median(region[v]) * 1e3, 2),
                     "p10_p90_us": [round(x * 1e3, 2) for x in
                                    statistics.quantiles(times[v], n=10)[::8]],
                     "tbps": round(3 * nb / (ms * 1e-3) / 1e12, 3),
                     "frac": round(3 * nb / (ms * 1e-3) / 1e9 / PEAK_GBPS, 4)})
    print(json.dumps({"tune": rows}))


def tune_tree(args) -> None:
    """A/B of the N-input tree kernel forms (float SUM), interleaved."""
    import ctypes
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    h = torch.cuda.current_stream().cuda_stream
    rows = []
    for nsrc in (2, 4, 8, 16):
        blk = (256 * 1024 * 1024 // 4) // nsrc           # 256 MiB of inputs
        sets = []
        for _ in range(2):
            srcs = [torch.rand(blk, device="cuda") for _ in range(nsrc)]
            sets.append((srcs, torch.empty(blk, device="cuda"),
                         (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs])))
        variants = [int(x) for x in args.variants.split(",")] if args.variants else [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, -1]
        ref = None
        for v in variants:  # correctness: every form equals the product's bits
            srcs, out, arr = sets[0]
            out.fill_(float("nan"))           # a form that wrote nothing fails
            torch.cuda.synchronize()
            assert L.lfa__tune_tree_f32(v, out.data_ptr(), arr, nsrc, blk, h) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif not torch.equal(ref, out):
                raise SystemExit(f"tree variant {v} nsrc={nsrc} WRONG")
        times = {v: [] for v in variants}
        for _ in range(args.tune_rounds):
            for v in variants:
                evs = [(torch.cuda.Event(enable_timing=True),
                        torch.cuda.Event(enable_timing=True)) for _ in range(10)]
                for i, (a, b) in enumerate(evs):
                    srcs, out, arr = sets[i % 2]
                    a.record()
                    L.lfa__tune_tree_f32(v, out.data_ptr(), arr, nsrc, blk, h)
                    b.record()
                torch.cuda.synchronize()
                times[v].extend(a.elapsed_time(b) for a, b in evs[2:])
        for v in variants:
            ms = statistics.median(times[v])
            gbps = (nsrc + 1) * blk * 4 / (ms * 1e-3) / 1e9
            rows.append({"nsrc": nsrc, "variant": v, "median_us": round(ms * 1e3, 2),
                         "gbs": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4)})
        del sets
        torch.cuda.empty_cache()
    print(json.dumps({"tune_tree": rows}))


def tune_treeput(args) -> None:
    """A/B of reduce_tree_put forms on LOCAL memory (float SUM, 8 x 32 MiB
    inputs -> 1 and 8 outputs): the product vs variants without system-scope
    bits or with other tiling (lfa__tune_treeput_f32, liblfa_tune.so)."""
    import ctypes
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    h = torch.cuda.current_stream().cuda_stream
    nsrc, blk = 8, 32 * 1024 * 1024 // 4
    variants = ([int(x) for x in args.variants.split(",")] if args.variants
                else [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
    # --treeput-layout skew: every input and output block in one allocation,
    # block k at k * (B + 6 KiB) (the collective's slot skew);
    # sep: separate allocations (adjacent 32 MiB blocks, the same HBM
    # channels at the same offset)
    skew = args.treeput_layout == "skew"
    rows = []
    nsets = args.tune_sets
    for ndst in [int(x) for x in args.tune_ndst.split(",")]:
        sets = []
        for _ in range(nsets):
            if skew:
                pitch = blk * 4 + 6144
                pool = torch.empty((nsrc + ndst) * pitch, dtype=torch.uint8, device="cuda")
                blocks = [pool[k * pitch:k * pitch + blk * 4].view(torch.float32)
                          for k in range(nsrc + ndst)]
                for b in blocks[:nsrc]:
                    b.uniform_()
                srcs, dsts = blocks[:nsrc], blocks[nsrc:]
            else:
                pool = None
                srcs = [torch.rand(blk, device="cuda") for _ in range(nsrc)]
                dsts = [torch.empty(blk, device="cuda") for _ in range(ndst)]
            sets.append((srcs, dsts, (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs]),
                         (ctypes.c_void_p * ndst)(*[t.data_ptr() for t in dsts]), pool))
        ref = None
        for v in variants:
            srcs, dsts, sa, da, _ = sets[0]
            for d in dsts:
                d.fill_(float("nan"))         # a form that wrote nothing fails
            torch.cuda.synchronize()
            assert L.lfa__tune_treeput_f32(v, da, ndst, sa, nsrc, blk, h) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = dsts[0].clone()
            elif not all(torch.equal(ref, d) for d in dsts):
                raise SystemExit(f"treeput variant {v} ndst={ndst} WRONG")
        times = {v: [] for v in variants}
        for _ in range(args.tune_rounds):
            for v in variants:
                evs = [(torch.cuda.Event(enable_timing=True),
                        torch.cuda.Event(enable_timing=True)) for _ in range(10)]
                for i, (a, b) in enumerate(evs):
                    srcs, dsts, sa, da, _ = sets[i % nsets]
                    a.record()
                    L.lfa__tune_treeput_f32(v, da, ndst, sa, nsrc, blk, h)
                    b.record()
                torch.cuda.synchronize()
                times[v].extend(a.elapsed_time(b) for a, b in evs[2:])
        for v in variants:
            ms = statistics.median(times[v])
            gbps = (nsrc + ndst) * blk * 4 / (ms * 1e-3) / 1e9
            rows.append({"ndst": ndst, "variant": v, "layout": args.treeput_layout,
                         "median_us": round(ms * 1e3, 2),
                         "gbs": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4)})
        del sets
        torch.cuda.empty_cache()
    print(json.dumps({"tune_treeput": rows}))


def tune_tree_layout(args) -> None:
    """Where the N input blocks sit in HBM, for the product tree kernel
    (float SUM, 8 x 32 MiB): separate allocations; one contiguous workspace
    (the collective's layout: block k at ws + k*B); and the contiguous
    workspace with block k skewed by k*skew bytes."""
    import ctypes
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    h = torch.cuda.current_stream().cuda_stream
    nsrc, blk = 8, 32 * 1024 * 1024 // 4
    layouts = {"separate": None}
    for sk in (args.skews.split(",") if args.skews else
               ["0", "256", "4096", "4352", "65536", "1048576"]):
        layouts[f"skew_{int(sk)}"] = int(sk)
    sets = {}
    for name, skew in layouts.items():
        per = []
        for _ in range(2):
            if skew is None:
                srcs = [torch.rand(blk, device="cuda") for _ in range(nsrc)]
                ptrs = [t.data_ptr() for t in srcs]
                keep = srcs
            else:
                stride = blk * 4 + skew
                ws = torch.rand((stride * nsrc) // 4 + 1024, device="cuda")
                ptrs = [ws.data_ptr() + k * stride for k in range(nsrc)]
                keep = ws
            per.append((keep, torch.empty(blk, device="cuda"),
                        (ctypes.c_void_p * nsrc)(*ptrs)))
        sets[name] = per
    times = {n: [] for n in layouts}
    for _ in range(args.tune_rounds):
        for name in layouts:
            evs = [(torch.cuda.Event(enable_timing=True),
                    torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for i, (a, b) in enumerate(evs):
                _, out, arr = sets[name][i % 2]
                a.record()
                L.lfa__tune_tree_f32(-1, out.data_ptr(), arr, nsrc, blk, h)
                b.record()
            torch.cuda.synchronize()
            times[name].extend(a.elapsed_time(b) for a, b in evs[2:])
    rows = []
    for name in layouts:
        ms = statistics.median(times[name])
        gbps = (nsrc + 1) * blk * 4 / (ms * 1e-3) / 1e9
        rows.append({"layout": name, "median_us": round(ms * 1e3, 2),
                     "gbs": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4)})
    print(json.dumps({"tune_tree_layout": rows}))


def sweep_ops(args) -> None:
    """Every (op, datatype) of the write table at 256 MiB: kernel time and
    fraction of the HBM roofline (3·S bytes per launch)."""
    from libfabric_amd import atomic
    import oracle
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    nbytes = S_BYTES
    sets = [(torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda"),
             torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda"))
            for _ in range(3)]
    rows = []
    for opname, op in oracle.OPS.items():
        for dtname, (dt, _) in oracle.DATATYPES.items():
            if not oracle.has_handler(op, dt):
                continue
            cnt = nbytes // oracle.datatype_size(dt)

            def fn(i, op=op, dt=dt, cnt=cnt):
                d, s = sets[i % 3]
                atomic.write(op, dt, d, s, cnt, stream)
            for i in range(6):
                fn(i)
            ms = _kernel_events(fn, 12, stream)
            gbps = 3 * nbytes / (ms * 1e-3) / 1e9
            rows.append({"op": opname, "dt": dtname, "us": round(ms * 1e3, 1),
                         "frac": round(gbps / PEAK_GBPS, 3)})
    print(json.dumps({"sweep_ops": rows}))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true", help="skip cpu_baseline")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--tune-rounds", type=int, default=10)
    ap.add_argument("--variants", default="", help="comma list for --tune")
    ap.add_argument("--tune-bytes", type=int, default=S_BYTES)
    ap.add_argument("--tune-tree", action="store_true")
    ap.add_argument("--tune-tree-layout", action="store_true")
    ap.add_argument("--tune-ndst", default="1,8",
                    help="--tune-treeput: output counts to time (8 inputs each)")
    ap.add_argument("--tune-sets", type=int, default=2,
                    help="--tune-treeput: buffer sets rotated (each 9 or 16 x 32 MiB)")
    ap.add_argument("--tune-treeput", action="store_true")
    ap.add_argument("--treeput-layout", choices=("sep", "skew"), default="sep",
                    help="--tune-treeput: separate allocations or one skewed pool")
    ap.add_argument("--skews", default="", help="comma list of byte skews")
    ap.add_argument("--sweep-ops", action="store_true")
    ap.add_argument("--only-extra", default="", help="run one extra: tree_put, host_rs, config3, sizes, fetch, buckets (dev); "
                    "crossover (the one-shot / tree crossover child), "
                    "coll (the isolated N>1 provider extras, started by run_isolated)")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-extras-coll", action="store_true",
                    help="skip the provider (RCCL) extras at N=1")
    ap.add_argument("--extras-timeout", type=float, default=300.0)
    ap.add_argument("--sizes-reps", type=int, default=100,
                    help="--only-extra sizes: timed launches per size")
    ap.add_argument("--prewarm-s", type=float, default=0.25,
                    help="untimed clock-ramp launches before the W warmup steps (s)")
    args = ap.parse_args()

    if args.tune:
        tune(args)
        return
    if args.tune_tree_layout:
        tune_tree_layout(args)
        return
    if args.tune_treeput:
        tune_treeput(args)
        return
    if args.tune_tree:
        tune_tree(args)
        return
    if args.sweep_ops:
        sweep_ops(args)
        return
    if args.only_extra == "host_rs":
        from libfabric_amd import coll
        torch.cuda.set_device(0)
        ep = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
        try:
            print(json.dumps({"host_rs": extra_host_reduce_scatter(ep, 0, 1),
                              "host_allreduce": extra_host_allreduce(ep, 1, sweep=True)}))
        finally:
            ep.close()
        return
    if args.only_extra == "config3":
        torch.cuda.set_device(0)
        print(json.dumps({"config3": extra_config3(torch.device("cuda", 0),
                                                   torch.cuda.current_stream())}))
        return
    if args.only_extra == "sizes":
        torch.cuda.set_device(0)
        print(json.dumps({"sizes": extra_sizes(torch.device("cuda", 0),
                                               torch.cuda.current_stream(),
                                               args.sizes_reps, args.prewarm_s)}))
        return
    if args.only_extra == "fetch":
        torch.cuda.set_device(0)
        print(json.dumps({"fetch": extra_fetch_tables(torch.device("cuda", 0),
                                                      torch.cuda.current_stream())}))
        return
    if args.only_extra == "buckets":
        torch.cuda.set_device(0)
        print(json.dumps({"buckets_two_streams": extra_two_streams(
            torch.device("cuda", 0), [COUNT // 8])}))
        return
    if args.only_extra == "tree_put":
        torch.cuda.set_device(0)
        print(json.dumps({"tree_put": extra_tree_put(torch.device("cuda", 0),
                                                     torch.cuda.current_stream())}))
        return

    if args.gpus > 1 and "RANK" not in os.environ:
        # Self-launch: one process per GPU, before this process touches one.
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__),
                                          *sys.argv[1:]]))
    rank, world, local = init_dist(args.gpus)
    from libfabric_amd import lib
    lib()  # no fallback: raises if liblfa.so is missing
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()
    if args.only_extra in ("coll", "crossover"):
        # the isolated child of run_isolated: the provider extras only
        def show(o):
            if rank == 0:
                print(json.dumps(o), flush=True)
                log(f"bench.py: provider extras rows so far: {len(o)}")
        try:
            if args.only_extra == "crossover":
                show({"oneshot_crossover": extra_oneshot_crossover(
                    rank, world, lambda o: show({"oneshot_crossover": o}))})
            else:
                extra_collectives(rank, world, stream, show)
        except Exception as e:  # noqa: BLE001
            show({"error": f"{type(e).__name__}: {e}"[:300]})
        finally:
            if world > 1:
                bye = threading.Timer(60.0, lambda: os._exit(0))
                bye.daemon = True
                bye.start()
                dist.destroy_process_group()
        return

    # Headline: every rank its own 256 MiB buffer pair per step (weak: the
    # combine partitions with no exchange, so N GPUs do N independent units).
    cnt = COUNT
    r = timed_combine(dev, stream, cnt, 1000 + rank, args, world)
    elapsed, kern_ms, kern_med = r["elapsed"], r["kern_ms"], r["kern_med"]
    shard_bytes = cnt * 4
    value = 3 * S_BYTES * world * args.steps / elapsed / 2**30
    achieved = 3 * shard_bytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = read_traffic()

    line = {
        "metric": "device-resident GiB/s, float32 FI_SUM reduce, 256 MiB buffers",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform[-1,1) float32, torch.Generator seeds 1000+rank)",
        "config": {
            "workload": "float32 FI_SUM local combine of one 256 MiB device-resident "
                        "buffer pair per step (BASELINE.json configs[1]), dst += src "
                        "through lfa_atomic_write_async; at N>1 every GPU combines its "
                        "own pair per step, no exchange (weak; SURVEY §8(e))",
            "count": COUNT, "buffer_bytes": S_BYTES,
            "bytes_per_gpu_per_step": 3 * shard_bytes,
            "buffer_sets": r["nsets"],
            "bytes_per_step": 3 * S_BYTES * world,
            "buffer_rate_gib_s": round(S_BYTES * world * args.steps / elapsed / 2**30, 2),
            "prewarm_launches": r["prewarm"],
            "parallelism": f"dp{world} (one independent 256 MiB pair per GPU, no exchange)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_GBPS, 4),
            "traffic": traffic,
            "kernel": "combine_lds<FI_SUM,float,U=4> (LDS-DMA staged; nt stores at "
                      ">= 192 MiB per operand, sc1 write-through below)",
            "kernel_us": round(kern_ms * 1e3, 2),
            "kernel_us_isolated_median": round(kern_med * 1e3, 2),
            "timing": "HIP event pair around the timed region on the launch stream, "
                      "divided by steps (includes inter-kernel dispatch gaps), max over "
                      "ranks; isolated per-launch event median beside it; rocprofv3 "
                      "kernel-trace summary in profiles/",
            "algorithmic_bytes_per_launch": 3 * shard_bytes,
            "traffic_source": traffic_src,
            # HBM's own rate for this 2-read/1-write mix, measured apart
            # (tools/probe_hbm.py): the practical ceiling beside the 8 TB/s spec
            "access_mix_ceiling": {
                "gb_s": ACCESS_MIX_CEILING_GBPS,
                "frac": round(achieved / ACCESS_MIX_CEILING_GBPS, 4),
                "source": "reads 7.00 TB/s, writes 6.32 TB/s alone; 3/(2/7.00+1/6.32) "
                          "(profiles/r02_probe_hbm_access_mix.log)"},
        },
    }
    if REHEARSE:
        line["rehearsal"] = "LFA_BENCH_REHEARSE: ranks share GPUs; not a measurement"
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.cpu_reps)
        line["cpu_baseline"]["config3_int64_64mib"] = cpu_baseline_config3(args.cpu_reps)
        line["cpu_baseline"]["config1_2rank_4kib_allreduce_host"] = cpu_config1_peer()
        line["cpu_baseline"]["config5_double_prod"] = cpu_baseline_config5()

    # Extras (never the headline).  A watchdog prints the line collected so
    # far and exits if an extra stalls, so the metric is always reported.
    def _emit(note=None):
        if note:
            line.setdefault("extras", {})["status"] = note
        if rank == 0:
            print(json.dumps(line), flush=True)

    def _overrun():
        if _CHILD is not None:
            _CHILD.kill()
        _emit("extras timed out")
        os._exit(0)

    if not args.no_extras:
        torch.cuda.empty_cache()
        t_extras = time.time()
        wd = threading.Timer(args.extras_timeout, _overrun)
        wd.daemon = True
        wd.start()
        ex = line.setdefault("extras", {})
        try:
            if world > 1:
                strong_scaling(line, dev, stream, args, world, rank)
            # independent buckets two streams at a time, at this rank's
            # shard (and at N = 1 at the N = 8 shard, 32 MiB) — only below
            # 192 MiB per operand: at 256 MiB two streams contend and lose
            # (tools/probe_streams.py), and the headline kernel's rocprofv3
            # statistics stay those of the one-stream headline
            ex["buckets_two_streams"] = extra_two_streams(
                dev, [c for c in [shard_of(COUNT, world, rank)[1]] + ([COUNT // 8] if world == 1 else [])
                      if c * 4 < (192 << 20)])
            torch.cuda.empty_cache()
            if world == 1:
                ex["config3_int64_64mib"] = extra_config3(dev, stream)
                ex["config1_2rank_4kib_loopback"] = extra_config1_loopback(dev, stream)
                ex["config1_2rank_4kib_two_processes"] = extra_config1_two_process()
                ex["tree8_fused_combine"] = extra_tree(dev, stream)
                ex["tree8_put_p2p_kernel_local"] = extra_tree_put(dev, stream)
                ex["fetch_compare_tables_256mib"] = extra_fetch_tables(dev, stream)
                ex["e2e_host_float_sum_256mib"] = extra_e2e_host(dev, stream)
                ex["e2e_host_staged_float_sum_256mib"] = extra_e2e_staged()
            if world > 1:
                # first N-GPU run of the transports: in a child job, so a
                # fault there cannot take the headline with it
                budget = args.extras_timeout - (time.time() - t_extras) - 20.0
                ex.update(run_isolated(
                    [sys.executable, os.path.abspath(__file__), "--gpus", str(world),
                     "--only-extra", "coll"], rank, world, max(budget - 60.0, 10.0)))
                # the one-shot / tree crossover per bucket, with the one-shot
                # bounds lifted in that child only
                budget = args.extras_timeout - (time.time() - t_extras) - 20.0
                if budget > 20.0:
                    res = run_isolated(
                        [sys.executable, os.path.abspath(__file__), "--gpus", str(world),
                         "--only-extra", "crossover"], rank, world, budget,
                        {"LFA_OS_AG_BYTES": str(OS_CROSSOVER_BOUND),
                         "LFA_OS_RS_BYTES": str(OS_CROSSOVER_BOUND)})
                    ex["oneshot_crossover"] = res.get("oneshot_crossover", res)
                    if "isolated_status" in res:
                        ex["oneshot_crossover"]["isolated_status"] = res["isolated_status"]
                    # the same buckets through P2P's two-barrier schedule
                    # (both bounds at 1 byte), AUTO's choice above the bounds
                    budget = args.extras_timeout - (time.time() - t_extras) - 20.0
                    if budget > 20.0:
                        bres = run_isolated(
                            [sys.executable, os.path.abspath(__file__), "--gpus", str(world),
                             "--only-extra", "crossover"], rank, world, budget,
                            {"LFA_OS_AG_BYTES": "1", "LFA_OS_RS_BYTES": "1"})
                        merge_crossover(ex["oneshot_crossover"],
                                        bres.get("oneshot_crossover", bres), world)
            elif not args.no_extras_coll:
                ex.update(extra_collectives(rank, world, stream))
        except Exception as e:  # noqa: BLE001 — extras must not hide the metric
            ex["error"] = f"{type(e).__name__}: {e}"[:300]
        wd.cancel()
    _emit()
    if world > 1:
        # The line is out; a peer stuck in a collective must not hold this
        # rank in teardown past the driver's clock.
        bye = threading.Timer(60.0, lambda: os._exit(0))
        bye.daemon = True
        bye.start()
        dist.destroy_process_group()


def strong_scaling(line, dev, stream, args, world, rank) -> None:
    """Strong scaling beside the weak headline, with equal prominence
    (ADVICE r5), at the top level of the line.  Timed first among the
    extras, under their watchdog, so a stalled rank cannot keep the line from
    printing.  ONE 256 MiB pair per step split into N contiguous 4 KiB-aligned
    shards (BASELINE configs[3]'s "8 GPUs each combine S/8").
    Rounds 1-4 reported THIS as `value`; since round 5 `value` is the weak
    form (the tier's rule for a path that partitions), so rounds compare on
    the matching field."""
    off, scnt = shard_of(COUNT, world, rank)
    w = timed_combine(dev, stream, scnt, 2000 + rank, args, world)
    line["strong_scaling"] = {
        "value": round(3 * S_BYTES * args.steps / w["elapsed"] / 2**30, 2),
        "unit": "GiB/s", "scaling": "strong",
        "ms_per_step": round(w["elapsed"] / args.steps * 1e3, 4),
        "workload": "one 256 MiB float32 pair per step, sharded over the N GPUs",
        "shard_bytes_per_gpu": scnt * 4,
        "kernel_us": round(w["kern_ms"] * 1e3, 2),
        "frac": round(3 * scnt * 4 / (w["kern_ms"] * 1e-3) / 1e9 / PEAK_GBPS, 4),
        "traffic": read_traffic_shard(scnt * 4)[0]}
    line["scaling_note"] = ("value: weak (every GPU its own 256 MiB pair per step) since "
                            "round 5; rounds 1-4 reported the strong form, now "
                            "strong_scaling.value")
    torch.cuda.empty_cache()


def timed_combine(dev, stream, count: int, seed: int, args, world: int) -> dict:
    """The bench step on this rank: float FI_SUM combine of `count` elements,
    rotating over enough buffer pairs to defeat the MALL.  W warmup launches
    (after a short time-based clock prewarm), then EXACTLY K timed launches
    between a barrier + synchronize on both sides; wall time and the launch
    stream's event time are maxed over ranks."""
    from libfabric_amd import atomic
    sets = make_buffers(dev, seed, count)
    nsets = len(sets)

    def step(i):
        d, s = sets[i % nsets]
        atomic.write(FI_SUM, FI_FLOAT, d, s, count, stream)

    npre = prewarm(step, args.prewarm_s) if args.prewarm_s > 0 else 0
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    # Timed region: K back-to-back launches, nothing else in the queue but
    # one HIP event pair around the whole region (on the launch stream).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(t1 - t0, world)
    # roofline: average launch duration = region GPU time / K (keeps the
    # ~1 us dispatch gap between consecutive kernels in: conservative).
    kern_ms = max_over_ranks(ev0.elapsed_time(ev1) / args.steps, world)
    # Diagnostic only (not timed): per-launch event pairs, median.
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(min(args.steps, 30))]
    for i, (a, b) in enumerate(evs):
        a.record(stream)
        step(i)
        b.record(stream)
    torch.cuda.synchronize()
    durs = [a.elapsed_time(b) for a, b in evs][3:] or [kern_ms]
    del sets
    return {"elapsed": elapsed, "kern_ms": kern_ms, "kern_med": statistics.median(durs),
            "nsets": nsets, "prewarm": npre}


if __name__ == "__main__":
    main()
