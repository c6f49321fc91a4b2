"""bench.py's N-rank launch and sharding, on CPU (no GPU call is made).

`python bench.py --gpus N` without RANK in the environment must start N rank
processes itself (the driver may invoke it that way), each with the
torch.distributed.run environment, and a job whose world size differs from
--gpus must fail instead of reporting n_gpus = 1.
"""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

_STUB = (
    "import json, os, sys\n"
    "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT',\n"
    "        'HSA_ENABLE_IPC_MODE_LEGACY']\n"
    "d = {k: os.environ.get(k) for k in keys}\n"
    "open(os.path.join(sys.argv[1], 'rank%s.json' % d['RANK']), 'w').write(json.dumps(d))\n"
)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_launch_starts_n_ranks(tmp_path, n):
    rc = bench.launch_ranks(n, [sys.executable, "-c", _STUB, str(tmp_path)], timeout_s=60)
    assert rc == 0
    seen = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(n)]
    assert [int(d["RANK"]) for d in seen] == list(range(n))
    assert [int(d["LOCAL_RANK"]) for d in seen] == list(range(n))
    assert {d["WORLD_SIZE"] for d in seen} == {str(n)}
    assert {d["MASTER_ADDR"] for d in seen} == {"127.0.0.1"}
    assert len({d["MASTER_PORT"] for d in seen}) == 1
    assert {d["HSA_ENABLE_IPC_MODE_LEGACY"] for d in seen} == {"0"}


def test_launch_failed_rank_stops_peers():
    # rank 1 fails at once; rank 0 would sleep a minute and must be stopped
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)\n")
    t0 = time.time()
    rc = bench.launch_ranks(2, [sys.executable, "-c", code], timeout_s=120)
    assert rc == 3
    assert time.time() - t0 < 30


def test_world_size_mismatch_fails_before_gpu():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""


def test_check_world():
    bench.check_world(4, 4)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1)


@pytest.mark.parametrize("world", range(1, 9))
def test_shards_partition_the_buffer(world):
    """Contiguous, 4 KiB-aligned shards that cover [0, COUNT) exactly."""
    pos = 0
    for r in range(world):
        off, ln = bench.shard_of(bench.COUNT, world, r)
        assert off == pos
        assert off * 4 % 4096 == 0
        pos += ln
    assert pos == bench.COUNT
    # ragged sizes too
    for count in (1, 1023, 1025, 10_000_019):
        pos = 0
        for r in range(world):
            off, ln = bench.shard_of(count, world, r)
            assert off == pos or ln == 0
            pos += ln
        assert pos == count


def test_rotation_defeats_mall():
    for world in range(1, 9):
        _, ln = bench.shard_of(bench.COUNT, world, 0)
        assert bench.n_sets(ln) * 2 * ln * 4 >= (1 << 30)


def test_config3_data_distribution():
    import numpy as np
    x = bench.config3_data(3, 1 << 16)
    special = np.isin(x, [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]).sum()
    assert 0.009 < special / x.size < 0.011
    assert x.min() < -(1 << 60) and x.max() > (1 << 60)   # full range


def _xgmi_worker(rank, world, port, q):
    try:
        import os as _os
        _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        import bench
        bench.REHEARSE = True               # max over ranks on the CPU
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = bench.extra_xgmi(rank, world, device="cpu", nbytes=1 << 20)
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_xgmi_probe_flow_on_gloo():
    """bench.extra_xgmi's all-to-all and ring send/recv, run over gloo on
    CPU tensors (the flow; the numbers come from RCCL on a GPU node)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_xgmi_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
    for r in range(2):
        assert isinstance(res[r], dict), res[r]
        # the flow, not the rate: CPU tensors over gloo on a loaded machine
        # can round to 0.0 GB/s
        assert res[r]["alltoall_egress_gbs"] >= 0 and res[r]["one_link_gbs"] >= 0


_ISO_CHILD = (
    "import json, os, sys, time\n"
    "mode, rank = sys.argv[1], int(os.environ['RANK'])\n"
    "if mode == 'crash' and rank == 1:\n"
    "    os.abort()\n"
    "if mode in ('crash', 'hang'):\n"
    "    time.sleep(120)\n"
    "import torch, torch.distributed as dist\n"
    "dist.init_process_group('gloo')\n"
    "t = torch.tensor([rank + 1.0])\n"
    "dist.all_reduce(t)\n"
    "if rank == 0:\n"
    "    print(json.dumps({'partial': 1}), flush=True)\n"
    "    print(json.dumps({'sum': float(t), 'port': os.environ['MASTER_PORT'],\n"
    "                      'elastic': [k for k in os.environ if k.startswith('TORCHELASTIC_')]}),\n"
    "          flush=True)\n"
    "dist.destroy_process_group()\n"
)


def _iso_worker(rank, world, port, mode, q):
    try:
        import os as _os
        _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        import bench
        dist.init_process_group("gloo", rank=rank, world_size=world)
        # as under torch.distributed.run: the child must not inherit it
        _os.environ["TORCHELASTIC_USE_AGENT_STORE"] = "True"
        t0 = time.time()
        out = bench.run_isolated([sys.executable, "-c", _ISO_CHILD, mode], rank, world,
                                 budget_s=20.0)
        dt = time.time() - t0
        dist.destroy_process_group()
        q.put((rank, (out, dt)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("mode", ["ok", "crash", "hang"])
def test_isolated_extras_child_job(mode):
    """bench.run_isolated (the N>1 provider extras' child job) over gloo:
    a fresh rendezvous that works without the elastic agent's store; rank 0's
    last JSON line comes back; a child that aborts on one rank stops every
    rank's child at once; a hung child is stopped at the budget."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_iso_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=120) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert isinstance(res[r], tuple), res[r]
    (out0, dt0), (out1, dt1) = res[0], res[1]
    if mode == "ok":
        assert out0["sum"] == 3.0 and out0["elastic"] == [] and out0["port"] != str(port)
        assert "isolated_status" not in out0 and out1 == {}
    elif mode == "crash":
        assert "code" in out1["isolated_status"]
        assert "stopped" in out0["isolated_status"]
        assert max(dt0, dt1) < 15
    else:
        assert "overran" in out0["isolated_status"] or "stopped" in out0["isolated_status"]
        assert max(dt0, dt1) < 40


def test_crossover_prices_the_one_shot_against_autos_bulk_choice():
    """The N > 1 crossover: the one-shot child's
    tree / one-shot times and the bulk child's P2P two-barrier times per
    bucket are merged, and `suggested_bound` is the largest bucket up to
    which the one-shot beats what AUTO runs above the bound — the two-barrier
    schedule by default (LFA_AUTO_BULK), not the tree."""
    out = {"allreduce": {"by_bucket_bytes_per_rank": {
               "16384": {"tree_us": 30.0, "oneshot_us": 9.0},
               "65536": {"tree_us": 40.0, "oneshot_us": 14.0},
               "262144": {"tree_us": 60.0, "oneshot_us": 20.0}}},
           "reduce_scatter": {"by_bucket_bytes_per_rank": {
               "65536": {"tree_us": 30.0, "oneshot_us": 11.0},
               "262144": {"tree_us": 9.0, "oneshot_us": 12.0}}}}
    bulk = {"allreduce": {"by_bucket_bytes_per_rank": {
                "16384": {"p2p_bulk_us": 12.0}, "65536": {"p2p_bulk_us": 13.0},
                "262144": {"p2p_bulk_us": 15.0}}},
            "reduce_scatter": {"by_bucket_bytes_per_rank": {
                "65536": {"p2p_bulk_us": 12.0}, "262144": {"p2p_bulk_us": 13.0}}},
            "isolated_status": "ok"}
    bench.merge_crossover(out, bulk, 8)
    assert out["auto_above_bound"] == "p2p_bulk"
    ar, rs = out["allreduce"], out["reduce_scatter"]
    assert ar["by_bucket_bytes_per_rank"]["65536"]["p2p_bulk_us"] == 13.0
    # allreduce: the one-shot wins at 16 KiB only (14 > 13 at 64 KiB), although
    # it beats the tree everywhere; the knob is summed over the 8 members
    assert ar["oneshot_wins_up_to_bytes_per_rank"] == 16384
    assert ar["suggested_bound"] == 8 * 16384 and ar["priced_against"] == "p2p_bulk"
    # reduce_scatter: the one-shot beats the two-barrier schedule at 256 KiB
    # too (12 < 13), even where the tree is faster still
    assert rs["oneshot_wins_up_to_bytes_per_rank"] == 262144
    assert rs["suggested_bound"] == 262144
    assert out["bulk_isolated_status"] == "ok"


def test_crossover_keeps_the_tree_pricing_without_the_bulk_child():
    """A bulk child that failed (no two-barrier rows) leaves the first
    child's tree-priced bound as it was, with its status on the line."""
    out = {"allreduce": {"by_bucket_bytes_per_rank": {
               "16384": {"tree_us": 30.0, "oneshot_us": 9.0},
               "65536": {"tree_us": 40.0, "oneshot_us": 14.0}}}}
    bench.merge_crossover(out, {"isolated_status": "rank 1: child exited with code 1"}, 4)
    ar = out["allreduce"]
    assert ar["priced_against"] == "tree"
    assert ar["oneshot_wins_up_to_bytes_per_rank"] == 65536
    assert ar["suggested_bound"] == 4 * 65536
    assert out["bulk_isolated_status"].startswith("rank 1")
