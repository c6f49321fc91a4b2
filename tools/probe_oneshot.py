#!/usr/bin/env python3
"""GPU time of LFA_ALGO_P2P's small-bucket forms, one process (dev probe).

Two "ranks" live in one process on one MI355X, each with its own symmetric
workspace and its own stream (so their kernels run concurrently, as on two
GPUs).  Per iteration every rank enqueues either

  oneshot  one lfa_oneshot_reduce_async launch (push, flags, tree), or
  4-step   the form it replaces: copy into the own workspace, flag barrier,
           tree_put over every rank's workspace, flag barrier,

and the per-iteration GPU time of each stream (one HIP event pair around K
iterations, enqueued while a sleep kernel holds the stream, so the launches
run back to back) is reported for float SUM allreduce of 4 KiB .. 256 KiB.  Not
xGMI: the peers' workspaces are this GPU's HBM, so this is the kernels' own
cost (launch, fences, flag round trips through HBM), not link latency.
Every result is checked against the two-input sum.  Waits are bounded
(2 s), so a schedule that could not make progress ends in an error flag,
not a hang.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    from libfabric_amd import lib
    from libfabric_amd.coll import OneShot
    L = lib()
    L.lfa_oneshot_reduce_async.argtypes = [ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(OneShot), ctypes.c_void_p]
    L.lfa_flag_barrier_async.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p]
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.set_device(0)
    n, k_iters = 2, 200
    region = 8 << 20
    flag_off = 2 * region
    from libfabric_amd.coll import sig_area_bytes
    ws = [torch.zeros(2 * region + sig_area_bytes(), dtype=torch.uint8, device="cuda")
          for _ in range(n)]
    sym = (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws])
    status = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(status), ctypes.c_size_t(8), 0x40000000) == 0
    ctypes.c_uint64.from_address(status.value).value = 0xFFFFFFFFFFFFFFFF   # LFA_SIG_NONE
    streams = [torch.cuda.Stream() for _ in range(n)]
    torch.cuda.synchronize()
    out = {}
    epoch = [0]
    bar = [0]

    def oneshot(r, x, y, count):
        a = OneShot(x[r].data_ptr(), y[r].data_ptr(), count, -1,
                    ctypes.cast(sym, ctypes.c_void_p), (count * 4 + 255) // 256 * 256,
                    region // 2, flag_off, n, r, epoch[0], status.value, 1, 2_000_000)
        assert L.lfa_oneshot_reduce_async(2, 8, ctypes.byref(a),
                                          ctypes.c_void_p(streams[r].cuda_stream)) == 0

    def barrier(r):
        post = (ctypes.c_void_p * n)(*[0 if k == r else ws[k].data_ptr() + flag_off + 4 * r
                                       for k in range(n)])
        assert L.lfa_flag_barrier_async(post, ctypes.c_void_p(ws[r].data_ptr() + flag_off), n,
                                        r, bar[0], status.value, 1, 2_000_000,
                                        ctypes.c_void_p(streams[r].cuda_stream)) == 0

    def four_step(r, x, y, count):
        nb = count * 4
        with torch.cuda.stream(streams[r]):
            ws[r][:nb].copy_(x[r].view(torch.uint8))
        barrier(r)
        srcs = (ctypes.c_void_p * n)(*[x[k].data_ptr() if k == r else ws[k].data_ptr()
                                       for k in range(n)])
        dsts = (ctypes.c_void_p * 1)(y[r].data_ptr())
        assert L.lfa_reduce_tree_put_async(2, 8, dsts, 1, srcs, n, count,
                                           ctypes.c_void_p(streams[r].cuda_stream)) == 0

    for nbytes in (4096, 65536, 131072):
        count = nbytes // 4
        x = [torch.rand(count, device="cuda") for _ in range(n)]
        y = [torch.zeros(count, device="cuda") for _ in range(n)]
        want = x[1] + x[0]
        torch.cuda.synchronize()
        row = {}
        for form in ("oneshot", "4step"):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(n)]
            for it in range(k_iters + 20):
                if it == 20:
                    torch.cuda.synchronize()
                    if ctypes.c_uint64.from_address(status.value).value != 0xFFFFFFFFFFFFFFFF:
                        # a wait timed out: the streams did not run together
                        print(json.dumps({"error": f"{form} {nbytes}: wait timed out"}))
                        sys.exit(1)
                    # hold each stream in a sleep kernel while the host
                    # enqueues the K timed iterations, so the events time the
                    # GPU's work back to back, not the host's enqueue rate
                    for r in range(n):
                        with torch.cuda.stream(streams[r]):
                            torch.cuda._sleep(int(1.5e8))
                        evs[r][0].record(streams[r])
                if form == "oneshot":
                    epoch[0] += 1
                    for r in range(n):
                        oneshot(r, x, y, count)
                else:
                    bar[0] += 1
                    for r in range(n):
                        four_step(r, x, y, count)
                    bar[0] += 1
                    for r in range(n):
                        barrier(r)
            for r in range(n):
                evs[r][1].record(streams[r])
            torch.cuda.synchronize()
            us = max(evs[r][0].elapsed_time(evs[r][1]) for r in range(n)) * 1e3 / k_iters
            ok = all(torch.equal(y[r], want) for r in range(n))
            row[form] = {"us_per_op": round(us, 2), "bitwise_equal": ok}
            for r in range(n):
                y[r].zero_()
            torch.cuda.synchronize()
        out[str(nbytes)] = row
    out["timeouts"] = int(ctypes.c_uint64.from_address(status.value).value != 0xFFFFFFFFFFFFFFFF)
    print(json.dumps({"ranks_in_one_process": n, "per_op_gpu_time": out}), flush=True)


if __name__ == "__main__":
    main()
