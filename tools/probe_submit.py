#!/usr/bin/env python3
"""Where a small collective's time goes on one GPU (dev probe, GPU box).

A 4 KiB float SUM allreduce through the RCCL endpoint at world size 1 (the
schedule is one COPY) next to its parts: the bare device copy with a stream
synchronize, the combine kernel with a stream synchronize, an empty
lfa_cq_read (the progress call the wait loop spins on), and the submit call
alone.  Medians over 2000 calls after 200 warm-up calls.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med_us(fn, n=2000, warm=200):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def main() -> None:
    import torch
    from libfabric_amd import atomic, coll
    torch.cuda.set_device(0)
    a = torch.rand(1024, device="cuda")
    b = torch.empty_like(a)
    s = torch.cuda.Stream()
    out = {}

    def copy_sync():
        b.copy_(a)
        torch.cuda.current_stream().synchronize()
    out["torch_copy_4kib_sync_us"] = med_us(copy_sync)

    def combine_sync():
        atomic.write(2, 8, b, a, 1024, s)
        s.synchronize()
    out["combine_4kib_sync_us"] = med_us(combine_sync)

    def empty_launch_sync():
        s.synchronize()
    out["stream_sync_idle_us"] = med_us(empty_launch_sync)

    # host cost of one enqueue alone (the stream drained every 100 calls)
    def per_call(fn, reps=20, k=100):
        t = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            t.append((time.perf_counter() - t0) / k)
            torch.cuda.synchronize()
        return round(statistics.median(t) * 1e6, 2)
    with torch.cuda.stream(s):
        out["enqueue_torch_copy_4kib_us"] = per_call(lambda: b.copy_(a))
    out["enqueue_combine_4kib_us"] = per_call(lambda: atomic.write(2, 8, b, a, 1024, s))
    out["enqueue_copy_as_atomic_write_4kib_us"] = per_call(
        lambda: atomic.write(11, 1, b, a, 4096, s))
    cudart = ctypes.CDLL("libamdhip64.so")
    attr = ctypes.create_string_buffer(256)
    out["hipPointerGetAttributes_us"] = per_call(
        lambda: cudart.hipPointerGetAttributes(attr, ctypes.c_void_p(a.data_ptr())))
    hs = ctypes.c_void_p(s.cuda_stream)
    out["enqueue_hipMemcpyAsync_d2d_4kib_us"] = per_call(
        lambda: cudart.hipMemcpyAsync(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                      ctypes.c_size_t(4096), 3, hs))
    ev = ctypes.c_void_p()
    cudart.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    out["enqueue_hipEventRecord_us"] = per_call(lambda: cudart.hipEventRecord(ev, hs))

    ep = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    try:
        torch.cuda.synchronize()
        out["allreduce_4kib_wait_us"] = med_us(lambda: ep.wait(ep.allreduce(a, b, 1024, 8, 2)))
        out["cq_read_empty_us"] = med_us(lambda: ep.cq_read())
        L = coll.lib()
        ents = (coll.CqEntry * 1)()
        out["lfa_cq_read_empty_raw_us"] = med_us(lambda: L.lfa_cq_read(ep.ep, ents, 1))
        ctxs = []

        def submit():
            ctxs.append(ep.allreduce(a, b, 1024, 8, 2))
        t = []
        for _ in range(20):
            ctxs.clear()
            t0 = time.perf_counter()
            for _ in range(100):
                submit()
            t.append((time.perf_counter() - t0) / 100)
            done = []
            while len(done) < len(ctxs):
                done += ep.cq_read(128)
        out["allreduce_submit_only_us"] = round(statistics.median(t) * 1e6, 2)
    finally:
        ep.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
