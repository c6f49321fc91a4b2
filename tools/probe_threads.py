"""Host-buffer combines from several threads at once.

For each size: the median of 7 single calls, then 4 threads calling at
once (median of 5 rounds), for pageable operands (registered per call),
pinned operands (no registration) and, with --staged, LFA_HOST_ZERO_COPY=0
(the chunked H2D / kernel / D2H pipeline).  Per-thread durations too, to
see whether calls overlap or queue.  One JSON line per (kind, size).

  python tools/probe_threads.py [--sizes 2,8,32] [--threads 4]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2,8,32")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--pre-alloc-gib", type=int, default=0,
                    help="hold this much device memory first (torch), as a test process does")
    ap.add_argument("--kinds", default="pageable,pinned")
    a = ap.parse_args()
    import numpy as np
    import torch
    from libfabric_amd import atomic, lib
    lib()
    torch.cuda.init()
    hold = (torch.empty(a.pre_alloc_gib << 30, dtype=torch.uint8, device="cuda")
            if a.pre_alloc_gib else None)
    fn = atomic.write_handler(2, 8)
    T = a.threads
    for mib in (int(x) for x in a.sizes.split(",")):
        n = (mib << 20) // 4
        for kind in a.kinds.split(","):
            if kind == "pinned":
                bufs = [(torch.rand(n).pin_memory().numpy(), torch.rand(n).pin_memory().numpy())
                        for _ in range(T)]
            else:
                bufs = [(np.random.rand(n).astype(np.float32), np.random.rand(n).astype(np.float32))
                        for _ in range(T)]
            # warm every staging slot: T threads once
            def one(k, out=None):
                t0 = time.perf_counter()
                fn(bufs[k][0].ctypes.data, bufs[k][1].ctypes.data, n)
                if out is not None:
                    out[k] = time.perf_counter() - t0
            singles = []
            for _ in range(7):
                t0 = time.perf_counter()
                one(0)
                singles.append(time.perf_counter() - t0)
            walls, per = [], []
            for rep in range(6):
                out = [0.0] * T
                bar = threading.Barrier(T + 1)

                def run(k):
                    bar.wait()
                    one(k, out)
                ts = [threading.Thread(target=run, args=(k,)) for k in range(T)]
                for t in ts:
                    t.start()
                bar.wait()
                t0 = time.perf_counter()
                for t in ts:
                    t.join()
                w = time.perf_counter() - t0
                if rep:             # rep 0 creates the other staging slots
                    walls.append(w)
                    per.append(max(out))
            s1 = statistics.median(singles)
            wm = statistics.median(walls)
            print(json.dumps({"kind": kind, "mib": mib, "threads": T,
                              "one_call_ms": round(s1 * 1e3, 3),
                              "threads_wall_ms": round(wm * 1e3, 3),
                              "slowest_thread_call_ms": round(statistics.median(per) * 1e3, 3),
                              "ratio_to_one": round(wm / s1, 2),
                              "walls_ms": [round(w * 1e3, 3) for w in walls],
                              "pre_alloc_gib": a.pre_alloc_gib,
                              "zero_copy": os.environ.get("LFA_HOST_ZERO_COPY", "1")}),
                  flush=True)


if __name__ == "__main__":
    main()
