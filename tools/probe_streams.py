#!/usr/bin/env python3
"""Independent buckets on one stream vs round-robin over 2 / 4 streams
(dev probe, GPU box).

On one stream every combine waits for the previous one to retire, so each
launch pays its own ramp (first loads' latency) and drain (last stores):
≈2.1 µs that a 32 MiB-per-operand launch — the N = 8 shard of the headline —
cannot hide.  Buckets that do not depend on each other (prov/coll
progresses several collectives at once) may go to different streams, where
the next launch's waves fill the CUs the previous one's are leaving.  This
probe measures the per-bucket time both ways at the headline's operand sizes:
K launches rotating over >= 1 GiB of operands, wall time between two device
synchronizes, after a clock prewarm, repeated and alternated.

Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    from libfabric_amd import atomic
    torch.cuda.set_device(0)
    sizes = [int(x) for x in (sys.argv[1:] or ["32", "64", "256"])]
    out = {}
    k = 100
    for mib in sizes:
        count = mib * (1 << 20) // 4
        nsets = max(4, (1 << 30) // (8 * count))
        sets = [(torch.rand(count, device="cuda"), torch.rand(count, device="cuda"))
                for _ in range(nsets)]
        streams = [torch.cuda.Stream() for _ in range(4)]
        torch.cuda.synchronize()

        def run(nstreams):
            for i in range(k):
                d, s = sets[i % nsets]
                atomic.write(2, 8, d, s, count, streams[i % nstreams])

        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            run(1)
        torch.cuda.synchronize()
        res = {1: [], 2: [], 4: []}
        for _ in range(10):
            for ns in (1, 2, 4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(ns)
                torch.cuda.synchronize()
                res[ns].append((time.perf_counter() - t0) / k)
        row = {}
        for ns, v in res.items():
            us = statistics.median(v) * 1e6
            row[f"{ns}_stream_us"] = round(us, 2)
            row[f"{ns}_stream_frac"] = round(3 * mib * (1 << 20) / (us * 1e-6) / 8e12, 4)
        out[str(mib)] = row
        del sets
        torch.cuda.empty_cache()
    print(json.dumps({"per_bucket_by_streams": out, "launches": k,
                      "note": "wall time / K between device synchronizes, median of 10"}),
          flush=True)


if __name__ == "__main__":
    main()
