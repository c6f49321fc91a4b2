#!/usr/bin/env python3
"""Per-step cost of back-to-back combines: stream launches vs one HIP graph
(dev probe, GPU box).

bench.py's step is one lfa_atomic_write_async launch.  Between two launches
on one stream the GPU idles for the kernel boundary (completion signal,
barrier, next dispatch).  A HIP graph of the same K launches replays the
identical kernels with the launch work done once; this probe measures what
that boundary costs per step at the operand sizes the headline uses
(256 MiB at N = 1, 32 MiB per GPU at N = 8) and between.

Prints one JSON line per (operand size, form, K).
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
    sizes = [int(x) for x in (sys.argv[1:] or ["256", "128", "64", "32"])]
    for mib in sizes:
        count = mib * (1 << 20) // 4
        nsets = max(4, (1 << 30) // (8 * count))
        sets = [(torch.rand(count, device="cuda"), torch.rand(count, device="cuda"))
                for _ in range(nsets)]
        for k in (20, 100):
            side = torch.cuda.Stream()

            def launches(stream, base=0):
                for i in range(k):
                    d, s = sets[(base + i) % nsets]
                    atomic.write(2, 8, d, s, count, stream)

            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                launches(side)          # warm the launch path on this stream
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=side):
                launches(torch.cuda.current_stream())
            torch.cuda.synchronize()
            stream = torch.cuda.current_stream()
            # clock prewarm
            t = time.perf_counter()
            while time.perf_counter() - t < 0.3:
                launches(stream)
            torch.cuda.synchronize()
            res = {"stream": [], "graph": []}
            for rep in range(15):
                for form in ("stream", "graph"):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record(stream)
                    if form == "stream":
                        launches(stream, rep)
                    else:
                        g.replay()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res[form].append(e0.elapsed_time(e1) * 1e3 / k)
            for form, v in res.items():
                us = statistics.median(v)
                print(json.dumps({"mib": mib, "k": k, "form": form,
                                  "us_per_step": round(us, 2),
                                  "p10_p90": [round(x, 2) for x in
                                              statistics.quantiles(v, n=10)[::8]],
                                  "frac_of_8tbs": round(3 * mib * (1 << 20) / (us * 1e-6)
                                                        / 8e12, 4)}), flush=True)
            del g
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
