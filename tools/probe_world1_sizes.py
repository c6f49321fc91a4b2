#!/usr/bin/env python3
"""World-1 reducing collectives by size through the provider, timed in C
(lfa_bench_samples: submit, then lfa_cq_read until that operation's
completion): double PROD reduce_scatter, 4 KiB .. 64 MiB, median / p10 / p90
of `--reps` operations, every result checked against its input (a one-member
reduce_scatter is a copy).  Prints one JSON line.  LFA_SOLO_BYTES moves the
bound between the solo copy (completion word) and the TREE plan's copy
(event)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    import torch
    from libfabric_amd import coll
    torch.cuda.set_device(0)
    ep = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    out = {}
    try:
        for nbytes in [4096 << (2 * k) for k in range(8)]:       # 4 KiB .. 64 MiB
            cnt = nbytes // 8
            x = torch.rand(cnt, device="cuda", dtype=torch.float64)
            y = torch.zeros_like(x)
            torch.cuda.synchronize()
            ep.wait(ep.reduce_scatter(x, y, cnt, 9, 3))
            torch.cuda.synchronize()
            ok = bool(torch.equal(x, y))
            s = sorted(ep.bench_samples(5, x, y, cnt, 9, 3, reps=a.reps))
            out[str(nbytes)] = {"median_us": round(statistics.median(s), 2),
                                "p10_us": round(s[len(s) // 10], 2),
                                "p90_us": round(s[9 * len(s) // 10], 2), "exact": ok}
            print(json.dumps({str(nbytes): out[str(nbytes)]}), flush=True)
    finally:
        ep.close()
    print(json.dumps({"world1_rs_us": out,
                      "solo_bytes": os.environ.get("LFA_SOLO_BYTES", "default")}), flush=True)


if __name__ == "__main__":
    main()
