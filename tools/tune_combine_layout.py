#!/usr/bin/env python3
"""Where dst and src sit relative to each other, for the product combine
(float FI_SUM, lfa_atomic_write_async) — dev probe, GPU box.

The elementwise combine reads d[i] and s[i] together, so the distance
src - dst decides whether the two streams meet on the same HBM channels and
banks at the same time.  Layouts, each rotated over >= 1 GiB of sets:
  separate      two torch allocations per set (what bench.py does)
  gap_<k>       one allocation per set, src = dst + S + k bytes
Per operand size (256 MiB and the 32 MiB strong-scaling shard): one HIP
event pair around 40 back-to-back launches, median of rounds, interleaved.
"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from libfabric_amd import atomic  # noqa: E402

GAPS = [0, 4096, 6144, 12288, 65536, 1 << 20, (1 << 20) + 6144, 2 << 20]


def main() -> None:
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    rows = []
    for mib in (256, 32):
        nbytes = mib << 20
        count = nbytes // 4
        nsets = max(4, (1 << 30) // (2 * nbytes))
        layouts = {}
        keep = []
        sets = []
        for _ in range(nsets):
            a, b = torch.rand(count, device="cuda"), torch.rand(count, device="cuda")
            keep.append((a, b))
            sets.append((a.data_ptr(), b.data_ptr()))
        layouts["separate"] = sets
        for gap in GAPS:
            sets = []
            for _ in range(nsets):
                ws = torch.rand((2 * nbytes + gap) // 4, device="cuda")
                keep.append(ws)
                sets.append((ws.data_ptr(), ws.data_ptr() + nbytes + gap))
            layouts[f"gap_{gap}"] = sets
        times = {k: [] for k in layouts}
        for rnd in range(12):
            for name, sets in layouts.items():
                def step(i):
                    d, s = sets[i % len(sets)]
                    assert atomic.write_ptr(2, 8, d, s, count, stream) == 0
                reps = 40
                for i in range(8):
                    step(i)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(reps):
                    step(i)
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[name].append(e0.elapsed_time(e1) / reps)
        for name in layouts:
            ms = statistics.median(times[name])
            rows.append({"operand_mib": mib, "layout": name, "us": round(ms * 1e3, 2),
                         "frac": round(3 * nbytes / (ms * 1e-3) / 8e12, 4)})
            print(json.dumps(rows[-1]), flush=True)
        del keep, layouts, sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
