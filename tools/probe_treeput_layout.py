#!/usr/bin/env python3
"""Where the 8 -> 8 reduce_tree_put's time goes on local HBM.

The product kernel (float SUM, 8 x 32 MiB inputs -> 8 outputs, the P2P
allreduce's push) timed per buffer SET rather than as a median over sets:

  sep_sets      three sets of 16 separate allocations (wherever the allocator
                puts them)
  pool_pitch    one allocation per set, block k at k * (32 MiB + s), for
                skews s from 0 to 2 MiB + 4 KiB, two pools per skew

Launches rotate over a layout's sets (1-1.5 GiB together) so the Infinity
Cache serves no reads; the median of 12 launches per set.

Same instructions, same traffic (the PMC passes show WRITE_SIZE = 8 x 32 MiB
and FETCH_SIZE x 2 = 8 x 32 MiB on every dispatch); only where the 16 streams
sit in HBM differs.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NSRC = NDST = 8
BLK = 32 << 20


def main():
    import torch
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    h = torch.cuda.current_stream().cuda_stream
    cnt = BLK // 4

    def run(sets, reps=12):
        """Launches rotate over the sets (>= 1 GiB together, so the 256 MB
        Infinity Cache serves none of a launch's reads); median per set."""
        args = [((ctypes.c_void_p * NSRC)(*[t.data_ptr() for t in srcs]),
                 (ctypes.c_void_p * NDST)(*[t.data_ptr() for t in dsts])) for srcs, dsts in sets]
        for sa, da in args:
            assert L.lfa__tune_treeput_f32(0, da, NDST, sa, NSRC, cnt, h) == 0
        evs = []
        for _ in range(reps):
            for k, (sa, da) in enumerate(args):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                L.lfa__tune_treeput_f32(0, da, NDST, sa, NSRC, cnt, h)
                b.record()
                evs.append((k, a, b))
        torch.cuda.synchronize()
        res = []
        for k in range(len(args)):
            us = statistics.median(a.elapsed_time(b) for kk, a, b in evs if kk == k) * 1e3
            res.append((round(us, 2), round((NSRC + NDST) * BLK / (us * 1e-6) / 8e12, 4)))
        return res

    out = {"sep_sets": [], "pool_pitch": {}}
    keep = []
    for _ in range(3):
        srcs = [torch.rand(cnt, device="cuda") for _ in range(NSRC)]
        dsts = [torch.empty(cnt, device="cuda") for _ in range(NDST)]
        keep.append((srcs, dsts))
    for (us, frac), (srcs, dsts) in zip(run(keep), keep):
        out["sep_sets"].append({"us": us, "frac": frac,
                                "va_mib_mod_64": [(t.data_ptr() >> 20) % 64 for t in srcs + dsts]})
    del keep
    torch.cuda.empty_cache()
    for skew in (0, 4096, 6144, 8192, 65536, 262144, (1 << 20) + 4096, (2 << 20) + 4096):
        pools, sets = [], []
        for _ in range(2):
            pitch = BLK + skew
            pool = torch.empty((NSRC + NDST) * pitch, dtype=torch.uint8, device="cuda")
            blocks = [pool[k * pitch:k * pitch + BLK].view(torch.float32)
                      for k in range(NSRC + NDST)]
            for b in blocks[:NSRC]:
                b.uniform_()
            pools.append(pool)
            sets.append((blocks[:NSRC], blocks[NSRC:]))
        out["pool_pitch"][str(skew)] = [{"us": u, "frac": f} for u, f in run(sets)]
        del sets, pools
        torch.cuda.empty_cache()
    print(json.dumps({"probe_treeput_layout": out}), flush=True)


if __name__ == "__main__":
    main()
