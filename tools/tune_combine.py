"""Back-to-back A/B of combine-kernel forms (float FI_SUM) at several sizes.

bench.py --tune brackets every launch with its own event pair, which puts a
gap between launches and lets each one ramp up from an idle chip; the
product runs launches back to back (the headline's timed region, the
collective's stream).  Here every measurement is K back-to-back launches of
one form between ONE event pair, operands rotating over >= 1 GiB so the
256 MB Infinity Cache cannot serve repeats; forms are interleaved round by
round after a clock prewarm.  Variants are bench.py --tune's ids (30 = the
product launch; 70.. drained forms and 77 = the round-2 product, through
liblfa_tune.so; 80.. the dynamically scheduled forms).

    python tools/tune_combine.py --sizes 32,64,256 --variants 30,77,70 [--rounds 15]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libfabric_amd import _native  # noqa: E402

PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32,64,256", help="MiB per operand")
    ap.add_argument("--variants", default="30,77")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--prewarm-s", type=float, default=0.3)
    args = ap.parse_args()
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    variants = [int(v) for v in args.variants.split(",")]

    def fn(v):
        return (L.lfa__tune_sum_f32 if v < 12 or v == 30 else
                L.lfa__tune3_sum_f32 if 70 <= v < 100 else L.lfa__tune2_sum_f32)

    # correctness first, odd size (partial last tile)
    n = (1 << 20) + 77
    for v in variants:
        a = torch.rand(n * 4, device="cuda")
        b = torch.rand(n * 4, device="cuda")
        want = a + b
        assert fn(v)(v, a.data_ptr(), b.data_ptr(), n, h) == 0
        torch.cuda.synchronize()
        if not torch.equal(a, want):
            raise SystemExit(f"variant {v} is WRONG")
    out = []
    for mib in (int(x) for x in args.sizes.split(",")):
        nbytes = mib << 20
        count = nbytes // 4
        nsets = max(2, (1 << 30) // (2 * nbytes))
        g = torch.Generator(device="cuda").manual_seed(mib)
        sets = [(torch.rand(count, device="cuda", generator=g),
                 torch.rand(count, device="cuda", generator=g)) for _ in range(nsets)]
        nvec = nbytes // 16
        t_end = time.time() + args.prewarm_s
        while time.time() < t_end:
            for d, s in sets:
                fn(30)(30, d.data_ptr(), s.data_ptr(), nvec, h)
            torch.cuda.synchronize()
        per = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(args.k):
                    d, s = sets[i % nsets]
                    fn(v)(v, d.data_ptr(), s.data_ptr(), nvec, h)
                e1.record(stream)
                torch.cuda.synchronize()
                per[v].append(e0.elapsed_time(e1) * 1e3 / args.k)
        # exactness at this size too (every form's whole-step / remainder split)
        d0, s0 = sets[0]
        for v in variants:
            a = d0.clone()
            assert fn(v)(v, a.data_ptr(), s0.data_ptr(), nvec, h) == 0
            torch.cuda.synchronize()
            if not torch.equal(a, d0 + s0):
                raise SystemExit(f"variant {v} is WRONG at {mib} MiB")
            del a
        for v in variants:
            us = statistics.median(per[v])
            row = {"variant": v, "mib": mib, "us": round(us, 3),
                   "min_us": round(min(per[v]), 3), "max_us": round(max(per[v]), 3),
                   "frac": round(3 * nbytes / (us * 1e-6) / PEAK, 4)}
            out.append(row)
            print(json.dumps(row), flush=True)
        del sets
        torch.cuda.empty_cache()
    print(json.dumps({"tune_combine": out}))


if __name__ == "__main__":
    main()
