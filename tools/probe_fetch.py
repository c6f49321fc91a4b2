#!/usr/bin/env python3
"""Fetch and compare tables at 256 MiB per operand (dev probe, GPU box):
lfa_atomic_readwrite_async (res = dst; dst = dst OP src: 2 reads + 2 writes
per element) and lfa_atomic_swap_async (res = dst; dst = src where cmp OP
dst: 3 reads + 2 writes), float / int64, rotated over >= 1 GiB per operand
kind; one HIP event pair around 20 launches, median of 5 rounds.  Prints one
JSON line per (table, op, datatype) with the HBM roofline fraction of the
algorithmic bytes."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libfabric_amd import atomic  # noqa: E402

S = int(os.environ.get("FETCH_MIB", "256")) << 20   # bytes per operand


def run(name, fn, nbytes_per_launch):
    for i in range(6):
        fn(i)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(20):
            fn(i)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 20)
    t = statistics.median(ts)
    print(json.dumps({"case": name, "us": round(t * 1e3, 1),
                      "frac": round(nbytes_per_launch / (t * 1e-3) / 8e12, 4)}), flush=True)


def main():
    torch.cuda.set_device(0)
    for dtn, dt, tdt in (("float", 8, torch.float32), ("int64", 6, torch.int64)):
        n = S // torch.tensor([], dtype=tdt).element_size()
        sets = [[torch.ones(n, dtype=tdt, device="cuda") for _ in range(4)]
                for _ in range(2)]
        # readwrite: SUM (float) / BOR (int64); ATOMIC_READ (1 read + 1 write)
        op = 2 if dt == 8 else 6
        run(f"readwrite_{dtn}_{'sum' if op == 2 else 'bor'}",
            lambda i: atomic.readwrite(op, dt, sets[i % 2][0], sets[i % 2][1], sets[i % 2][2]),
            4 * S)
        run(f"readwrite_{dtn}_atomic_read",
            lambda i: atomic.readwrite(10, dt, sets[i % 2][0], None, sets[i % 2][2]), 2 * S)
        # swap: CSWAP (op 12 = FI_CSWAP): reads dst, src, cmp; writes res, dst
        run(f"swap_{dtn}_cswap",
            lambda i: atomic.swap(12, dt, sets[i % 2][0], sets[i % 2][1], sets[i % 2][3],
                                  sets[i % 2][2]), 5 * S)
        del sets
        torch.cuda.empty_cache()


def tune():
    """--tune: the fetch bodies of liblfa_tune.so (lfa__tune_fetch_f32),
    interleaved rounds, float SUM readwrite and float CSWAP, 256 MiB each
    operand, two rotating sets; every variant checked against variant 0."""
    from libfabric_amd import _native
    L = _native.lib("tune")
    torch.cuda.set_device(0)
    h = torch.cuda.current_stream().cuda_stream
    n = S // 4
    nvec = n // 4
    variants = [int(v) for v in os.environ.get("FETCH_VARIANTS", "0,1,2,3,4,5,6,7").split(",")]
    # 8..11: the compare body with cmp in registers (U 4 sc1 / 4 nt / 2 sc1 / 2 nt)
    for swap, nbytes in ((0, 4 * S), (1, 5 * S)):
        g = torch.Generator(device="cuda").manual_seed(3)
        sets = [[torch.rand(n, device="cuda", generator=g) for _ in range(4)]
                for _ in range(2)]
        for t in sets:                      # cmp == dst on half the lanes
            t[3][::2] = t[0][::2]
        vs = [v for v in variants if swap or not 8 <= v <= 11]    # 8..11: compare only
        ref = None
        for v in vs:                        # correctness on a fresh copy
            d, sr, c, r = (x.clone() for x in sets[0])
            assert L.lfa__tune_fetch_f32(v, swap, d.data_ptr(), sr.data_ptr(), c.data_ptr(),
                                         r.data_ptr(), nvec, h) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = (d, r)
            elif not (torch.equal(ref[0], d) and torch.equal(ref[1], r)):
                raise SystemExit(f"fetch variant {v} swap={swap} WRONG")
        del ref
        times = {v: [] for v in vs}
        for _ in range(int(os.environ.get("FETCH_ROUNDS", "8"))):
            for v in vs:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(10):
                    d, sr, c, r = sets[i % 2]
                    L.lfa__tune_fetch_f32(v, swap, d.data_ptr(), sr.data_ptr(), c.data_ptr(),
                                          r.data_ptr(), nvec, h)
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / 10)
        for v in vs:
            t = statistics.median(times[v][2:])
            print(json.dumps({"tune_fetch": "cswap" if swap else "readwrite_sum", "variant": v,
                              "us": round(t * 1e3, 1),
                              "frac": round(nbytes / (t * 1e-3) / 8e12, 4)}), flush=True)
        del sets
        torch.cuda.empty_cache()


def sweep():
    """--sweep: every entry of the fetch (readwrite) and compare (swap)
    tables at 256 MiB per operand; entries the table lacks are skipped (the
    product's -EOPNOTSUPP).  Bytes: readwrite 4·S (ATOMIC_READ 2·S), swap
    5·S."""
    from libfabric_amd.atomic import LfaError
    torch.cuda.set_device(0)
    sets = [[torch.randint(0, 255, (S,), dtype=torch.uint8, device="cuda")
             for _ in range(4)] for _ in range(2)]
    rows = []
    for dt in range(16):
        if not atomic.datatype_size(dt):
            continue
        for op in list(range(12)) + list(range(12, 19)):
            if op < 12:
                fn = lambda i, op=op, dt=dt: atomic.readwrite(
                    op, dt, sets[i % 2][0], sets[i % 2][1], sets[i % 2][2],
                    S // atomic.datatype_size(dt))
                nb = 2 * S if op == 10 else 4 * S
            else:
                fn = lambda i, op=op, dt=dt: atomic.swap(
                    op, dt, sets[i % 2][0], sets[i % 2][1], sets[i % 2][3], sets[i % 2][2],
                    S // atomic.datatype_size(dt))
                nb = 5 * S
            try:
                fn(0)
            except LfaError:
                continue
            for i in range(3):
                fn(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for i in range(8):
                fn(i)
            b.record()
            torch.cuda.synchronize()
            t = a.elapsed_time(b) / 8
            rows.append({"table": "readwrite" if op < 12 else "swap", "op": op, "dt": dt,
                         "us": round(t * 1e3, 1),
                         "frac": round(nb / (t * 1e-3) / 8e12, 4)})
    fr = [r["frac"] for r in rows]
    print(json.dumps({"sweep_fetch": rows, "entries": len(rows), "min_frac": min(fr),
                      "median_frac": statistics.median(fr)}), flush=True)


if __name__ == "__main__":
    tune() if "--tune" in sys.argv else sweep() if "--sweep" in sys.argv else main()
