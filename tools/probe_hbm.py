#!/usr/bin/env python3
"""What HBM gives each access mix on this MI355X (dev probe, GPU box): the
practical ceiling the combine is measured against.

Per 256 MiB operand, rotating over >= 1 GiB, 0.3 s clock prewarm, then 100
back-to-back launches between one HIP event pair (bench.py's timing):

  read1      one input  HBM -> LDS (nt global_load_lds), nothing stored
  read2      two inputs, the combine's load side alone
  write_nt   one output, nt stores (the combine's policy at >= 192 MiB)
  write_sc1  one output, sc1 write-through stores (its policy below)
  copy       read + write: the write table's ATOMIC_WRITE entry (product)
  combine    the headline: float SUM dst += src (product), 2 reads + 1 write

If reads and writes shared the bus serially, 2 reads + 1 write of S bytes
would take 2S/R_read + S/R_write; the line reports that prediction beside the
measured combine.  Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

S = 256 << 20
NVEC = S // 16


def main() -> None:
    import torch
    from libfabric_amd import _native, atomic
    T = _native.lib("tune")
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    sets = [(torch.empty(S, dtype=torch.uint8, device="cuda"),
             torch.empty(S, dtype=torch.uint8, device="cuda")) for _ in range(4)]
    for a, b in sets:
        a.view(torch.float32).uniform_()
        b.view(torch.float32).uniform_()
    sink = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")

    def launcher(kind):
        if kind == "copy":
            return lambda i: atomic.write(11, 1, sets[i % 4][0], sets[i % 4][1], S, stream)
        if kind == "combine":
            return lambda i: atomic.write(2, 8, sets[i % 4][0].view(torch.float32),
                                          sets[i % 4][1].view(torch.float32), S // 4, stream)
        if kind.startswith("combine_v"):
            v = int(kind[len("combine_v"):])

            def var(i):
                d, s = sets[i % 4]
                assert T.lfa__tune2_sum_f32(v, d.data_ptr(), s.data_ptr(), NVEC, h) == 0
            return var
        code = {"read1": 0, "read2": 1, "write_nt": 2, "write_sc1": 3}[kind]

        def go(i):
            d, s = sets[i % 4]
            dst = sink.data_ptr() if code < 2 else d.data_ptr()
            assert T.lfa__tune_stream(code, dst, s.data_ptr(), d.data_ptr(), NVEC, h) == 0
        return go

    traffic = {"read1": S, "read2": 2 * S, "write_nt": S, "write_sc1": S, "copy": 2 * S,
               "combine": 3 * S, "combine_v50": 3 * S, "combine_v51": 3 * S,
               "combine_v53": 3 * S}
    out = {}
    # combine_v50 / v51 / v53: the same LDS-DMA body with buffer stores of
    # policy nt / sc1 / sc0 sc1 (lfa_tune.hip variants), for the store A/B
    for kind in ("read1", "read2", "write_nt", "write_sc1", "copy", "combine",
                 "combine_v50", "combine_v51", "combine_v53", "combine"):
        fn = launcher(kind)
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < 0.3:
            fn(i)
            i += 1
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(100):
                fn(i)
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 100
            best = us if best is None else min(best, us)
        tbs = traffic[kind] / (best * 1e-6) / 1e12
        out[kind] = {"us": round(best, 2), "tb_s": round(tbs, 3), "frac_of_8tbs": round(tbs / 8, 4)}
    rr, rw = out["read2"]["tb_s"], min(out["write_nt"]["tb_s"], out["write_sc1"]["tb_s"])
    rw_best = max(out["write_nt"]["tb_s"], out["write_sc1"]["tb_s"])
    pred = 3 / (2 / rr + 1 / rw_best)
    out["serial_mix_prediction_2r1w_tb_s"] = round(pred, 3)
    out["combine_vs_prediction"] = round(out["combine"]["tb_s"] / pred, 4)
    out["note"] = ("prediction = 3 / (2 / read2 + 1 / best write): reads and writes "
                   "sharing the bus one after the other; min write " + str(rw))
    print(json.dumps({"probe_hbm_256mib": out}), flush=True)


def _timed(fn, stream, torch, reps=100):
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 0.3:
        fn(i)
        i += 1
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def tree(nin: int = 8, block: int = 32 << 20) -> None:
    """--tree: the N -> 1 fused tree (atomic.reduce_tree, the product body)
    against what HBM gives its access mix, in two input layouts: separate
    allocations, and the collective's slots (round_up(B, 256) + 6 KiB apart in
    one allocation).  Per layout: the read side alone (nin
    streams in the product's load shape, lfa__tune_read_n), the write side
    alone (sc1, the product's store policy at this size), and the tree; the
    prediction is (nin + 1) / (nin / R + 1 / W)."""
    import ctypes
    import torch
    from libfabric_amd import _native, atomic
    T = _native.lib("tune")
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    n = block // 4
    nsets = max(4, -(-(1 << 30) // (nin * block)))
    sink = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    outs = [torch.empty(n, device="cuda") for _ in range(nsets)]
    pitch = (block + 255) // 256 * 256 + (6 << 10)
    layouts = {
        "separate": [[torch.rand(n, device="cuda") for _ in range(nin)] for _ in range(nsets)],
        "slots": [],
    }
    slabs = []
    for _ in range(nsets):
        slab = torch.rand(nin * pitch // 4, device="cuda")
        slabs.append(slab)
        layouts["slots"].append([slab[k * pitch // 4: k * pitch // 4 + n] for k in range(nin)])
    res = {"nin": nin, "block_mib": block >> 20, "sets": nsets}
    for name, sets in layouts.items():
        ptrs = [(ctypes.c_void_p * nin)(*[x.data_ptr() for x in s]) for s in sets]

        def rd(i):
            assert T.lfa__tune_read_n(ptrs[i % nsets], nin, sink.data_ptr(), block // 16, h) == 0

        def wr(i):
            assert T.lfa__tune_stream(3, outs[i % nsets].data_ptr(), None, None, block // 16,
                                      h) == 0

        def tr(i):
            atomic.reduce_tree(2, 8, outs[i % nsets], sets[i % nsets], n, stream)
        r_us, w_us, t_us = (_timed(f, stream, torch) for f in (rd, wr, tr))
        R, W = nin * block / r_us / 1e6, block / w_us / 1e6
        pred = (nin + 1) / (nin / R + 1 / W)
        got = (nin + 1) * block / t_us / 1e6
        res[name] = {"read_us": round(r_us, 2), "read_tb_s": round(R, 3),
                     "write_us": round(w_us, 2), "write_tb_s": round(W, 3),
                     "tree_us": round(t_us, 2), "tree_tb_s": round(got, 3),
                     "tree_frac_of_8tbs": round(got / 8, 4),
                     "mix_prediction_tb_s": round(pred, 3),
                     "tree_vs_prediction": round(got / pred, 4)}
    print(json.dumps({"probe_hbm_tree": res}), flush=True)


if __name__ == "__main__":
    if "--tree" in sys.argv:
        for k in (8, 2):
            tree(k)
    else:
        main()
