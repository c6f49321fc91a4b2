#!/usr/bin/env python3
"""Where one combine launch's fixed cost goes, GPU box.

The product body (float SUM combine, LDS-DMA staged, 4 KiB per operand per
wave) built with a timestamp pair per wave (lfa__tune_combine_stamped,
liblfa_tune.so; s_memrealtime, 100 MHz) and the XCC each wave ran on.  At 32
and 256 MiB per operand, after a clock prewarm, K back-to-back stamped
launches over rotating operands; per launch:

  span         first wave start -> last wave end (the kernel as the waves see it)
  steady_tbs   the HBM rate of the launch's middle (bytes of the waves
               running, spread over each wave's lifetime, 0.25 us bins)
  ramp_us      time lost before the rate first reaches 95 % of steady
               (integral of (steady - rate) over those bins / steady)
  drain_us     the same after the rate last left 95 % of steady
  tail_waves   waves still running in the drain window, and their lifetimes
               against the median wave's
  xcc_end_us   per XCC, when its last wave ended (imbalance between XCDs)

Medians over the launches.  Prints one JSON line.
   python tools/probe_ramp.py [--launches 30]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01          # s_memrealtime: 100 MHz
BIN_US = 0.25


def analyse(st, wave_bytes):
    import numpy as np
    st = st.reshape(-1, 4).astype(np.int64)
    t0 = st[:, 0].min()
    s = (st[:, 0] - t0) * TICK_US
    e = (st[:, 1] - t0) * TICK_US
    span = float(e.max())
    nb = int(np.ceil(span / BIN_US)) + 1
    edges = np.arange(nb + 1) * BIN_US
    d = np.maximum(e - s, 1e-3)
    # each wave's bytes spread evenly over its lifetime: bytes done by time t
    # = sum_w bytes * clip(t - s_w, 0, d_w) / d_w, evaluated at the bin edges
    done = np.zeros(nb + 1)
    conc = np.zeros(nb)
    mids = edges[:-1] + BIN_US / 2
    for j in range(0, len(s), 4096):
        a, dd = s[j:j + 4096, None], d[j:j + 4096, None]
        done += (wave_bytes * np.clip(edges[None, :] - a, 0, dd) / dd).sum(axis=0)
        conc += ((a <= mids[None, :]) & (a + dd > mids[None, :])).sum(axis=0)
    rate_tbs = np.diff(done) / (BIN_US * 1e-6) / 1e12
    mid = rate_tbs[nb // 4: 3 * nb // 4]
    steady = float(np.median(mid)) if mid.size else float(rate_tbs.max())
    above = np.nonzero(rate_tbs >= 0.95 * steady)[0]
    first, last = (int(above[0]), int(above[-1])) if above.size else (0, nb - 1)
    ramp = float(np.sum(steady - rate_tbs[:first]) * BIN_US / steady)
    drain = float(np.sum(steady - rate_tbs[last + 1:]) * BIN_US / steady)
    life = e - s
    order = np.argsort(s)
    k = max(len(order) // 10, 1)
    drain_start = (last + 1) * BIN_US
    tail = e > drain_start
    xcc = st[:, 2]
    xcc_end = {int(x): round(float(e[xcc == x].max()), 2) for x in np.unique(xcc)}
    return {"span_us": round(span, 2), "steady_tbs": round(steady, 3),
            "ramp_us": round(ramp, 3), "drain_us": round(drain, 3),
            "waves": int(len(s)), "max_concurrent_waves": int(conc.max()),
            "first_wave_end_us": round(float(e.min()), 2),
            "last_wave_start_us": round(float(s.max()), 2),
            "wave_life_median_us": round(float(np.median(life)), 3),
            "wave_life_first10pct_us": round(float(np.median(life[order[:k]])), 3),
            "wave_life_last10pct_us": round(float(np.median(life[order[-k:]])), 3),
            "drain_window_start_us": round(drain_start, 2),
            "tail_waves": int(tail.sum()),
            "tail_wave_life_median_us": round(float(np.median(life[tail])), 3) if tail.any() else None,
            "xcc_end_us": xcc_end}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch
    from libfabric_amd import _native, atomic
    L = _native.lib("tune")
    L.lfa__tune_combine_stamped.restype = ctypes.c_int
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    h = stream.cuda_stream
    out = {}
    for mib in (32, 64, 256):
        nbytes = mib << 20
        nvec = nbytes // 16
        npairs = max(4, (1 << 30) // nbytes // 2)
        pairs = [(torch.rand(nbytes // 4, device="cuda"), torch.rand(nbytes // 4, device="cuda"))
                 for _ in range(npairs)]
        sc1 = 1 if nbytes < (192 << 20) else 0
        nwaves = -(-nvec // (4 * 64))
        stamps = [torch.zeros(nwaves * 4, dtype=torch.int64, device="cuda")
                  for _ in range(args.launches)]
        # prewarm: steady clocks (bench.py's 0.25 s)
        t_end = time.time() + 0.3
        i = 0
        while time.time() < t_end:
            d, s_ = pairs[i % npairs]
            atomic.write(2, 8, d, s_, nbytes // 4, stream)
            i += 1
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.launches)]
        for k in range(args.launches):
            d, s_ = pairs[k % npairs]
            evs[k][0].record()
            g = L.lfa__tune_combine_stamped(ctypes.c_void_p(d.data_ptr()),
                                            ctypes.c_void_p(s_.data_ptr()),
                                            ctypes.c_size_t(nvec), sc1,
                                            ctypes.c_void_p(stamps[k].data_ptr()),
                                            ctypes.c_void_p(h))
            evs[k][1].record()
            assert g > 0, g
        torch.cuda.synchronize()
        rows = [analyse(st.cpu().numpy(), 3 * 4096) for st in stamps[args.launches // 3:]]
        ev_us = [a.elapsed_time(b) * 1e3 for a, b in evs[args.launches // 3:]]
        med = {key: (statistics.median([r[key] for r in rows])
                     if isinstance(rows[0][key], (int, float)) else rows[len(rows) // 2][key])
               for key in rows[0] if rows[0][key] is not None}
        med["event_us"] = round(statistics.median(ev_us), 2)
        med["frac_of_8tbs_event"] = round(3 * nbytes / (med["event_us"] * 1e-6) / 8e12, 4)
        med["store_policy"] = "sc1" if sc1 else "nt"
        out[f"{mib}mib"] = med
        del pairs, stamps
        torch.cuda.empty_cache()
        print(json.dumps({f"{mib}mib": med}), flush=True)
    print(json.dumps({"probe_ramp": out}), flush=True)


if __name__ == "__main__":
    main()
