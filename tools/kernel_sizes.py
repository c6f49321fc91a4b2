#!/usr/bin/env python3
"""Per-grid durations of the float SUM combine from a rocprofv3 kernel trace.

  python tools/kernel_sizes.py <run_kernel_trace.csv> [--fit]

One row per grid size: operand MiB (a 256-thread workgroup covers 16 KiB of
each operand), launches, median / mean / min duration in us, and the HBM rate
of the algorithmic bytes (3 x operand) at the median.  --fit adds the least
squares line t = a + bytes / bw over the rows from 32 MiB up.
"""
import csv
import json
import statistics
import sys

KERNEL = "combine_lds<2, float"


def main():
    path = sys.argv[1]
    by = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
            by.setdefault(int(r["Grid_Size_X"]), []).append(us)
    rows = []
    for g in sorted(by):
        v = by[g]
        op = g * 64                     # bytes per operand
        med = statistics.median(v)
        rows.append({"operand_kib": op >> 10, "launches": len(v), "median_us": round(med, 2),
                     "mean_us": round(statistics.mean(v), 2), "min_us": round(min(v), 2),
                     "gbs_at_median": round(3 * op / (med * 1e-6) / 1e9, 1)})
    out = {"rows": rows}
    if "--fit" in sys.argv:
        pts = [(3 * r["operand_kib"] * 1024, r["median_us"]) for r in rows
               if r["operand_kib"] >= 32 * 1024]
        if len(pts) >= 2:
            mx = statistics.mean(p[0] for p in pts)
            my = statistics.mean(p[1] for p in pts)
            sl = (sum((x - mx) * (y - my) for x, y in pts) /
                  sum((x - mx) ** 2 for x, _ in pts))
            out["fit"] = {"intercept_us": round(my - sl * mx, 3),
                          "steady_tb_s": round(1e-6 / sl, 3) if sl else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
