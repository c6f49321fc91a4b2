#!/usr/bin/env python3
"""Per-launch HBM traffic of the headline kernel at every operand size of
`bench.py --only-extra sizes`, from two rocprofv3 PMC passes.

  python tools/pmc_sizes.py <fetch_counter_collection.csv> \
      <write_counter_collection.csv> <out.json>

Rows of combine_lds<2, float, ...> are grouped by Grid_Size (threads): one
workgroup of 256 threads covers 1024 16-byte vectors, so an operand of B bytes
launches B / 64 threads.  gfx950 correction as tools/pmc_traffic.py: reads =
2 x FETCH_SIZE, writes = WRITE_SIZE, both KiB.  bench.py reads the result for
roofline.traffic at the strong-scaling shard size.
"""
import csv
import json
import statistics
import sys

KERNEL = "combine_lds<2, float"


def by_grid(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out.setdefault(int(r["Grid_Size"]), []).append(float(r["Counter_Value"]))
    return out


def main():
    fetch, write, dst = sys.argv[1:4]
    f, w = by_grid(fetch, "FETCH_SIZE"), by_grid(write, "WRITE_SIZE")
    res = {}
    for grid in sorted(set(f) & set(w)):
        operand = grid * 64
        rd = 2 * statistics.median(f[grid]) * 1024
        wr = statistics.median(w[grid]) * 1024
        res[str(operand >> 20)] = {
            "operand_bytes": operand, "read_bytes": int(rd), "write_bytes": int(wr),
            "hbm_bytes_per_launch": int(rd + wr), "algorithmic_bytes": 3 * operand,
            "ratio": round((rd + wr) / (3 * operand), 5),
            "dispatches": [len(f[grid]), len(w[grid])]}
    d = {"kernel": KERNEL + ", U=4, ...>", "by_operand_mib": res,
         "correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; KiB -> bytes",
         "source": dst}
    json.dump(d, open(dst, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
