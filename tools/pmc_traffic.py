#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into per-launch HBM traffic of a kernel.

  python tools/pmc_traffic.py <fetch_counter_collection.csv> \
      <write_counter_collection.csv> <kernel-substring> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly HALF the bytes of a
wide coalesced streaming read (16 B/lane global_load and LDS-DMA alike), so
it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.  The two
counters come from separate passes (they do not fit one pass together).
"""
import csv
import json
import statistics
import sys


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel!r} in {path}")
    return statistics.median(vals), len(vals)


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    fkb, nf = per_launch(fetch_csv, kernel, "FETCH_SIZE")
    wkb, nw = per_launch(write_csv, kernel, "WRITE_SIZE")
    read_b = 2 * fkb * 1024
    write_b = wkb * 1024
    d = {
        "kernel": kernel,
        "hbm_bytes_per_launch": int(read_b + write_b),
        "read_bytes": int(read_b), "write_bytes": int(write_b),
        "raw": {"FETCH_SIZE_KiB": fkb, "WRITE_SIZE_KiB": wkb,
                "dispatches": [nf, nw]},
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count on wide streaming "
                      "reads), write = WRITE_SIZE; KiB -> bytes",
        "source": out,
    }
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
