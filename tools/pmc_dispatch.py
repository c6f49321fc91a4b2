#!/usr/bin/env python3
"""Per-dispatch counter table from rocprofv3 --pmc CSVs (counter_collection).

    python tools/pmc_dispatch.py <dir>... [--kernel SUBSTR] [--json]

Rows are merged across the given pass directories by (kernel, dispatch order
within that kernel), so separate passes of the same program line up.  Prints
per dispatch: duration (us) and every counter."""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, sub):
    rows = defaultdict(dict)     # (kernel, k-th dispatch) -> counters
    seen = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if sub and sub not in r["Kernel_Name"]:
                    continue
                key = (r["Kernel_Name"], int(r["Dispatch_Id"]))
                if key not in seen[r["Kernel_Name"]]:
                    seen[r["Kernel_Name"]].append(key)
                rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
                rows[key]["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                rows[key]["_grid"] = int(r["Grid_Size"])
                rows[key]["_vgpr"] = int(r["VGPR_Count"])
    out = {}
    for k, keys in seen.items():
        for i, key in enumerate(sorted(keys, key=lambda x: x[1])):
            out[(k, i)] = rows[key]
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sub = None
    if "--kernel" in sys.argv:
        sub = sys.argv[sys.argv.index("--kernel") + 1]
        args.remove(sub)
    merged = defaultdict(dict)
    for d in args:
        for key, vals in load(d, sub).items():
            for c, v in vals.items():
                if c.startswith("_") and c in merged[key]:
                    merged[key][c + "_" + os.path.basename(d.rstrip("/"))] = v
                else:
                    merged[key][c] = v
    res = [{"kernel": k[:60], "n": i, **v} for (k, i), v in sorted(merged.items())]
    if "--json" in sys.argv:
        print(json.dumps(res))
    else:
        for r in res:
            print(json.dumps(r))


if __name__ == "__main__":
    main()
