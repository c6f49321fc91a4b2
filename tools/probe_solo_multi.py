#!/usr/bin/env python3
"""World-1 solo copy above one workgroup: launch -> completion word by the
way each workgroup orders its stores before the counter (lfa_tune.hip
lfa__tune_solo_multi, modes 0-4), 4 KiB .. 1 MiB, interleaved rounds, result
bytes checked after every mode.  Prints one JSON line (median us per mode
and size)."""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    from libfabric_amd import _native
    L = _native.lib("tune")
    L.lfa__tune_solo_multi.restype = ctypes.c_int
    torch.cuda.set_device(0)
    names = {0: "product_hip", 1: "product_direct", 2: "replica_hip",
             3: "relaxed_counter_acquire_last", 4: "relaxed_counter",
             5: "tile_8k", 6: "tile_16k", 7: "tile_32k"}
    out = {}
    for nbytes in (4096, 16384, 65536, 262144, 1 << 20):
        src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        times = {m: [] for m in names}
        for _ in range(5):
            for m in names:
                dst = torch.zeros_like(src)
                torch.cuda.synchronize()
                us = ctypes.c_double()
                rc = L.lfa__tune_solo_multi(m, ctypes.c_void_p(dst.data_ptr()),
                                            ctypes.c_void_p(src.data_ptr()),
                                            ctypes.c_size_t(nbytes), 400, ctypes.byref(us))
                torch.cuda.synchronize()
                if rc != 0:
                    raise SystemExit(f"mode {m} size {nbytes}: rc {rc}")
                if not torch.equal(dst, src):
                    raise SystemExit(f"mode {m} size {nbytes}: WRONG bytes")
                times[m].append(us.value)
        out[str(nbytes)] = {names[m]: round(statistics.median(v), 2) for m, v in times.items()}
        print(json.dumps({str(nbytes): out[str(nbytes)]}), flush=True)
    print(json.dumps({"solo_multi_us": out}), flush=True)


if __name__ == "__main__":
    main()
