#!/usr/bin/env python3
"""The e2e host-buffer combine (lfa_atomic_write_staged on pinned host dst /
src), zero-copy — one combine on the mapped buffers, reading and writing host
memory over PCIe — against the staged pipeline (LFA_HOST_ZERO_COPY=0: H2D /
combine / D2H chunked through HBM on two streams), float SUM at 1 MiB ..
256 MiB, median of 5, every result checked.  One JSON line per size."""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FI_SUM, FI_FLOAT = 2, 8


def main() -> None:
    import torch
    from libfabric_amd import _native
    L = _native.lib()
    torch.cuda.set_device(0)
    out = {}
    for mib in (1, 4, 16, 64, 256):
        n = (mib << 20) // 4
        hd = torch.rand(n).pin_memory()
        hs = torch.rand(n).pin_memory()
        row = {}
        for name, zc, chunk in (("zero_copy", "1", 0), ("staged_16mib", "0", 16 << 20),
                                ("staged_32mib", "0", 32 << 20)):
            os.environ["LFA_HOST_ZERO_COPY"] = zc

            def fn():
                assert L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, ctypes.c_void_p(hd.data_ptr()),
                                                 ctypes.c_void_p(hs.data_ptr()), ctypes.c_size_t(n),
                                                 ctypes.c_size_t(chunk)) == 0
            base = hd.clone()
            fn()
            ok = bool(torch.equal(hd, base + hs))
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            t = statistics.median(ts)
            row[name] = {"ms": round(t * 1e3, 3), "buffer_gib_s": round(n * 4 / t / 2**30, 2),
                         "exact": ok}
        out[f"{mib}mib"] = row
        print(json.dumps({f"{mib}mib": row}), flush=True)
    print(json.dumps({"e2e_host_float_sum": out}), flush=True)


if __name__ == "__main__":
    main()
