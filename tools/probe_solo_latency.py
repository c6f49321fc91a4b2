#!/usr/bin/env python3
"""Launch-to-completion-word latency of one small GPU operation, by part
(lfa__tune_solo_latency, liblfa_tune.so): the product's
n = 1 one-shot kernel, its body copied with and without the system-scope
releases, with write-through data stores, and the word alone.  4 KiB,
mean of 5000 after 50 untimed.  Prints one JSON line."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = ("product_oneshot_n1", "body_copy_with_releases", "body_no_releases_diag",
         "body_writethrough_stores", "word_only_with_releases", "word_only_no_releases",
         "product_solo_copy", "direct_solo_copy")
COPIES = {0, 6, 7}      # modes whose result must equal the input


def main():
    import torch
    from libfabric_amd import _native
    L = _native.lib("tune")
    L.lfa__tune_solo_latency.restype = ctypes.c_int
    torch.cuda.set_device(0)
    a = torch.rand(1024, device="cuda")
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    out = {}
    for rnd in range(2):
        for m, name in enumerate(MODES):
            us = ctypes.c_double()
            b.zero_()
            torch.cuda.synchronize()
            rc = L.lfa__tune_solo_latency(m, ctypes.c_void_p(b.data_ptr()),
                                          ctypes.c_void_p(a.data_ptr()), ctypes.c_size_t(4096),
                                          5000, ctypes.byref(us))
            torch.cuda.synchronize()
            out.setdefault(name, []).append(round(us.value, 3) if rc == 0 else f"rc {rc}")
            if m in COPIES and rc == 0:
                out.setdefault("copy_exact", {})[name] = bool(torch.equal(a, b))
    print(json.dumps({"probe_solo_latency_us": out}), flush=True)


if __name__ == "__main__":
    main()
