#!/usr/bin/env python3
"""The e2e host-buffer combine (lfa_atomic_write_staged on pinned host dst /
src), zero-copy — one combine on the mapped buffers, reading and writing host
memory over PCIe — against the staged pipeline (LFA_HOST_ZERO_COPY=0: H2D /
combine / D2H chunked through HBM on two streams), float SUM at 1 MiB ..
256 MiB, median of 5, every result checked.  One JSON line per size.
--small: pinned buffers of 4 KiB .. 2 MiB, the host loop (lfa_host_write,
what the synchronous table runs up to LFA_HOST_SMALL_BYTES) against the
zero-copy combine, median of 50.
--cross: 1 MiB .. 64 MiB, the same two with the caches hot (one buffer pair,
repeated) and cold (a rotating pool of pairs, 512 MiB per operand, so every
call touches memory the last calls did not), median of 9 — where the host
loop stops winning (the synchronous table's LFA_HOST_SMALL_BYTES)."""
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


def small(L, torch) -> None:
    out = {}
    for kib in (4, 16, 64, 256, 512, 1024, 2048):
        n = (kib << 10) // 4
        hd = torch.rand(n).pin_memory()
        hs = torch.rand(n).pin_memory()
        row = {}
        for name, fn in (("host_loop", lambda: L.lfa_host_write(FI_SUM, FI_FLOAT, hd.data_ptr(),
                                                                 hs.data_ptr(), n)),
                         ("zero_copy", lambda: L.lfa_atomic_write_staged(
                             FI_SUM, FI_FLOAT, hd.data_ptr(), hs.data_ptr(), n, 0))):
            base = hd.clone()
            assert fn() == 0
            ok = bool(torch.equal(hd, base + hs))
            ts = []
            for _ in range(50):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            row[name] = {"us": round(statistics.median(ts) * 1e6, 1), "exact": ok}
        out[f"{kib}kib"] = row
        print(json.dumps({f"{kib}kib": row}), flush=True)
    print(json.dumps({"host_loop_vs_zero_copy_pinned": out}), flush=True)


def cross(L, torch) -> None:
    out = {}
    for mib in (1, 2, 4, 8, 16, 32, 64):
        n = (mib << 20) // 4
        k = max(2, 512 // mib)
        ds = [torch.rand(n).pin_memory() for _ in range(k)]
        ss = [torch.rand(n).pin_memory() for _ in range(k)]
        row = {}
        for name in ("host_loop", "zero_copy"):
            for temp in ("hot", "cold"):
                def fn(i):
                    d, s = (ds[0], ss[0]) if temp == "hot" else (ds[i % k], ss[i % k])
                    if name == "host_loop":
                        return L.lfa_host_write(FI_SUM, FI_FLOAT, d.data_ptr(), s.data_ptr(), n)
                    return L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, d.data_ptr(),
                                                     s.data_ptr(), n, 0)
                base = ds[0].clone()
                assert fn(0) == 0
                ok = bool(torch.equal(ds[0], base + ss[0]))
                ts = []
                for i in range(1, 10):
                    t0 = time.perf_counter()
                    fn(i)
                    ts.append(time.perf_counter() - t0)
                row[f"{name}_{temp}"] = {"us": round(statistics.median(ts) * 1e6, 1), "exact": ok}
        del ds, ss
        out[f"{mib}mib"] = row
        print(json.dumps({f"{mib}mib": row}), flush=True)
    print(json.dumps({"host_loop_vs_zero_copy_cross": out}), flush=True)


def copy(L, torch) -> None:
    """--copy: a world-1 allreduce of pinned host buffers is a copy.  The
    provider (zero-copy on the mappings: the solo copy up to 4 MiB, the
    ATOMIC_WRITE body above), the provider with LFA_HOST_ZERO_COPY=0 (H2D /
    device copy / D2H on three streams), the ATOMIC_WRITE body called
    directly, and a hipMemcpyAsync between the two pinned buffers."""
    import numpy as np
    from libfabric_amd import coll
    hip = ctypes.CDLL("libamdhip64.so")
    ep = coll.Endpoint(0, 1, 0, coll.Endpoint.unique_id())
    s = torch.cuda.current_stream()
    out = {}
    for kib in (4, 256, 4096, 32768, 262144):
        n = (kib << 10) // 4
        hx = torch.rand(n).pin_memory()
        hy = torch.empty(n).pin_memory()
        row = {}

        def provider():
            ep.wait(ep.allreduce(hx, hy, n, 8, 2))

        def provider_staged():
            os.environ["LFA_HOST_ZERO_COPY"] = "0"
            try:
                ep.wait(ep.allreduce(hx, hy, n, 8, 2))
            finally:
                del os.environ["LFA_HOST_ZERO_COPY"]

        px = hx.numpy().copy()          # pageable twins
        py = np.zeros_like(px)

        def provider_pageable():
            ep.wait(ep.allreduce(px, py, n, 8, 2))

        def provider_pageable_staged():
            os.environ["LFA_HOST_ZERO_COPY"] = "0"
            try:
                ep.wait(ep.allreduce(px, py, n, 8, 2))
            finally:
                del os.environ["LFA_HOST_ZERO_COPY"]

        def zero_copy():
            assert L.lfa_atomic_write_async(11, 1, ctypes.c_void_p(hy.data_ptr()),
                                            ctypes.c_void_p(hx.data_ptr()),
                                            ctypes.c_size_t(n * 4),
                                            ctypes.c_void_p(s.cuda_stream)) == 0
            torch.cuda.synchronize()

        def memcpy_async():
            assert hip.hipMemcpyAsync(ctypes.c_void_p(hy.data_ptr()),
                                      ctypes.c_void_p(hx.data_ptr()),
                                      ctypes.c_size_t(n * 4), 4,
                                      ctypes.c_void_p(s.cuda_stream)) == 0
            torch.cuda.synchronize()

        for name, fn in (("provider", provider), ("provider_staged", provider_staged),
                         ("provider_pageable", provider_pageable),
                         ("provider_pageable_staged", provider_pageable_staged),
                         ("zero_copy", zero_copy),
                         ("hip_memcpy", memcpy_async)):
            hy.zero_()
            py[:] = 0
            fn()
            ok = bool(torch.equal(hy, hx)) if "pageable" not in name else \
                bool(np.array_equal(py, px))
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            row[name] = {"ms": round(statistics.median(ts) * 1e3, 3), "exact": ok}
        out[f"{kib}kib"] = row
        print(json.dumps({f"{kib}kib": row}), flush=True)
    ep.close()
    print(json.dumps({"world1_host_allreduce_copy": out}), flush=True)


def pageable(L, torch) -> None:
    """--pageable: PAGEABLE (numpy) dst / src, float SUM at 4 .. 256 MiB: the
    staged pipeline (the runtime stages pageable memory itself), the host
    loop, hipHostRegister of both buffers + the zero-copy combine +
    hipHostUnregister from Python, and the entry point's default (which does
    that registration itself), each timed whole, median of 5, results
    checked."""
    import numpy as np
    hip = ctypes.CDLL("libamdhip64.so")
    out = {}
    for mib in (4, 32, 256):
        n = (mib << 20) // 4
        rng = np.random.default_rng(mib)
        d0 = rng.random(n, dtype=np.float32)
        sv = rng.random(n, dtype=np.float32)
        want = d0 + sv
        row = {}

        def staged(d):
            os.environ["LFA_HOST_ZERO_COPY"] = "0"
            try:
                assert L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, d.ctypes.data, sv.ctypes.data,
                                                 n, 0) == 0
            finally:
                del os.environ["LFA_HOST_ZERO_COPY"]

        def host_loop(d):
            assert L.lfa_host_write(FI_SUM, FI_FLOAT, d.ctypes.data, sv.ctypes.data, n) == 0

        def register(d):
            for a in (d, sv):
                assert hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data),
                                           ctypes.c_size_t(a.nbytes), 0) == 0
            try:
                assert L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, d.ctypes.data, sv.ctypes.data,
                                                 n, 0) == 0
            finally:
                for a in (d, sv):
                    hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))

        def default(d):
            assert L.lfa_atomic_write_staged(FI_SUM, FI_FLOAT, d.ctypes.data, sv.ctypes.data,
                                             n, 0) == 0

        for name, fn in (("staged", staged), ("host_loop", host_loop),
                         ("register_zero_copy", register), ("default", default)):
            ts, ok = [], True
            for _ in range(5):
                d = d0.copy()
                t0 = time.perf_counter()
                fn(d)
                ts.append(time.perf_counter() - t0)
                ok = ok and d.tobytes() == want.tobytes()
            row[name] = {"ms": round(statistics.median(ts) * 1e3, 3), "exact": ok}
        out[f"{mib}mib"] = row
        print(json.dumps({f"{mib}mib": row}), flush=True)
    print(json.dumps({"pageable_host_combine": out}), flush=True)


def main() -> None:
    import torch
    from libfabric_amd import _native
    L = _native.lib()
    torch.cuda.set_device(0)
    if "--small" in sys.argv:
        return small(L, torch)
    if "--pageable" in sys.argv:
        return pageable(L, torch)
    if "--copy" in sys.argv:
        return copy(L, torch)
    if "--cross" in sys.argv:
        return cross(L, torch)
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
