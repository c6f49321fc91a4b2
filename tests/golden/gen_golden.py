#!/usr/bin/env python3
"""Generate the committed golden fixtures (run in the build container).

combine_<OP>_<DT>.npz   — (dst, src, out) for every (op, datatype) handler of
    the shipping write table.  ``out`` comes from the REFERENCE's own
    fabtests restatement, oracle/_ref/libft_atomic.so, compiled from
    /root/reference/fabtests/common/ofi_atomic.c (oracle/Makefile).  Inputs are
    seeded random lanes plus the edge lanes the survey lists (§8(c)):
    ±0, ±inf, qNaN in dst and in src, min denormal, FLT_MAX, INT_MIN/MAX, 0, ±1.

allreduce_<OP>_<DT>_n<N>.npz — per-rank sends and the allreduce result.
    prov/coll cannot be compiled here (configure-generated config.h), so
    these come from our restatement of coll_coll.c:349-449 (oracle/),
    whose combine steps are pinned by the fixtures above and whose
    schedule is pinned by the reference's known-answer test
    (fabtests/multinode/src/core_coll.c:230-277, also stored here).

Usage:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
N_LANES = 256


def edge_values(dt: int) -> list:
    nd = oracle.DT_NP[dt]
    if nd.kind in "iu":
        info = np.iinfo(nd)
        vals = [0, 1, info.max, info.min, info.max - 1, info.min + 1, 2, 3]
        if nd.kind == "i":
            vals += [-1, -2]
        return [np.array(v).astype(nd) for v in vals]
    if nd.kind == "f":
        f = nd.type
        info = np.finfo(nd)
        tiny_den = np.array(1, dtype=np.uint32 if nd.itemsize == 4 else np.uint64).view(nd)[()]
        nan = np.array(np.nan, dtype=nd)[()]
        return [f(0.0), f(-0.0), f(np.inf), f(-np.inf), nan, -nan, tiny_den,
                -tiny_den, f(info.max), f(-info.max), f(1.0), f(-1.0),
                f(info.tiny), f(2.0), f(0.5)]
    return []


def rand_lanes(dt: int, n: int, rng: np.random.Generator) -> np.ndarray:
    nd = oracle.DT_NP[dt]
    if nd.kind == "V":  # 128-bit integers: raw little-endian bytes
        raw = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        # small-magnitude lanes too, so MIN/MAX/PROD see sign structure
        small = rng.integers(-1000, 1000, size=n // 2).astype(np.int64)
        lo = small.view(np.uint64)
        hi = np.where(small < 0, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0))
        raw[: n // 2, :8] = lo.view(np.uint8).reshape(-1, 8)
        raw[: n // 2, 8:] = hi.view(np.uint8).reshape(-1, 8)
        # edge lanes: 0, 1, -1, INT128 max/min
        raw[-1] = 0
        raw[-2] = 0
        raw[-2, 0] = 1
        raw[-3] = 0xFF
        raw[-4] = 0xFF
        raw[-4, 15] = 0x7F
        raw[-5] = 0
        raw[-5, 15] = 0x80
        return raw.reshape(-1).view(nd)
    if nd.kind == "c":
        re = rand_lanes(oracle.DT_CODE["FLOAT"], n, rng)
        im = rand_lanes(oracle.DT_CODE["FLOAT"], n, rng)
        rng.shuffle(im)
        return np.stack([re, im], axis=1).reshape(-1).view(np.complex64)
    if nd.kind in "iu":
        info = np.iinfo(nd)
        a = rng.integers(info.min, info.max, size=n, dtype=nd, endpoint=True)
        small = rng.integers(-3 if nd.kind == "i" else 0, 4, size=n // 4).astype(nd)
        a[: n // 4] = small
    else:
        a = rng.uniform(-1, 1, size=n).astype(nd)
        # a quarter raw bit patterns: NaNs, infinities, denormals, huge
        ut = np.uint32 if nd.itemsize == 4 else np.uint64
        bits = rng.integers(0, np.iinfo(ut).max, size=n // 4, dtype=ut, endpoint=True)
        a[: n // 4] = bits.view(nd)
        a[n // 4: n // 2] = rng.standard_normal(n // 4).astype(nd) * nd.type(1e30 if nd.itemsize == 8 else 1e20)
    ev = edge_values(dt)
    k = len(ev)
    if k:
        # all (dst, src) pairs of edge values are produced by the caller
        pass
    return a


def combine_case(op: int, dt: int, seed: int):
    rng = np.random.default_rng(seed)
    dst = rand_lanes(dt, N_LANES, rng)
    src = rand_lanes(dt, N_LANES, rng)
    ev = edge_values(dt)
    if ev:  # every ordered pair of edge values
        pairs = [(a, b) for a in ev for b in ev]
        m = min(len(pairs), N_LANES)
        dst[-m:] = np.array([p[0] for p in pairs[:m]], dtype=dst.dtype)
        src[-m:] = np.array([p[1] for p in pairs[:m]], dtype=src.dtype)
    if oracle.DT_NP[dt].kind == "c":  # complex: inf/nan lanes for __mulsc3 path
        sp = [(np.inf, 0.0), (np.nan, np.nan), (0.0, np.inf), (np.inf, np.nan),
              (1.0, 1.0), (-0.0, 0.0)]
        specials = np.array(sp, dtype=np.float32).reshape(-1).view(np.complex64)
        k = len(specials)
        for i in range(k):
            dst[i * k:(i + 1) * k] = specials[i]
            src[i * k:(i + 1) * k] = specials
    out = dst.copy()
    oracle.ref_write(op, dt, out, src)
    return dst, src, out


def main() -> None:
    oracle.build()
    if not oracle.ref_available():
        raise SystemExit("needs /root/reference to build oracle/_ref")
    manifest = {"combine": [], "allreduce": [], "source": {}}
    manifest["source"]["combine"] = (
        "out = reference fabtests/common/ofi_atomic.c ofi_atomic_write_handlers"
        "[op][dt](dst, src, cnt), compiled by oracle/Makefile")
    for opname, op in oracle.OPS.items():
        for dtname, (dt, _) in oracle.DATATYPES.items():
            if not oracle.has_handler(op, dt):
                continue
            seed = 1000 * op + dt
            dst, src, out = combine_case(op, dt, seed)
            fn = f"combine_{opname}_{dtname}.npz"
            np.savez_compressed(os.path.join(OUT, fn), dst=dst.view(np.uint8),
                                src=src.view(np.uint8), out=out.view(np.uint8))
            manifest["combine"].append({"file": fn, "op": op, "dt": dt,
                                        "n": int(dst.shape[0]), "seed": seed})

    # fetch (readwrite) and compare (swap) tables, also from the reference
    manifest["readwrite"], manifest["swap"] = [], []
    manifest["source"]["readwrite"] = ("out/res = reference fabtests "
                                       "ofi_atomic_readwrite_handlers[op][dt]")
    manifest["source"]["swap"] = (
        "out/res = reference fabtests ofi_atomic_swap_handlers (open-coded: CSWAP "
        "compares VALUES); the shipping CAS build compares BITS — see test_oracle")
    for opname, op in oracle.OPS.items():
        for dtname, (dt, _) in oracle.DATATYPES.items():
            if not oracle.has_readwrite(op, dt):
                continue
            dst, src, _ = combine_case(op if op <= 9 else 2, dt, 5000 + 100 * op + dt)
            out, res = dst.copy(), np.zeros_like(dst)
            oracle.ref_readwrite_handler(op, dt)(out.ctypes.data, src.ctypes.data,
                                                 res.ctypes.data, dst.shape[0])
            fn = f"readwrite_{opname}_{dtname}.npz"
            np.savez_compressed(os.path.join(OUT, fn), dst=dst.view(np.uint8),
                                src=src.view(np.uint8), out=out.view(np.uint8),
                                res=res.view(np.uint8))
            manifest["readwrite"].append({"file": fn, "op": op, "dt": dt,
                                          "n": int(dst.shape[0])})
    for opname, op in oracle.SWAP_OPS.items():
        for dtname, (dt, _) in oracle.DATATYPES.items():
            if not oracle.has_swap(op, dt):
                continue
            rng = np.random.default_rng(7000 + 100 * op + dt)
            dst, src, _ = combine_case(2, dt, 7000 + 100 * op + dt)
            cmp = rand_lanes(dt, dst.shape[0], rng)
            # a third of the lanes compare equal, a third as the other zero /
            # the same NaN bits, the rest random
            k = dst.shape[0]
            eq = rng.random(k) < 0.34
            cmp[eq] = dst[eq]
            if oracle.DT_NP[dt].kind in "fc":
                ft = np.float32 if oracle.DT_NP[dt].kind == "c" or dt == 8 else np.float64
                dv, cv = dst.view(ft), cmp.view(ft)
                dv[:16] = np.array([0.0, -0.0, np.nan, -np.nan] * 4, ft)
                cv[:16] = np.array([-0.0, 0.0, np.nan, -np.nan, 0.0, -0.0, 1.0, np.nan] * 2, ft)
            out, res = dst.copy(), np.zeros_like(dst)
            oracle.ref_swap_handler(op, dt)(out.ctypes.data, src.ctypes.data,
                                            cmp.ctypes.data, res.ctypes.data, k)
            fn = f"swap_{opname}_{dtname}.npz"
            np.savez_compressed(os.path.join(OUT, fn), dst=dst.view(np.uint8),
                                src=src.view(np.uint8), cmp=cmp.view(np.uint8),
                                out=out.view(np.uint8), res=res.view(np.uint8))
            manifest["swap"].append({"file": fn, "op": op, "dt": dt,
                                     "n": int(k)})

    manifest["source"]["allreduce"] = (
        "oracle restatement of prov/coll/src/coll_coll.c:349-449 "
        "(prov/coll itself is unbuildable here: needs configure's config.h)")
    cases = [("SUM", "FLOAT"), ("PROD", "FLOAT"), ("SUM", "DOUBLE"),
             ("PROD", "DOUBLE"), ("MIN", "INT64"), ("BOR", "INT64"),
             ("MAX", "FLOAT"), ("BXOR", "UINT32")]
    for n in (2, 3, 5, 8):
        for opname, dtname in cases:
            op, dt = oracle.OPS[opname], oracle.DT_CODE[dtname]
            rng = np.random.default_rng(0x5EED + 97 * n + op)
            nd = oracle.DT_NP[dt]
            if nd.kind == "f":
                lo, hi = (0.9, 1.1) if opname == "PROD" else (-1.0, 1.0)
                sends = [rng.uniform(lo, hi, 1024).astype(nd) for _ in range(n)]
            else:
                info = np.iinfo(nd)
                sends = [rng.integers(info.min, info.max, 1024, dtype=nd,
                                      endpoint=True) for _ in range(n)]
            res = oracle.allreduce(op, dt, sends)
            for r in range(1, n):
                assert res[r].tobytes() == res[0].tobytes()
            fn = f"allreduce_{opname}_{dtname}_n{n}.npz"
            np.savez_compressed(os.path.join(OUT, fn), sends=np.stack(sends),
                                out=res[0])
            manifest["allreduce"].append({"file": fn, "op": op, "dt": dt,
                                          "nranks": n, "count": 1024})
    # the reference's own known answer (core_coll.c:230-277): uint64 SUM,
    # count 1, rank r sends 1234 + r, all ranks expect sum(1234 + r)
    manifest["known_answer"] = {
        "source": "fabtests/multinode/src/core_coll.c:230-277",
        "op": oracle.OPS["SUM"], "dt": oracle.DT_CODE["UINT64"],
        "base": 1234,
        "expect": {str(n): int(sum(1234 + r for r in range(n)))
                   for n in (1, 2, 3, 4, 5, 7, 8)},
    }
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    total = sum(os.path.getsize(os.path.join(OUT, x)) for x in os.listdir(OUT))
    print(f"wrote {len(manifest['combine'])} combine + {len(manifest['readwrite'])} "
          f"readwrite + {len(manifest['swap'])} swap + "
          f"{len(manifest['allreduce'])} allreduce fixtures, {total/1024:.0f} KiB")


if __name__ == "__main__":
    main()
