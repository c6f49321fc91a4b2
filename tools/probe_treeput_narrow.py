"""reduce_tree_put with a forced tile on narrow lanes, lane by lane against
the oracle.

The product uses U = 4 KiB per wave only up to 8 leaves of >= 4-byte lanes
because U = 4 "gave wrong uint8 results at 16 leaves" (round 2).  This probe
builds U = 1 / 2 / 4 for 1-, 2- and 4-byte lanes at 2…32 inputs through
liblfa_tune.so (lfa__tune_treeput_u) and, for every wrong output, records
how many lanes differ and where: byte offset mod 16, vector index within
the wave's tile, wave, workgroup, and which outputs.

    python tools/probe_treeput_narrow.py [--out gpurun_out/treeput_narrow.json]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (the checker)
from libfabric_amd import _native  # noqa: E402

CASES = [(2, 1), (2, 0), (2, 3), (2, 2), (0, 0), (3, 1), (9, 1), (2, 8)]  # (op, dt)


def run_case(L, u, op, dt, nsrc, ndst, n, head):
    nd = oracle.DT_NP[dt]
    esz = nd.itemsize
    rng = np.random.default_rng(nsrc * 1009 + dt * 17 + op)
    if nd.kind == "f":
        sends = [rng.uniform(0.9, 1.1, n + 2).astype(nd) for _ in range(nsrc)]
    else:
        info = np.iinfo(nd)
        sends = [rng.integers(info.min, info.max, n + 2, dtype=nd, endpoint=True)
                 for _ in range(nsrc)]
    want = oracle.allreduce(op, dt, [s[head:head + n].copy() for s in sends])[0]
    srcs = [torch.from_numpy(s.view(np.uint8).copy()).cuda() for s in sends]
    outs = [torch.zeros((n + 2) * esz, dtype=torch.uint8, device="cuda") for _ in range(ndst)]
    sa = (ctypes.c_void_p * nsrc)(*[t.data_ptr() + head * esz for t in srcs])
    da = (ctypes.c_void_p * ndst)(*[t.data_ptr() + head * esz for t in outs])
    rc = L.lfa__tune_treeput_u(u, op, dt, da, ndst, sa, nsrc, n, None)
    torch.cuda.synchronize()
    if rc:
        return {"rc": rc}
    bad_outs = []
    for j, o in enumerate(outs):
        got = o.cpu().numpy()[head * esz:(head + n) * esz].view(nd)
        diff = np.nonzero(got.view(np.uint8).reshape(n, esz) !=
                          want.view(np.uint8).reshape(n, esz))
        if diff[0].size == 0:
            continue
        el = np.unique(diff[0])
        # the vector body starts at the first 16-B boundary of the output
        p0 = (da[j] + 0) % 16
        hd = ((16 - p0) % 16) // esz
        byte = (el - hd) * esz
        vec = byte // 16
        tile = 64 * u
        bad_outs.append({
            "out": j, "wrong_elems": int(el.size),
            "first": el[:8].tolist(),
            "byte_mod16": np.unique(byte % 16).tolist()[:16],
            "vec_in_tile": np.unique(vec % tile).tolist()[:32],
            "lane": np.unique(vec % 64).tolist()[:64],
            "step_u": np.unique((vec % tile) // 64).tolist(),
            "wave": np.unique((vec // tile) % 4).tolist(),
            "nwg_bad": int(np.unique(vec // (4 * tile)).size),
            "sample": [[int(e), got[e].item(), want[e].item()] for e in el[:4]],
        })
    return {"ok": not bad_outs, "bad": bad_outs}


def probe_forms(L):
    """lfa__tp_probe's four register regimes of the int8 SUM 16-leaf U = 4
    body (lfa_probe.hip), 16 and 17 inputs, 1 and 3 outputs."""
    out = []
    for form in (0, 1, 2, 3):
        for nsrc, ndst, n in ((16, 1, 1 << 20), (17, 3, 70_000), (16, 2, 4096)):
            rng = np.random.default_rng(nsrc * 7 + form)
            sends = [rng.integers(-128, 127, n, dtype=np.int8, endpoint=True)
                     for _ in range(nsrc)]
            want = oracle.allreduce(2, 0, sends)[0]
            srcs = [torch.from_numpy(s.copy()).cuda() for s in sends]
            outs = [torch.zeros(n, dtype=torch.int8, device="cuda") for _ in range(ndst)]
            sa = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs])
            da = (ctypes.c_void_p * ndst)(*[t.data_ptr() for t in outs])
            rc = L.lfa__tp_probe(form, da, ndst, sa, nsrc, n, None)
            torch.cuda.synchronize()
            wrong = []
            for o in outs:
                got = o.cpu().numpy()
                bad = np.nonzero(got != want)[0]
                vec = bad // 16
                wrong.append({"elems": int(bad.size),
                              "step_u": np.unique((vec % 256) // 64).tolist(),
                              "wave": np.unique((vec // 256) % 4).tolist()})
            row = {"form": form, "nsrc": nsrc, "ndst": ndst, "n": n, "rc": rc,
                   "ok": rc == 0 and all(w["elems"] == 0 for w in wrong), "outs": wrong}
            print(json.dumps(row), flush=True)
            out.append(row)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/treeput_narrow.json")
    ap.add_argument("--probe", action="store_true",
                    help="also the four register regimes of lfa__tp_probe")
    args = ap.parse_args()
    L = _native.lib("tune")
    _native.lib("lfa")
    forms = probe_forms(L) if args.probe else []
    rows = []
    for op, dt in CASES:
        for u in (1, 2, 4):
            for nsrc in (2, 8, 9, 16, 17, 32):
                for ndst, n, head in ((1, 70_001, 1), (3, 5_003, 0), (1, 1 << 20, 0)):
                    r = run_case(L, u, op, dt, nsrc, ndst, n, head)
                    row = {"op": op, "dt": dt, "u": u, "nsrc": nsrc, "ndst": ndst, "n": n,
                           "head": head, **r}
                    rows.append(row)
                    if not r.get("ok", False):
                        print(json.dumps(row), flush=True)
            print(f"op {op} dt {dt} u {u} done", flush=True)
    bad = [r for r in rows if not r.get("ok", False)]
    summary = {"cases": len(rows), "wrong": len(bad),
               "wrong_keys": sorted({(r["op"], r["dt"], r["u"], r["nsrc"]) for r in bad}),
               "probe_forms_wrong": sorted({r["form"] for r in forms if not r["ok"]})}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"summary": summary, "probe_forms": forms, "rows": rows}, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
