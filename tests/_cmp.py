"""Parity comparison helpers.

Integers, bitwise and index results: bit-exact.
float / double / float complex: bit-exact on every non-NaN lane; NaN lanes
must be NaN on both sides (x86 and gfx950 differ in NaN payload/sign
propagation — SURVEY §7 "Hard parts"), compared per component.
"""
import numpy as np

FLOAT_DTS = {8: np.float32, 9: np.float64, 10: np.float32}


def assert_parity(dt: int, got_bytes: np.ndarray, want_bytes: np.ndarray,
                  what: str = "") -> None:
    got_bytes = np.ascontiguousarray(got_bytes).view(np.uint8)
    want_bytes = np.ascontiguousarray(want_bytes).view(np.uint8)
    assert got_bytes.shape == want_bytes.shape, what
    if dt not in FLOAT_DTS:
        if not np.array_equal(got_bytes, want_bytes):
            bad = np.nonzero(got_bytes != want_bytes)[0]
            raise AssertionError(f"{what}: {bad.size} bytes differ, first at {bad[:8]}")
        return
    ft = FLOAT_DTS[dt]
    g, w = got_bytes.view(ft), want_bytes.view(ft)
    gn, wn = np.isnan(g), np.isnan(w)
    if not np.array_equal(gn, wn):
        idx = np.nonzero(gn != wn)[0][:8]
        raise AssertionError(f"{what}: NaN class differs at {idx}: got {g[idx]} want {w[idx]}")
    ub = np.uint32 if ft == np.float32 else np.uint64
    gb, wb = g.view(ub), w.view(ub)
    diff = (gb != wb) & ~gn
    if diff.any():
        idx = np.nonzero(diff)[0][:8]
        raise AssertionError(f"{what}: {int(diff.sum())} lanes differ, e.g. {idx}: "
                             f"got {g[idx]} want {w[idx]}")
