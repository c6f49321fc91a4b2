"""The oracle pinned against the reference (CPU only).

* every (op, datatype) handler of oracle/liboracle.so — CAS and plain
  variants — is bit-exact with the reference's own restatement
  (oracle/_ref/libft_atomic.so, built from fabtests/common/ofi_atomic.c);
* the committed golden fixtures reproduce through the oracle;
* the allreduce restatement (coll_coll.c:349-449) hits the reference's
  known answer (fabtests/multinode/src/core_coll.c:230-277) and the
  committed multi-rank fixtures.
"""
import json
import os

import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def manifest(golden_dir):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        return json.load(f)


def _load(golden_dir, case):
    z = np.load(os.path.join(golden_dir, case["file"]))
    nd = oracle.DT_NP[case["dt"]]
    return z["dst"].view(nd), z["src"].view(nd), z["out"].view(nd)


def test_table_shape_matches_shipping_table():
    # op rows (util_atomic.c:907-922): REALNO for MIN/MAX, ALL for
    # SUM/PROD/LOR/LAND/LXOR/WRITE, INT for BOR/BAND/BXOR, READ row empty.
    real = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 14, 15]
    allt = real + [10]
    ints = [0, 1, 2, 3, 4, 5, 6, 7, 14, 15]
    rows = {0: real, 1: real, 2: allt, 3: allt, 4: allt, 5: allt, 6: ints,
            7: ints, 8: allt, 9: ints, 10: [], 11: allt}
    for op, dts in rows.items():
        for dt in range(16):
            assert oracle.has_handler(op, dt) == (dt in dts), (op, dt)


def test_datatype_size():
    sizes = [1, 1, 2, 2, 4, 4, 8, 8, 4, 8, 8, 16, 16, 32, 16, 16]
    for dt, s in enumerate(sizes):
        assert oracle.datatype_size(dt) == s
    assert oracle.datatype_size(16) == 0  # FI_FLOAT16: no entry (util_atomic.c:58-63)


def test_atomic_valid():
    assert oracle.atomic_valid(8, 2) == 0                     # float SUM
    assert oracle.atomic_valid(8, 6) == -95                   # float BOR: EOPNOTSUPP
    assert oracle.atomic_valid(6, 10) == -95                  # ATOMIC_READ row
    assert oracle.atomic_valid(16, 2) == -95                  # datatype >= 16
    assert oracle.atomic_valid(6, 2, 1 << 40) == -260         # unknown flag: EBADFLAGS
    assert oracle.atomic_valid(6, 2, (1 << 58) | (1 << 59)) == -260
    assert oracle.atomic_valid(6, 2, (1 << 3) | (1 << 58)) == -38  # tagged fetch: ENOSYS


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("variant", [oracle.CAS, oracle.PLAIN])
def test_oracle_bit_exact_vs_reference(manifest, golden_dir, variant):
    for case in manifest["combine"]:
        dst, src, _ = _load(golden_dir, case)
        a, b = dst.copy(), dst.copy()
        oracle.write(case["op"], case["dt"], a, src, variant)
        oracle.ref_write(case["op"], case["dt"], b, src)
        assert a.tobytes() == b.tobytes(), case["file"]


def test_golden_fixtures_reproduce(manifest, golden_dir):
    assert len(manifest["combine"]) == 132
    for case in manifest["combine"]:
        dst, src, out = _load(golden_dir, case)
        got = dst.copy()
        oracle.write(case["op"], case["dt"], got, src)
        assert got.tobytes() == out.tobytes(), case["file"]


def test_semantic_spot_checks():
    f32 = oracle.DT_CODE["FLOAT"]
    # no denormal flush: 1e-45f + 1e-45f = 0x00000002
    d = np.array([1], np.uint32).view(np.float32).copy()
    oracle.write(2, f32, d, d.copy())
    assert d.view(np.uint32)[0] == 2
    # dst-biased MIN: NaN in dst stays, NaN in src ignored, ties keep dst
    d = np.array([np.nan, 1.0, -0.0, 0.0], np.float32)
    s = np.array([1.0, np.nan, 0.0, -0.0], np.float32)
    oracle.write(0, f32, d, s)
    assert np.isnan(d[0]) and d[1] == 1.0
    assert np.signbit(d[2]) and not np.signbit(d[3])
    # integer wrap: INT32_MAX + 1 = INT32_MIN; 65536^2 = 0
    i32 = oracle.DT_CODE["INT32"]
    d = np.array([2**31 - 1, 65536], np.int32)
    oracle.write(2, i32, d[:1], np.array([1], np.int32))
    oracle.write(3, i32, d[1:], np.array([65536], np.int32))
    assert d[0] == -2**31 and d[1] == 0


def test_known_answer_uint64_sum(manifest):
    ka = manifest["known_answer"]
    for n, expect in ka["expect"].items():
        n = int(n)
        sends = [np.array([ka["base"] + r], np.uint64) for r in range(n)]
        res = oracle.allreduce(ka["op"], ka["dt"], sends)
        assert all(int(x[0]) == expect for x in res)


def test_allreduce_fixtures(manifest, golden_dir):
    for case in manifest["allreduce"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        sends = list(z["sends"])
        res = oracle.allreduce(case["op"], case["dt"], sends)
        for r in res:
            assert r.tobytes() == z["out"].tobytes(), case["file"]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 12, 16])
def test_allreduce_tree_order(n):
    """Recursive doubling reduces as (hi OP lo) at every level
    (coll_coll.c:409-430).  With a non-commutative-in-bits op (dst-biased
    MIN over signed zeros) the result equals the explicit tree."""
    f32 = oracle.DT_CODE["FLOAT"]
    rng = np.random.default_rng(n)
    sends = [rng.uniform(-1, 1, 64).astype(np.float32) for _ in range(n)]
    res = oracle.allreduce(2, f32, sends)

    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    leaves = []
    for i in range(pof2):
        leaves.append(sends[2 * i + 1] + sends[2 * i] if i < rem else sends[i + rem])
    while len(leaves) > 1:
        leaves = [leaves[i + 1] + leaves[i] for i in range(0, len(leaves), 2)]
    for r in res:
        assert r.tobytes() == leaves[0].tobytes()


def test_reduce_scatter_slices():
    i64 = oracle.DT_CODE["INT64"]
    sends = [np.arange(10, dtype=np.int64) * (r + 1) for r in range(3)]
    out = oracle.reduce_scatter(2, i64, sends)
    assert [len(o) for o in out] == [4, 3, 3]
    assert np.concatenate(out).tolist() == (np.arange(10) * 6).tolist()


# ------------------------------------------------ fetch / compare tables --

def test_fetch_and_compare_table_membership():
    """Shipping CAS tables (util_atomic.c:924-980) vs the reference fabtests
    tables: identical except the columns the CAS build leaves NULL
    (double complex, long double, long double complex)."""
    for op in range(12):
        for dt in range(16):
            if dt in (11, 12, 13):
                assert not oracle.has_readwrite(op, dt)
                continue
            assert oracle.has_readwrite(op, dt) == \
                (oracle.ref_readwrite_handler(op, dt) is not None), (op, dt)
    for op in range(12, 19):
        for dt in range(16):
            if dt in (11, 12, 13):
                assert not oracle.has_swap(op, dt)
                continue
            assert oracle.has_swap(op, dt) == \
                (oracle.ref_swap_handler(op, dt) is not None), (op, dt)


@pytest.mark.parametrize("variant", [oracle.CAS, oracle.PLAIN])
def test_readwrite_fixtures(manifest, golden_dir, variant):
    assert len(manifest["readwrite"]) == 145
    for case in manifest["readwrite"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        nd = oracle.DT_NP[case["dt"]]
        d = z["dst"].view(nd).copy()
        r = np.zeros_like(d)
        oracle.readwrite(case["op"], case["dt"], d, z["src"].view(nd).copy(), r, variant)
        assert d.tobytes() == z["out"].tobytes(), case["file"]
        assert r.tobytes() == z["res"].tobytes(), case["file"]


def _bits_vs_value_lanes(dt, d, c):
    """Lanes where a bytewise compare and a value compare disagree."""
    nd = oracle.DT_NP[dt]
    if nd.kind not in "fc":
        return np.zeros(d.shape[0], bool)
    ft = np.float32 if nd.kind == "c" or dt == 8 else np.float64
    dv, cv = d.view(ft), c.view(ft)
    if nd.kind == "c":
        dv, cv = dv.reshape(-1, 2), cv.reshape(-1, 2)
        val = (dv == cv).all(axis=1)
        bits = (dv.view(np.uint32) == cv.view(np.uint32)).all(axis=1)
    else:
        ut = np.uint32 if ft == np.float32 else np.uint64
        val = dv == cv
        bits = dv.view(ut) == cv.view(ut)
    return val != bits


def test_swap_fixtures_both_builds(manifest, golden_dir):
    """Open-coded oracle == reference fixtures everywhere.  The shipping
    CAS build (__atomic_compare_exchange, a BYTEWISE compare) differs from
    them on FI_CSWAP exactly where bits and values disagree: ±0 pairs and
    identical NaNs — and nowhere else."""
    assert len(manifest["swap"]) == 84
    seen_divergence = 0
    for case in manifest["swap"]:
        z = np.load(os.path.join(golden_dir, case["file"]))
        nd = oracle.DT_NP[case["dt"]]
        d0, s, c = (z[k].view(nd).copy() for k in ("dst", "src", "cmp"))
        for variant in (oracle.PLAIN, oracle.CAS):
            d, r = d0.copy(), np.zeros_like(d0)
            oracle.swap(case["op"], case["dt"], d, s, c, r, variant)
            assert r.tobytes() == z["res"].tobytes(), case["file"]
            if variant == oracle.PLAIN or case["op"] != 12:
                assert d.tobytes() == z["out"].tobytes(), (case["file"], variant)
            else:
                esz = oracle.datatype_size(case["dt"])
                got = d.view(np.uint8).reshape(-1, esz)
                ref = z["out"].reshape(-1, esz)
                differ = (got != ref).any(axis=1)
                expect = _bits_vs_value_lanes(case["dt"], d0, c)
                assert np.array_equal(differ, expect), case["file"]
                seen_divergence += int(differ.sum())
    assert seen_divergence > 0
