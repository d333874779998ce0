"""Pins the CPU oracle (oracle/, test infrastructure) to the reference's own known-answer
tests (tests/golden/kats.json, transcribed by tests/golden/make_kats.py)."""
import numpy as np
import pytest

from conftest import kat_array, load_kats
from oracle import oracle

KATS = load_kats()


def _oracle_binners(specs):
    out = []
    for s in specs:
        data = kat_array(s)
        if s["kind"] == "scalar":
            out.append(oracle.Binner("scalar", data, vmin=s["vmin"], vmax=s["vmax"], bins=s["bins"]))
        else:
            out.append(oracle.Binner("ordinal", data, ordinal_count=s["ordinal_count"],
                                     min_value=s["min_value"]))
    return out


@pytest.mark.parametrize("kat", KATS["superagg"], ids=[k["name"] for k in KATS["superagg"]])
def test_superagg_kat(kat):
    binners = _oracle_binners(kat["binners"])
    agg = kat["agg"]
    data = np.array(agg["data"], dtype=agg["dtype"]) if "data" in agg else None
    grid = oracle.compute_grid(binners, agg["kind"], data=data)
    if "expected" in kat:
        assert grid.tolist() == kat["expected"]
    if "expected_diagonal" in kat:
        assert [grid[k, k] for k in range(grid.shape[0])] == kat["expected_diagonal"]
    if "expected_central" in kat:
        assert oracle.extract_central_part(grid).tolist() == kat["expected_central"]
    if "expected_central_diagonal" in kat:
        assert np.diagonal(oracle.extract_central_part(grid)).tolist() == kat["expected_central_diagonal"]


@pytest.mark.parametrize("nmaps", [1, 2, 3])
@pytest.mark.parametrize("nan", [False, True])
@pytest.mark.parametrize("missing", [False, True])
def test_ordered_set_kat(nmaps, nan, missing):
    """tests/internal/hash_test.py:54-126 on the OrderedSet restatement."""
    spec = KATS["hash_sets"][0]
    ar = np.array(spec["keys"], dtype="f8")
    expected = list(ar)
    mask = None
    if missing:
        mask = np.zeros(4, bool)
        mask[spec["null_row"]] = True
        expected[spec["null_row"]] = None
    if nan:
        ar[spec["nan_row"]] = np.nan
        expected[spec["nan_row"]] = "nan"
    s = oracle.OrderedSet(nmaps)
    s.update(ar, mask, return_values=True)
    keys = s.key_array("f8").tolist()
    if missing:
        keys[s.null_value] = None
    norm = lambda v: "nan" if isinstance(v, float) and v != v else v
    assert sorted(map(str, map(norm, keys))) == sorted(map(str, expected))
    ords = s.map_ordinal(np.array([k if k is not None else 0.0 for k in keys], dtype="f8"))
    assert ords.dtype.name == spec["expected_map_ordinal_dtype"]
    ords = ords.tolist()
    if missing:
        ords[s.null_value] = s.null_value
    assert ords == list(range(4))


def test_ordered_set_c_matches_python():
    """The C set (used by the CPU baseline) and the Python restatement agree on ordinals."""
    rng = np.random.default_rng(0)
    keys = rng.integers(-50, 50, size=500).astype(np.int64)
    for nmaps in (1, 3, 7):
        py = oracle.OrderedSet(nmaps)
        py.update(keys)
        L = oracle.lib()
        h = L.or_set_create(nmaps)
        L.or_set_update(h, keys.ctypes.data, len(keys))
        n = L.or_set_length(h)
        ka = np.empty(n, np.int64)
        L.or_set_key_array(h, ka.ctypes.data)
        mo = np.empty(len(keys), np.int64)
        L.or_set_map_ordinal(h, keys.ctypes.data, len(keys), mo.ctypes.data)
        L.or_set_destroy(h)
        assert ka.tolist() == py.key_array(np.int64).tolist()
        assert mo.tolist() == py.map_ordinal(keys).astype(np.int64).tolist()
        assert (ka[mo] == keys).all()


def test_count_vs_numpy_histogram():
    """tests/count_test.py:23-38: equal to np.histogram except the last bin (max -> overflow)."""
    rng = np.random.default_rng(1)
    x = rng.normal(size=10000)
    lo, hi = oracle.minmax_f64(x)
    g = oracle.compute_grid([oracle.Binner("scalar", x, vmin=lo, vmax=hi, bins=4)], "count")
    counts = oracle.extract_central_part(g)
    ref, _ = np.histogram(x, bins=4, range=(lo, hi))
    assert counts[:-1].tolist() == ref[:-1].tolist()
    assert counts.sum() == len(x) - 1  # the max lands in the overflow bin


def test_groupby_reference_order_independent():
    rng = np.random.default_rng(2)
    k = rng.integers(0, 100, 5000).astype(np.int32)
    v = rng.normal(size=5000)
    v[::97] = np.nan
    uk, s, c = oracle.groupby_reference(k, v)
    for key in uk[:10]:
        sel = (k == key) & ~np.isnan(v)
        assert c[np.searchsorted(uk, key)] == sel.sum()
        assert np.isclose(s[np.searchsorted(uk, key)], v[sel].sum())


def test_bench_drivers_match_restatement():
    """The threaded CPU-baseline drivers compute the same grids as the restated superagg."""
    rng = np.random.default_rng(3)
    n = 200_000
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    bins = 64
    L = oracle.lib()
    cnt = np.zeros((bins + 3) ** 2, np.int64)
    sm = np.zeros((bins + 3) ** 2, np.float64)
    L.or_bench_grid2d(x.ctypes.data, y.ctypes.data, w.ctypes.data, n, -4.0, 4.0, -4.0, 4.0, bins, 4, 4,
                      1 << 14, cnt.ctypes.data, sm.ctypes.data)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=bins)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=bins)
    ref_c = oracle.compute_grid([bx, by], "count")
    ref_s = oracle.compute_grid([bx, by], "sum", data=w)
    assert (cnt.reshape((bins + 3, bins + 3), order="F") == ref_c).all()
    np.testing.assert_allclose(sm.reshape((bins + 3, bins + 3), order="F"), ref_s, rtol=1e-12)
    keys = rng.integers(5, 1005, n).astype(np.int32)
    ko, so, co = np.empty(2000, np.int64), np.empty(2000), np.empty(2000, np.int64)
    ng = L.or_bench_groupby_i32(keys.ctypes.data, w.ctypes.data, n, 4, 2, 1 << 14, 2000,
                                ko.ctypes.data, so.ctypes.data, co.ctypes.data)
    uk, s, c = oracle.groupby_reference(keys, w)
    order = np.argsort(ko[:ng])
    assert ko[:ng][order].tolist() == uk.tolist()
    assert co[:ng][order].tolist() == c.tolist()
    np.testing.assert_allclose(so[:ng][order], s, rtol=1e-12)


@pytest.mark.parametrize("combine", ["auto", True, False])
@pytest.mark.parametrize("name", ["groupby_1d", "groupby_1d_nan", "groupby_2d"])
def test_groupby_agg_restatement_kats(name, combine):
    """oracle.groupby_agg (the multi-key / multi-aggregate groupby restatement) against the
    reference's groupby KATs (tests/groupby_test.py:103-109,149-155,199-207), whether the
    keys are combined (_combine) or binned as a cartesian grid."""
    kat = next(k for k in KATS["api"] if k["name"] == name)
    call = kat["calls"][0]
    cols = {c: np.array([np.nan if v == "nan" or (isinstance(v, float) and v != v) else v for v in vals],
                        dtype="f8" if any(isinstance(v, float) for v in vals) else "i8")
            for c, vals in kat["columns"].items()}
    by = call["by"]
    got = oracle.groupby_agg(cols, by, [("count", "count", None)], combine=combine)
    keys = call["expected_keys"] if isinstance(by, list) else [call["expected_keys"]]
    for b, want in zip(by if isinstance(by, list) else [by], keys):
        g = got[b].tolist()
        if want[-1] == "nan":
            assert g[:-1] == want[:-1] and np.isnan(g[-1])
        else:
            assert g == want
    assert got["count"].tolist() == call["expected_count"]


def test_groupby_agg_restatement_combines_past_63_bits():
    """_combine's recursion (groupby.py:256-287): six keys whose cartesian span passes 2**63
    give the same groups, labels and sums as a plain lexicographic unique."""
    rng = np.random.default_rng(1)
    n = 5000
    cols = {f"k{i}": rng.integers(0, 2000 if i % 2 else 3_000_000, n) for i in range(6)}
    cols["v"] = rng.normal(size=n)
    got = oracle.groupby_agg(cols, [f"k{i}" for i in range(6)], [("s", "sum", "v"), ("n", "count", None)])
    tup = np.stack([cols[f"k{i}"] for i in range(6)], axis=1)
    uniq, inv = np.unique(tup, axis=0, return_inverse=True)
    for i in range(6):
        np.testing.assert_array_equal(got[f"k{i}"], uniq[:, i])
    np.testing.assert_array_equal(got["n"], np.bincount(inv.ravel()))
    np.testing.assert_allclose(got["s"], np.bincount(inv.ravel(), weights=cols["v"]), rtol=1e-12)
