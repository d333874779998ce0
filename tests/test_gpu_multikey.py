"""Multi-key groupby (groupby.py:248-333 ``_combine`` / ``combine='auto'``): the keys are
combined on the GPU into one int64 cartesian ordinal (``vh_combine_keys``) and take the
single-key routes (dense grid, fused hash pass, set grouper for other aggregators), or,
with >= 10 rows per cell, the cartesian grid of dense groupers.

The checker is the oracle's groupby restatement (oracle.groupby_agg: Grouper sort=True,
_combine, GroupBy.agg; pinned by the reference's groupby KATs in test_oracle_kats.py): the
groups in lexicographic order of the sorted labels (the reference's ``sort=True`` order),
counts, sums, min / max per group.  Counts, labels, integer sums and min / max are
bit-exact; float sums within 1e-6 relative (north_star)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _expected(keys, v, extra=()):
    """(labels as an (n_groups, n_keys) int64 array, count(*), sum(v), count(v), *extra) from
    the oracle; extra: more (name, op) aggregates of v."""
    cols = {f"k{i}": k for i, k in enumerate(keys)}
    cols["v"] = v
    names = [f"k{i}" for i in range(len(keys))]
    r = oracle.groupby_agg(cols, names, [("n", "count", None), ("s", "sum", "v"), ("c", "count", "v")] +
                           [(name, op, "v") for name, op in extra])
    uniq = np.stack([r[nm].astype(np.int64) for nm in names], axis=1)
    return (uniq, r["n"], r["s"], r["c"]) + tuple(r[name] for name, _ in extra)


def _frame(keys, v, device):
    import vaex_amd
    from vaex_amd.device import DeviceArray
    cols = {f"k{i}": k for i, k in enumerate(keys)}
    cols["v"] = v
    if device:
        cols = {name: DeviceArray.from_numpy(c) for name, c in cols.items()}
    return vaex_amd.from_arrays(**cols)


def _check(keys, v, res, sort_result=False):
    uniq, cnt, s, nn = _expected(keys, v)
    names = [f"k{i}" for i in range(len(keys))]
    got = [res[n].to_numpy() for n in names]
    order = np.lexsort(got[::-1]) if sort_result else np.arange(len(got[0]))
    for j, g in enumerate(got):
        np.testing.assert_array_equal(g[order].astype(np.int64), uniq[:, j])
    np.testing.assert_array_equal(res["n"].to_numpy()[order], cnt)
    np.testing.assert_array_equal(res["v_count"].to_numpy()[order], nn)
    np.testing.assert_allclose(res["v_sum"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)
    with np.errstate(invalid="ignore", divide="ignore"):
        np.testing.assert_allclose(res["v_mean"].to_numpy()[order], s / nn, rtol=1e-6, atol=1e-9)


def _agg():
    import vaex_amd
    return {"n": "count", "v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v"),
            "v_mean": vaex_amd.agg.mean("v")}


def _spy(monkeypatch):
    from vaex_amd import _lib
    calls = []
    orig = _lib.call
    monkeypatch.setattr(_lib, "call", lambda name, *a: (calls.append(name), orig(name, *a))[1])
    return calls


@pytest.mark.parametrize("device", [False, True])
def test_sparse_keys_combine_into_fused_hash(monkeypatch, device):
    """Two int32 keys whose cartesian span (1e10) is far beyond the rows: combined key,
    fused hash pass; groups in lexicographic key order."""
    rng = np.random.default_rng(1)
    n = 1_000_000
    k0 = (rng.integers(-50_000, 50_000, n)).astype(np.int32)
    k1 = (rng.integers(0, 3, n) * 40_000 + 7).astype(np.int32)
    v = rng.normal(size=n)
    v[::41] = np.nan
    df = _frame([k0, k1], v, device)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg())
    assert "vh_combine_keys" in calls and "vh_hashagg_create" in calls
    assert res.get_column_names()[:2] == ["k0", "k1"]
    _check([k0, k1], v, res, sort_result=True)
    _check_first_appearance([k0, k1], res, ["k0", "k1"])


def test_combined_dense_range_takes_grid_path(monkeypatch):
    """Spans 300 x 400 with 100k rows: occupancy < 10 -> combined, and the combined range
    (120000 <= 4 n) bins as a dense BinnerOrdinal grid."""
    rng = np.random.default_rng(2)
    n = 100_000
    k0 = rng.integers(-150, 150, n).astype(np.int16)
    k1 = rng.integers(1000, 1400, n).astype(np.uint32)
    v = rng.normal(size=n)
    df = _frame([k0, k1], v, True)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg())
    assert "vh_combine_keys" in calls
    _check([k0, k1], v, res, sort_result=True)
    _check_first_appearance([k0, k1], res, ["k0", "k1"])
    assert res["k0"].to_numpy().dtype == np.int16 and res["k1"].to_numpy().dtype == np.uint32
    # sort=True: lexicographic (the dense combined range bins as a BinnerOrdinal grid)
    calls.clear()
    res = df.groupby(["k0", "k1"], agg=_agg(), sort=True)
    assert "vh_combine_keys" in calls and "vh_hashagg_create" not in calls
    _check([k0, k1], v, res)


def test_high_occupancy_keeps_cartesian_grid(monkeypatch):
    """10 x 20 cells over 100k rows: >= 10 rows per cell, no combine (groupby.py:329-333)."""
    rng = np.random.default_rng(3)
    n = 100_000
    k0 = rng.integers(0, 10, n).astype(np.int8)
    k1 = rng.integers(-10, 10, n).astype(np.int64)
    v = rng.normal(size=n)
    df = _frame([k0, k1], v, False)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg())
    assert "vh_combine_keys" not in calls
    _check([k0, k1], v, res)


def test_three_keys_mixed_dtypes_other_aggregators():
    """min / max are not fused aggregators: the combined key goes through the set grouper;
    compared against numpy per group.  Result order: lexicographic after sorting."""
    rng = np.random.default_rng(4)
    n = 300_000
    k0 = rng.integers(0, 60_000, n).astype(np.uint16)
    k1 = (rng.integers(-5, 5, n) * 10 ** 9).astype(np.int64)
    k2 = rng.integers(-100, 100, n).astype(np.int8)
    v = rng.normal(size=n)
    import vaex_amd
    df = _frame([k0, k1, k2], v, True)
    res = df.groupby(["k0", "k1", "k2"], agg={"lo": vaex_amd.agg.min("v"), "hi": vaex_amd.agg.max("v"),
                                              "n": "count"})
    uniq, cnt, _, _, lo, hi = _expected([k0, k1, k2], v, extra=(("lo", "min"), ("hi", "max")))
    got = [res[c].to_numpy() for c in ("k0", "k1", "k2")]
    order = np.lexsort(got[::-1])
    for j, g in enumerate(got):
        np.testing.assert_array_equal(g[order].astype(np.int64), uniq[:, j])
    np.testing.assert_array_equal(res["n"].to_numpy()[order], cnt)
    np.testing.assert_array_equal(res["lo"].to_numpy()[order], lo)
    np.testing.assert_array_equal(res["hi"].to_numpy()[order], hi)


def _first_appearance_order(keys):
    """Row index of each key combination's first appearance, in appearance order (the
    ordered_set order of GrouperCombined with one thread, groupby.py:248-288)."""
    combined = np.zeros(len(keys[0]), np.int64)
    for k in keys:  # NaN keys are one group (the oracle's Grouper)
        labels, ordinal = oracle._grouper(k)
        _, combined = np.unique(combined * len(labels) + ordinal, return_inverse=True)
        combined = combined.astype(np.int64).ravel()
    _, first = np.unique(combined, return_index=True)
    return np.sort(first)


def _check_first_appearance(keys, res, names):
    """Without sort, combined keys ('auto' below the occupancy, or True) come out in the order
    each combination first appears: GrouperCombined over an ordered_set (groupby.py:313-333)."""
    first = _first_appearance_order(keys)
    for nm, k in zip(names, keys):
        np.testing.assert_array_equal(res[nm].to_numpy(), k[first])


def _check_combined(keys, v, res, names, sort):
    """res (groupby(..., assume_sparse=True)) against oracle.groupby_agg(combine=True):
    the same groups and aggregates; without sort the groups in first-appearance order, with
    sort lexicographic."""
    cols = {nm: k for nm, k in zip(names, keys)}
    cols["v"] = v
    exp = oracle.groupby_agg(cols, names, [("n", "count", None), ("v_sum", "sum", "v"), ("v_count", "count", "v"),
                                           ("v_mean", "mean", "v")], combine=True)
    got = [res[nm].to_numpy() for nm in names]
    order = np.lexsort(got[::-1])
    for nm, g in zip(names, got):
        np.testing.assert_array_equal(g[order], exp[nm])
    np.testing.assert_array_equal(res["n"].to_numpy()[order], exp["n"])
    np.testing.assert_array_equal(res["v_count"].to_numpy()[order], exp["v_count"])
    np.testing.assert_allclose(res["v_sum"].to_numpy()[order], exp["v_sum"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(res["v_mean"].to_numpy()[order], exp["v_mean"], rtol=1e-6, atol=1e-9)
    if sort:
        np.testing.assert_array_equal(order, np.arange(len(order)))
    else:
        first = _first_appearance_order(keys)
        for nm, k in zip(names, keys):
            np.testing.assert_array_equal(res[nm].to_numpy(), k[first])


@pytest.mark.parametrize("nkeys", [2, 3, 6])
@pytest.mark.parametrize("sort", [False, True])
def test_assume_sparse_combines_like_reference(monkeypatch, nkeys, sort):
    """assume_sparse=True is the reference's combine=True (dataframe.py:6679,
    groupby.py:313-315): the keys are always combined into one grouper, even when the
    cartesian grid would be small (2 and 3 keys below have >= 10 rows per cell, where
    'auto' bins the cartesian grid).  Six keys: the h2o q10 key set (id1 / id2 / id4 / id5
    one int8 column in [5, 105), id3 / id6 one int32 column in [5, 1e6 + 5), 1e20 cells:
    the 64-bit recursion).  Checked against oracle.groupby_agg(combine=True)."""
    rng = np.random.default_rng(70 + nkeys)
    n = 600_000 if nkeys == 6 else 200_000
    if nkeys == 6:
        a = rng.integers(5, 105, n).astype(np.int8)
        b = rng.integers(5, 1_000_005, n).astype(np.int32)
        keys = [a, a, b, a, a, b]
    elif nkeys == 3:
        keys = [rng.integers(0, 4, n).astype(np.int16), rng.integers(-3, 3, n).astype(np.int64),
                rng.integers(10, 20, n).astype(np.uint8)]
    else:
        keys = [rng.integers(0, 30, n).astype(np.int32), rng.integers(-50, 50, n).astype(np.int32)]
    v = rng.normal(size=n)
    v[::17] = np.nan
    names = [f"k{i}" for i in range(nkeys)]
    df = _frame(keys, v, True)
    calls = _spy(monkeypatch)
    res = df.groupby(names, agg=_agg(), sort=sort, assume_sparse=True)
    assert "vh_combine_keys" in calls
    _check_combined(keys, v, res, names, sort)


def test_assume_sparse_false_bins_the_cartesian_grid(monkeypatch):
    """assume_sparse=False = combine=False: never combined, the cartesian grid filtered by
    count > 0 (groupby.py:334-335, :484-533)."""
    rng = np.random.default_rng(77)
    n = 50_000
    keys = [rng.integers(0, 300, n).astype(np.int32), rng.integers(0, 200, n).astype(np.int32)]
    v = rng.normal(size=n)
    df = _frame(keys, v, True)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg(), assume_sparse=False, sort=True)
    assert "vh_combine_keys" not in calls
    _check(keys, v, res)


@pytest.mark.parametrize("assume_sparse", [True, "auto"])
@pytest.mark.parametrize("device", [False, True])
def test_float_keys_combine_through_set_ordinals(monkeypatch, assume_sparse, device):
    """Keys that are not plain integer columns (float64 with NaN, float32): per-key GPU
    ordered_sets, every row's set ordinal (map_ordinal), the ordinals combined -- the
    reference's _combine over Groupers (groupby.py:248-288).  'auto' combines here too
    (2000 x 1500 cells over 1e5 rows: occupancy < 10, groupby.py:318-333)."""
    rng = np.random.default_rng(78)
    n = 100_000
    k0 = rng.integers(0, 2000, n).astype(np.float64) / 8
    k0[::97] = np.nan
    k1 = (rng.integers(0, 1500, n) - 700).astype(np.float32)
    keys = [k0, k1]
    v = rng.normal(size=n)
    df = _frame(keys, v, device)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg(), assume_sparse=assume_sparse)
    assert "vh_combine_keys" in calls and "vh_set_map_ordinal" in calls
    _check_combined(keys, v, res, ["k0", "k1"], sort=False)
    assert res["k1"].to_numpy().dtype == np.float32


def test_float_keys_high_occupancy_auto_keeps_cartesian(monkeypatch):
    """'auto' with >= 10 rows per cell of the sets' sizes: the cartesian grid (no combine)."""
    rng = np.random.default_rng(79)
    n = 100_000
    keys = [rng.integers(0, 20, n).astype(np.float64), rng.integers(0, 30, n).astype(np.float64)]
    v = rng.normal(size=n)
    df = _frame(keys, v, False)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], agg=_agg(), sort=True)
    assert "vh_combine_keys" not in calls
    _check_combined(keys, v, res, ["k0", "k1"], sort=True)


@pytest.mark.parametrize("device", [False, True])
def test_spans_overflowing_62_bits_recombine(device, monkeypatch):
    """Cartesian span >= 2**62 (the reference's 64-bit overflow recursion, groupby.py:256-287):
    leading keys are combined, re-ordinalised through sorted GPU sets, then combined with the
    rest; the h2o q10 shape (six keys, aliased columns) included."""
    rng = np.random.default_rng(44)
    n = 40_000
    keys = [(rng.integers(0, 60, n) * (2 ** 21) - 2 ** 25).astype(np.int64) for _ in range(4)]
    keys[2] = rng.integers(-3, 4, n).astype(np.int8)
    v = rng.normal(size=n)
    v[::13] = np.nan
    calls = _spy(monkeypatch)
    res = _frame(keys, v, device).groupby([f"k{i}" for i in range(4)], agg=_agg(), sort=True)
    assert calls.count("vh_combine_keys") >= 2
    _check(keys, v, res)
    # h2o q10: id1/id2/id4/id5 alias one int8 column, id3/id6 one int32 column
    a = rng.integers(5, 105, n).astype(np.int8)
    b = rng.integers(5, 1_000_005, n).astype(np.int32)
    six = [a, a, b, a, a, b]
    res = _frame(six, v, device).groupby([f"k{i}" for i in range(6)], agg=_agg())
    _check(six, v, res, sort_result=True)


def test_groupby_then_agg_takes_the_same_routes(monkeypatch):
    """``df.groupby(by).agg(actions)`` (the h2o benchmark's form) == ``df.groupby(by,
    agg=actions)``, through the GPU combine, with the grouper-built GroupBy still reachable."""
    rng = np.random.default_rng(45)
    n = 30_000
    keys = [rng.integers(0, 300, n).astype(np.int32) * 1000, rng.integers(-50, 50, n).astype(np.int16)]
    v = rng.normal(size=n)
    df = _frame(keys, v, True)
    calls = _spy(monkeypatch)
    res = df.groupby(["k0", "k1"], sort=True).agg(_agg())
    assert "vh_combine_keys" in calls
    _check(keys, v, res)
    g = df.groupby(["k0", "k1"])
    assert g.groupby_expression == ["k0", "k1"]


@pytest.mark.parametrize("n", [1, 2, 1000, 300_001])
@pytest.mark.parametrize("keyset", ["signed", "nonneg_47bit", "zeros_and_ones", "nonneg_wide"])
def test_dense_rank_i64(n, keyset):
    """vh_dense_rank_i64 == np.unique(return_inverse): ranks bit-exact, distinct keys sorted
    (signed order across negative keys and the int64 extremes; non-negative keys take the
    unsigned sort over only the bits their maximum needs)."""
    import ctypes
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(n)
    if keyset == "signed":
        pool = np.concatenate([rng.integers(-2 ** 62, 2 ** 62, 50), [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]])
    elif keyset == "nonneg_47bit":
        pool = np.concatenate([rng.integers(0, 10 ** 14, 200), [0, 10 ** 14 - 1]])
    elif keyset == "zeros_and_ones":
        pool = np.array([0, 1])
    else:
        pool = np.concatenate([rng.integers(0, 2 ** 62, 50), [np.iinfo(np.int64).max, 0]])
    keys = pool[rng.integers(0, len(pool), n)].astype(np.int64)
    d_keys = DeviceArray.from_numpy(keys)
    rank = DeviceArray.empty(n, np.int32)
    distinct = DeviceArray.empty(n, np.int64)
    m = ctypes.c_uint64()
    _lib.call("vh_dense_rank_i64", n, d_keys.ptr, rank.ptr, distinct.ptr, ctypes.byref(m))
    uniq, inv = np.unique(keys, return_inverse=True)
    assert m.value == len(uniq)
    np.testing.assert_array_equal(rank.to_numpy(), inv.ravel())
    np.testing.assert_array_equal(distinct[:m.value].to_numpy(), uniq)


@pytest.mark.parametrize("n", [300_000, 3_000_000])
def test_aliased_key_columns_share_one_minmax(n, monkeypatch):
    """Keys that alias one column (groupbyh2o.py: id1 / id2 / id4 / id5 = df['i1_100']) get one
    min / max pass per distinct column; the result equals the oracle's on the same values
    (cartesian grid at n = 3e6: 1e4 cells, combined hash key at 3e5 rows)."""
    import vaex_amd
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(11)
    a = rng.integers(5, 105, n).astype(np.int8)
    b = rng.integers(5, 1005, n).astype(np.int32)
    v = rng.normal(size=n)
    df = vaex_amd.from_arrays(a=DeviceArray.from_numpy(a), b=DeviceArray.from_numpy(b), v=DeviceArray.from_numpy(v))
    df.columns["id1"] = df.columns["a"]
    df.columns["id2"] = df.columns["a"]
    df.columns["id3"] = df.columns["b"]
    calls = []
    real = DataFrame.minmax
    monkeypatch.setattr(DataFrame, "minmax", lambda self, expr, *x, **kw: calls.append(str(expr)) or real(self, expr, *x, **kw))
    by = ["id1", "id2"] if n > 1_000_000 else ["id1", "id2", "id3"]
    got = df.groupby(by, agg={"n": "count", "s": vaex_amd.agg.sum("v"), "c": vaex_amd.agg.count("v")}, sort=True)
    assert sorted(c for c in calls if c in by) == sorted({"id1", "id3"} & set(by))
    keys = [a, a] if n > 1_000_000 else [a, a, b]
    uniq, cnt, s, c = _expected(keys, v)
    np.testing.assert_array_equal(np.stack([got[k].to_numpy().astype(np.int64) for k in by], axis=1), uniq)
    np.testing.assert_array_equal(got["n"].to_numpy(), cnt)
    np.testing.assert_array_equal(got["c"].to_numpy(), c)
    np.testing.assert_allclose(got["s"].to_numpy(), s, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("assume_sparse", [True, "auto"])
def test_masked_integer_keys_combine_with_null_labels(assume_sparse):
    """Masked integer keys take the set-ordinal combine (_groupby_combine_sets): a masked row
    is its key's null group, whose label is masked (None in Grouper.labels, groupby.py:
    158-168), never the raw value under the mask.  sort=True puts the null group last per
    key; checked against oracle.groupby_agg(combine=True) on the keys with masked rows
    replaced by a value above every key (which sorts the same way)."""
    import vaex_amd
    rng = np.random.default_rng(81)
    n = 120_000
    k0 = rng.integers(0, 700, n).astype(np.int32)
    k1 = rng.integers(-40, 40, n).astype(np.int32)
    m0 = np.zeros(n, bool)
    m0[::13] = True
    k0_raw = k0.copy()
    k0_raw[m0] = 5  # the value under the mask must not become a label
    v = rng.normal(size=n)
    df = vaex_amd.from_arrays(k0=np.ma.masked_array(k0_raw, mask=m0), k1=k1, v=v)
    res = df.groupby(["k0", "k1"], agg=_agg(), sort=True, assume_sparse=assume_sparse)
    sentinel = np.int32(10_000)
    k0s = np.where(m0, sentinel, k0)
    exp = oracle.groupby_agg({"k0": k0s, "k1": k1, "v": v}, ["k0", "k1"],
                             [("n", "count", None), ("v_sum", "sum", "v")], combine=True)
    g0 = res["k0"].to_numpy()
    null = exp["k0"] == sentinel
    assert np.ma.isMaskedArray(g0) and np.array_equal(np.ma.getmaskarray(g0), null)
    np.testing.assert_array_equal(np.asarray(g0)[~null], exp["k0"][~null])
    np.testing.assert_array_equal(res["k1"].to_numpy(), exp["k1"])
    np.testing.assert_array_equal(res["n"].to_numpy(), exp["n"])
    np.testing.assert_allclose(res["v_sum"].to_numpy(), exp["v_sum"], rtol=1e-6, atol=1e-9)
