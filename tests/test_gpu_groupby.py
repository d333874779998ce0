"""GPU ordered_set (hash_primitives.hpp) and groupby parity against the oracle.

The GPU set assigns ordinals in first-appearance order, which is exactly what the
reference's ordered_set produces for a single-threaded update with nmaps=1; the oracle's
OrderedSet(1) is that restatement, so ordinals and key_array are compared bit-exactly.
groupby results are compared as key -> (sum, count) maps."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def su():
    import vaex_amd.superutils as m
    return m


@pytest.mark.parametrize("dtype", ["int64", "int32", "int16", "int8", "uint64", "uint32", "uint8", "float64", "float32"])
def test_set_matches_single_thread_reference(dtype):
    rng = np.random.default_rng(1)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        keys = rng.integers(-50, 50, 20000).astype(dt)
        keys[::97] = np.nan
    else:
        info = np.iinfo(dt)
        keys = rng.integers(max(info.min, -100), min(info.max, 100), 20000).astype(dt)
    s = getattr(su(), "ordered_set_" + dtype)(7)
    s.update(keys[:12000])
    s.update(keys[12000:])
    ref = oracle.OrderedSet(1)
    ref.update(keys[:12000])
    ref.update(keys[12000:])
    ka, rka = s.key_array(), ref.key_array(dtype)
    assert len(s) == len(ref)
    np.testing.assert_array_equal(ka, rka)
    np.testing.assert_array_equal(s.map_ordinal(keys), ref.map_ordinal(keys))
    assert s.map_ordinal(keys).dtype == ref.map_ordinal(keys).dtype


@pytest.mark.parametrize("nan", [False, True])
@pytest.mark.parametrize("missing", [False, True])
def test_set_float_kat(nan, missing):
    """tests/internal/hash_test.py:54-126."""
    ar = np.arange(4, dtype="f8")[::-1].copy()
    expected = list(ar)
    mask = None
    if missing:
        mask = np.array([0, 0, 1, 0], dtype=bool)
        expected[2] = None
    if nan:
        ar[1] = np.nan
        expected[1] = "nan"
    oset = su().ordered_set_float64(3)
    ordinals, map_index = oset.update(ar, mask, return_values=True)
    keys = oset.key_array().tolist()
    if missing:
        keys[oset.null_value] = None
    norm = lambda v: "nan" if isinstance(v, float) and v != v else v
    assert [norm(keys[o]) for o in ordinals] == [norm(e) for e in expected]
    assert oset.map_ordinal(np.array([0.0])).dtype.name == "int8"
    ka = oset.key_array()
    ords = oset.map_ordinal(ka).tolist()
    if missing:
        ords[oset.null_value] = oset.null_value
    assert ords == list(range(4))
    # the create() constructor round trip
    copy = su().ordered_set_float64(ka, oset.null_value, oset.nan_count, oset.null_count, "")
    ords = copy.map_ordinal(copy.key_array()).tolist()
    if missing:
        ords[copy.null_value] = copy.null_value
    assert ords == list(range(4))


def test_set_special_keys_and_growth():
    """int64 -1 (the EMPTY bit pattern) and >1e5 distinct keys (table growth)."""
    rng = np.random.default_rng(2)
    keys = rng.integers(-1, 300000, 1_000_000).astype(np.int64)
    keys[5] = -1
    s = su().ordered_set_int64()
    s.update(keys)
    ref = oracle.OrderedSet(1)
    uniq, first = np.unique(keys, return_index=True)
    order = uniq[np.argsort(first)]
    np.testing.assert_array_equal(s.key_array(), order)
    mo = s.map_ordinal(keys)
    np.testing.assert_array_equal(s.key_array()[mo], keys)
    assert (s.map_ordinal(np.array([10 ** 12], np.int64)) == -1).all()


@pytest.mark.parametrize("sort", [False, True])
def test_groupby_sum_count_matches_reference(sort):
    import vaex_amd
    rng = np.random.default_rng(3)
    n = 2_000_000
    keys = (5 + rng.integers(0, 100000, n)).astype(np.int32)
    v = rng.normal(size=n)
    v[::101] = np.nan
    df = vaex_amd.from_arrays(key=keys, v=v)
    dfg = df.groupby("key", agg={"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v"),
                                 "n": "count"}, sort=sort)
    uk, s, c = oracle.groupby_reference(keys, v)
    # the 'count' string is count(*) (groupby.py:390-391): NaN values still count
    np.testing.assert_array_equal(np.sort(dfg["n"].to_numpy()), np.sort(np.bincount(keys)[uk]))
    gk = dfg["key"].to_numpy()
    order = np.argsort(gk)
    assert gk[order].tolist() == uk.tolist()
    if sort:
        assert (np.diff(gk) > 0).all()
    np.testing.assert_array_equal(dfg["v_count"].to_numpy()[order], c)
    np.testing.assert_allclose(dfg["v_sum"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)


def test_groupby_device_resident_keys():
    import vaex_amd
    from vaex_amd.device import DeviceArray
    n = 3_000_000
    dk = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 50000, dtype="int32")
    dv = DeviceArray.random(n, "normal", seed=6)
    df = vaex_amd.from_arrays(key=dk, v=dv)
    dfg = df.groupby("key", agg={"v": ["sum", "count"]})
    # {'v': ['sum', 'count']} -> columns v_sum and v (= count(*)), groupby.py:386-398
    dfg["v_count"] = dfg["v"].to_numpy()
    keys, v = dk.to_numpy(), dv.to_numpy()
    uk, s, c = oracle.groupby_reference(keys, v)
    gk = dfg["key"].to_numpy()
    order = np.argsort(gk)
    assert gk[order].tolist() == uk.tolist()
    np.testing.assert_array_equal(dfg["v_count"].to_numpy()[order], c)
    np.testing.assert_allclose(dfg["v_sum"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("dense", [True, False])
def test_dense_and_hash_groupers_agree(dense):
    """Dense integer keys bin like a categorical (GrouperDense); assume_sparse=True forces the
    hash set path (Grouper); both must give the oracle's key -> (sum, count) map."""
    import vaex_amd
    from vaex_amd import groupby as vg
    rng = np.random.default_rng(9)
    n = 1_500_000
    keys = rng.integers(-300, 4000, n).astype(np.int64)
    keys[keys % 7 == 0] = 10 ** 6  # a gap: most of the range is empty
    v = rng.normal(size=n)
    df = vaex_amd.from_arrays(key=keys, v=v)
    g = vg.GroupBy(df, "key", dense=dense)
    assert isinstance(g.by[0], vg.GrouperDense if dense else vg.Grouper)
    dfg = g.agg({"v_sum": vaex_amd.agg.sum("v"), "n": vaex_amd.agg.count()})
    uk, s, c = oracle.groupby_reference(keys, v)
    gk = dfg["key"].to_numpy()
    order = np.argsort(gk)
    assert gk[order].tolist() == uk.tolist()
    np.testing.assert_array_equal(dfg["n"].to_numpy()[order], c)
    np.testing.assert_allclose(dfg["v_sum"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("spread", [1, 1000])
@pytest.mark.parametrize("kdtype", ["int8", "int16", "int32", "uint32", "int64"])
def test_set_ordinal_grid_through_hash_aggregation(kdtype, spread):
    """assume_sparse=True with count / sum aggregators over >= 2^22 rows: the set-ordinal
    grid is filled by the fused hash aggregation (per-key totals added at each key's
    ordinal cell, hashagg_bin_set_ordinal) -- groups in first-appearance order, counts
    exact, sums within 1e-6, NaN values skipped by sum and count(v), keys of every width
    including negative 1- and 2-byte keys (sign- vs zero-extended bits); dense (spread 1) and
    sparse (spread 1000, >= 4-byte keys) key ranges."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(21)
    n = (1 << 22) + 3
    info = np.iinfo(kdtype)
    lo, hi = max(info.min, -40_000), min(info.max, 60_000)
    keys = rng.integers(lo, hi, n, endpoint=True)
    if np.dtype(kdtype).itemsize >= 4:
        keys = keys * spread
    keys = keys.astype(kdtype)
    v = rng.normal(size=n)
    v[rng.random(n) < 0.01] = np.nan
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    dfg = df.groupby("key", agg={"s": vaex_amd.agg.sum("v"), "c": vaex_amd.agg.count("v"), "n": vaex_amd.agg.count()},
                     assume_sparse=True)
    gk = dfg["key"].to_numpy()
    first = np.unique(keys, return_index=True)
    expect_order = first[0][np.argsort(first[1])]
    np.testing.assert_array_equal(gk, expect_order)
    uk, s, c = oracle.groupby_reference(keys, v)
    order = np.argsort(gk, kind="stable")
    np.testing.assert_array_equal(gk[order], uk)
    np.testing.assert_array_equal(dfg["c"].to_numpy()[order], c)
    np.testing.assert_array_equal(dfg["n"].to_numpy()[order], np.bincount(np.searchsorted(uk, keys), minlength=len(uk)))
    np.testing.assert_allclose(dfg["s"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("spread", [1, 1000])
@pytest.mark.parametrize("vdtype", ["float64", "float32", "int32", "int64"])
def test_set_ordinal_min_max_tile_path(vdtype, spread):
    """assume_sparse=True with min / max (+ count): the set-ordinal binner's fused LUT probe
    (k_tile_scatter_ord<SET = true>) feeding the tile path's min / max slots -- exact per-key
    extrema (NaN skipped, as AggMin/AggMax do), groups in first-appearance order.  spread 1:
    a dense key range (BinnerOrdinal grid + vh_dense_first_order); spread 1000: the set route."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(33)
    n = (1 << 22) + 5
    keys = (rng.integers(-5_000, 200_000, n) * spread).astype(np.int32)
    if vdtype.startswith("float"):
        v = rng.normal(size=n).astype(vdtype)
        v[rng.random(n) < 0.01] = np.nan
    else:
        info = np.iinfo(vdtype)
        v = rng.integers(max(info.min, -(1 << 40)), min(info.max, 1 << 40), n).astype(vdtype)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    dfg = df.groupby("key", agg={"lo": vaex_amd.agg.min("v"), "hi": vaex_amd.agg.max("v"),
                                 "n": vaex_amd.agg.count()}, assume_sparse=True)
    gk = dfg["key"].to_numpy()
    first = np.unique(keys, return_index=True)
    np.testing.assert_array_equal(gk, first[0][np.argsort(first[1])])
    uk, inv = np.unique(keys, return_inverse=True)
    wide = v.astype(np.float64) if vdtype.startswith("float") else v.astype(np.int64)
    if vdtype.startswith("float"):
        lo = np.full(len(uk), np.inf)
        hi = np.full(len(uk), -np.inf)
        np.fmin.at(lo, inv, wide)
        np.fmax.at(hi, inv, wide)
    else:
        lo = np.full(len(uk), np.iinfo(np.int64).max)
        hi = np.full(len(uk), np.iinfo(np.int64).min)
        np.minimum.at(lo, inv, wide)
        np.maximum.at(hi, inv, wide)
    order = np.argsort(gk, kind="stable")
    np.testing.assert_array_equal(gk[order], uk)
    np.testing.assert_array_equal(dfg["lo"].to_numpy()[order].astype(lo.dtype), lo)
    np.testing.assert_array_equal(dfg["hi"].to_numpy()[order].astype(hi.dtype), hi)
    np.testing.assert_array_equal(dfg["n"].to_numpy()[order], np.bincount(inv, minlength=len(uk)))


def test_large_grid_mixed_aggregators_split_routes():
    """count(*) + sum + min + max on a grid beyond the LDS sub-grid size with > 2^20 rows:
    count / sum take the tile path, min / max the generic one (run_bin splits the mix);
    every column equals numpy's per-key result."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(77)
    n = 1_300_001
    key = rng.integers(-20_000, 30_000, n).astype(np.int32)
    v = rng.integers(-100, 100, n).astype(np.int8)
    w = rng.normal(size=n).astype(np.float32)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(key), v=DeviceArray.from_numpy(v),
                              w=DeviceArray.from_numpy(w))
    res = df.groupby("key", sort=True).agg({"n": "count", "vs": vaex_amd.agg.sum("v"),
                                            "vmax": vaex_amd.agg.max("v"), "wmin": vaex_amd.agg.min("w")})
    uk, inv = np.unique(key, return_inverse=True)
    np.testing.assert_array_equal(res["key"].to_numpy(), uk)
    np.testing.assert_array_equal(res["n"].to_numpy(), np.bincount(inv))
    np.testing.assert_array_equal(res["vs"].to_numpy(),
                                  np.bincount(inv, weights=v.astype(np.float64)).astype(np.int64))
    vmax = np.full(len(uk), -128, np.int8)
    np.maximum.at(vmax, inv, v)
    np.testing.assert_array_equal(res["vmax"].to_numpy(), vmax)
    wmin = np.full(len(uk), np.inf, np.float32)
    np.minimum.at(wmin, inv, w)
    np.testing.assert_array_equal(res["wmin"].to_numpy(), wmin)


def test_two_small_int_keys_narrow_lds_cells():
    """A 10^4-cell grid of two int8 keys (h2o q2 shape): counts and 8/16-bit integer sums
    aggregate in 32-bit LDS cells (k_agg_lds_c<..., NARROW>); exact against numpy,
    including extreme values and a float count with NaNs."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(78)
    n = 2_000_003
    k1 = rng.integers(5, 105, n).astype(np.int8)
    k2 = rng.integers(-50, 50, n).astype(np.int8)
    v8 = rng.choice(np.array([-128, 127, -1, 3], np.int8), n)
    v16 = rng.choice(np.array([-32768, 32767, 7], np.int16), n)
    u8 = rng.integers(0, 256, n).astype(np.uint8)
    f = rng.normal(size=n)
    f[::11] = np.nan
    cols = dict(k1=k1, k2=k2, v8=v8, v16=v16, u8=u8, f=f)
    df = vaex_amd.from_arrays(**{c: DeviceArray.from_numpy(a) for c, a in cols.items()})
    res = df.groupby(["k1", "k2"], sort=True).agg({"n": "count", "s8": vaex_amd.agg.sum("v8"),
                                                   "s16": vaex_amd.agg.sum("v16"), "su": vaex_amd.agg.sum("u8"),
                                                   "nf": vaex_amd.agg.count("f")})
    tup = np.stack([k1.astype(np.int64), k2.astype(np.int64)], axis=1)
    uniq, inv = np.unique(tup, axis=0, return_inverse=True)
    inv = inv.ravel()
    np.testing.assert_array_equal(res["k1"].to_numpy(), uniq[:, 0])
    np.testing.assert_array_equal(res["k2"].to_numpy(), uniq[:, 1])
    np.testing.assert_array_equal(res["n"].to_numpy(), np.bincount(inv))
    for name, col in (("s8", v8), ("s16", v16), ("su", u8)):
        exp = np.zeros(len(uniq), np.int64)
        np.add.at(exp, inv, col.astype(np.int64))
        np.testing.assert_array_equal(res[name].to_numpy().astype(np.int64), exp, err_msg=name)
    np.testing.assert_array_equal(res["nf"].to_numpy(), np.bincount(inv[~np.isnan(f)], minlength=len(uniq)))


def test_small_grid_shared_plain_counts():
    """h2o q4 shape: count(*) and counts of integer columns (never NaN) share one LDS
    sub-grid in the fused small-grid pass; a float count with NaNs and the means stay
    separate.  Exact against numpy."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(79)
    n = 1_500_007
    key = rng.integers(5, 105, n).astype(np.int8)
    v1 = rng.integers(5, 15, n).astype(np.int8)
    v2 = rng.integers(-300, 300, n).astype(np.int16)
    v3 = rng.normal(size=n).astype(np.float32)
    v3[::7] = np.nan
    df = vaex_amd.from_arrays(**{c: DeviceArray.from_numpy(a) for c, a in dict(key=key, v1=v1, v2=v2, v3=v3).items()})
    res = df.groupby(["key"], sort=True).agg({"n": "count", "c1": vaex_amd.agg.count("v1"), "c2": vaex_amd.agg.count("v2"),
                                              "c3": vaex_amd.agg.count("v3"), "m1": vaex_amd.agg.mean("v1"),
                                              "m2": vaex_amd.agg.mean("v2")})
    uk, inv = np.unique(key, return_inverse=True)
    cnt = np.bincount(inv)
    np.testing.assert_array_equal(res["key"].to_numpy(), uk)
    for c in ("n", "c1", "c2"):
        np.testing.assert_array_equal(res[c].to_numpy(), cnt, err_msg=c)
    np.testing.assert_array_equal(res["c3"].to_numpy(), np.bincount(inv[~np.isnan(v3)], minlength=len(uk)))
    s1 = np.zeros(len(uk), np.int64)
    np.add.at(s1, inv, v1.astype(np.int64))
    s2 = np.zeros(len(uk), np.int64)
    np.add.at(s2, inv, v2.astype(np.int64))
    np.testing.assert_allclose(res["m1"].to_numpy(), s1 / cnt, rtol=1e-12)
    np.testing.assert_allclose(res["m2"].to_numpy(), s2 / cnt, rtol=1e-12)


def test_small_grid_wide_cells_beyond_fused_budget():
    """grids of 6145..12288 cells whose count / sum need 8-byte LDS cells
    exceed the fused pass's 48 KB budget on their own; they must take the per-aggregator
    LDS path (the host loop once stopped advancing there).  Two int8 keys (~10^4 cells) with
    sums of int32 / float32 / float64 and a count of an int column, and a 100x100 binby
    sum of float32; exact (integers) / 1e-6 (floats) against numpy."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(80)
    n = 1_200_011
    k1 = rng.integers(5, 105, n).astype(np.int8)
    k2 = rng.integers(-50, 50, n).astype(np.int8)
    i32 = rng.integers(-2 ** 31, 2 ** 31 - 1, n, dtype=np.int64).astype(np.int32)
    f32 = rng.normal(size=n).astype(np.float32)
    f64 = rng.normal(size=n)
    cols = dict(k1=k1, k2=k2, i32=i32, f32=f32, f64=f64)
    df = vaex_amd.from_arrays(**{c: DeviceArray.from_numpy(a) for c, a in cols.items()})
    res = df.groupby(["k1", "k2"], sort=True).agg({"si": vaex_amd.agg.sum("i32"), "sf": vaex_amd.agg.sum("f32"),
                                                   "sd": vaex_amd.agg.sum("f64"), "ci": vaex_amd.agg.count("i32")})
    tup = np.stack([k1.astype(np.int64), k2.astype(np.int64)], axis=1)
    uniq, inv = np.unique(tup, axis=0, return_inverse=True)
    inv = inv.ravel()
    si = np.zeros(len(uniq), np.int64)
    np.add.at(si, inv, i32.astype(np.int64))
    np.testing.assert_array_equal(res["si"].to_numpy(), si)
    np.testing.assert_array_equal(res["ci"].to_numpy(), np.bincount(inv))
    np.testing.assert_allclose(res["sf"].to_numpy(), np.bincount(inv, weights=f32.astype(np.float64)), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(res["sd"].to_numpy(), np.bincount(inv, weights=f64), rtol=1e-6, atol=1e-9)
    x, y = rng.normal(size=n), rng.normal(size=n)
    df2 = vaex_amd.from_arrays(x=DeviceArray.from_numpy(x), y=DeviceArray.from_numpy(y), f32=DeviceArray.from_numpy(f32))
    got = df2.sum("f32", binby=["x", "y"], limits=[[-3, 3], [-3, 3]], shape=100)
    bx = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=100)
    by = oracle.Binner("scalar", y, vmin=-3, vmax=3, bins=100)
    exp = oracle.extract_central_part(oracle.compute_grid([bx, by], "sum", data=f32))
    np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("layout", ["holes", "outliers", "host_key"])
def test_dense_first_order_device_finish(layout):
    """assume_sparse=True with min / max / sum / count over a dense key range: the grids stay in
    HBM and vh_dense_first_take gathers the occupied cells in first-appearance order before the
    read-back (groupby.py:97-168 ordered_set order).  holes: only even keys occur (the
    occupied cells are compacted on the device); outliers: keys outside the sampled range
    (the speculative range misses, the exact range reruns); host_key: the key column in host
    memory (staged for the first-row scan).  Against numpy per key."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(91)
    n = (1 << 22) + 3
    keys = rng.integers(0, 150_000, n).astype(np.int32)
    if layout == "holes":
        keys = keys * 2
    out_rows = rng.integers(0, n, 7)
    if layout == "outliers":
        keys[out_rows] = np.array([-40_000, -39_999, 400_000, 400_001, 399_000, -1, 150_001], np.int32)
    v = rng.normal(size=n)
    v[::29] = np.nan
    v[out_rows] = 1.5  # one-row groups: not NaN (an all-NaN group keeps the min / max fill)
    kcol = keys if layout == "host_key" else DeviceArray.from_numpy(keys)
    df = vaex_amd.from_arrays(key=kcol, v=DeviceArray.from_numpy(v))
    got = df.groupby("key", agg={"lo": vaex_amd.agg.min("v"), "hi": vaex_amd.agg.max("v"), "s": vaex_amd.agg.sum("v"),
                                 "n": vaex_amd.agg.count()}, assume_sparse=True)
    u, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    order = np.argsort(first)
    np.testing.assert_array_equal(got["key"].to_numpy(), u[order])
    assert got["key"].to_numpy().dtype == np.int32
    lo = np.full(len(u), np.inf)
    hi = np.full(len(u), -np.inf)
    np.fmin.at(lo, inv, v)
    np.fmax.at(hi, inv, v)
    s = np.bincount(inv, weights=np.nan_to_num(v), minlength=len(u))
    np.testing.assert_array_equal(got["lo"].to_numpy(), lo[order])
    np.testing.assert_array_equal(got["hi"].to_numpy(), hi[order])
    np.testing.assert_array_equal(got["n"].to_numpy(), np.bincount(inv, minlength=len(u))[order])
    np.testing.assert_allclose(got["s"].to_numpy(), s[order], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("kdt,vdt", [("int8", "float32"), ("uint16", "int32"), ("int64", "datetime64[ns]"),
                                     ("uint32", "timedelta64[us]"), ("int32", "int64")])
def test_dense_device_finish_dtypes(kdt, vdt):
    """The device-finish route (vh_dense_first_take) over narrow / wide / unsigned keys near the
    top of their range and 4-byte, integer and datetime / timedelta value columns: the result
    columns keep the descriptor's output dtype (min / max of a datetime column are datetimes,
    an int32 sum is int64), values equal numpy per key in first-appearance order."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(5)
    n = (1 << 21) + 17
    kt = np.dtype(kdt)
    info = np.iinfo(kt)
    lo_k = 0 if kt.kind == "u" else int(info.min) + 7
    span = min(int(info.max) - lo_k, 60_000)
    base = int(info.max) - span  # keys up to the dtype's max (unsigned: near the top of the range)
    keys = (base + rng.integers(0, span + 1, n)).astype(kt)
    vt = np.dtype(vdt)
    if vt.kind in "mM":
        raw = rng.integers(-10 ** 12, 10 ** 12, n)
        vals = raw.astype(np.int64).view(vt) if vt.kind == "M" else raw.astype(vt)
        vcol = vals
    else:
        vals = (rng.normal(size=n) * 100).astype(vt) if vt.kind == "f" else rng.integers(-1000, 1000, n).astype(vt)
        vcol = DeviceArray.from_numpy(vals)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=vcol)
    aggs = {"lo": vaex_amd.agg.min("v"), "hi": vaex_amd.agg.max("v"), "n": vaex_amd.agg.count()}
    if vt.kind not in "mM":
        aggs["s"] = vaex_amd.agg.sum("v")
    got = df.groupby("key", agg=aggs, assume_sparse=True)
    u, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    order = np.argsort(first)
    np.testing.assert_array_equal(got["key"].to_numpy(), u[order])
    srt = np.argsort(inv, kind="stable")
    bounds = np.r_[0, np.cumsum(np.bincount(inv, minlength=len(u)))]
    lo = np.array([vals[srt[bounds[i]:bounds[i + 1]]].min() for i in range(len(u))], dtype=vals.dtype)
    hi = np.array([vals[srt[bounds[i]:bounds[i + 1]]].max() for i in range(len(u))], dtype=vals.dtype)
    glo, ghi = got["lo"].to_numpy(), got["hi"].to_numpy()
    assert glo.dtype == vals.dtype and ghi.dtype == vals.dtype
    np.testing.assert_array_equal(glo, lo[order])
    np.testing.assert_array_equal(ghi, hi[order])
    np.testing.assert_array_equal(got["n"].to_numpy(), np.bincount(inv, minlength=len(u))[order])
    if "s" in aggs:
        s = np.bincount(inv, weights=vals.astype(np.float64), minlength=len(u))
        gs = got["s"].to_numpy()
        if vt.kind in "iu":
            assert gs.dtype == np.int64
            np.testing.assert_array_equal(gs, s[order].astype(np.int64))
        else:
            np.testing.assert_allclose(gs, s[order], rtol=1e-5, atol=1e-3)


def test_dense_device_finish_row_limit_and_reuse():
    """row_limit on the device-finish route raises what the set build raises; a count
    descriptor reused across queries carries no per-query state (occupancy) into the next."""
    import vaex_amd
    from vaex_amd.dataframe import RowLimitException
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(6)
    keys = rng.integers(0, 5000, 1 << 20).astype(np.int32)
    v = rng.normal(size=1 << 20)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    with pytest.raises(RowLimitException):
        df.groupby("key", agg={"m": vaex_amd.agg.max("v")}, assume_sparse=True, row_limit=100)
    cnt = vaex_amd.agg.count()
    a = df.groupby("key", agg={"n": cnt, "m": vaex_amd.agg.max("v")}, assume_sparse=True)
    assert not hasattr(cnt, "occupancy") and not getattr(cnt, "want_occupancy", False)
    keys2 = keys[: 1 << 19] + 10_000
    df2 = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys2), v=DeviceArray.from_numpy(v[: 1 << 19]))
    b = df2.groupby("key", agg={"n": cnt, "m": vaex_amd.agg.max("v")}, assume_sparse=True)
    for d, k in ((a, keys), (b, keys2)):
        u, first, inv = np.unique(k, return_index=True, return_inverse=True)
        np.testing.assert_array_equal(d["key"].to_numpy(), u[np.argsort(first)])
        np.testing.assert_array_equal(d["n"].to_numpy(), np.bincount(inv)[np.argsort(first)])
