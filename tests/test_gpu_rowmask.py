"""A keep mask shared by every aggregator (a selection / filter) on the fast pass A
(k_tile_scatter_f64<..., MK = true>): masked rows are dropped per row before
the exchange.  Grids against the oracle with the same mask (counts exact, sums within 1e-6
relative) and against the generic pass A (VH_TILE_ROWMASK=0): float64 and float32 columns,
count-only, 1- and 3-d grids, odd n (the last row alone), mask bytes other than 0 / 1 (only
1 keeps, as the generic path reads them), and a selection through the DataFrame API on HBM
columns.  Aggregators with different masks keep the generic pass A."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def sa():
    import vaex_amd.superagg as m
    return m


def _run(xs, w, keep, bins, dt, masks=None):
    from vaex_amd.device import DeviceArray
    bs = []
    for i, x in enumerate(xs):
        b = getattr(sa(), "BinnerScalar_" + dt)(f"x{i}", -4, 4, bins)
        b.set_data(DeviceArray.from_numpy(x))
        bs.append(b)
    grid = sa().Grid(bs)
    aggs = [sa().AggCount_int64(grid)]
    if w is not None:
        s = getattr(sa(), "AggSum_" + dt)(grid)
        s.set_data(DeviceArray.from_numpy(w), 0)
        aggs.append(s)
    dk = DeviceArray.from_numpy(keep)
    for k, a in enumerate(aggs):
        a.set_data_mask(DeviceArray.from_numpy(masks[k]) if masks is not None else dk)
    grid.bin(aggs)
    return [np.asarray(a).copy() for a in aggs]


def _case(seed, n, nd, dt, with_sum):
    rng = np.random.default_rng(seed)
    xs = [rng.normal(size=n).astype(dt) for _ in range(nd)]
    for x in xs:
        x[::991] = np.nan
    w = rng.random(n).astype(dt) if with_sum else None
    if w is not None:
        w[::97] = np.nan
    keep = (rng.random(n) < 0.6).astype(np.uint8)
    keep[::13] = 2  # not 1: dropped
    return xs, w, keep


@pytest.mark.parametrize("nd,bins,dt,with_sum,n", [(2, 1024, "float64", True, 3_000_000),
                                                   (2, 1024, "float64", False, 3_000_000),
                                                   (2, 1024, "float64", True, 3_000_001),
                                                   (1, 1 << 20, "float64", True, 2_000_000),
                                                   (3, 100, "float64", True, 2_000_000),
                                                   (2, 1024, "float32", True, 3_000_000),
                                                   (2, 1024, "float32", False, 3_000_000)])
def test_shared_mask_matches_oracle(monkeypatch, nd, bins, dt, with_sum, n):
    xs, w, keep = _case(nd * 31 + n % 7, n, nd, dt, with_sum)
    out = _run(xs, w, keep, bins, dt)
    ob = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=bins) for x in xs]
    np.testing.assert_array_equal(out[0], oracle.compute_grid(ob, "count", mask=keep))
    if with_sum:
        np.testing.assert_allclose(out[1], oracle.compute_grid(ob, "sum", data=w, mask=keep), rtol=1e-6, atol=1e-9)
    monkeypatch.setenv("VH_TILE_ROWMASK", "0")
    gen = _run(xs, w, keep, bins, dt)
    np.testing.assert_array_equal(out[0], gen[0])
    if with_sum:
        np.testing.assert_allclose(out[1], gen[1], rtol=1e-9, atol=1e-9)


def test_different_masks_keep_generic_path():
    """count and sum with different masks (one plan): the generic pass A's per-aggregator
    flags, same oracle grids."""
    xs, w, keep = _case(3, 2_000_000, 2, "float64", True)
    other = (np.random.default_rng(4).random(len(keep)) < 0.5).astype(np.uint8)
    out = _run(xs, w, keep, 1024, "float64", masks=[keep, other])
    ob = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024) for x in xs]
    np.testing.assert_array_equal(out[0], oracle.compute_grid(ob, "count", mask=keep))
    np.testing.assert_allclose(out[1], oracle.compute_grid(ob, "sum", data=w, mask=other), rtol=1e-6, atol=1e-9)


def test_selection_on_hbm_frame():
    """df.select(...) then count / sum with selection=True over HBM columns: one device keep
    mask for both aggregators (the MK kernel), against the oracle."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(9)
    n = 3_000_000
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    df = vaex_amd.from_arrays(x=DeviceArray.from_numpy(x), y=DeviceArray.from_numpy(y), w=DeviceArray.from_numpy(w))
    df.select("w > 0.3")
    lim = [[-4, 4], [-4, 4]]
    c = np.asarray(df.count(binby=["x", "y"], limits=lim, shape=1024, selection=True))
    s = np.asarray(df.sum("w", binby=["x", "y"], limits=lim, shape=1024, selection=True))
    keep = (w > 0.3).astype(np.uint8)
    ob = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024), oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)]
    np.testing.assert_array_equal(c, oracle.extract_central_part(oracle.compute_grid(ob, "count", mask=keep)))
    np.testing.assert_allclose(s, oracle.extract_central_part(oracle.compute_grid(ob, "sum", data=w, mask=keep)),
                               rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("vdt", ["float64", "int64"])
def test_filtered_groupby_dense_route(vdt):
    """groupby on a filtered HBM frame (df[df.w > 0.4]) takes the dense-grid route with the
    filter as every aggregator's keep mask (float64 values: the ordinal kernel's MK
    instantiation; int64 values: the generic pass A): groups, counts and sums equal
    oracle.groupby_agg over the filtered rows, keys in sorted order (GrouperDense)."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(21)
    n = 3_000_000
    keys = rng.integers(5, 200_005, n).astype(np.int32)
    w = rng.random(n)
    v = rng.normal(size=n) if vdt == "float64" else rng.integers(-1000, 1000, n).astype(np.int64)
    if vdt == "float64":
        v[::89] = np.nan
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), w=DeviceArray.from_numpy(w), v=DeviceArray.from_numpy(v))
    g = df[df.w > 0.4].groupby("key", agg={"v": ["sum", "count"]})
    keep = w > 0.4
    # the string 'count' is count(*) under the column's name (parse_actions: vaex.agg.count())
    want = oracle.groupby_agg({"key": keys[keep], "v": v[keep]}, ["key"], [("v_sum", "sum", "v"), ("v_count", "count", None)])
    np.testing.assert_array_equal(g["key"].to_numpy(), want["key"])
    np.testing.assert_array_equal(g["v"].to_numpy(), want["v_count"])
    if vdt == "float64":
        np.testing.assert_allclose(g["v_sum"].to_numpy(), want["v_sum"], rtol=1e-9, atol=1e-9)
    else:
        np.testing.assert_array_equal(g["v_sum"].to_numpy(), want["v_sum"])


def test_filtered_groupby_empty_and_narrow_filters():
    """A filter no row passes (no groups) and one that leaves a few keys (most dense cells
    empty: compaction) give the oracle's groups."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(22)
    n = 2_000_000
    keys = rng.integers(0, 50_000, n).astype(np.int64)
    v = rng.normal(size=n)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    g0 = df[df.v > 100].groupby("key", agg={"v": "sum"})
    assert len(g0) == 0
    sel = (keys >= 20_000) & (keys < 20_300) & (v > 0)
    g1 = df[(df.key >= 20_000) & (df.key < 20_300) & (df.v > 0)].groupby("key", agg={"v": "sum"})
    want = oracle.groupby_agg({"key": keys[sel], "v": v[sel]}, ["key"], [("v", "sum", "v")])
    np.testing.assert_array_equal(g1["key"].to_numpy(), want["key"])
    np.testing.assert_allclose(g1["v"].to_numpy(), want["v"], rtol=1e-9, atol=1e-12)


def test_filter_mask_cache_follows_columns():
    """A filtered HBM frame keeps its filter mask between queries (the reference's per-block
    filter-mask cache) and evaluates it again when a column is replaced."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(23)
    n = 2_000_000
    keys = rng.integers(0, 10_000, n).astype(np.int32)
    v = rng.normal(size=n)
    base = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    dff = base[base.v > 0]
    for _ in range(2):  # the second query reuses the mask
        g = dff.groupby("key", agg={"v": "sum"})
        want = oracle.groupby_agg({"key": keys[v > 0], "v": v[v > 0]}, ["key"], [("v", "sum", "v")])
        np.testing.assert_allclose(g["v"].to_numpy(), want["v"], rtol=1e-9, atol=1e-12)
    v2 = rng.normal(size=n)
    dff.columns["v"] = DeviceArray.from_numpy(v2)
    g = dff.groupby("key", agg={"v": "sum"})
    want = oracle.groupby_agg({"key": keys[v2 > 0], "v": v2[v2 > 0]}, ["key"], [("v", "sum", "v")])
    np.testing.assert_array_equal(g["key"].to_numpy(), want["key"])
    np.testing.assert_allclose(g["v"].to_numpy(), want["v"], rtol=1e-9, atol=1e-12)


def test_selection_mask_cache_follows_select():
    """Selection masks of an HBM frame are kept per block (cpu.py:548 asks for cached masks);
    a new df.select() expression or a replaced column evaluates again."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(24)
    n = 2_000_000
    x, w = rng.normal(size=n), rng.random(n)
    df = vaex_amd.from_arrays(x=DeviceArray.from_numpy(x), w=DeviceArray.from_numpy(w))
    spec = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=64)
    for thr in (0.3, 0.3, 0.7):
        df.select(f"w > {thr}")
        got = np.asarray(df.count(binby="x", limits=[-4, 4], shape=64, selection=True))
        want = oracle.extract_central_part(oracle.compute_grid([spec], "count", mask=(w > thr).astype(np.uint8)))
        np.testing.assert_array_equal(got, want)
    w2 = rng.random(n)
    df.columns["w"] = DeviceArray.from_numpy(w2)
    got = np.asarray(df.count(binby="x", limits=[-4, 4], shape=64, selection=True))
    want = oracle.extract_central_part(oracle.compute_grid([spec], "count", mask=(w2 > 0.7).astype(np.uint8)))
    np.testing.assert_array_equal(got, want)
