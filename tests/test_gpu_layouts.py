"""Row-order robustness of the partitioned engines (tile path, fused hash groupby, ordered_set
build): sorted and clustered layouts give the same results as shuffled rows, and almost no
pass-A row misses its region (vh_stat_read overflow counters).

* tiled.hip / hashagg.hip / hashset.hip: pass-A workgroup w takes batches w, w + W, ... so
  every workgroup's partition distribution is the global one;
* hashagg.hip: clustered keys (the sample sees most rows equal to their neighbour) fold
  each run of equal keys into one HBM-table update;
* hashset.hip: a row whose key equals the previous row's is not a first appearance and is
  dropped in pass A.

Expected values: oracle.groupby_reference / np.unique (the oracle's key -> sum/count maps),
and first-appearance order for the ordered_set (oracle.OrderedSet with nmaps = 1 is that
order; tests/test_gpu_set_insert.py pins it at small sizes)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _stat(name):
    from vaex_amd import _lib
    return _lib.stat_read(name, reset=True)


def _layout(keys, layout, rng, block=100_000):
    if layout == "sorted":
        return np.sort(keys, kind="stable")
    if layout == "clustered":  # sorted runs of `block` rows, the blocks shuffled
        s = np.sort(keys, kind="stable")
        blocks = [s[i:i + block] for i in range(0, len(s), block)]
        rng.shuffle(blocks)
        return np.concatenate(blocks)
    return keys


def _check_groups(keys, v, out):
    gk, cnt, sums, nn = out
    uniq, inv = np.unique(keys, return_inverse=True)
    np.testing.assert_array_equal(gk, uniq)
    np.testing.assert_array_equal(cnt, np.bincount(inv, minlength=len(uniq)))
    if v is not None:
        _, es, ec = oracle.groupby_reference(inv.astype(np.int64), v)
        np.testing.assert_array_equal(nn[0], ec)
        np.testing.assert_allclose(sums[0], es, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("layout", ["sorted", "clustered", "shuffled"])
@pytest.mark.parametrize("card", [1_000, 100_000, 2_000_000])
@pytest.mark.parametrize("kdtype", ["int32", "uint32"])
def test_hashagg_layouts(layout, card, kdtype):
    from vaex_amd.device import DeviceArray
    from vaex_amd.hashagg import HashAgg
    rng = np.random.default_rng(card)
    n = 8_000_000
    keys = _layout((rng.integers(0, card, n) * 7 + 3).astype(kdtype), layout, rng)
    v = rng.normal(size=n)
    v[::11] = np.nan
    _stat("hashagg_overflow_rows")
    ha = HashAgg(keys.dtype, [v.dtype])
    ha.update(DeviceArray.from_numpy(keys), [DeviceArray.from_numpy(v)])
    out = ha.finish()
    assert _stat("hashagg_overflow_rows") <= n // 100
    _check_groups(keys, v, out)
    # count(*) only (no value column)
    ha0 = HashAgg(keys.dtype, [])
    ha0.update(DeviceArray.from_numpy(keys), [])
    _check_groups(keys, None, ha0.finish())


@pytest.mark.parametrize("layout", ["sorted", "clustered"])
def test_groupby_routes_on_sorted_keys(layout):
    """C3's query on a sorted / clustered key column through every route: the dense
    BinnerOrdinal grid (auto), the fused hash path (sparse keys) and the ordered_set build
    (assume_sparse, the reference's structure)."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(3)
    n = 6_000_000
    key = _layout(rng.integers(5, 5 + 200_000, n).astype(np.int32), layout, rng)
    skey = (key.astype(np.int64) * 104729 - 10 ** 9).astype(np.int32)  # sparse: the fused path
    v = rng.normal(size=n)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(key), skey=DeviceArray.from_numpy(skey),
                              v=DeviceArray.from_numpy(v))
    for col, k in (("key", key), ("skey", skey)):
        uniq, inv = np.unique(k, return_inverse=True)
        _, es, ec = oracle.groupby_reference(inv.astype(np.int64), v)
        for sparse in ("auto", True):
            for name in ("tile_overflow_rows", "hashagg_overflow_rows", "set_overflow_rows"):
                _stat(name)
            g = df.groupby(col, agg={"v": ["sum", "count"]}, sort=True, assume_sparse=sparse)
            np.testing.assert_array_equal(g[col].to_numpy(), uniq, err_msg=f"{col} {sparse}")
            np.testing.assert_array_equal(g["v"].to_numpy(), ec)
            np.testing.assert_allclose(g["v_sum"].to_numpy(), es, rtol=1e-6, atol=1e-9)
            over = sum(_stat(name) for name in ("tile_overflow_rows", "hashagg_overflow_rows", "set_overflow_rows"))
            assert over <= n // 100, (col, sparse, over)


@pytest.mark.parametrize("layout", ["sorted", "clustered", "shuffled"])
@pytest.mark.parametrize("dtype", ["int32", "int64"])
def test_ordered_set_layouts(layout, dtype):
    """ordered_set over sorted / clustered keys (pass A drops rows equal to their previous
    row): key_array in first-appearance order, map_ordinal exact."""
    from vaex_amd import superutils
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(17)
    n = 8_000_000
    keys = _layout(rng.integers(-300_000, 300_000, n).astype(dtype), layout, rng)
    s = getattr(superutils, f"ordered_set_{dtype}")()
    _stat("set_overflow_rows")
    s.update(DeviceArray.from_numpy(keys))
    assert _stat("set_overflow_rows") <= n // 100
    uniq, first = np.unique(keys, return_index=True)
    want = keys[np.sort(first)]
    np.testing.assert_array_equal(s.key_array(), want)
    probe = keys[::997]
    ordinal = {k: i for i, k in enumerate(want.tolist())}
    np.testing.assert_array_equal(s.map_ordinal(probe).astype(np.int64), np.array([ordinal[k] for k in probe.tolist()]))


def test_ordered_set_sorted_small_matches_oracle():
    """The same dedup against the pinned restatement itself (small input, several runs)."""
    from vaex_amd import superutils
    rng = np.random.default_rng(2)
    keys = np.sort(rng.integers(0, 500, 40_000)).astype(np.int32)[::-1].copy()
    ref = oracle.OrderedSet(nmaps=1)
    ref.update(keys)
    s = superutils.ordered_set_int32()
    s.update(keys)
    np.testing.assert_array_equal(s.key_array(), ref.key_array(np.int32))
    np.testing.assert_array_equal(s.map_ordinal(keys).astype(np.int64), ref.map_ordinal(keys).astype(np.int64))


def test_tile_path_sorted_y_overflow_counter():
    """The C2 query with y sorted at 2e7 rows: bit-exact counts and (almost) no pass-A row
    beyond its region."""
    from vaex_amd import superagg
    from vaex_amd.device import DeviceArray
    n = 20_000_000
    x = DeviceArray.random(n, "normal", seed=2)
    y = DeviceArray.random(n, "sorted_normal", a=0.0, b=1.0)
    hy = y.to_numpy()
    assert np.all(np.diff(hy) >= 0)
    bx, by = superagg.BinnerScalar_float64("x", -4, 4, 1024), superagg.BinnerScalar_float64("y", -4, 4, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    c = superagg.AggCount_int64(grid)
    _stat("tile_overflow_rows")
    grid.bin([c])
    assert _stat("tile_overflow_rows") <= n // 100
    spec = [oracle.Binner("scalar", x.to_numpy(), vmin=-4, vmax=4, bins=1024),
            oracle.Binner("scalar", hy, vmin=-4, vmax=4, bins=1024)]
    np.testing.assert_array_equal(np.asarray(c), oracle.compute_grid(spec, "count"))
