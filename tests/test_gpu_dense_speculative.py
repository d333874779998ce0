"""Dense single-key groupby with a sampled key range (groupby._dense_range speculative=True).

The dense route bins an integer key like a categorical (BinnerOrdinal over [min, max],
superagg_binners.cpp:104-142).  For HBM columns of >= SPECULATE_MIN_ROWS rows the range is
guessed from a row sample instead of a full min/max pass; keys outside the guess land in the
binner's under/overflow cells, which the query checks before it returns, redoing it with the
exact range on a miss.  Every layout here must give exactly the exact-range result (labels,
label dtype, counts, sums) and the oracle's key -> (sum, count) map."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

N = (1 << 22) + 37


def _keys(layout, dtype, rng):
    dt = np.dtype(dtype)
    info = np.iinfo(dt)
    if layout == "uniform":
        lo, hi = (5, 105) if dt.itemsize == 1 else (5, 5 + 20000)
        return rng.integers(lo, hi, N).astype(dt)
    if layout == "sorted":
        return np.sort(rng.integers(0, 20000 if dt.itemsize > 1 else 120, N)).astype(dt)
    if layout == "outlier_high":  # one far key the sample cannot see
        k = rng.integers(0, 1000, N).astype(dt)
        k[N // 3 + 1] = min(int(info.max), 60000)
        return k
    if layout == "outlier_low":
        k = rng.integers(0, 1000, N).astype(dt)
        k[7] = max(int(info.min), -5000) if dt.kind == "i" else 0
        return k
    if layout == "normal":  # tails beyond the sample's extremes
        return np.clip(np.round(rng.normal(0, 2000, N)), info.min, info.max).astype(dt)
    if layout == "wide":  # more values than the dtype's max: ordinal_count (a T) cannot hold them
        return rng.integers(int(info.min) + 1, int(info.max), N, dtype=np.int64).astype(dt)
    if layout == "dtype_edge":  # keys at the dtype's limits: the widened guess is clipped
        return rng.integers(int(info.max) - 50, int(info.max) + 1, N, dtype=np.int64).astype(dt)
    raise ValueError(layout)


CASES = [("uniform", "int32"), ("uniform", "int8"), ("uniform", "uint16"), ("uniform", "int64"),
         ("sorted", "int32"), ("sorted", "int8"), ("outlier_high", "int32"), ("outlier_high", "int16"),
         ("outlier_low", "int32"), ("outlier_low", "int64"), ("normal", "int32"), ("dtype_edge", "int8"),
         ("dtype_edge", "uint8"), ("dtype_edge", "int16"), ("wide", "int8")]


@pytest.mark.parametrize("layout,dtype", CASES)
def test_sampled_range_equals_exact_range(layout, dtype, monkeypatch):
    import vaex_amd
    from vaex_amd import groupby as vg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(CASES.index((layout, dtype)))
    keys = _keys(layout, dtype, rng)
    v = rng.normal(size=N)
    v[::1013] = np.nan
    guesses = []
    real = vg._sampled_range

    def spy(*a):
        r = real(*a)
        guesses.append(r)
        return r

    monkeypatch.setattr(vg, "_sampled_range", spy)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), v=DeviceArray.from_numpy(v))
    agg = {"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v"), "n": "count"}
    got = df.groupby("key", agg=agg)
    assert guesses and (guesses[0] is not None) == (layout != "wide")  # the sampled route ran
    exact = df.groupby("key", agg=agg, _speculate=False)
    for name in ["key", "v_sum", "v_count", "n"]:
        a, b = got[name].to_numpy(), exact[name].to_numpy()
        assert a.dtype == b.dtype, name
        if name == "v_sum":  # float sums: the atomic order differs run to run
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12, err_msg=name)
        else:
            np.testing.assert_array_equal(a, b, err_msg=name)
    uk, s, c = oracle.groupby_reference(keys, v)
    gk = got["key"].to_numpy()
    assert gk.tolist() == uk.tolist()  # dense and hash routes: sorted by key
    np.testing.assert_array_equal(got["v_count"].to_numpy(), c)
    np.testing.assert_allclose(got["v_sum"].to_numpy(), s, rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(got["n"].to_numpy(), np.unique(keys, return_counts=True)[1])


def test_sampled_range_host_columns_use_exact_pass():
    """Host (numpy) key columns and short columns keep the exact min/max pass (the sample
    reads HBM and only pays off at size)."""
    import vaex_amd
    from vaex_amd import groupby as vg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(2)
    keys = rng.integers(0, 3000, N).astype(np.int32)
    assert vg._sampled_range(keys, N, keys.dtype) is None
    short = DeviceArray.from_numpy(keys[:1000])
    assert vg._sampled_range(short, 1000, keys.dtype) is None
    lo, hi = vg._sampled_range(DeviceArray.from_numpy(keys), N, keys.dtype)
    assert lo <= keys.min() and hi >= keys.max()
    df = vaex_amd.from_arrays(key=keys, v=np.ones(N))
    got = df.groupby("key", agg={"n": "count"})
    np.testing.assert_array_equal(got["n"].to_numpy(), np.bincount(keys)[np.unique(keys)])


def test_cached_device_blocks_are_reused_and_trimmed():
    """vh_malloc / vh_free go through the device block cache (multi-GB query temporaries
    are reused instead of re-allocated); trim_caches hands everything back and later
    allocations still work."""
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    _lib.trim_caches()  # no other cached block of this size from earlier tests
    a = DeviceArray.from_numpy(np.arange(1 << 20, dtype=np.int64))
    p = a.ptr
    del a
    b = DeviceArray.empty(1 << 20, np.int64)
    assert b.ptr == p  # the freed block came back
    del b
    _lib.trim_caches()
    c = DeviceArray.from_numpy(np.arange(1000, dtype=np.int32))
    np.testing.assert_array_equal(c.to_numpy(), np.arange(1000, dtype=np.int32))
    np.testing.assert_array_equal(c.to_numpy(pinned=True), np.arange(1000, dtype=np.int32))
