"""DataFrame-level parity (count/sum/mean/min/max/first/minmax, groupby, binby) on the GPU,
against the reference's own test expectations (tests/golden/kats.json) and the oracle."""
import numpy as np
import pytest

from conftest import load_kats
from oracle import oracle

pytestmark = pytest.mark.gpu

KATS = load_kats()
API = {k["name"]: k for k in KATS["api"]}


def vx():
    import vaex_amd
    return vaex_amd


def _df(name):
    k = API[name]
    return vx().from_arrays(**{c: np.array(v, dtype="f8" if any(isinstance(e, float) for e in v) else "i8")
                                for c, v in k["columns"].items()})


def _run(df, call):
    op = call["op"]
    kw = {}
    for key in ("binby", "limits", "shape"):
        if key in call:
            kw[key] = call[key]
    if "selection" in call:
        df.select(call["selection"])
        kw["selection"] = True
    if op == "first":
        order = call["order"]
        if order.startswith("-"):
            df.add_virtual_column("neg_" + order[1:], "-" + order[1:])
            order = "neg_" + order[1:]
        return df.first(call["expression"], order, **kw)
    f = getattr(df, op)
    return f(call.get("expression"), **kw) if op == "count" else f(call["expression"], **kw)


@pytest.mark.parametrize("name", ["mean_basics", "count_basics_1d", "first"])
def test_api_kats(name):
    for call in API[name]["calls"]:
        df = _df(name)
        got = _run(df, call)
        assert np.asarray(got).tolist() == call["expected"], call


def test_count_1d_edges():
    """tests/agg_test.py:150-158 through df._agg with edges=True."""
    df = vx().from_arrays(x=np.array([-1, -2, 0.5, 1.5, 4.5, 5], dtype="f8"))
    binner = df._binner_scalar("x", [0, 5], 5)
    grid = df._agg(vx().agg.count(edges=True), (binner,))
    assert grid.tolist() == [0, 2, 1, 1, 0, 0, 1, 1]


def test_count_1d_ordinal_delay():
    """tests/agg_test.py:171-181: add_tasks + df.execute()."""
    df = vx().from_arrays(x=np.array([-1, -2, 0, 1, 4, 5], dtype="i8"))
    binner = df._binner_ordinal("x", 5)
    agg = vx().agg.count(edges=True)
    tasks, result = agg.add_tasks(df, (binner,))
    df.execute()
    assert result.get().tolist() == [0, 2, 1, 1, 0, 0, 1, 1]


def test_big_endian_and_strides():
    """tests/agg_test.py:257-281."""
    x = np.arange(10, dtype=">f8")
    y = np.zeros(10, dtype=">f8")
    df = vx().from_arrays(x=x, y=y)
    counts = df.count(binby=[df.x, df.y], limits=[[-0.5, 9.5], [-0.5, 0.5]], shape=[10, 1])
    assert counts.ravel().tolist() == np.ones(10).tolist()
    ar = np.zeros((10, 2)).reshape(20)
    x = ar[::2]
    x[:] = np.arange(10)
    df = vx().from_arrays(x=x)
    assert df.count(binby=df.x, limits=[-0.5, 9.5], shape=10).tolist() == np.ones(10).tolist()


def test_count_vs_numpy_minmax_limits():
    """tests/count_test.py:23-38: limits='minmax' runs the GPU min/max pre-pass; counts equal
    np.histogram except the last bin (the max lands in the overflow cell)."""
    rng = np.random.default_rng(3)
    x = rng.normal(size=100000)
    df = vx().from_arrays(x=x)
    counts = df.count(binby="x", shape=4, limits="minmax")
    lo, hi = df.minmax("x")
    assert (lo, hi) == oracle.minmax_f64(x)
    ref, _ = np.histogram(x, bins=4, range=(lo, hi))
    assert counts[:-1].tolist() == ref[:-1].tolist()


def test_delay_merges_into_one_pass():
    rng = np.random.default_rng(4)
    x, w = rng.normal(size=50000), rng.random(50000)
    df = vx().from_arrays(x=x, w=w)
    before = df.executor.passes
    c = df.count(binby="x", limits=[-3, 3], shape=64, delay=True)
    s = df.sum("w", binby="x", limits=[-3, 3], shape=64, delay=True)
    m = df.mean("w", binby="x", limits=[-3, 3], shape=64, delay=True)
    df.execute()
    assert df.executor.passes == before + 1
    spec = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=64)
    ec = oracle.extract_central_part(oracle.compute_grid([spec], "count"))
    es = oracle.extract_central_part(oracle.compute_grid([spec], "sum", data=w))
    assert c.get().tolist() == ec.tolist()
    np.testing.assert_allclose(s.get(), es, rtol=1e-6)
    with np.errstate(invalid="ignore", divide="ignore"):
        np.testing.assert_allclose(m.get(), es / ec, rtol=1e-6)


def test_masked_column_and_selection():
    rng = np.random.default_rng(8)
    n = 40000
    x = rng.normal(size=n)
    w = np.ma.array(rng.normal(size=n), mask=rng.random(n) < 0.2)
    df = vx().from_arrays(x=x, w=w)
    df.select("x > 0")
    got = df.sum("w", binby="x", limits=[-3, 3], shape=10, selection=True)
    keep = ((x > 0) & ~np.ma.getmaskarray(w)).astype(np.uint8)
    spec = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=10)
    exp = oracle.extract_central_part(oracle.compute_grid([spec], "sum", data=w.data, mask=keep))
    np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-12)
    cnt = df.count("w", binby="x", limits=[-3, 3], shape=10)
    keep2 = (~np.ma.getmaskarray(w)).astype(np.uint8)
    exp2 = oracle.extract_central_part(oracle.compute_grid([spec], "count", data=w.data, mask=keep2))
    assert cnt.tolist() == exp2.tolist()


def test_small_chunks_multi_chunk_path(monkeypatch):
    """small_buffer (tests/common.py:45-56): chunk_size=3 exercises many chunks + reduce."""
    monkeypatch.setenv("VAEX_CHUNK_SIZE", "3")
    x = np.arange(10, dtype="f8")
    y = x ** 2
    df = vx().from_arrays(x=x, y=y)
    assert df.first("y", "x", binby="x", limits=[0, 10], shape=2).tolist() == [0, 25]
    assert df.sum("y", binby="x", limits=[0, 10], shape=10).tolist() == y.tolist()
    assert df.count().item() == 10


@pytest.mark.parametrize("name", ["groupby_1d", "groupby_1d_nan", "groupby_2d"])
def test_groupby_kats(name):
    call = API[name]["calls"][0]
    df = _df(name)
    by = call["by"]
    dfg = df.groupby(by=by, agg={"count": vx().agg.count()}, sort=call["sort"])
    if name == "groupby_1d_nan":
        dfg = dfg.sort("g")
    keys = call["expected_keys"]
    if isinstance(by, list):
        for k, col in zip(keys, by):
            assert dfg[col].tolist() == k
    else:
        got = dfg[by].tolist()
        if keys[-1] == "nan":
            assert got[:-1] == keys[:-1] and np.isnan(got[-1])
        else:
            assert got == keys
    assert dfg["count"].tolist() == call["expected_count"]


def test_binby_2d_kat():
    call = API["binby_2d"]["calls"][0]
    df = _df("binby_2d")
    ar = df.binby(by=call["by"], agg=vx().agg.count(), sort=True)
    assert ar.data.tolist() == call["expected"]
    assert ar.dims == ("g", "h")


def test_categorical_groupby():
    """tests/groupby_test.py:127-141: categorized ints bin by BinnerOrdinal(min, N) directly."""
    g = np.array([0, 0, 0, 0, 1, 1, 1, 1, 2, 2])
    df = vx().from_arrays(g=g)
    df.categorize("g", labels=["cat", "dog", "snake"], inplace=True)
    dfg = df.groupby(by="g", agg="count")
    assert dfg.g.tolist() == ["cat", "dog", "snake"]
    assert dfg["count"].tolist() == [4, 4, 2]


@pytest.mark.parametrize("dtype,lo,hi", [("int64", 3_500_000_000, 5_000_000_000),
                                         ("int32", -2 ** 31, 2 ** 31 - 1),
                                         ("int8", -128, 127), ("float32", -1e3, 1e3)])
@pytest.mark.parametrize("hbm", [False, True])
def test_var_std_cast_to_float64(dtype, lo, hi, hbm):
    """agg.py:196-224: var/std take the moments of astype(x, 'float64').  Integer squares
    here overflow int64 (int64 >= 3.04e9, int32 near 2^31), so an integer moment grid would
    wrap; the result must equal the oracle's float64 restatement within 1e-6."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(11)
    n = 200_000
    g = rng.normal(size=n)
    if dtype.startswith("float"):
        v = rng.uniform(lo, hi, n).astype(dtype)
    else:
        v = rng.integers(lo, hi, n, endpoint=True, dtype=np.int64).astype(dtype)
    cols = dict(g=g, v=v)
    df = vx().from_arrays(**({k: DeviceArray.from_numpy(a) for k, a in cols.items()} if hbm else cols))
    spec = oracle.Binner("scalar", g, vmin=-3, vmax=3, bins=16)
    exp = oracle.extract_central_part(oracle.var_grid([spec], v))
    got = df.var("v", binby="g", limits=[-3, 3], shape=16)
    assert got.dtype == np.float64
    np.testing.assert_allclose(got, exp, rtol=1e-6)
    np.testing.assert_allclose(df.std("v", binby="g", limits=[-3, 3], shape=16), exp ** 0.5, rtol=1e-6)
    # no binby: one cell (the whole column)
    whole = oracle.var_grid([], v, n=n)
    np.testing.assert_allclose(df.var("v"), whole, rtol=1e-6)


def test_zero_d_grid_after_binned_query():
    """Aggregations without binby (one cell) right after binned ones on the same frame: the
    small-grid pass's cell scratch must be cell 0 for every row, not what a previous query
    left there."""
    rng = np.random.default_rng(12)
    n = 300_000
    x = rng.normal(size=n)
    v = rng.integers(-1000, 1000, n)
    df = vx().from_arrays(x=x, v=v)
    df.count(binby="x", limits=[-3, 3], shape=100)
    assert int(df.sum("v")) == int(v.sum())
    assert int(df.count("v")) == n
    assert int(df.min("v")) == int(v.min()) and int(df.max("v")) == int(v.max())


def test_minmax_binby_and_empty_cells():
    """minmax(expr, binby=...) (dataframe.py:1276-1333): per cell [min, max] of the
    expression, NaN ignored, empty cells [inf, -inf] (the OP_MIN_MAX initial values)."""
    import vaex_amd
    rng = np.random.default_rng(31)
    n = 200_000
    x = rng.normal(size=n)
    y = rng.normal(size=n)
    y[::17] = np.nan
    df = vaex_amd.from_arrays(x=x, y=y)
    got = df.minmax("y", binby="x", shape=12, limits=[-6, 6])
    assert got.shape == (12, 2)
    b = oracle.Binner("scalar", x, vmin=-6, vmax=6, bins=12)
    cell = oracle.bin_indices([b], n).astype(np.int64) - 2  # central cells 0..11
    for c in range(12):
        sel = (cell == c) & ~np.isnan(y)
        if sel.any():
            assert got[c, 0] == np.min(y[sel]) and got[c, 1] == np.max(y[sel])
        else:
            assert got[c, 0] == np.inf and got[c, 1] == -np.inf
    two = df.minmax(["x", "y"], binby="x", shape=4, limits=[-1, 1])
    assert two.shape == (2, 4, 2)


def test_limits_percentage_matches_restatement():
    """limits('x', '90%') / limits_percentage (dataframe.py:1570-1614): the cumulative
    16384-bin count over [min, max] interpolated at (1 -+ p) / 2 -- the same counts the
    oracle bins (the max row falls in the overflow cell there too)."""
    import vaex_amd
    rng = np.random.default_rng(32)
    x = rng.standard_t(3, size=300_000)
    df = vaex_amd.from_arrays(x=x)
    vmin, vmax = x.min(), x.max()
    size = 16384
    b = oracle.Binner("scalar", x, vmin=vmin, vmax=vmax, bins=size)
    counts = oracle.extract_central_part(oracle.compute_grid([b], "count"))
    cum = np.concatenate([[0], np.cumsum(counts)])
    cum = cum / cum.max()
    for pct in (90, 99.7):
        f = (1 - pct / 100.) / 2
        exp = np.interp([f, 1 - f], cum, np.linspace(vmin, vmax, size + 1))
        np.testing.assert_allclose(df.limits("x", f"{pct}%"), exp, rtol=0, atol=0)
        np.testing.assert_allclose(df.limits_percentage("x", pct), exp, rtol=0, atol=0)
    # limits of a binby given as a percentage string
    c = df.count(binby="x", limits="90%", shape=10)
    assert int(np.asarray(c).sum()) < len(x)
    with pytest.raises(AttributeError):
        df.limits("x", "3sigma")
