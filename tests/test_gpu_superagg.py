"""Parity of the HIP superagg surface (libvaexhip through the C-ABI) with the CPU oracle.

Integer counts and bin indices must be bit-exact; float64 sums within 1e-6 relative
(north_star); min/max/first are exact."""
import zlib

import numpy as np
import pytest

from conftest import kat_array, load_kats
from oracle import oracle

pytestmark = pytest.mark.gpu

KATS = load_kats()
DTYPES = ["float64", "float32", "int64", "int32", "int16", "int8", "uint64", "uint32", "uint16", "uint8", "bool"]


def sa():
    import vaex_amd.superagg as m
    return m


def _binner_cls(kind, ar):
    from vaex_amd.utils import find_type_from_dtype
    return find_type_from_dtype(sa(), "BinnerScalar_" if kind == "scalar" else "BinnerOrdinal_", ar.dtype)


def _agg_cls(kind, dtype):
    from vaex_amd.utils import find_type_from_dtype
    name = {"count": "AggCount_", "sum": "AggSum_", "min": "AggMin_", "max": "AggMax_", "first": "AggFirst_",
            "sum_moment": "AggSumMoment_"}[kind]
    return find_type_from_dtype(sa(), name, dtype)


@pytest.mark.parametrize("kat", KATS["superagg"], ids=[k["name"] for k in KATS["superagg"]])
def test_superagg_kat(kat):
    binners = []
    for s in kat["binners"]:
        ar = kat_array(s)
        ar = np.ascontiguousarray(ar)
        if s["kind"] == "scalar":
            b = _binner_cls("scalar", ar)("x", s["vmin"], s["vmax"], s["bins"])
        else:
            b = _binner_cls("ordinal", ar)("x", s["ordinal_count"], s["min_value"])
        b.set_data(ar)
        binners.append(b)
    grid = sa().Grid(binners)
    a = kat["agg"]
    if "data" in a:
        data = np.array(a["data"], dtype=a["dtype"])
        agg = _agg_cls(a["kind"], data.dtype)(grid)
        agg.set_data(data, 0)
    else:
        agg = _agg_cls(a["kind"], np.dtype("float64"))(grid)
    view = np.asarray(agg)
    grid.bin([agg])
    if "expected" in kat:
        assert view.tolist() == kat["expected"]
    if "expected_diagonal" in kat:
        assert [view[k, k] for k in range(view.shape[0])] == kat["expected_diagonal"]
    if "expected_central" in kat:
        assert view[(slice(2, -1),) * view.ndim].tolist() == kat["expected_central"]
    if "expected_central_diagonal" in kat:
        assert np.diagonal(view[2:-1, 2:-1]).tolist() == kat["expected_central_diagonal"]


def test_live_view_mutation_before_bin():
    """tests/internal/superagg_tests.py:86-106 pattern: the array view is live and writable."""
    x = np.array([-1, -1, 0, 0, 4, 6, 10], dtype="i8")
    y = np.array([-1, 2, 4, 1, 9, 6, 10], dtype="i8")
    b = sa().BinnerOrdinal_int64("x", 5, 0)
    b.set_data(x)
    grid = sa().Grid([b])
    agg = sa().AggMax_int64(grid)
    view = np.asarray(agg)
    view[:] = -100
    agg.set_data(y, 0)
    grid.bin([agg])
    assert view.tolist() == [-100, 2, 4, -100, -100, -100, 9, 10]
    agg = sa().AggMin_int64(grid)
    view = np.asarray(agg)
    view[:] = 100
    agg.set_data(y, 0)
    grid.bin([agg])
    assert view.tolist() == [100, -1, 1, 100, 100, 100, 9, 6]


def test_errors():
    b = sa().BinnerScalar_float64("x", 0, 1, 4)
    with pytest.raises(RuntimeError, match="Expected a 1d array"):
        b.set_data(np.zeros((2, 2)))
    with pytest.raises(RuntimeError, match="Itemsize of data and binner are not equal"):
        b.set_data(np.zeros(4, dtype="f4"))
    grid = sa().Grid([])
    with pytest.raises(RuntimeError, match="no binners set and no length given"):
        grid.bin([sa().AggCount_int64(grid)])
    b.set_data(np.zeros(4))
    grid = sa().Grid([b])
    with pytest.raises(RuntimeError, match="data not set"):
        grid.bin([sa().AggSum_float64(grid)])
    agg = sa().AggFirst_float64(grid)
    agg.set_data(np.zeros(4), 0)
    with pytest.raises(RuntimeError, match="data2 not set"):
        grid.bin([agg])


def _random_column(rng, dtype, n, with_nan=True):
    dt = np.dtype(dtype)
    if dt.kind == "f":
        a = rng.normal(0, 3, n).astype(dt)
        if with_nan:
            a[rng.random(n) < 0.05] = np.nan
    elif dt.kind == "b":
        a = rng.random(n) < 0.5
    else:
        info = np.iinfo(dt)
        lo, hi = max(info.min, -20), min(info.max, 40)
        a = rng.integers(lo, hi, n).astype(dt)
    return a


def _oracle_grid(binner_specs, kind, data=None, data2=None, mask=None, moment=2):
    return oracle.compute_grid(binner_specs, kind, data=data, data2=data2, mask=mask, moment=moment)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("flip", [False, True])
def test_binners_random_parity(dtype, flip):
    """Both binner kinds, every dtype, native and byte-swapped, with a binner mask."""
    rng = np.random.default_rng(zlib.crc32(f"{dtype}{flip}".encode()))
    n = 5000
    a = _random_column(rng, dtype, n)
    b2 = _random_column(rng, "float64", n)
    if flip:
        a = a.astype(a.dtype.newbyteorder(">"))
    mask = (rng.random(n) < 0.1).astype(np.uint8)
    for kind in ("scalar", "ordinal"):
        if kind == "scalar":
            spec = oracle.Binner("scalar", a, vmin=-7.5, vmax=25.0, bins=13, mask=mask)
            gb = _binner_cls("scalar", a)("a", -7.5, 25.0, 13)
        else:
            spec = oracle.Binner("ordinal", a, ordinal_count=17, min_value=-3 if np.dtype(dtype).kind == "i" else 2,
                                 mask=mask)
            gb = _binner_cls("ordinal", a)("a", 17, spec.min_value)
        gb.set_data(a)
        gb.set_data_mask(mask)
        spec2 = oracle.Binner("scalar", b2, vmin=-4, vmax=4, bins=5)
        gb2 = sa().BinnerScalar_float64("b", -4, 4, 5)
        gb2.set_data(b2)
        grid = sa().Grid([gb, gb2])
        agg = sa().AggCount_int64(grid)
        grid.bin([agg])
        expected = _oracle_grid([spec, spec2], "count")
        assert np.asarray(agg).tolist() == expected.tolist(), kind


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("kind", ["count", "sum", "min", "max", "first", "sum_moment"])
def test_aggregators_random_parity(dtype, kind):
    rng = np.random.default_rng(zlib.crc32(f"{dtype}{kind}".encode()))
    n = 20000
    x = rng.normal(0, 1, n)
    data = _random_column(rng, dtype, n)
    data2 = _random_column(rng, dtype, n)
    keep = (rng.random(n) < 0.8).astype(np.uint8)
    spec = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=32)
    gb = sa().BinnerScalar_float64("x", -3, 3, 32)
    gb.set_data(x)
    grid = sa().Grid([gb])
    agg = _agg_cls(kind, data.dtype)(grid, *([2] if kind == "sum_moment" else []))
    agg.set_data(data, 0)
    if kind == "first":
        agg.set_data(data2, 1)
        expected = _oracle_grid([spec], "first", data=data, data2=data2)
    else:
        agg.set_data_mask(keep)
        expected = _oracle_grid([spec], kind, data=data, mask=keep, moment=2)
    grid.bin([agg])
    got = np.asarray(agg)
    if kind in ("sum", "sum_moment") and got.dtype.kind == "f":
        np.testing.assert_allclose(got, expected, rtol=1e-6, atol=1e-9)
    else:
        np.testing.assert_array_equal(got, expected)


def test_count_with_data_skips_nan_and_mask():
    rng = np.random.default_rng(5)
    n = 10000
    x = rng.normal(size=n)
    w = rng.normal(size=n)
    w[::7] = np.nan
    keep = (rng.random(n) < 0.7).astype(np.uint8)
    spec = oracle.Binner("scalar", x, vmin=-2, vmax=2, bins=20)
    gb = sa().BinnerScalar_float64("x", -2, 2, 20)
    gb.set_data(x)
    grid = sa().Grid([gb])
    c = sa().AggCount_float64(grid)
    c.set_data(w, 0)
    c.set_data_mask(keep)
    s = sa().AggSum_float64(grid)
    s.set_data(w, 0)
    s.set_data_mask(keep)
    grid.bin([c, s])
    np.testing.assert_array_equal(np.asarray(c), _oracle_grid([spec], "count", data=w, mask=keep))
    np.testing.assert_allclose(np.asarray(s), _oracle_grid([spec], "sum", data=w, mask=keep), rtol=1e-6, atol=1e-12)


def test_scalar_grid_no_binners():
    """Grid([]) with an explicit length: everything lands in cell 0 (df.count() without binby)."""
    grid = sa().Grid([])
    c = sa().AggCount_int64(grid)
    s = sa().AggSum_float64(grid)
    w = np.arange(100, dtype="f8")
    s.set_data(w, 0)
    grid.bin([c, s], 100)
    assert np.asarray(c).item() == 100
    assert np.asarray(s).item() == w.sum()


@pytest.mark.parametrize("kind", ["count", "sum", "min", "max", "first"])
def test_reduce_parts(kind):
    rng = np.random.default_rng(7)
    n = 30000
    x = rng.normal(size=n)
    w = rng.normal(size=n)
    o = rng.permutation(n).astype("f8")
    spec = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=16)
    expected = _oracle_grid([spec], kind, data=w, data2=o) if kind != "count" else _oracle_grid([spec], "count")
    parts = []
    for p in range(3):
        sl = slice(p * n // 3, (p + 1) * n // 3)
        gb = sa().BinnerScalar_float64("x", -3, 3, 16)
        gb.set_data(x[sl])
        grid = sa().Grid([gb])
        agg = _agg_cls(kind, np.dtype("f8"))(grid)
        if kind != "count":
            agg.set_data(w[sl], 0)
        if kind == "first":
            agg.set_data(o[sl], 1)
        grid.bin([agg])
        parts.append(agg)
    parts[0].reduce(parts[1:])
    got = np.asarray(parts[0])
    if kind == "sum":
        np.testing.assert_allclose(got, expected, rtol=1e-6, atol=1e-9)
    else:
        np.testing.assert_array_equal(got, expected)


def test_device_resident_columns_match_host():
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(11)
    n = 200000
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=100)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=100)
    exp_c = _oracle_grid([bx, by], "count")
    exp_s = _oracle_grid([bx, by], "sum", data=w)
    dx, dy, dw = DeviceArray.from_numpy(x), DeviceArray.from_numpy(y), DeviceArray.from_numpy(w)
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 100), sa().BinnerScalar_float64("y", -4, 4, 100)
    gx.set_data(dx)
    gy.set_data(dy)
    grid = sa().Grid([gx, gy])
    c, s = sa().AggCount_int64(grid), sa().AggSum_float64(grid)
    s.set_data(dw, 0)
    grid.bin([c, s])
    np.testing.assert_array_equal(np.asarray(c), exp_c)
    np.testing.assert_allclose(np.asarray(s), exp_s, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("dist,n", [("normal", 4_000_000), ("uniform", 4_000_000), ("normal", 1_048_577)])
@pytest.mark.parametrize("with_sum", [False, True])
def test_tiled_path_large_grid(dist, n, with_sum):
    """1027x1027 grid (the C2 shape) over >1M rows takes the tile-partitioned LDS path
    (odd n: the last row goes through the global-atomic path)."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(13)
    if dist == "normal":
        x, y = rng.normal(size=n), rng.normal(size=n)
    else:
        x, y = rng.uniform(-4.5, 4.5, n), rng.uniform(-4.5, 4.5, n)
    x[::1001] = np.nan
    w = rng.random(n)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    exp_c = _oracle_grid([bx, by], "count")
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    aggs = [sa().AggCount_int64(grid)]
    if with_sum:
        s = sa().AggSum_float64(grid)
        s.set_data(DeviceArray.from_numpy(w), 0)
        aggs.append(s)
    grid.bin(aggs)
    np.testing.assert_array_equal(np.asarray(aggs[0]), exp_c)
    if with_sum:
        np.testing.assert_allclose(np.asarray(aggs[1]), _oracle_grid([bx, by], "sum", data=w), rtol=1e-6, atol=1e-12)


def _layout(x, y, w, layout):
    """The same rows in another order: sorted by y (the slow binby dimension), sorted by x,
    or clustered (runs of 50 000 rows from random places)."""
    if layout == "shuffled":
        return x, y, w
    if layout == "sorted_y":
        o = np.argsort(y, kind="stable")
    elif layout == "sorted_x":
        o = np.argsort(x, kind="stable")
    else:  # runs of 50 000 rows of similar y, the runs in random order
        o = np.argsort(y, kind="stable")
        chunks = [o[b:b + 50_000] for b in range(0, len(x), 50_000)]
        np.random.default_rng(5).shuffle(chunks)
        o = np.concatenate(chunks)
    return x[o], y[o], w[o]


@pytest.mark.parametrize("layout", ["shuffled", "sorted_y", "sorted_x", "clustered"])
@pytest.mark.parametrize("with_sum", [False, True])
def test_tile_path_row_layouts_match_oracle(layout, with_sum):
    """Pass-A workgroups take batches w, w + W, ... so sorted or clustered rows spread over
    every workgroup like shuffled ones: bit-exact counts, sums within 1e-6, for every row
    order of the C2-shape query (1027^2 grid, NaN rows included)."""
    from vaex_amd.device import DeviceArray
    n = 6_000_000
    rng = np.random.default_rng(29)
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    x[::997] = np.nan
    w[::13] = np.nan
    x, y, w = _layout(x, y, w, layout)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    dw = DeviceArray.from_numpy(w)
    aggs = [sa().AggCount_int64(grid)]
    if with_sum:
        s = sa().AggSum_float64(grid)
        s.set_data(dw, 0)
        cw = sa().AggCount_float64(grid)  # count(w) of float64 data: keyed on w NaN-ness
        cw.set_data(dw, 0)
        aggs += [s, cw]
    grid.bin(aggs)
    np.testing.assert_array_equal(np.asarray(aggs[0]), _oracle_grid([bx, by], "count"))
    if with_sum:
        np.testing.assert_allclose(np.asarray(aggs[1]), _oracle_grid([bx, by], "sum", data=w), rtol=1e-6, atol=1e-12)
        np.testing.assert_array_equal(np.asarray(aggs[2]), _oracle_grid([bx, by], "count", data=w))


def test_removed_experiment_switches_change_nothing(monkeypatch):
    """The product library reads no ablation switch: the old experiment variables (results
    wrong by design) and the removed XCD-resident switch leave every result unchanged."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    n = 4_000_000
    rng = np.random.default_rng(3)
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    keys = rng.integers(0, 300_000, n).astype(np.int32) * 13
    cols = {"x": DeviceArray.from_numpy(x), "y": DeviceArray.from_numpy(y), "w": DeviceArray.from_numpy(w),
            "k": DeviceArray.from_numpy(keys)}

    def run():
        df = vaex_amd.from_arrays(**cols)
        c = np.asarray(df.count(binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024))
        s = np.asarray(df.sum("w", binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024))
        g = df.groupby("k", agg={"n": "count", "s": vaex_amd.agg.sum("w")}, sort=True)
        h = df.groupby("k", agg={"n": "count"}, sort=True, assume_sparse=True)
        return c, s, g["k"].to_numpy(), g["n"].to_numpy(), g["s"].to_numpy(), h["k"].to_numpy(), h["n"].to_numpy()

    ref = run()
    for var in ("VH_TILE_DEBUG", "VH_HA_DEBUG", "VH_SI_DEBUG"):
        monkeypatch.setenv(var, "4095")  # every experiment bit
        got = run()
        monkeypatch.delenv(var)
        for a, b in zip(got, ref):
            if a.dtype.kind == "f":
                np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12, err_msg=var)
            else:
                np.testing.assert_array_equal(a, b, err_msg=var)
    monkeypatch.setenv("VH_RESIDENT", "1")
    got = run()
    np.testing.assert_array_equal(got[0], ref[0])


@pytest.mark.parametrize("dtype", ["float64", "float32", "int16"])
def test_tile_path_min_max_large_grid(dtype):
    """AggMin / AggMax on the C2-shape 1027^2 grid take the tile path (LDS min / max cells,
    typed CAS flush); equal to the oracle, NaN rows skipped, untouched cells keep the fill."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(41)
    n = 3_000_000
    x, y = rng.normal(size=n), rng.normal(size=n)
    if dtype.startswith("float"):
        w = rng.normal(size=n).astype(dtype)
        w[::17] = np.nan
    else:
        w = rng.integers(-30000, 30000, n).astype(dtype)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    dw = DeviceArray.from_numpy(w)
    mx = getattr(sa(), "AggMax_" + dtype)(grid)
    mn = getattr(sa(), "AggMin_" + dtype)(grid)
    mx.set_data(dw, 0)
    mn.set_data(dw, 0)
    grid.bin([mx, mn])
    np.testing.assert_array_equal(np.asarray(mx), _oracle_grid([bx, by], "max", data=w))
    np.testing.assert_array_equal(np.asarray(mn), _oracle_grid([bx, by], "min", data=w))


@pytest.mark.parametrize("dtype", ["float64", "float32", "int32"])
def test_tile_path_shared_value_slots(dtype):
    """sum / min / max of one column and the sum of a second on the 1027^2 grid: one tile
    group carrying two value slots (the three aggregators of the first column share one);
    equal to the oracle (integer sums exact, float sums to 1e-9)."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(43)
    n = 3_000_000
    x, y = rng.normal(size=n), rng.normal(size=n)
    if dtype.startswith("float"):
        w = rng.normal(size=n).astype(dtype)
        w[::19] = np.nan
    else:
        w = rng.integers(-30000, 30000, n).astype(dtype)
    w2 = rng.normal(size=n)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    dw, dw2 = DeviceArray.from_numpy(w), DeviceArray.from_numpy(w2)
    up = "float64" if dtype.startswith("float") else "int64"
    s = getattr(sa(), "AggSum_" + dtype)(grid)
    mn = getattr(sa(), "AggMin_" + dtype)(grid)
    mx = getattr(sa(), "AggMax_" + dtype)(grid)
    s2 = sa().AggSum_float64(grid)
    for a in (s, mn, mx):
        a.set_data(dw, 0)
    s2.set_data(dw2, 0)
    grid.bin([s, mn, mx, s2])
    np.testing.assert_array_equal(np.asarray(mx), _oracle_grid([bx, by], "max", data=w))
    np.testing.assert_array_equal(np.asarray(mn), _oracle_grid([bx, by], "min", data=w))
    ref_s = _oracle_grid([bx, by], "sum", data=w)
    if up == "int64":
        np.testing.assert_array_equal(np.asarray(s), ref_s)
    else:
        np.testing.assert_allclose(np.asarray(s), ref_s, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(np.asarray(s2), _oracle_grid([bx, by], "sum", data=w2), rtol=1e-9, atol=1e-9)


def test_host_staging_multiple_chunks():
    """Host columns longer than one staging chunk (16 Mi rows)."""
    n = (1 << 24) + 12345
    rng = np.random.default_rng(17)
    x = rng.normal(size=n)
    spec = oracle.Binner("scalar", x, vmin=-5, vmax=5, bins=256)
    gb = sa().BinnerScalar_float64("x", -5, 5, 256)
    gb.set_data(x)
    grid = sa().Grid([gb])
    c = sa().AggCount_int64(grid)
    grid.bin([c])
    np.testing.assert_array_equal(np.asarray(c), _oracle_grid([spec], "count"))


@pytest.mark.parametrize("bins,nsums", [(3000, 1), (4000, 2), (2000, 0)])
def test_tiled_path_many_tiles(bins, nsums):
    """Grids with 1000-4000 tiles: the multi-batch staging of pass A no longer fits the LDS,
    so the one-batch fast kernel (or the global-atomic path) takes over; same results."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(bins)
    n = 3_000_000
    x, y = rng.uniform(-1.1, 1.1, n), rng.uniform(-1.1, 1.1, n)
    ws = [rng.random(n) for _ in range(nsums)]
    bx = oracle.Binner("scalar", x, vmin=-1, vmax=1, bins=bins)
    by = oracle.Binner("scalar", y, vmin=-1, vmax=1, bins=bins)
    gx, gy = sa().BinnerScalar_float64("x", -1, 1, bins), sa().BinnerScalar_float64("y", -1, 1, bins)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    aggs = [sa().AggCount_int64(grid)]
    for w in ws:
        s = sa().AggSum_float64(grid)
        s.set_data(DeviceArray.from_numpy(w), 0)
        aggs.append(s)
    grid.bin(aggs)
    np.testing.assert_array_equal(np.asarray(aggs[0]), _oracle_grid([bx, by], "count"))
    for a, w in zip(aggs[1:], ws):
        np.testing.assert_allclose(np.asarray(a), _oracle_grid([bx, by], "sum", data=w), rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("dtype", ["int8", "int32", "uint16", "uint64", "float32", "bool", "int64"])
def test_tile_path_generic_dtype_sums(dtype):
    """count / sum of non-float64 columns over a 1e5+ cell grid take the tile path with
    per-dtype loads (integer sums accumulate as 64-bit integers, float32 as float64):
    bit-exact integer sums and counts, float sums within 1e-6."""
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(len(dtype))
    n = 3_000_001
    key = rng.integers(0, 200_000, n).astype(np.int32)
    if dtype == "bool":
        v = rng.random(n) > 0.5
    elif dtype == "float32":
        v = rng.normal(size=n).astype(np.float32)
        v[::77] = np.nan
    else:
        info = np.iinfo(dtype)
        v = rng.integers(max(info.min, -100), min(info.max, 100), n).astype(dtype)
        if dtype == "uint64":
            v[::5] = np.uint64(2 ** 63 + 12345)
    spec = oracle.Binner("ordinal", key, ordinal_count=200_000, min_value=0)
    b = sa().BinnerOrdinal_int32("key", 200_000, 0)
    b.set_data(DeviceArray.from_numpy(key))
    grid = sa().Grid([b])
    s = getattr(sa(), "AggSum_" + dtype)(grid)
    s.set_data(DeviceArray.from_numpy(v), 0)
    c = getattr(sa(), "AggCount_" + dtype)(grid)
    c.set_data(DeviceArray.from_numpy(v), 0)
    _lib.timing_reset()
    _lib.timing_enable(True)
    grid.bin([s, c])
    _lib.synchronize()
    _lib.timing_enable(False)
    assert _lib.timing_read("tile_reduce")[0] >= 1, "tile path not used"
    exp_s = _oracle_grid([spec], "sum", data=v)
    exp_c = _oracle_grid([spec], "count", data=v)
    np.testing.assert_array_equal(np.asarray(c), exp_c)
    if dtype == "float32":
        np.testing.assert_allclose(np.asarray(s), exp_s, rtol=1e-6, atol=1e-9)
    else:
        np.testing.assert_array_equal(np.asarray(s), exp_s)


def test_tile_path_three_sums_in_groups():
    """Three sums (h2o q5's shape: two int8 columns and a float32 one) run as two tile
    passes of at most two carried values each."""
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(5)
    n = 2_000_000
    key = rng.integers(0, 300_000, n).astype(np.int32)
    v1 = rng.integers(5, 15, n).astype(np.int8)
    v2 = rng.integers(-5, 5, n).astype(np.int8)
    v3 = rng.normal(size=n).astype(np.float32)
    spec = oracle.Binner("ordinal", key, ordinal_count=300_000, min_value=0)
    b = sa().BinnerOrdinal_int32("key", 300_000, 0)
    b.set_data(DeviceArray.from_numpy(key))
    grid = sa().Grid([b])
    aggs = []
    for v in (v1, v2, v3):
        a = getattr(sa(), "AggSum_" + v.dtype.name)(grid)
        a.set_data(DeviceArray.from_numpy(v), 0)
        aggs.append(a)
    c = sa().AggCount_int64(grid)
    _lib.timing_reset()
    _lib.timing_enable(True)
    grid.bin(aggs + [c])
    _lib.synchronize()
    _lib.timing_enable(False)
    assert _lib.timing_read("tile_reduce")[0] == 2
    np.testing.assert_array_equal(np.asarray(aggs[0]), _oracle_grid([spec], "sum", data=v1))
    np.testing.assert_array_equal(np.asarray(aggs[1]), _oracle_grid([spec], "sum", data=v2))
    np.testing.assert_allclose(np.asarray(aggs[2]), _oracle_grid([spec], "sum", data=v3), rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(np.asarray(c), _oracle_grid([spec], "count"))
