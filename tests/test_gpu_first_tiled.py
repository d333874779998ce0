"""AggFirst over grids too large for one workgroup's LDS: the tile-partitioned engine
(vaex_amd/csrc/first.hip) against the oracle's serial AggFirst (superagg.cpp:436-511,
oracle/superagg_oracle.c or_agg_first): value and order grids bit-exact, including order ties
(the earliest row wins), NaN values / orders (skipped), order values equal to the dtype's max
(never taken: strict `<` against the max-filled order grid), several chunks of host columns
(rows past the first chunk), sorted and clustered row layouts, and binners the fast f64
index does not take (plan_index)."""
import zlib

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _oracle_first(binners, v, o):
    shape = oracle.grid_shape(binners)
    idx = oracle.bin_indices(binners, len(v))
    grid, grid2 = oracle.new_grid("first", oracle._dtype_info(np.asarray(v))[0], shape)
    oracle.aggregate("first", idx, grid, data=v, data2=o, grid2=grid2)
    return grid, grid2


def _run(binner_specs, v, o, device=True):
    """binner_specs: [(superagg class name, column, args...)]; returns (value grid, order grid,
    tiled chunks) flattened in F order like the oracle."""
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    put = DeviceArray.from_numpy if device else (lambda a: a)
    bs = []
    keep = []
    for cls, col, *args in binner_specs:
        b = getattr(superagg, cls)("c", *args)
        dc = put(col)
        keep.append(dc)
        b.set_data(dc)
        bs.append(b)
    grid = superagg.Grid(bs)
    a = getattr(superagg, "AggFirst_" + v.dtype.name)(grid)
    dv, do = put(v), put(o)
    a.set_data(dv, 0)
    a.set_data(do, 1)
    _lib.stat_read("first_tiled_chunks", reset=True)
    grid.bin([a])
    chunks = _lib.stat_read("first_tiled_chunks", reset=True)
    return (np.asarray(a).ravel(order="F").copy(), np.asarray(a.order_grid()).ravel(order="F").copy(), chunks)


def _check(got, exp, o_dtype):
    gv, go, chunks = got
    ev, eo = exp
    assert chunks >= 1, "the tiled AggFirst engine did not run"
    np.testing.assert_array_equal(go.view(f"u{go.dtype.itemsize}") if go.dtype.kind == "f" else go,
                                  eo.view(f"u{eo.dtype.itemsize}") if eo.dtype.kind == "f" else eo)
    np.testing.assert_array_equal(gv.view(f"u{gv.dtype.itemsize}") if gv.dtype.kind == "f" else gv,
                                  ev.view(f"u{ev.dtype.itemsize}") if ev.dtype.kind == "f" else ev)


@pytest.mark.parametrize("order", ["random", "ties", "ascending", "descending", "nan_and_max"])
def test_first_c2_grid(order):
    """first(w, order=o, binby=[x, y], limits=[[-4, 4]] * 2, shape=1024) at 4 Mi rows."""
    rng = np.random.default_rng(zlib.crc32(order.encode()))
    n = (1 << 22) + 3
    x, y = rng.normal(size=n), rng.normal(size=n)
    w = rng.normal(size=n)
    if order == "random":
        o = rng.random(n)
    elif order == "ties":  # few distinct order values: the earliest row of each cell's minimum
        o = rng.integers(0, 5, n).astype(np.float64)
    elif order == "ascending":
        o = np.arange(n, dtype=np.float64)
    elif order == "descending":
        o = np.arange(n, 0, -1, dtype=np.float64)
    else:
        o = rng.integers(0, 40, n).astype(np.float64)
        o[rng.random(n) < 0.05] = np.nan
        w[rng.random(n) < 0.05] = np.nan
        o[rng.random(n) < 0.3] = np.finfo(np.float64).max  # never taken (strict <)
        o[::7] = -0.0  # -0.0 == 0.0: ties by row
        o[3::7] = 0.0
    specs = [("BinnerScalar_float64", x, -4.0, 4.0, 1024), ("BinnerScalar_float64", y, -4.0, 4.0, 1024)]
    got = _run(specs, w, o)
    exp = _oracle_first([oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024),
                         oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)], w, o)
    _check(got, exp, o.dtype)


@pytest.mark.parametrize("dtype", ["int32", "int64", "float32", "uint16", "int8"])
def test_first_dtypes_plan_index(dtype):
    """Value / order columns of other dtypes (the order column shares the value dtype, as the
    reference reinterprets it) under an int32 scalar binner x an ordinal binner: the generic
    plan_index cell path; small integer orders give many ties."""
    rng = np.random.default_rng(7)
    n = 3_000_001
    kx = rng.integers(-1000, 1000, n).astype(np.int32)
    ky = rng.integers(0, 700, n).astype(np.int16)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        v = rng.normal(size=n).astype(dt)
        o = rng.integers(0, 1000, n).astype(dt)
        o[::11] = np.nan
    else:
        info = np.iinfo(dt)
        v = rng.integers(info.min, info.max, n, endpoint=True).astype(dt)
        o = rng.integers(max(info.min, -50), min(info.max, 50), n).astype(dt)
        o[::13] = info.max
    specs = [("BinnerScalar_int32", kx, -1000.0, 1000.0, 2000), ("BinnerOrdinal_int16", ky, 700, 0)]
    got = _run(specs, v, o)
    exp = _oracle_first([oracle.Binner("scalar", kx, vmin=-1000, vmax=1000, bins=2000),
                         oracle.Binner("ordinal", ky, ordinal_count=700, min_value=0)], v, o)
    _check(got, exp, o.dtype)


@pytest.mark.parametrize("layout", ["y_sorted", "clustered"])
def test_first_row_layouts(layout):
    """Rows sorted along the slow grid axis (a tile's rows contiguous) and clustered runs:
    the per-(XCD, tile) streams and spill areas hold them; bit-exact."""
    rng = np.random.default_rng(11)
    n = 1 << 22
    x = rng.normal(size=n)
    if layout == "y_sorted":
        y = np.sort(rng.normal(size=n))
    else:
        runs = rng.integers(1, 20000, n // 1000)
        y = np.repeat(rng.normal(size=len(runs)), runs)[:n]
        y = np.concatenate([y, rng.normal(size=n - len(y))])
    w = rng.random(n)
    o = rng.integers(0, 1000, n).astype(np.float64)
    specs = [("BinnerScalar_float64", x, -4.0, 4.0, 1024), ("BinnerScalar_float64", y, -4.0, 4.0, 1024)]
    got = _run(specs, w, o)
    exp = _oracle_first([oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024),
                         oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)], w, o)
    _check(got, exp, o.dtype)


@pytest.mark.parametrize("layout", ["random", "y_sorted", "clustered"])
def test_first_commit_index_boundaries(layout, monkeypatch):
    """Pass A capped at 2 workgroups (VH_FIRST_MAX_WG): ~640 commits per workgroup, so region
    entries carry the commit index mod 256 and pass B recovers its high bits from the positions
    where it crossed 256 and 512 -- including regions that see fewer than 8 entries between two
    crossings (sorted / clustered rows); order ties resolved by row; bit-exact."""
    monkeypatch.setenv("VH_FIRST_MAX_WG", "2")
    rng = np.random.default_rng(5)
    n = (5 << 20) + 77
    x = rng.normal(size=n)
    if layout == "y_sorted":
        y = np.sort(rng.normal(size=n))
    elif layout == "clustered":
        runs = rng.integers(1, 40000, n // 4000)
        y = np.repeat(rng.normal(size=len(runs)), runs)[:n]
        y = np.concatenate([y, rng.normal(size=n - len(y))])
    else:
        y = rng.normal(size=n)
    w = rng.random(n)
    o = rng.integers(0, 50, n).astype(np.float64)  # ties: the earliest row must win
    specs = [("BinnerScalar_float64", x, -4.0, 4.0, 512), ("BinnerScalar_float64", y, -4.0, 4.0, 512)]
    got = _run(specs, w, o)
    exp = _oracle_first([oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=512),
                         oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=512)], w, o)
    _check(got, exp, o.dtype)


def test_first_host_columns_several_chunks():
    """Host columns staged in 16 Mi-row chunks: chunks after the first carry their global row
    offset (ties between chunks go to the earlier chunk)."""
    rng = np.random.default_rng(12)
    n = (1 << 24) + (1 << 21) + 5
    x, y = rng.normal(size=n), rng.normal(size=n)
    w = rng.normal(size=n)
    o = rng.integers(0, 3, n).astype(np.float64)
    specs = [("BinnerScalar_float64", x, -4.0, 4.0, 512), ("BinnerScalar_float64", y, -4.0, 4.0, 512)]
    got = _run(specs, w, o, device=False)
    assert got[2] >= 2
    exp = _oracle_first([oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=512),
                         oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=512)], w, o)
    _check(got, exp, o.dtype)


def test_first_dataframe_api_large_grid():
    """df.first(w, o, binby=[x, y], shape=1024) through the DataFrame API (tiled engine):
    the central part equals the oracle's grid."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(13)
    n = 1 << 21
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.normal(size=n)
    o = rng.permutation(n).astype(np.float64)
    df = vaex_amd.from_arrays(x=DeviceArray.from_numpy(x), y=DeviceArray.from_numpy(y), w=DeviceArray.from_numpy(w),
                              o=DeviceArray.from_numpy(o))
    got = np.asarray(df.first("w", "o", binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024))
    exp = oracle.extract_central_part(oracle.compute_grid(
        [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024), oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)],
        "first", data=w, data2=o))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("dtype", ["float64", "int32", "float32"])
@pytest.mark.parametrize("order", ["ties", "descending"])
def test_first_small_grid_lds(dtype, order):
    """Small grids (12 B of LDS per cell fit a workgroup): per-workgroup LDS (key, row) cells
    + a fold of the partials (k_first_small) instead of per-row global atomics on few cells;
    bit-exact with ties, NaN and max-valued orders."""
    rng = np.random.default_rng(31)
    n = 3_000_007
    x = rng.normal(size=n)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        v = rng.normal(size=n).astype(dt)
        o = (rng.integers(0, 4, n) if order == "ties" else np.arange(n, 0, -1)).astype(dt)
        v[::19] = np.nan
        o[5::23] = np.nan
        o[::29] = np.finfo(dt).max
    else:
        v = rng.integers(-(1 << 30), 1 << 30, n).astype(dt)
        o = (rng.integers(0, 4, n) if order == "ties" else np.arange(n, 0, -1)).astype(dt)
        o[::29] = np.iinfo(dt).max
    specs = [("BinnerScalar_float64", x, -3.0, 3.0, 256)]
    gv, go, _ = _run(specs, v, o)
    ev, eo = _oracle_first([oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=256)], v, o)
    np.testing.assert_array_equal(go.view(f"u{dt.itemsize}"), eo.view(f"u{dt.itemsize}"))
    np.testing.assert_array_equal(gv.view(f"u{dt.itemsize}"), ev.view(f"u{dt.itemsize}"))


def test_first_small_grid_host_chunks():
    """Host columns in several pipeline chunks on a small 2-d grid: row offsets per chunk."""
    rng = np.random.default_rng(32)
    n = (1 << 24) + 12345
    x, y = rng.normal(size=n), rng.normal(size=n)
    v = rng.normal(size=n)
    o = rng.integers(0, 2, n).astype(np.float64)
    specs = [("BinnerScalar_float64", x, -3.0, 3.0, 40), ("BinnerScalar_float64", y, -3.0, 3.0, 50)]
    gv, go, _ = _run(specs, v, o, device=False)
    ev, eo = _oracle_first([oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=40),
                            oracle.Binner("scalar", y, vmin=-3, vmax=3, bins=50)], v, o)
    np.testing.assert_array_equal(go, eo)
    np.testing.assert_array_equal(gv, ev)


def test_first_large_chunk_index_path_pieces():
    """An AggFirst-only bin of more than 2^26 HBM rows on a grid neither the tiled engine
    (grids of <= 12288 cells count as small) nor the LDS kernels (12 B per cell > 96 KB past
    8192 cells) take: the index path runs in 2^26-row pieces (the chunk itself may be up to
    2^32 rows); values, order ties across the pieces (earliest row) and NaN orders bit-exact."""
    rng = np.random.default_rng(31)
    n = (1 << 26) + 12345
    x = rng.random(n)
    y = rng.random(n)
    v = rng.random(n)
    o = rng.integers(0, 50, n).astype(np.float64)  # many ties per cell, across the pieces
    o[::97] = np.nan
    specs = [("BinnerScalar_float64", x, 0.0, 1.0, 100), ("BinnerScalar_float64", y, 0.0, 1.0, 100)]
    from vaex_amd import superagg, _lib  # noqa: F401
    gv, go, _ = _run(specs, v, o)
    bs = [oracle.Binner("scalar", x, vmin=0.0, vmax=1.0, bins=100), oracle.Binner("scalar", y, vmin=0.0, vmax=1.0, bins=100)]
    ev, eo = _oracle_first(bs, v, o)
    np.testing.assert_array_equal(go.view("u8"), eo.ravel(order="F").view("u8"))
    np.testing.assert_array_equal(gv.view("u8"), ev.ravel(order="F").view("u8"))
