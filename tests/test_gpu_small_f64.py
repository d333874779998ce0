"""Small grids over float64 scalar binners (k_small_f64: 16-B pair loads, LDS sub-grids written
out as partials, folded by k_small_f64_fin) and the limits pre-pass (k_minmax* partials folded
by k_minmax_fin), against the oracle (Grid::bin_, agg.hpp:106-136; BinnerScalar::to_bins,
superagg_binners.cpp:14-56; nanmin/nanmax, tasks.py:173-185).

Counts bit-exact; float64 sums within 1e-9 relative (the atomic fold order differs)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _cols(rng, n, nd, nan_frac=0.03):
    cols = []
    for d in range(nd):
        x = rng.normal(0, 1.5, n)
        x[rng.random(n) < nan_frac] = np.nan
        x[rng.random(n) < 0.01] = 4.0  # exactly vmax: the overflow cell
        cols.append(x)
    return cols


@pytest.mark.parametrize("n", [2, 3, 17, 1001, (1 << 20) + 3])
@pytest.mark.parametrize("nd", [1, 2, 3])
@pytest.mark.parametrize("device", [True, False])
def test_small_f64_grid_matches_oracle(n, nd, device):
    from vaex_amd import superagg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(1000 * n + 10 * nd + device)
    bins = {1: 256, 2: 30, 3: 9}[nd]
    xs = _cols(rng, n, nd)
    w = rng.random(n) - 0.25
    w[rng.random(n) < 0.02] = np.nan
    put = DeviceArray.from_numpy if device else (lambda a: a)
    binners, specs = [], []
    for d, x in enumerate(xs):
        b = superagg.BinnerScalar_float64(f"x{d}", -4, 4, bins)
        b.set_data(put(x))
        binners.append(b)
        specs.append(oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=bins))
    grid = superagg.Grid(binners)
    c_all = superagg.AggCount_int64(grid)
    c_w = superagg.AggCount_float64(grid)
    c_w.set_data(put(w), 0)
    s_w = superagg.AggSum_float64(grid)
    s_w.set_data(put(w), 0)
    s_x = superagg.AggSum_float64(grid)
    s_x.set_data(put(xs[0]), 0)  # a binner column summed too: the same column read twice
    grid.bin([c_all, c_w, s_w, s_x])
    assert np.array_equal(np.asarray(c_all), oracle.compute_grid(specs, "count"))
    assert np.array_equal(np.asarray(c_w), oracle.compute_grid(specs, "count", data=w))
    np.testing.assert_allclose(np.asarray(s_w), oracle.compute_grid(specs, "sum", data=w), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(np.asarray(s_x), oracle.compute_grid(specs, "sum", data=xs[0]), rtol=1e-9, atol=1e-9)
    # binning again accumulates (the grid is not reset by bin)
    grid.bin([c_all])
    assert np.array_equal(np.asarray(c_all), 2 * oracle.compute_grid(specs, "count"))


def test_small_f64_misaligned_column_falls_back():
    """A column view starting at an odd row is not 16-B aligned: the per-row kernel takes it."""
    from vaex_amd import superagg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(5)
    n = 100_001
    x = rng.normal(size=n + 1)
    dx = DeviceArray.from_numpy(x)[1:]
    b = superagg.BinnerScalar_float64("x", -4, 4, 256)
    b.set_data(dx)
    grid = superagg.Grid([b])
    c = superagg.AggCount_int64(grid)
    grid.bin([c])
    spec = oracle.Binner("scalar", x[1:], vmin=-4, vmax=4, bins=256)
    assert np.array_equal(np.asarray(c), oracle.compute_grid([spec], "count"))


def test_dataframe_c1_count_matches_oracle():
    """C1 (BASELINE configs[0]) through the DataFrame API at 1e6 rows: minmax limits, then the bin."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    n = 1_000_000
    x = DeviceArray.random(n, "normal", seed=11)
    hx = x.to_numpy()
    df = vaex_amd.from_arrays(x=x)
    lo, hi = df.minmax("x")
    assert lo == np.nanmin(hx) and hi == np.nanmax(hx)
    c = df.count(binby="x", shape=256)
    spec = oracle.Binner("scalar", hx, vmin=lo, vmax=hi, bins=256)
    assert np.array_equal(np.asarray(c), oracle.compute_grid([spec], "count")[2:-1])


@pytest.mark.parametrize("dtype", ["float64", "float32", "int64", "int32", "int16", "uint8"])
@pytest.mark.parametrize("n", [1, 7, 4099, 3_000_001])
def test_minmax_partials_match_numpy(dtype, n):
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    import ctypes
    rng = np.random.default_rng(n)
    a = (rng.normal(0, 1000, n)).astype(dtype)
    if np.dtype(dtype).kind == "f" and n > 2:
        a[rng.random(n) < 0.1] = np.nan
    for src, off in ((DeviceArray.from_numpy(a), 0), (DeviceArray.from_numpy(np.concatenate([a[:1], a]))[1:], 1), (a, 0)):
        lo, hi = ctypes.c_double(), ctypes.c_double()
        code, flip = _lib.dtype_code(a.dtype)
        ptr = src.ptr if hasattr(src, "ptr") else src.ctypes.data
        _lib.call("vh_minmax", ctypes.c_void_p(ptr), n, code, flip, None, 0, ctypes.byref(lo), ctypes.byref(hi))
        assert lo.value == float(np.nanmin(a)) and hi.value == float(np.nanmax(a)), off


def test_minmax_all_nan_is_nan():
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    import ctypes
    a = np.full(1000, np.nan)
    lo, hi = ctypes.c_double(), ctypes.c_double()
    _lib.call("vh_minmax", ctypes.c_void_p(DeviceArray.from_numpy(a).ptr), 1000, _lib.dtype_code(a.dtype)[0], 0, None, 0,
              ctypes.byref(lo), ctypes.byref(hi))
    assert np.isnan(lo.value) and np.isnan(hi.value)
