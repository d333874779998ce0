"""var / std over a grid too large for one workgroup's LDS (agg.py:191-229: AggSumMoment(2),
AggSum and count of the float64-cast expression): the moment cell rides on the tile path
beside the sum's (one carried value slot; superagg.cpp:391-434 adds pow(value, 2) per
non-NaN row), checked against the oracle's serial grids.  Float sums / moments within 1e-6
relative (north_star); the tile path must carry it (no generic scattered-atomic pass)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _frame(cols):
    import vaex_amd
    from vaex_amd.device import DeviceArray
    return vaex_amd.from_arrays(**{k: DeviceArray.from_numpy(v) for k, v in cols.items()})


def _timed(fn):
    from vaex_amd import _lib
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    try:
        out = fn()
        _lib.synchronize()
    finally:
        _lib.timing_enable(False)
    names = ("tile_reduce", "bin_aggregate", "bin_indices")
    return out, {k: _lib.timing_read(k)[0] for k in names}


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("stat", ["var", "std"])
def test_var_std_c2_grid_tile_path(dtype, stat):
    rng = np.random.default_rng(21)
    n = (1 << 22) + 6
    x, y = rng.normal(size=n), rng.normal(size=n)
    w = (rng.random(n) * 3 + 1).astype(dtype)
    w[rng.random(n) < 0.02] = np.nan
    df = _frame({"x": x, "y": y, "w": w})
    lim = [[-4, 4], [-4, 4]]
    got, timers = _timed(lambda: np.asarray(getattr(df, stat)("w", binby=["x", "y"], limits=lim, shape=1024)))
    assert timers["tile_reduce"] >= 1 and timers["bin_aggregate"] == 0, timers
    bs = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024), oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)]
    var = oracle.extract_central_part(oracle.var_grid(bs, w))
    if stat == "var":
        np.testing.assert_allclose(got, var, rtol=1e-6, atol=1e-12, equal_nan=True)
        return
    # std = sqrt(m2 / n - mean^2), checked per class of cell:
    cnt = oracle.extract_central_part(oracle.compute_grid(bs, "count", data=w.astype(np.float64)))
    empty, one, many = cnt == 0, cnt == 1, cnt >= 2
    # empty cells: 0 / 0 on both sides
    assert np.isnan(got[empty]).all() and np.isnan(var[empty]).all()
    # one-row cells: the moment is v * v here, so m2 / 1 - (v / 1)^2 is exactly 0 and std is
    # exactly 0.0; the reference adds pow(v, 2) (superagg.cpp:420,429), which glibc may round one
    # ulp away from v * v, leaving a +-1-ulp residue there -- a negative one is NaN std
    np.testing.assert_array_equal(got[one], 0.0)
    residue = var[one]
    ulp = np.spacing(np.nanmax(np.square(w.astype(np.float64))))
    assert np.all(np.abs(residue) <= ulp), "oracle residue beyond one ulp of v^2"
    negative = np.flatnonzero(one.ravel() & (var.ravel() < 0))  # the reference's NaN std cells
    assert np.all(got.ravel()[negative] == 0.0) and np.all(var.ravel()[negative] < 0)
    # several rows: m2 / n - mean^2 subtracts two numbers of size m2 / n, so its rounding
    # residue is a few ulps of m2 / n whatever the summation order; the GPU's variance
    # (got^2) must match the oracle's within rtol 1e-6 plus that residue, and where the
    # variance itself is inside the residue (two nearly equal values in a cell) the sign is
    # the summation order's: std is NaN or below sqrt(residue) -- those cells are few
    m2n = oracle.extract_central_part(oracle.compute_grid(bs, "sum_moment", data=w.astype(np.float64), moment=2)) / np.maximum(cnt, 1)
    resid = 16 * np.finfo(np.float64).eps * m2n
    inside = many & (np.abs(var) <= resid)
    clear = many & ~inside
    assert inside.sum() <= 1e-3 * many.sum(), int(inside.sum())
    np.testing.assert_array_less(np.abs(got[clear] ** 2 - var[clear]), 1e-6 * var[clear] + resid[clear])
    assert np.all(np.isfinite(got[clear]))
    g_in = got[inside]
    assert np.all(np.isnan(g_in) | (g_in ** 2 <= 2 * resid[inside]))


def test_sum_moment_with_count_sum_and_min_max():
    """AggSumMoment(2) beside count, sum, min and max of the same column in one tile pass
    (shared value slot, per-entry pass B), through the superagg surface."""
    from vaex_amd import superagg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(22)
    n = 3_000_000
    x = rng.normal(size=n)
    y = rng.normal(size=n)
    w = rng.normal(size=n)
    w[::17] = np.nan
    bx, by = superagg.BinnerScalar_float64("x", -4, 4, 1000), superagg.BinnerScalar_float64("y", -4, 4, 1000)
    dx, dy, dw = DeviceArray.from_numpy(x), DeviceArray.from_numpy(y), DeviceArray.from_numpy(w)
    bx.set_data(dx)
    by.set_data(dy)
    grid = superagg.Grid([bx, by])
    aggs = {"count": superagg.AggCount_float64(grid), "sum": superagg.AggSum_float64(grid),
            "m2": superagg.AggSumMoment_float64(grid, 2), "m3": superagg.AggSumMoment_float64(grid, 3),
            "min": superagg.AggMin_float64(grid), "max": superagg.AggMax_float64(grid)}
    for a in aggs.values():
        a.set_data(dw, 0)
    grid.bin(list(aggs.values()))
    bs = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1000), oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1000)]
    np.testing.assert_array_equal(np.asarray(aggs["count"]), oracle.compute_grid(bs, "count", data=w))
    np.testing.assert_array_equal(np.asarray(aggs["min"]), oracle.compute_grid(bs, "min", data=w))
    np.testing.assert_array_equal(np.asarray(aggs["max"]), oracle.compute_grid(bs, "max", data=w))
    np.testing.assert_allclose(np.asarray(aggs["sum"]), oracle.compute_grid(bs, "sum", data=w), rtol=1e-6, atol=1e-9)
    for m in (2, 3):
        np.testing.assert_allclose(np.asarray(aggs[f"m{m}"]), oracle.compute_grid(bs, "sum_moment", data=w, moment=m),
                                   rtol=1e-6, atol=1e-9)
