"""0-d aggregation (no binby: df.count() / df.sum('w') / df.mean('w')): the grid is one cell
(Grid::bin with a length and no binners, agg.hpp:76-105), computed by the reduction kernel
(binning.hip k_reduce0 + k_reduce0_fin).  Counts exact; float64 sums within 1e-12 of the
oracle's row-order sum (the reduction adds per lane, per wave, per workgroup, then the
workgroup partials in a fixed order -- run-to-run identical)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _cols(n, seed=3):
    rng = np.random.default_rng(seed)
    w = rng.normal(loc=0.5, size=n)
    w[::7] = np.nan
    x = rng.normal(size=n)
    return w, x


@pytest.mark.parametrize("n", [0, 1, 2, 3, 64, 1001, 1_000_003])
@pytest.mark.parametrize("where", ["hbm", "host"])
def test_zero_d_count_sum_mean(n, where):
    import vaex_amd
    from vaex_amd.device import DeviceArray
    w, x = _cols(n)
    cols = {"w": w, "x": x}
    if where == "hbm":
        cols = {k: DeviceArray.from_numpy(v) for k, v in cols.items()}
    df = vaex_amd.from_arrays(**cols)
    assert int(df.count()) == n
    cw = oracle.compute_grid([], "count", data=w, n=n)
    sw = oracle.compute_grid([], "sum", data=w, n=n)
    assert int(df.count("w")) == int(cw)
    np.testing.assert_allclose(float(df.sum("w")), float(sw), rtol=1e-12, atol=1e-12)
    with np.errstate(divide="ignore", invalid="ignore"):
        np.testing.assert_allclose(float(df.mean("w")), np.float64(sw) / np.float64(cw), rtol=1e-12, equal_nan=True)
    # a selection: the aggregator mask (1 = keep) of count(*), count(w) and sum(w)
    keep = (x > 0).astype(np.uint8)
    assert int(df.count(selection="x > 0")) == int(keep.sum())
    assert int(df.count("w", selection="x > 0")) == int(oracle.compute_grid([], "count", data=w, mask=keep, n=n))
    np.testing.assert_allclose(float(df.sum("w", selection="x > 0")),
                               float(oracle.compute_grid([], "sum", data=w, mask=keep, n=n)), rtol=1e-12, atol=1e-12)


def test_zero_d_superagg_accumulates_and_unaligned_columns():
    """Grid([]) with a length (agg.hpp:76-83): repeated bin() calls add into the cell; a column
    view that is not 16-B aligned takes the per-row fused kernel and agrees."""
    from vaex_amd import superagg
    from vaex_amd.device import DeviceArray
    n = 2_000_001
    w, _ = _cols(n, seed=9)
    d = DeviceArray.from_numpy(w)
    grid = superagg.Grid([])
    c, s, cw = superagg.AggCount_float64(grid), superagg.AggSum_float64(grid), superagg.AggCount_float64(grid)
    s.set_data(d, 0)
    cw.set_data(d, 0)
    grid.bin([c, s, cw], n)
    grid.bin([c, s, cw], n)
    nn = int(np.sum(~np.isnan(w)))
    assert int(np.asarray(c)) == 2 * n and int(np.asarray(cw)) == 2 * nn
    np.testing.assert_allclose(float(np.asarray(s)), 2 * np.nansum(w), rtol=1e-12)
    # unaligned view (8-byte offset)
    g2 = superagg.Grid([])
    s2, cw2 = superagg.AggSum_float64(g2), superagg.AggCount_float64(g2)
    s2.set_data(d[1:], 0)
    cw2.set_data(d[1:], 0)
    g2.bin([s2, cw2], n - 1)
    assert int(np.asarray(cw2)) == int(np.sum(~np.isnan(w[1:])))
    np.testing.assert_allclose(float(np.asarray(s2)), np.nansum(w[1:]), rtol=1e-12)


def test_zero_d_sum_is_deterministic():
    import vaex_amd
    from vaex_amd.device import DeviceArray
    d = DeviceArray.random(3_000_000, "normal", seed=4)
    df = vaex_amd.from_arrays(w=d)
    vals = {float(df.sum("w")) for _ in range(5)}
    assert len(vals) == 1
