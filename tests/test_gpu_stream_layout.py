"""The tile path's two exchange layouts: value-carrying plans of the fast
pass-A kernels write one stream per pass-A workgroup plus a per-commit tile table (default),
`VH_TILE_STREAM=0` keeps the per-(workgroup, tile) regions.  Both must give the oracle's
grids: counts / min / max exact, float sums within 1e-6 relative (north_star), for the C2
shape, the dense-key groupby grid (ordinal pass A, narrow and packed value slots), row orders
that skew the commits' tile runs, and sizes that leave workgroups with different commit
counts (the table's empty tail rows)."""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def sa():
    import vaex_amd.superagg as m
    return m


@pytest.fixture(params=["1", "0"])
def layout(request, monkeypatch):
    monkeypatch.setenv("VH_TILE_STREAM", request.param)
    return request.param


@pytest.mark.parametrize("n,order", [(4_000_000, "shuffled"), (3_000_001 + 1, "sorted_y"), (2_500_000, "clustered")])
def test_c2_count_sum_min_max(layout, n, order):
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(n)
    x, y = rng.normal(size=n), rng.normal(size=n)
    w = rng.random(n)
    w[::101] = np.nan
    if order == "sorted_y":
        o = np.argsort(y, kind="stable")
        x, y, w = x[o], y[o], w[o]
    elif order == "clustered":
        o = np.argsort(y, kind="stable")
        chunks = [o[b:b + 40_000] for b in range(0, n, 40_000)]
        rng.shuffle(chunks)
        o = np.concatenate(chunks)
        x, y, w = x[o], y[o], w[o]
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
    gx.set_data(DeviceArray.from_numpy(x))
    gy.set_data(DeviceArray.from_numpy(y))
    grid = sa().Grid([gx, gy])
    dw = DeviceArray.from_numpy(w)
    c, s = sa().AggCount_int64(grid), sa().AggSum_float64(grid)
    s.set_data(dw, 0)
    grid.bin([c, s])
    np.testing.assert_array_equal(np.asarray(c), oracle.compute_grid([bx, by], "count"))
    np.testing.assert_allclose(np.asarray(s), oracle.compute_grid([bx, by], "sum", data=w), rtol=1e-6, atol=1e-12)
    grid2 = sa().Grid([gx, gy])
    mn, mx = sa().AggMin_float64(grid2), sa().AggMax_float64(grid2)
    mn.set_data(dw, 0)
    mx.set_data(dw, 0)
    grid2.bin([mn, mx])
    np.testing.assert_array_equal(np.asarray(mn), oracle.compute_grid([bx, by], "min", data=w))
    np.testing.assert_array_equal(np.asarray(mx), oracle.compute_grid([bx, by], "max", data=w))


@pytest.mark.parametrize("vdt", ["float64", "int8", "float32"])
def test_dense_groupby_grid(layout, vdt):
    """The C3 shape (int32 key, 1e6 cells) through the ordinal pass A: float64 values (8-byte
    slots) and int8 + float32 (narrow 4-byte slots, two packed in one stream)."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(7)
    n = 3_000_000
    keys = rng.integers(5, 1_000_005, n).astype(np.int32)
    if vdt == "float64":
        v = rng.normal(size=n)
        cols = {"v": v}
        agg = {"v": ["sum", "count"]}
    else:
        v = rng.integers(-100, 100, n).astype(np.int8) if vdt == "int8" else rng.normal(size=n).astype(np.float32)
        v2 = rng.normal(size=n).astype(np.float32)
        cols = {"v": v, "v2": v2}
        agg = {"v": "sum", "v2": "sum"}
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(keys), **{k: DeviceArray.from_numpy(c) for k, c in cols.items()})
    g = df.groupby("key", agg=agg, sort=True)
    uk, inv = np.unique(keys, return_inverse=True)
    np.testing.assert_array_equal(g["key"].to_numpy(), uk)
    for name, col in cols.items():
        want = np.bincount(inv, weights=col.astype(np.float64), minlength=len(uk))
        out = "v_sum" if vdt == "float64" and name == "v" else name
        got = g[out].to_numpy().astype(np.float64)
        if col.dtype.kind in "iu":
            np.testing.assert_array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-5 if col.dtype == np.float32 else 1e-6, atol=1e-3)
    if vdt == "float64":
        np.testing.assert_array_equal(g["v"].to_numpy(), np.bincount(inv, minlength=len(uk)))


def test_layouts_agree_bitwise_on_counts():
    """Both layouts on the same columns in one process: count grids identical, sum grids
    within 1e-9 (the same entries, a different pass-B association order)."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(3)
    n = 5_000_000
    x = DeviceArray.from_numpy(rng.normal(size=n))
    y = DeviceArray.from_numpy(rng.normal(size=n))
    w = DeviceArray.from_numpy(rng.random(n))
    out = {}
    for mode in ("0", "1"):
        os.environ["VH_TILE_STREAM"] = mode
        try:
            gx, gy = sa().BinnerScalar_float64("x", -4, 4, 1024), sa().BinnerScalar_float64("y", -4, 4, 1024)
            gx.set_data(x)
            gy.set_data(y)
            grid = sa().Grid([gx, gy])
            c, s = sa().AggCount_int64(grid), sa().AggSum_float64(grid)
            s.set_data(w, 0)
            grid.bin([c, s])
            out[mode] = (np.asarray(c).copy(), np.asarray(s).copy())
        finally:
            os.environ.pop("VH_TILE_STREAM", None)
    np.testing.assert_array_equal(out["0"][0], out["1"][0])
    np.testing.assert_allclose(out["0"][1], out["1"][1], rtol=1e-9, atol=0)
