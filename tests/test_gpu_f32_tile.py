"""The fast float32 pass A (k_tile_scatter_f64<ND, NV, SB, float>): 1-, 2- and
3-d grids too large for LDS over float32 columns, count(*) with 0, 1 or 2 float32 sums and
the mean's keyed count, against the oracle's grids (counts exact, sums within 1e-6 relative,
as north_star states for floating point) and against the generic pass A it replaces
(VH_TILE_F32=0: identical counts).  NaNs in binner and value columns, odd n (the generic
path takes those), and an unaligned column view (the generic path too)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def sa():
    import vaex_amd.superagg as m
    return m


def _cols(rng, n, nd, nv):
    xs = [rng.normal(size=n).astype(np.float32) for _ in range(nd)]
    for x in xs:
        x[::997] = np.nan
    ws = [rng.random(n).astype(np.float32) for _ in range(nv)]
    for w in ws:
        w[::101] = np.nan
    return xs, ws


def _run(xs, ws, bins, extra_count=False, offset=0):
    from vaex_amd.device import DeviceArray

    def put(a):  # offset 1: a view one float32 past an aligned HBM block (4-byte aligned)
        if not offset:
            return DeviceArray.from_numpy(a)
        d = DeviceArray.from_numpy(np.concatenate([np.zeros(offset, a.dtype), a]))
        return d[offset:]
    bs = []
    for i, x in enumerate(xs):
        b = sa().BinnerScalar_float32(f"x{i}", -4, 4, bins)
        b.set_data(put(x))
        bs.append(b)
    grid = sa().Grid(bs)
    aggs = [sa().AggCount_int64(grid)]
    for w in ws:
        s = sa().AggSum_float32(grid)
        s.set_data(put(w), 0)
        aggs.append(s)
    if extra_count:  # the mean's count, keyed on the summed column's non-NaN rows
        c = sa().AggCount_float32(grid)
        c.set_data(put(ws[0]), 0)
        aggs.append(c)
    grid.bin(aggs)
    return [np.asarray(a).copy() for a in aggs]


def _check(xs, ws, bins, out, extra_count=False):
    ob = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=bins) for x in xs]
    np.testing.assert_array_equal(out[0], oracle.compute_grid(ob, "count"))
    for k, w in enumerate(ws):
        np.testing.assert_allclose(out[1 + k], oracle.compute_grid(ob, "sum", data=w), rtol=1e-6, atol=1e-9)
    if extra_count:
        np.testing.assert_array_equal(out[-1], oracle.compute_grid(ob, "count", data=ws[0]))


@pytest.mark.parametrize("nd,bins,nv", [(2, 1024, 0), (2, 1024, 1), (2, 1024, 2), (1, 1 << 20, 1), (3, 100, 1)])
def test_f32_tile_grid_matches_oracle(monkeypatch, nd, bins, nv):
    rng = np.random.default_rng(nd * 100 + nv)
    n = 3_000_000
    xs, ws = _cols(rng, n, nd, nv)
    out = _run(xs, ws, bins, extra_count=nv == 1)
    _check(xs, ws, bins, out, extra_count=nv == 1)
    monkeypatch.setenv("VH_TILE_F32", "0")  # the generic pass A on the same columns
    gen = _run(xs, ws, bins, extra_count=nv == 1)
    np.testing.assert_array_equal(out[0], gen[0])
    for a, b in zip(out[1:], gen[1:]):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("case", ["odd_n", "unaligned"])
def test_f32_tile_fallbacks_match_oracle(case):
    """Odd row counts and 4-byte-aligned column views leave the fast kernel's pair loads out:
    the generic pass A gives the same oracle grids."""
    rng = np.random.default_rng(5)
    n = 2_000_001 if case == "odd_n" else 2_000_002
    xs, ws = _cols(rng, n, 2, 1)
    out = _run(xs, ws, 1024, offset=1 if case == "unaligned" else 0)
    _check(xs, ws, 1024, out)


@pytest.mark.parametrize("nd,bins,n,offset", [(1, 256, 3_000_001, 0), (2, 64, 3_000_000, 0), (3, 16, 2_000_000, 0),
                                              (2, 64, 2_000_000, 1)])
def test_f32_small_grid_count_matches_oracle(monkeypatch, nd, bins, n, offset):
    """Small grids (LDS sub-grids, k_small_f64 with float32 row pairs): count(*) over float32
    binner columns with NaNs, odd n (the last row alone) and a 4-byte-aligned view (k_fused
    takes it), against the oracle and against k_fused (VH_SMALL_F32=0)."""
    rng = np.random.default_rng(nd * 7 + offset)
    xs, _ = _cols(rng, n, nd, 0)
    out = _run(xs, [], bins, offset=offset)
    _check(xs, [], bins, out)
    monkeypatch.setenv("VH_SMALL_F32", "0")
    np.testing.assert_array_equal(_run(xs, [], bins, offset=offset)[0], out[0])


@pytest.mark.parametrize("bdt,vdt,nv", [("float64", "float32", 1), ("float64", "float32", 2), ("float32", "float64", 1),
                                        ("float32", "float64", 2)])
def test_mixed_column_types_match_oracle(monkeypatch, bdt, vdt, nv):
    """Mixed plans on the fast pass A (float64 binners with float32 sums, float32 binners with
    float64 sums: the value columns in a second register array of their own pair type),
    against the oracle and the generic pass A (VH_TILE_F32=0)."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(31 + nv)
    n = 3_000_000
    xs = [rng.normal(size=n).astype(bdt) for _ in range(2)]
    for x in xs:
        x[::997] = np.nan
    ws = [rng.random(n).astype(vdt) for _ in range(nv)]
    for w in ws:
        w[::101] = np.nan

    def run():
        bs = []
        for i, x in enumerate(xs):
            b = getattr(sa(), "BinnerScalar_" + bdt)(f"x{i}", -4, 4, 1024)
            b.set_data(DeviceArray.from_numpy(x))
            bs.append(b)
        grid = sa().Grid(bs)
        aggs = [sa().AggCount_int64(grid)]
        for w in ws:
            s = getattr(sa(), "AggSum_" + vdt)(grid)
            s.set_data(DeviceArray.from_numpy(w), 0)
            aggs.append(s)
        grid.bin(aggs)
        return [np.asarray(a).copy() for a in aggs]

    out = run()
    _check(xs, ws, 1024, out)
    monkeypatch.setenv("VH_TILE_F32", "0")
    gen = run()
    np.testing.assert_array_equal(out[0], gen[0])
    for a, b in zip(out[1:], gen[1:]):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9)


def test_f32_plan_past_the_fast_kernels_lds():
    """A float32 plan whose tiles do not fit the fast kernel's LDS (2^25 bins: 4096 tiles)
    runs the generic pass A with its per-dtype loads (not an ND > 0 kernel that reads float64
    columns), against the oracle."""
    rng = np.random.default_rng(41)
    n = 2_000_000
    xs, ws = _cols(rng, n, 1, 1)
    out = _run(xs, ws, 1 << 25)
    _check(xs, ws, 1 << 25, out)


@pytest.mark.parametrize("bdt", ["int32", "int64"])
@pytest.mark.parametrize("vdt,nv", [(None, 0), ("float64", 1), ("float32", 1), ("float64", 2)])
def test_integer_binners_match_oracle(monkeypatch, bdt, vdt, nv):
    """Integer binby columns on the fast pass A (BinnerScalar<int>: the value widened to
    double before the index math), 1- and 2-d, with float64 / float32 sums or count only,
    against the oracle and the generic pass A (VH_TILE_F32=0)."""
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(51 + nv)
    n = 3_000_000
    for nd, bins in ((2, 1000), (1, 1 << 20)):
        hi = 1200 if nd == 2 else 1_100_000
        xs = [rng.integers(-100, hi, n).astype(bdt) for _ in range(nd)]
        ws = [rng.random(n).astype(vdt) for _ in range(nv)]
        for w in ws:
            w[::101] = np.nan
        lim = (0, 1000) if nd == 2 else (0, 1 << 20)

        def run():
            bs = []
            for i, x in enumerate(xs):
                b = getattr(sa(), "BinnerScalar_" + bdt)(f"x{i}", lim[0], lim[1], bins)
                b.set_data(DeviceArray.from_numpy(x))
                bs.append(b)
            grid = sa().Grid(bs)
            aggs = [sa().AggCount_int64(grid)]
            for w in ws:
                s = getattr(sa(), "AggSum_" + vdt)(grid)
                s.set_data(DeviceArray.from_numpy(w), 0)
                aggs.append(s)
            grid.bin(aggs)
            return [np.asarray(a).copy() for a in aggs]

        out = run()
        ob = [oracle.Binner("scalar", x, vmin=lim[0], vmax=lim[1], bins=bins) for x in xs]
        np.testing.assert_array_equal(out[0], oracle.compute_grid(ob, "count"))
        for k, w in enumerate(ws):
            np.testing.assert_allclose(out[1 + k], oracle.compute_grid(ob, "sum", data=w), rtol=1e-6, atol=1e-9)
        monkeypatch.setenv("VH_TILE_F32", "0")
        gen = run()
        monkeypatch.delenv("VH_TILE_F32")
        np.testing.assert_array_equal(out[0], gen[0])
        for a, b in zip(out[1:], gen[1:]):
            np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9)
