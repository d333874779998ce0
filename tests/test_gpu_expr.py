"""Device expression evaluation (csrc/expr.hip via vaex_amd/expr.py) on HBM frames, against
numpy evaluating the same expression on the host copies; then the paths that use it:
binning by an expression, selections, filters (aggregations, min/max, groupby set build)
and virtual columns, all against numpy on the filtered host arrays.

Integer, boolean and basic float arithmetic (+ - * / // %, comparisons, sqrt, floor) are
bit-exact; transcendental functions (pow, exp, log, sin, arctan2) within 4 ulp over a whole expression (device libm
vs glibc / numpy's SIMD kernels)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

N = 300_001


def _host():
    rng = np.random.default_rng(42)
    return dict(
        x=rng.normal(size=N), y=rng.normal(size=N) + 2, f=rng.normal(size=N).astype(np.float32),
        i=rng.integers(-50, 50, N).astype(np.int64), i32=rng.integers(-1000, 1000, N).astype(np.int32),
        i8=rng.integers(-100, 100, N).astype(np.int8), u8=rng.integers(0, 255, N).astype(np.uint8),
        b=rng.random(N) > 0.5, w=rng.random(N), key=rng.integers(0, 1000, N).astype(np.int32) * 7919)


def _device_frame(h):
    import vaex_amd
    from vaex_amd.device import DeviceArray
    return vaex_amd.from_arrays(**{k: DeviceArray.from_numpy(v) for k, v in h.items()})


EXACT = [
    "x + y", "x * 2 - y / 3", "(x > 0) & (y < 2.5)", "x ** 2 + sqrt(abs(y))", "i % 7", "i // 3", "-i", "~b",
    "where(x > 0, x, -x)", "i8 + i8", "i8 * 3", "f * 2.5 + f", "i32 / 2", "x // 0.7", "x % -1.3",
    "minimum(x, y)", "u8 + 1", "i << 2", "b & (i > 3)", "f + i8", "f + i32", "i32 + i8", "np.floor(x) + 1",
    "u8 > 200", "i == 3", "b | ~b", "where(b, i8, i32)", "maximum(i8, u8)", "i % -3", "i // -4",
    "x ** 0.5", "1 / f", "abs(i32) * 2", "isnan(sqrt(x))",
]
ULP = ["exp(x)", "log(y)", "sin(x) * cos(y)", "x ** 3", "arctan2(x, y)", "tanh(x) * log1p(abs(x))", "f ** 1.7"]


@pytest.mark.parametrize("e", EXACT + ULP)
def test_expression_matches_numpy(e):
    from vaex_amd.device import DeviceArray
    h = _host()
    df = _device_frame(h)
    got = df.evaluate(e)
    assert isinstance(got, DeviceArray), "evaluated off the GPU"
    got = got.to_numpy()
    ns = dict(np=np, **{k: getattr(np, k) for k in ("sqrt", "abs", "where", "minimum", "maximum", "isnan", "exp",
                                                      "log", "sin", "cos", "arctan2", "tanh", "log1p")})
    ns.update(h)
    with np.errstate(all="ignore"):
        expected = np.asarray(eval(e, {"__builtins__": {}}, ns))  # noqa: S307
    assert got.dtype == expected.dtype
    if e in ULP:
        # float32: numpy uses its own float32 SIMD libm (several ulp); the device computes in
        # float64 and rounds once
        np.testing.assert_array_max_ulp(got, expected, maxulp=4 if got.dtype == np.float64 else 16)
    else:
        np.testing.assert_array_equal(got, expected)


def _count(binners):
    return oracle.extract_central_part(oracle.compute_grid(binners, "count"))


def test_binby_expression_and_virtual_column():
    h = _host()
    df = _device_frame(h)
    df["r"] = df.x * df.x + df.y
    got = df.count(binby="x + y", limits=[-3, 7], shape=128)
    exp = _count([oracle.Binner("scalar", h["x"] + h["y"], vmin=-3, vmax=7, bins=128)])
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_allclose(df.sum("r"), np.sum(h["x"] * h["x"] + h["y"]), rtol=1e-9)


def test_selection_on_device_frame():
    h = _host()
    df = _device_frame(h)
    sel = (h["x"] > 0.5) & (h["i"] < 10)
    assert int(df.count(selection="(x > 0.5) & (i < 10)")) == int(sel.sum())
    np.testing.assert_allclose(df.sum("w", selection="(x > 0.5) & (i < 10)"), h["w"][sel].sum(), rtol=1e-9)
    got = df.count(binby="y", limits=[0, 4], shape=64, selection="b")
    exp = _count([oracle.Binner("scalar", h["y"][h["b"]], vmin=0, vmax=4, bins=64)])
    np.testing.assert_array_equal(got, exp)


def test_filter_on_device_frame():
    h = _host()
    df = _device_frame(h)
    dff = df[df.x > 0]
    m = h["x"] > 0
    assert len(dff) == int(m.sum())
    np.testing.assert_allclose(dff.sum("w"), h["w"][m].sum(), rtol=1e-9)
    got = dff.count(binby=["x", "y"], limits=[[-1, 4], [0, 4]], shape=[64, 32])
    exp = _count([oracle.Binner("scalar", h["x"][m], vmin=-1, vmax=4, bins=64),
                  oracle.Binner("scalar", h["y"][m], vmin=0, vmax=4, bins=32)])
    np.testing.assert_array_equal(got, exp)
    lo, hi = dff.minmax("y")
    assert lo == h["y"][m].min() and hi == h["y"][m].max()
    np.testing.assert_array_equal(dff.evaluate("i"), h["i"][m])
    # filter + selection
    sel = m & (h["i"] > 0)
    assert int(dff.count(selection="i > 0")) == int(sel.sum())


def test_groupby_on_filtered_device_frame():
    h = _host()
    df = _device_frame(h)
    dff = df[(df.i > -20) & (df.b)]
    m = (h["i"] > -20) & h["b"]
    res = dff.groupby("key", agg={"n": "count"})
    keys, counts = np.unique(h["key"][m], return_counts=True)
    order = np.argsort(res["key"].to_numpy())
    np.testing.assert_array_equal(res["key"].to_numpy()[order], keys)
    np.testing.assert_array_equal(res["n"].to_numpy()[order], counts)


TERMS = ["x > 0.4", "(x > 0.3) & (f < 2)", "(i >= -20) & (i < 30) & (w > 0.1)", "(x > 0.3) | (i32 == 3)",
         "~(y <= 2)", "u8 > 200", "i8 < -3", "(f > 0.5) & (i32 >= 0)", "x != x", "(i > 3) & (x > 0) & (y > 1) & (w < 0.9)",
         "i32 > 2.5", "f >= 0.1"]


@pytest.mark.parametrize("e", TERMS)
@pytest.mark.parametrize("offset", [0, 3])
def test_comparison_terms_kernel(monkeypatch, e, offset):
    """Conjunctions / disjunctions of column-vs-constant comparisons run the 8-rows-per-lane
    kernel (k_expr_terms); it must equal numpy and the interpreter (VH_EXPR_TERMS=0) byte for
    byte, on whole frames and on views starting mid-block (tail rows, unaligned columns),
    with NaNs in the float columns."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    h = _host()
    h["x"][::37] = np.nan
    h["f"][::41] = np.nan
    hv = {k: v[offset:] for k, v in h.items()}
    full = {k: DeviceArray.from_numpy(v) for k, v in h.items()}
    df = vaex_amd.from_arrays(**{k: d[offset:] for k, d in full.items()})
    got = df.evaluate(e).to_numpy()
    monkeypatch.setenv("VH_EXPR_TERMS", "0")
    interp = df.evaluate(e).to_numpy()
    ns = dict(hv)
    with np.errstate(all="ignore"):
        expected = np.asarray(eval(e, {"__builtins__": {}}, ns))  # noqa: S307
    np.testing.assert_array_equal(got, expected)
    np.testing.assert_array_equal(got, interp)
