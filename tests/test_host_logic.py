"""Host-side logic of the superagg mirror (no GPU needed)."""
import numpy as np
import pytest

from oracle import oracle


def test_class_registry_matches_reference_names():
    """superagg_binners.cpp:279-303 and superagg.cpp:614-624: 11 dtypes x {native, _non_native}."""
    from vaex_amd import superagg
    for dt in ["float64", "float32", "int64", "int32", "int16", "int8", "uint64", "uint32", "uint16", "uint8", "bool"]:
        for post in ("", "_non_native"):
            for pre in ("BinnerScalar_", "BinnerOrdinal_", "AggCount_", "AggSum_", "AggMin_", "AggMax_", "AggFirst_",
                        "AggSumMoment_"):
                assert hasattr(superagg, pre + dt + post)


@pytest.mark.parametrize("dtype,postfix", [("f8", "float64"), (">f8", "float64_non_native"), ("<i4", "int32"),
                                           (">u2", "uint16_non_native"), ("M8[ns]", "int64"), ("m8[s]", "int64"),
                                           ("?", "bool"), ("u1", "uint8")])
def test_find_type_from_dtype(dtype, postfix):
    from vaex_amd import superagg
    from vaex_amd.utils import find_type_from_dtype
    assert find_type_from_dtype(superagg, "AggCount_", np.dtype(dtype)).__name__ == "AggCount_" + postfix


def test_find_type_unsupported():
    from vaex_amd import superagg
    from vaex_amd.utils import find_type_from_dtype
    with pytest.raises(ValueError):
        find_type_from_dtype(superagg, "AggCount_", np.dtype("complex128"))


@pytest.mark.parametrize("value,dtype", [(-3, "int8"), (300, "int8"), (-1, "int64"), (2 ** 40, "int32"), (5, "uint16"),
                                         (-1.5, "float64"), (2.7, "float32"), (17, "bool"), (0, "bool"), (-7, "uint8")])
def test_ordinal_ctor_conversion_matches_oracle(value, dtype):
    """BinnerOrdinal_<T>(expr, T, T): pybind11 cast to T, then T -> uint64_t (superagg_binners.cpp:99)."""
    from vaex_amd.superagg import _u64_of
    assert _u64_of(value, dtype) == oracle.as_u64_bits(value, dtype)


def test_utils():
    from vaex_amd.utils import _expand_limits, _expand_shape, extract_central_part, required_dtype_for_max
    a = np.arange(5 * 6).reshape(5, 6)
    assert extract_central_part(a).tolist() == a[2:-1, 2:-1].tolist()
    assert required_dtype_for_max(127) == np.int8 and required_dtype_for_max(128) == np.int16
    assert required_dtype_for_max(2 ** 31) == np.int64
    assert _expand_shape(128, 2) == (128, 128)
    assert _expand_limits([0, 1], 2) == ([0, 1], [0, 1])
    assert _expand_limits([[0, 1], [2, 3]], 2) == ([0, 1], [2, 3])


def test_dtype_codes():
    from vaex_amd import _lib
    assert _lib.dtype_code(np.dtype(">f8")) == (_lib.DTYPE_CODE["float64"], 1)
    assert _lib.dtype_code(np.dtype("<f8")) == (_lib.DTYPE_CODE["float64"], 0)
    assert _lib.dtype_code(np.dtype("M8[ns]")) == (_lib.DTYPE_CODE["int64"], 0)
    with pytest.raises(ValueError):
        _lib.dtype_code(np.dtype("c16"))


def test_promise_and_delayed():
    from vaex_amd.promise import Promise, delayed
    a, b = Promise(), Promise()
    out = delayed(lambda x, y: x + y)(a, b)
    with pytest.raises(RuntimeError):
        out.get()
    a.fulfill(1)
    b.fulfill(2)
    assert out.get() == 3
    c = Promise()
    bad = delayed(lambda x: x)(c)
    c.reject(ValueError("x"))
    with pytest.raises(ValueError):
        bad.get()


def test_binner_specs_merge_tasks():
    """execution.py:47-73: aggregations with equal binners merge into one pass."""
    import vaex_amd
    from vaex_amd.execution import _merge
    from vaex_amd.tasks import TaskAggregation, TaskAggregations, TaskMinMax
    df = vaex_amd.from_arrays(x=np.arange(10.0), w=np.ones(10))
    b1 = df._binner_scalar("x", [0, 10], 4)
    b2 = df._binner_scalar("x", [0, 10], 4)
    b3 = df._binner_scalar("x", [0, 10], 5)
    assert b1 == b2 and hash(b1) == hash(b2) and b1 != b3
    aggs = [vaex_amd.agg.count(), vaex_amd.agg.sum("w")]
    for a in aggs:
        a._prepare_types(df)
    tasks = [TaskAggregation(df, (b1,), aggs[0]), TaskAggregation(df, (b2,), aggs[1]),
             TaskAggregation(df, (b3,), aggs[0]), TaskMinMax(df, "x")]
    merged = _merge(tasks, df)
    kinds = sorted(type(t).__name__ for t in merged)
    assert kinds == ["TaskAggregations", "TaskAggregations", "TaskMinMax"]
    big = [t for t in merged if isinstance(t, TaskAggregations) and len(t.aggregation_descriptions) == 2]
    assert len(big) == 1 and big[0].expressions == ["x", "w"]


def test_parse_ordinal_values():
    from vaex_amd.taskparts import parse_ordinal_values
    assert parse_ordinal_values("_ordinal_values(key, set_key)") == ("key", "set_key")
    assert parse_ordinal_values("_ordinal_values(a + b, s_1)") == ("a + b", "s_1")
    assert parse_ordinal_values("x") is None


def test_host_expression_evaluation():
    import vaex_amd
    x = np.arange(10.0)
    df = vaex_amd.from_arrays(x=x, y=x ** 2)
    assert df.evaluate("x + y").tolist() == (x + x ** 2).tolist()
    df.select("x < 3")
    assert df.evaluate_selection_mask(True).tolist() == (x < 3).tolist()
    assert str(df.x < 5) == "(x < 5)"
    df2 = df.filter("x > 4")
    assert df2.evaluate("x").tolist() == x[x > 4].tolist()
    assert df.data_type("x") == np.float64


def test_hostops_match_numpy():
    """Threaded host finishing (mean division, label ranges) equals the single numpy call."""
    from vaex_amd import hostops
    rng = np.random.default_rng(4)
    n = 3 * hostops.MIN_SPLIT + 17
    for a in [rng.normal(size=n), rng.integers(-10 ** 12, 10 ** 12, n), rng.integers(0, 2 ** 63, n).astype(np.uint64)]:
        b = rng.integers(0, 4, n)  # zeros: x / 0 -> inf, 0 / 0 -> nan
        a[::7] = 0
        with np.errstate(divide="ignore", invalid="ignore"):
            exp = a / b
        got = hostops.true_divide(a, b)
        assert got.dtype == exp.dtype
        np.testing.assert_array_equal(got, exp)
    for dtype, vmin in [("int32", 5), ("int64", -(2 ** 40)), ("uint16", 3), ("int8", -100)]:
        m = min(n, np.iinfo(dtype).max - vmin)
        got = hostops.arange(vmin, m, dtype)
        np.testing.assert_array_equal(got, np.arange(vmin, vmin + m, dtype=dtype))
        assert got.dtype == np.dtype(dtype)


def test_hostops_astype_minmax():
    from vaex_amd import hostops
    rng = np.random.default_rng(5)
    n = 2 * hostops.MIN_SPLIT + 3
    a = rng.integers(-(2 ** 40), 2 ** 40, n)
    assert hostops.minmax(a) == (a.min(), a.max())
    for dt in ["int32", "int16", "uint64", "int64"]:
        got = hostops.astype(a, dt)
        assert got.dtype == np.dtype(dt)
        np.testing.assert_array_equal(got, a.astype(dt))
