"""AggNUnique (agg_hash_primitive.cpp:6-102): the oracle restatement against the
reference's own known answers (tests/agg_test.py:293-316 test_nunique with its float
mapping, :318-333 test_nunique_filtered, :344-360 test_agg_selections with the strings
mapped to numbers), on CPU; then the HIP path against the oracle (-m gpu), including the
reference's drop arithmetic (dropmissing / dropnan subtract ROW counts), selections,
filters on HBM frames, reduce of parts, every dtype and byte order."""
import zlib

import numpy as np
import pytest

from oracle import oracle

X = np.array([0, 0, 0, 0, 0, 1, 1, 1, 2], np.int64)
S = np.array([1.2, 1.2, 2.5, 3.7, np.nan, 3.7, 4.8, 3.7, 1.2])  # agg_test.py:306 mapping
Y = np.array([1, 1, 0, 1, 0, 0, 0, 1, 1], np.int64)


def _groups(x, values, **kw):
    b = oracle.Binner("ordinal", x, ordinal_count=3, min_value=0)
    return oracle.extract_central_part(oracle.nunique_grid([b], values, **kw)).tolist()


def test_oracle_reference_kats():
    assert _groups(X, S) == [4, 2, 1]                       # agg_test.py:309-311
    assert _groups(X, S, dropnan=True) == [3, 2, 1]         # agg_test.py:313-315
    m = Y == 0                                              # agg_test.py:330-333 (filter)
    assert _groups(X[m], S[m])[:2] == [2, 2]
    # the string version's None as a missing value (agg_test.py:297-303)
    missing = np.isnan(S)
    assert _groups(X, np.where(missing, 0.0, S), mask=~missing) == [4, 2, 1]
    assert _groups(X, np.where(missing, 0.0, S), mask=~missing, dropmissing=True) == [3, 2, 1]


def test_oracle_selection_kat():
    # agg_test.py:344-360: w = dog, cat, mouse, dog, dog, dog, cat -> 1, 2, 3, 1, 1, 1, 2
    x = np.array([0, 0, 0, 1, 1, 2, 2], np.int64)
    y = np.array([1, 3, 5, 1, 7, 1, -1])
    w = np.array([1, 2, 3, 1, 1, 1, 2], np.int64)
    assert _groups(x, w, mask=y <= 3, selection=True, dropmissing=True, dropnan=True) == [2, 1, 2]


def test_oracle_drop_counts_rows_like_the_reference():
    # two NaNs in one cell: count() has +1 for NaN, dropnan subtracts the NaN ROW count (2)
    x = np.zeros(4, np.int64)
    assert _groups(x, np.array([1.0, np.nan, np.nan, 2.0]))[0] == 3
    assert _groups(x, np.array([1.0, np.nan, np.nan, 2.0]), dropnan=True)[0] == 1


# ---------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


def _agg_grid(values, x, mask=None, selection=None, dropmissing=False, dropnan=False, parts=1, device=False):
    from vaex_amd import superagg as sa
    from vaex_amd.device import DeviceArray
    dt = values.dtype
    postfix = dt.newbyteorder("=").name + ("" if dt.isnative else "_non_native")
    aggs = []
    bounds = np.linspace(0, len(x), parts + 1).astype(int)
    for a, b in zip(bounds[:-1], bounds[1:]):
        binner = sa.BinnerOrdinal_int64("x", 300, 0)
        xs, vs = x[a:b], values[a:b]
        if device:
            xs, vs = DeviceArray.from_numpy(xs), DeviceArray.from_numpy(np.ascontiguousarray(vs))
        binner.set_data(xs)
        grid = sa.Grid([binner])
        agg = getattr(sa, "AggNUnique_" + postfix)(grid, dropmissing, dropnan)
        agg.set_data(vs, 0)
        if mask is not None:
            agg.set_data_mask(np.ascontiguousarray(mask[a:b], dtype=np.uint8))
        if selection:
            agg.set_selection_mask(np.ascontiguousarray(mask[a:b], dtype=np.uint8))
        grid.bin([agg])
        aggs.append(agg)
    if parts > 1:
        aggs[0].reduce(aggs[1:])
    return np.asarray(aggs[0]).copy()


DTYPES = ["float64", "float32", "int64", "int32", "int16", "int8", "uint64", "uint32", "uint16", "uint8", "bool"]


@gpu
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("flip", [False, True])
def test_gpu_every_dtype(dtype, flip):
    rng = np.random.default_rng(zlib.crc32(f"{dtype}{flip}".encode()))
    n = 200_000
    x = rng.integers(-5, 305, n).astype(np.int64)
    if dtype == "bool":
        v = rng.random(n) > 0.5
    elif dtype.startswith("float"):
        v = rng.integers(-40, 40, n).astype(dtype) / 4
        v[::97] = np.nan
        v[::89] = -0.0
    else:
        info = np.iinfo(dtype)
        v = rng.integers(max(info.min, -200), min(info.max, 200), n).astype(dtype)
    if flip:
        v = v.astype(v.dtype.newbyteorder())
    mask = rng.random(n) > 0.1
    b = oracle.Binner("ordinal", x, ordinal_count=300, min_value=0)
    for kw in (dict(), dict(dropnan=True), dict(dropmissing=True), dict(dropnan=True, dropmissing=True)):
        exp = oracle.nunique_grid([b], v, mask=mask, **kw)
        got = _agg_grid(v, x, mask=mask, **kw)
        np.testing.assert_array_equal(got, exp, err_msg=str(kw))


@gpu
@pytest.mark.parametrize("parts,device", [(1, True), (3, False), (4, True)])
def test_gpu_selection_and_reduce(parts, device):
    rng = np.random.default_rng(parts)
    n = 300_000
    x = rng.integers(0, 300, n).astype(np.int64)
    v = rng.normal(size=n).round(2)
    v[::13] = np.nan
    sel = rng.random(n) > 0.3
    b = oracle.Binner("ordinal", x, ordinal_count=300, min_value=0)
    exp = oracle.nunique_grid([b], v, mask=sel, selection=True, dropnan=True)
    got = _agg_grid(v, x, mask=sel, selection=True, dropnan=True, parts=parts, device=device)
    np.testing.assert_array_equal(got, exp)


@gpu
@pytest.mark.parametrize("device", [False, True])
def test_gpu_dataframe_groupby_kats(device):
    """The reference's groupby KATs through DataFrame.groupby (host and HBM frames)."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    cols = dict(x=X, s=S, y=Y)
    if device:
        cols = {k: DeviceArray.from_numpy(v) for k, v in cols.items()}
    df = vaex_amd.from_arrays(**cols)
    g = df.groupby("x", agg={"nunique": vaex_amd.agg.nunique("s")})
    assert list(zip(g["x"].tolist(), g["nunique"].tolist())) == [(0, 4), (1, 2), (2, 1)]
    g = df.groupby("x", agg={"nunique": vaex_amd.agg.nunique("s", dropnan=True)})
    assert list(zip(g["x"].tolist(), g["nunique"].tolist())) == [(0, 3), (1, 2), (2, 1)]
    dff = df[df.y == 0] if device else df.filter("y == 0")
    g = dff.groupby("x", agg={"nunique": vaex_amd.agg.nunique("s")})
    assert list(zip(g["x"].tolist(), g["nunique"].tolist())) == [(0, 2), (1, 2)]
    g = df.groupby("x", agg={"nu": vaex_amd.agg.nunique("s", selection="y == 1", dropna=True), "n": "count"})
    assert g["nu"].tolist() == [2, 1, 1] and g["n"].tolist() == [5, 3, 1]


@gpu
def test_gpu_groupby_many_groups_vs_oracle():
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(7)
    n = 2_000_000
    key = rng.integers(0, 50_000, n).astype(np.int32)
    v = rng.integers(0, 40, n).astype(np.int64)
    df = vaex_amd.from_arrays(key=DeviceArray.from_numpy(key), v=DeviceArray.from_numpy(v))
    g = df.groupby("key", agg={"nu": vaex_amd.agg.nunique("v")})
    order = np.argsort(g["key"].to_numpy())
    pairs = np.unique(np.stack([key.astype(np.int64), v], axis=1), axis=0)
    keys, exp = np.unique(pairs[:, 0], return_counts=True)
    np.testing.assert_array_equal(g["key"].to_numpy()[order], keys)
    np.testing.assert_array_equal(g["nu"].to_numpy()[order], exp)


@gpu
@pytest.mark.parametrize("lds", ["0", "1"])
@pytest.mark.parametrize("card", [7, 300_000])
def test_gpu_workgroup_dedup_low_and_high_cardinality(monkeypatch, card, lds):
    """int32 / int8 values through the LDS-deduplicating collect: few distinct pairs per
    workgroup (all rows collapse in LDS) and more distinct pairs than the LDS table holds
    (table cleared between batches, probe misses appended as duplicates); VH_NU_LDS=0 is
    the plain collect with block-level slot reservation."""
    monkeypatch.setenv("VH_NU_LDS", lds)
    rng = np.random.default_rng(card)
    n = 3_000_000
    x = rng.integers(0, 300, n).astype(np.int64)
    v = rng.integers(0, card, n).astype(np.int32 if card > 127 else np.int8)
    b = oracle.Binner("ordinal", x, ordinal_count=300, min_value=0)
    exp = oracle.nunique_grid([b], v)
    got = _agg_grid(v, x, parts=1, device=True)
    np.testing.assert_array_equal(got, exp)
