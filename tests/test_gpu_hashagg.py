"""Fused hash groupby (hashagg.hip) against the oracle's key -> (sum, count) restatement
(oracle.groupby_reference: the reference's single-threaded AggSum / AggCount grids over
the ordered_set ordinals, superagg.cpp:155-192,349-389 + groupby.py:484-533).

Groups come out sorted by key, so keys, counts and integer sums are compared bit-exactly
and float sums within 1e-6 relative (north_star; the association order differs).
Covers every key dtype incl. the LDS table's sentinel bit patterns, every value kind,
direct (P = 1) and partitioned paths, closed LDS tables (more keys per bucket than fit),
region overflow (sorted / skewed keys), chunked updates, host and device columns."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _ha():
    from vaex_amd import hashagg
    return hashagg


def _expected_int_sums(keys, vals, uniq):
    inv = np.searchsorted(uniq, keys)
    out = np.zeros(len(uniq), np.int64 if vals.dtype.kind in "i" else np.uint64)
    np.add.at(out, inv, vals.astype(out.dtype))
    return out


def _run(keys, vals, chunks=1, device=False):
    from vaex_amd.device import DeviceArray
    ha = _ha().HashAgg(keys.dtype, [v.dtype for v in vals])
    n = len(keys)
    bounds = np.linspace(0, n, chunks + 1).astype(int)
    for a, b in zip(bounds[:-1], bounds[1:]):
        k, vs = keys[a:b], [v[a:b] for v in vals]
        if device:
            k, vs = DeviceArray.from_numpy(k), [DeviceArray.from_numpy(v) for v in vs]
        ha.update(k, vs)
    return ha.finish()


def _check(keys, vals, out):
    gk, cnt, sums, nn = out
    # sorted in the key's own order (uint64 keys above 2**63 sort last)
    uniq, first_inv = np.unique(keys, return_inverse=True)
    ordinal = first_inv.astype(np.int64)
    assert gk.dtype == (np.uint64 if keys.dtype == np.uint64 else np.int64)
    np.testing.assert_array_equal(gk, uniq)
    np.testing.assert_array_equal(cnt, np.bincount(first_inv, minlength=len(uniq)))
    for v, s, c in zip(vals, sums, nn):
        if v.dtype.kind == "f":
            uk, es, ec = oracle.groupby_reference(ordinal, v.astype(np.float64))
            np.testing.assert_array_equal(c, ec)
            np.testing.assert_allclose(s, es, rtol=1e-6, atol=1e-9)
        else:
            np.testing.assert_array_equal(s, _expected_int_sums(ordinal, v, np.arange(len(uniq))))
            np.testing.assert_array_equal(c, np.bincount(first_inv, minlength=len(uniq)))


def _keys(dtype, n, card, rng):
    dt = np.dtype(dtype)
    info = np.iinfo(dt)
    span = min(card, int(info.max) - int(info.min) + 1)
    lo = int(info.min) if dt.kind == "i" else 0
    if dt.itemsize == 8:
        # 64-bit keys: a sparse spread over the whole range (the hash, not the span, matters)
        pool = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, card, dtype=np.int64, endpoint=True)
        k = pool[rng.integers(0, card, n)].view(dt)
    else:
        k = (lo + rng.integers(0, span, n)).astype(dt)
    # the table sentinels (all-ones / all-ones - 1 key bits, the HBM table's side slot for
    # 64-bit keys) and extremes
    if dt.kind == "i":
        k[:4] = np.array([-1, -2, info.min, info.max], dtype=np.int64).astype(dt)
    else:
        k[:4] = np.array([info.max, info.max - 1, 0, 1], dtype=np.uint64).astype(dt)
    return k


@pytest.mark.parametrize("kdtype", ["int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64"])
@pytest.mark.parametrize("card", [3, 200, 60000])
def test_key_dtypes(kdtype, card):
    rng = np.random.default_rng(card)
    n = 400_000
    keys = _keys(kdtype, n, card, rng)
    v = rng.normal(size=n)
    v[::37] = np.nan
    _check(keys, [v], _run(keys, [v]))


@pytest.mark.parametrize("vdtypes", [[], ["float32"], ["int8", "float64"], ["uint16", "bool"], ["int64", "uint32"]])
def test_value_kinds(vdtypes):
    rng = np.random.default_rng(4)
    n = 300_000
    keys = rng.integers(-5000, 5000, n).astype(np.int32)
    vals = []
    for d in vdtypes:
        dt = np.dtype(d)
        if dt.kind == "f":
            a = (rng.normal(size=n) * 100).astype(dt)
            a[::13] = np.nan
        elif dt.kind == "b":
            a = rng.random(n) < 0.3
        else:
            info = np.iinfo(dt)
            a = rng.integers(max(info.min, -1000), min(info.max, 1000), n).astype(dt)
        vals.append(a)
    _check(keys, vals, _run(keys, vals))


@pytest.mark.parametrize("n,card", [(3_000_000, 1_000_000), (4_000_000, 4_000_000)])
def test_high_cardinality(n, card):
    rng = np.random.default_rng(5)
    if card >= n:
        keys = rng.permutation(n).astype(np.int32) * 7 - 12345
    else:
        keys = (5 + rng.integers(0, card, n)).astype(np.int32)
    v = rng.normal(size=n)
    _check(keys, [v], _run(keys, [v]))


def test_closed_lds_tables():
    """~8e6 distinct keys: more than P_max x 2560 fit in the LDS tables, so tables close
    and the rest goes through the HBM-table path; results must not change."""
    rng = np.random.default_rng(6)
    n = 9_000_000
    keys = rng.permutation(np.arange(n, dtype=np.int64) * 3 - 10 ** 9).astype(np.int32)[:n]
    keys[: n // 9] = keys[n // 9: 2 * (n // 9)]  # some repeats
    v = rng.random(n)
    _check(keys, [v], _run(keys, [v], device=True))


@pytest.mark.parametrize("kdtype,nvals,n,card", [("int64", 1, 16_000_000, 12_000_000),
                                                  ("int64", 2, 16_000_000, 12_000_000),
                                                  ("int32", 1, 24_000_000, 20_000_000)])
def test_repartitioned_high_cardinality(kdtype, nvals, n, card):
    """More keys per bucket than an LDS table holds with P at its cap: pass-B entries are
    re-split into sub-buckets first (k_ha_repart); packed {key, value} and separate-array
    entry formats, wide (8-byte keys) and narrow (int32) tables."""
    rng = np.random.default_rng(card + nvals)
    keys = (rng.integers(0, card, n) * 2654435761 - 77).astype(kdtype)
    vals = [rng.normal(size=n)]
    if nvals > 1:
        vals.append(rng.integers(-1000, 1000, n).astype(np.int32))
    _check(keys, vals, _run(keys, vals, device=True))


@pytest.mark.parametrize("layout", ["sorted", "heavy", "runs"])
def test_skewed_and_sorted_keys(layout):
    """Per-workgroup bucket fractions far from the sampled global ones: region overflow
    rows take the HBM-table path."""
    rng = np.random.default_rng(7)
    n = 2_000_000
    if layout == "sorted":
        keys = np.sort(rng.integers(0, 300_000, n)).astype(np.int32)
    elif layout == "heavy":
        keys = rng.integers(0, 100_000, n).astype(np.int32)
        keys[rng.random(n) < 0.6] = 42
    else:
        keys = np.repeat(np.arange(20, dtype=np.int32) * 1000, n // 20)
    v = rng.normal(size=len(keys))
    _check(keys, [v], _run(keys, [v]))


@pytest.mark.parametrize("device", [False, True])
def test_chunked_updates(device):
    rng = np.random.default_rng(8)
    n = 3_000_000
    keys = rng.integers(0, 500_000, n).astype(np.uint32)
    keys[n // 2:] += 400_000  # later chunks bring new keys: the HBM table grows across updates
    v = rng.normal(size=n)
    v2 = rng.integers(-50, 50, n).astype(np.int16)
    _check(keys, [v, v2], _run(keys, [v, v2], chunks=5, device=device))


def test_empty_and_tiny():
    keys = np.array([], np.int32)
    gk, cnt, sums, nn = _run(keys, [np.array([], np.float64)])
    assert len(gk) == 0 and len(cnt) == 0
    keys = np.array([7, -1, 7], np.int32)
    v = np.array([1.0, np.nan, 2.0])
    gk, cnt, sums, nn = _run(keys, [v])
    assert gk.tolist() == [-1, 7] and cnt.tolist() == [1, 2] and nn[0].tolist() == [0, 2]
    assert sums[0].tolist() == [0.0, 3.0]


def test_dataframe_groupby_uses_fused_path(monkeypatch):
    """DataFrame.groupby takes the fused path for this query shape and returns the same
    frame as the grouper path (assume_sparse=True: ordered_set + BinnerOrdinal)."""
    import vaex_amd
    from vaex_amd import hashagg
    rng = np.random.default_rng(9)
    n = 1_000_000
    # sparse keys (value span >> rows): the dense-range grouper does not apply
    keys = (rng.integers(-100, 20000, n).astype(np.int64) * 104729 - 10 ** 9).astype(np.int32)
    df = vaex_amd.from_arrays(key=keys, v=rng.normal(size=n), w=rng.integers(0, 10, n).astype(np.int8))
    agg = {"v": ["sum", "count", "mean"], "w": "sum", "n": "count"}
    calls = []
    orig = hashagg.HashAgg.update
    monkeypatch.setattr(hashagg.HashAgg, "update", lambda self, *a: (calls.append(1), orig(self, *a))[1])
    fused = df.groupby("key", agg=agg)
    assert calls, "fused path not taken"
    ref = df.groupby("key", agg=agg, assume_sparse=True).sort("key")
    assert fused.get_column_names() == ref.get_column_names()
    for c in ref.get_column_names():
        a, b = fused[c].to_numpy(), ref[c].to_numpy()
        assert a.dtype == b.dtype, c
        if a.dtype.kind == "f":
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-9)
        else:
            np.testing.assert_array_equal(a, b)


def test_row_limit():
    import vaex_amd
    from vaex_amd.dataframe import RowLimitException
    df = vaex_amd.from_arrays(key=np.arange(1000, dtype=np.int32), v=np.ones(1000))
    with pytest.raises(RowLimitException):
        df.groupby("key", agg={"v": "sum"}, row_limit=10)


@pytest.mark.parametrize("n", [2_000_000, 2_000_001])
def test_dense_int32_keys_take_fast_ordinal_tile_path(n):
    """A dense int32 key range goes to the categorical-style grid (min/max pass +
    BinnerOrdinal) whose pass A is the fast ordinal kernel; the result equals the oracle
    map and the fused path's.  Odd n exercises the last-row split."""
    import vaex_amd
    from vaex_amd import _lib
    rng = np.random.default_rng(10)
    keys = (5 + rng.integers(0, 300_000, n)).astype(np.int32)
    v = rng.normal(size=n)
    v[::53] = np.nan
    df = vaex_amd.from_arrays(key=keys, v=v)
    _lib.timing_reset()
    _lib.timing_enable(True)
    dfg = df.groupby("key", agg={"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v"), "n": "count"})
    _lib.synchronize()
    _lib.timing_enable(False)
    assert _lib.timing_read("tile_scatter_ord")[0] >= 1, "fast ordinal pass A not used"
    uk, s, c = oracle.groupby_reference(keys, v)
    gk = dfg["key"].to_numpy()
    np.testing.assert_array_equal(gk, uk)
    np.testing.assert_array_equal(dfg["v_count"].to_numpy(), c)
    np.testing.assert_array_equal(dfg["n"].to_numpy(), np.bincount(keys)[uk])
    np.testing.assert_allclose(dfg["v_sum"].to_numpy(), s, rtol=1e-6, atol=1e-9)
    fk, fc, fs, fn = _run(keys, [v])
    np.testing.assert_array_equal(fk, uk)
    np.testing.assert_allclose(fs[0], s, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("vdtypes", [("int8", "float32"), ("int16", "uint8"), ("int32", "uint32"), ("bool", "int64"),
                                     ("uint16", "float64")])
@pytest.mark.parametrize("device", [False, True])
def test_dense_int32_keys_fast_ordinal_any_value_dtype(vdtypes, device):
    """The fast ordinal pass A with value columns of any native dtype (the h2o q3 / q5
    shape: int8 and float32 sums, mean of float32): exact integer sums, float sums within
    1e-6, NaN-keyed counts; 4-byte value slots when every column is <= 4 bytes."""
    import vaex_amd
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(len(vdtypes[0]) * 31 + len(vdtypes[1]))
    n = 2_000_000
    keys = (5 + rng.integers(0, 250_000, n)).astype(np.int32)
    cols = {"key": keys}
    for j, dt in enumerate(vdtypes):
        if dt == "bool":
            a = rng.random(n) > 0.5
        elif dt.startswith("float"):
            a = rng.normal(size=n).astype(dt)
            a[::37] = np.nan
        else:
            info = np.iinfo(dt)
            a = rng.integers(info.min, info.max, n, endpoint=True).astype(dt)
        cols[f"v{j}"] = a
    df = vaex_amd.from_arrays(**({k: DeviceArray.from_numpy(v) for k, v in cols.items()} if device else cols))
    agg = {}  # at most 4 aggregators: one tile-path pass (sum, sum, and a mean's sum + count)
    for j, dt in enumerate(vdtypes):
        agg[f"s{j}"] = vaex_amd.agg.sum(f"v{j}")
        if dt.startswith("float"):
            agg[f"m{j}"] = vaex_amd.agg.mean(f"v{j}")
    _lib.timing_reset()
    _lib.timing_enable(True)
    g = df.groupby("key", agg=agg)
    _lib.synchronize()
    _lib.timing_enable(False)
    assert _lib.timing_read("tile_scatter_ord")[0] >= 1, "fast ordinal pass A not used"
    uk, inv = np.unique(keys, return_inverse=True)
    np.testing.assert_array_equal(g["key"].to_numpy(), uk)
    for j, dt in enumerate(vdtypes):
        a = cols[f"v{j}"]
        if dt.startswith("float"):
            ok = ~np.isnan(a)
            es = np.bincount(inv[ok], weights=a[ok].astype(np.float64), minlength=len(uk))
            ec = np.bincount(inv[ok], minlength=len(uk))
            np.testing.assert_allclose(g[f"s{j}"].to_numpy(), es, rtol=1e-6, atol=1e-6)
            with np.errstate(divide="ignore", invalid="ignore"):
                np.testing.assert_allclose(g[f"m{j}"].to_numpy(), es / ec, rtol=1e-6, atol=1e-6)
        else:
            wide = np.uint64 if dt.startswith("uint") or dt == "bool" else np.int64
            es = np.zeros(len(uk), wide)
            np.add.at(es, inv, a.astype(wide))
            np.testing.assert_array_equal(g[f"s{j}"].to_numpy(), es)


@pytest.mark.parametrize("vdtype", ["int8", "float32", "float64", "int64", "uint16", "int32"])
@pytest.mark.parametrize("device", [False, True])
def test_dense_keys_min_max_through_tile_path(vdtype, device):
    """h2o q7's shape: max / min per group over a 2.5e5-group dense grid go through the
    tile path (LDS min / max cells) instead of per-row global atomics; equal to numpy."""
    import vaex_amd
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(len(vdtype))
    n = 2_000_000
    keys = (5 + rng.integers(0, 250_000, n)).astype(np.int32)
    if vdtype.startswith("float"):
        v = rng.normal(size=n).astype(vdtype)
        v[::29] = np.nan
    else:
        info = np.iinfo(vdtype)
        v = rng.integers(info.min, info.max, n, endpoint=True).astype(vdtype)
    cols = {"key": keys, "v": v}
    df = vaex_amd.from_arrays(**({k: DeviceArray.from_numpy(a) for k, a in cols.items()} if device else cols))
    _lib.timing_reset()
    _lib.timing_enable(True)
    g = df.groupby("key", agg={"mx": vaex_amd.agg.max("v"), "mn": vaex_amd.agg.min("v"), "n": "count"})
    _lib.synchronize()
    _lib.timing_enable(False)
    assert _lib.timing_read("bin_aggregate")[0] == 0, "min / max took the generic global-atomic path"
    uk, inv = np.unique(keys, return_inverse=True)
    np.testing.assert_array_equal(g["key"].to_numpy(), uk)
    np.testing.assert_array_equal(g["n"].to_numpy(), np.bincount(inv))
    order = np.argsort(inv, kind="stable")
    starts = np.r_[0, np.cumsum(np.bincount(inv))[:-1]]
    vs = v[order]
    if vdtype.startswith("float"):
        # NaN never enters (superagg.cpp AggMax/AggMin): an all-NaN group keeps the -inf / +inf fill
        exp_mx = np.nan_to_num(np.fmax.reduceat(vs, starts), nan=-np.inf)
        exp_mn = np.nan_to_num(np.fmin.reduceat(vs, starts), nan=np.inf)
    else:
        exp_mx = np.maximum.reduceat(vs, starts)
        exp_mn = np.minimum.reduceat(vs, starts)
    np.testing.assert_array_equal(g["mx"].to_numpy(), exp_mx)
    np.testing.assert_array_equal(g["mn"].to_numpy(), exp_mn)


@pytest.mark.parametrize("n,card", [(3_000_000, 1_000_000), (600_000, 3)])
@pytest.mark.parametrize("kdtype", ["int64", "uint64"])
def test_64bit_keys_partitioned_and_chunked(kdtype, n, card):
    """64-bit keys through the partitioned path (many buckets), chunked device updates, the
    all-ones key in the HBM table's side slot in every chunk."""
    rng = np.random.default_rng(card + 1)
    keys = _keys(kdtype, n, card, rng)
    keys[n // 2] = keys[0]
    v = rng.normal(size=n)
    w = rng.integers(-5, 5, n).astype(np.int32)
    _check(keys, [v, w], _run(keys, [v, w], chunks=3, device=True))


def test_64bit_keys_that_collide_in_low_bits():
    """Keys equal in their low 32 bits (and in their high 32 bits) stay distinct groups."""
    lo = np.arange(1000, dtype=np.int64)
    keys = np.concatenate([lo, lo + (1 << 32), lo + (7 << 40), (lo << 32) | 5, lo]).astype(np.int64)
    rng = np.random.default_rng(3)
    keys = keys[rng.permutation(len(keys))]
    v = rng.normal(size=len(keys))
    _check(keys, [v], _run(keys, [v]))


@pytest.mark.parametrize("dtypes", [["int32", "int8"], ["uint16", "int64", "int32"], ["uint32", "uint32"]])
def test_combine_keys(dtypes):
    """vh_combine_keys = the cartesian ordinal of groupby.py:248-288 (first key most
    significant), bit-exact against numpy."""
    import ctypes
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(len(dtypes))
    n = 1_000_003
    cols = []
    for d in dtypes:
        info = np.iinfo(d)
        lo = max(int(info.min), -1000)
        cols.append(rng.integers(lo, lo + 700, n).astype(d))
    mins = [int(c.min()) for c in cols]
    spans = [int(c.max()) - m + 1 for c, m in zip(cols, mins)]
    mults = [int(np.prod(spans[i + 1:], dtype=np.int64)) for i in range(len(cols))]
    expect = np.zeros(n, np.int64)
    for c, m, k in zip(cols, mins, mults):
        expect += (c.astype(np.int64) - m) * k
    dcols = [DeviceArray.from_numpy(c) for c in cols]
    out = DeviceArray.empty(n, np.int64)
    k = len(cols)
    _lib.call("vh_combine_keys", n, k, (ctypes.c_void_p * k)(*[c.ptr for c in dcols]),
              (ctypes.c_int * k)(*[_lib.dtype_code(np.dtype(d))[0] for d in dtypes]),
              (ctypes.c_int64 * k)(*mins), (ctypes.c_int64 * k)(*mults), out.ptr)
    np.testing.assert_array_equal(out.to_numpy(), expect)
