"""groupby(key, assume_sparse=True) with count / sum / mean: the fused hash aggregation plus
vh_hashagg_order_first (groups in the order their keys first appear) must equal the ordered_set
grouper route -- the reference's structure, hash_primitives.hpp:96-281 + groupby.py:97-168 --
and the oracle's OrderedSet(1) key order, for every row layout (random keys found in a short
prefix, sorted / reverse-sorted runs scanned by run heads, keys that first appear at the very
end, which take the ordered_set fallback).  Counts and keys exact, float64 sums rtol 1e-9."""
import zlib

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _keys(layout, n, card, dtype, rng):
    if layout == "random":
        k = rng.integers(0, card, n)
    elif layout == "sorted":
        k = np.sort(rng.integers(0, card, n))
    elif layout == "reverse":
        k = np.sort(rng.integers(0, card, n))[::-1]
    elif layout == "late":  # 300 keys appear only in the last rows: the prefix scan gives up
        k = rng.integers(0, card, n)
        k[-600:] = card + np.arange(600) % 300
    else:  # clustered: runs of random lengths of random keys
        runs = rng.integers(1, 64, n // 8)
        k = np.repeat(rng.integers(0, card, len(runs)), runs)[:n]
        k = np.concatenate([k, rng.integers(0, card, n - len(k))])
    info = np.iinfo(dtype)
    k = k + max(info.min, -card // 2) if info.min < 0 else k
    return k.astype(dtype)


def _first_order(keys):
    u, first = np.unique(keys, return_index=True)
    return u[np.argsort(first)]


@pytest.mark.parametrize("layout", ["random", "sorted", "reverse", "late", "clustered"])
@pytest.mark.parametrize("kdtype", ["int32", "int64", "uint64", "int16"])
@pytest.mark.parametrize("device", [True, False])
def test_order_first_matches_ordered_set_route(layout, kdtype, device):
    import vaex_amd
    from vaex_amd import groupby as vg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(zlib.crc32(f"{layout}{kdtype}{device}".encode()))
    n = (1 << 22) + 5
    card = 20_000 if kdtype == "int16" else 200_000
    keys = _keys(layout, n, card, kdtype, rng)
    v = rng.normal(size=n)
    v[rng.random(n) < 0.01] = np.nan
    put = DeviceArray.from_numpy if device else (lambda a: a)
    df = vaex_amd.from_arrays(key=put(keys), v=put(v))
    agg = {"s": vaex_amd.agg.sum("v"), "c": vaex_amd.agg.count("v"), "n": vaex_amd.agg.count(),
           "m": vaex_amd.agg.mean("v")}
    got = df.groupby("key", agg=agg, assume_sparse=True)
    gk = got["key"].to_numpy()
    np.testing.assert_array_equal(gk, _first_order(keys))
    # the ordered_set grouper route (set build + set-ordinal grid) the same frame
    ref = vg.GroupBy(df, "key", dense=False).agg(agg)
    np.testing.assert_array_equal(ref["key"].to_numpy(), gk)
    assert got["key"].to_numpy().dtype == ref["key"].to_numpy().dtype
    for col in ("c", "n"):
        np.testing.assert_array_equal(got[col].to_numpy(), ref[col].to_numpy())
    for col in ("s", "m"):
        np.testing.assert_allclose(got[col].to_numpy(), ref[col].to_numpy(), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("layout", ["random", "sorted", "late"])
def test_order_first_matches_oracle_ordered_set(layout):
    """Key order = the single-thread OrderedSet restatement's key_array (hash_primitives.hpp
    :96-281,289-312, nmaps = 1) on a size the pure-Python oracle finishes quickly."""
    import vaex_amd
    rng = np.random.default_rng(zlib.crc32(layout.encode()))
    keys = _keys(layout, 30_000, 2_000, "int64", rng)
    df = vaex_amd.from_arrays(key=keys, v=rng.random(len(keys)))
    got = df.groupby("key", agg={"n": vaex_amd.agg.count()}, assume_sparse=True)
    s = oracle.OrderedSet(1)
    s.update(keys)
    np.testing.assert_array_equal(got["key"].to_numpy(), s.key_array(keys.dtype))
    np.testing.assert_array_equal(got["n"].to_numpy()[np.argsort(s.map_ordinal(got["key"].to_numpy()))],
                                  np.bincount(s.map_ordinal(keys), minlength=len(s)))


def test_order_first_sort_true_is_key_order():
    import vaex_amd
    rng = np.random.default_rng(4)
    keys = rng.integers(-5000, 5000, 1 << 20).astype(np.int32)
    df = vaex_amd.from_arrays(key=keys, v=rng.random(len(keys)))
    got = df.groupby("key", agg={"s": vaex_amd.agg.sum("v")}, assume_sparse=True, sort=True)
    np.testing.assert_array_equal(got["key"].to_numpy(), np.unique(keys))


def test_order_first_rejects_another_column():
    """A key column the aggregation never saw fails loudly (no hang, no partial order)."""
    from vaex_amd import _lib
    from vaex_amd.hashagg import HashAgg
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(8)
    keys = DeviceArray.from_numpy(rng.integers(0, 1000, 1 << 20).astype(np.int32))
    other = DeviceArray.from_numpy(rng.integers(5000, 6000, 1 << 20).astype(np.int32))
    ha = HashAgg(np.int32, [])
    ha.update(keys, [])
    with pytest.raises(_lib.HipError):
        ha.finish(first_order_keys=other)


def test_order_first_tiny_inputs():
    import vaex_amd
    for keys in ([7], [3, 3, 3], [2, 1], [5, 4, 5, 4, 9]):
        k = np.array(keys, np.int64)
        df = vaex_amd.from_arrays(key=k, v=np.ones(len(k)))
        got = df.groupby("key", agg={"n": vaex_amd.agg.count()}, assume_sparse=True)
        np.testing.assert_array_equal(got["key"].to_numpy(), _first_order(k))
        np.testing.assert_array_equal(got["n"].to_numpy(), [int((k == x).sum()) for x in _first_order(k)])


def test_order_first_wave_straddling_the_grid_stride():
    """The first-row scan (k_ha_first) takes each row's predecessor from the neighbour lane.
    A chunk whose vector count is not a multiple of the grid stride leaves one wave with
    lanes in the two-vector loop and lanes in the one-vector remainder; the scan must still
    compare each row with its true predecessor.  Layout (for the MI355X grid of 2048 x 256
    lanes, 4 int32 keys per lane step): run-structured keys so the second scan chunk spans
    [2^20, n) rows, a key K that first appears at the first row of the remainder wave's
    first remainder lane, K again in the rows the neighbour lane held last, and a key M
    first appearing right after K's first run: K must come before M."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(123)
    S = 2048 * 256  # grid stride in 16-B vectors (blocks_for cap: 256 CUs x 8)
    R = 3_000_148  # rows of the second chunk: 750037 vectors, boundary 225749 (lane 21 of its wave)
    c0 = 1 << 20
    n = c0 + R
    keys = np.repeat(rng.integers(0, 1000, n // 64 + 1), 64)[:n].astype(np.int32)
    K, M = 5000, 5001
    b = R // 4 - S
    row = lambda v: c0 + 4 * v  # noqa: E731
    keys[row(b) - 1] = 7  # the true predecessor differs from K
    keys[row(b):row(b) + 8] = K
    keys[row(b) + 8:row(b) + 12] = M
    keys[row(b) + 12:row(b) + 16] = K
    keys[row(b - 1 + S):row(b + S)] = K  # what the neighbour lane loaded last
    keys[row(b - 1 + S) + 4:row(b - 1 + S) + 8] = M
    dkeys = DeviceArray.from_numpy(keys)
    exp = _first_order(keys)
    u, cnt = np.unique(keys, return_counts=True)
    # the hash aggregation's scan (k_ha_first) ...
    from vaex_amd.hashagg import HashAgg
    ha = HashAgg(np.int32, [])
    ha.update(dkeys, [])
    hk, hc, _, _ = ha.finish(first_order_keys=dkeys)
    np.testing.assert_array_equal(hk, exp)
    np.testing.assert_array_equal(hc, cnt[np.searchsorted(u, exp)])
    # ... and the dense-range grid route's (k_dense_first), through groupby(assume_sparse=True)
    # with an aggregator the hash aggregation does not carry (min)
    df = vaex_amd.from_arrays(key=dkeys, v=DeviceArray.from_numpy(np.ones(n)))
    got = df.groupby("key", agg={"n": vaex_amd.agg.count(), "lo": vaex_amd.agg.min("v")}, assume_sparse=True)
    np.testing.assert_array_equal(got["key"].to_numpy(), exp)
    gk = list(got["key"].to_numpy())
    assert gk.index(K) < gk.index(M)
    np.testing.assert_array_equal(got["n"].to_numpy(), cnt[np.searchsorted(u, exp)])
