"""The hash-partitioned ordered_set update (hashset.hip: sample, pass A partition, pass B
LDS dedup + one HBM insert per distinct key per unit, direct mode for few keys) against the
single-threaded reference restatement (oracle.OrderedSet, hash_primitives.hpp:96-281,
289-312, 543-583): key_array bit-exact in first-appearance order, map_ordinal exact.

Edge cases the partitioned design has to get right: keys whose bits equal the LDS table's
EMPTY / CLOSED markers (-1 / -2 of every width), the 8-byte key whose bits equal the HBM
table's EMPTY marker (the side slot), a distinct-key estimate that misses badly (the
sample sees one key, the column holds millions: HBM table overflow, grow, re-run), LDS
tables that close (far more keys per unit than slots), NaN / null / unselected rows, and
several update calls (row numbering across calls)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _check(s, keys_list, dtype, masks=None):
    ref = oracle.OrderedSet(nmaps=1)
    for i, k in enumerate(keys_list):
        ref.update(k, None if masks is None else masks[i])
    np.testing.assert_array_equal(s.key_array(), ref.key_array(dtype))
    assert len(s) == len(ref)
    allk = np.concatenate(keys_list)
    np.testing.assert_array_equal(s.map_ordinal(allk).astype(np.int64), ref.map_ordinal(allk).astype(np.int64))


@pytest.mark.parametrize("dtype", ["int64", "int32", "uint32", "int16", "uint8", "uint64"])
def test_marker_valued_keys(dtype):
    from vaex_amd import superutils
    rng = np.random.default_rng(1)
    info = np.iinfo(dtype)
    n = 300_000
    keys = rng.integers(max(info.min, -50_000), min(info.max, 50_000), n, endpoint=True).astype(dtype)
    # all-ones / all-ones-minus-one bit patterns of the key width
    ones = np.array(-1).astype(dtype) if info.min < 0 else np.array(info.max, dtype)
    keys[rng.random(n) < 0.01] = ones
    keys[rng.random(n) < 0.01] = (ones - 1).astype(dtype)
    keys[:3] = [ones, (ones - 1).astype(dtype), keys[5]]
    s = getattr(superutils, "ordered_set_" + dtype)()
    s.update(keys)
    _check(s, [keys], dtype)


def test_estimate_miss_overflow_rerun():
    """The sample (evenly spaced 4096-row blocks) sees only key 0; every other row holds a
    distinct key, so the pre-sized table overflows and the chunk is re-run after growing."""
    from vaex_amd import superutils
    n = 1 << 22
    keys = np.arange(n, dtype=np.int64) * 7 + 11
    stride = n // 256
    for b in range(256):
        keys[b * stride:b * stride + 4096] = 0
    s = superutils.ordered_set_int64()
    s.update(keys)
    _check(s, [keys], "int64")


def test_direct_mode_lds_close():
    """Few distinct keys in the sample but each workgroup sees more keys than its LDS table
    holds: keys spill to the HBM table through the CLOSED slots; results unchanged."""
    from vaex_amd import superutils
    rng = np.random.default_rng(2)
    n = 2_000_000
    keys = rng.integers(0, 3000, n).astype(np.int32)
    keys[::3] = rng.integers(-(1 << 30), 1 << 30, len(keys[::3])).astype(np.int32)
    s = superutils.ordered_set_int32()
    s.update(keys)
    _check(s, [keys], "int32")


def test_many_keys_partitioned_multi_update():
    from vaex_amd import superutils
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(3)
    parts = [rng.integers(-2_000_000, 2_000_000, 3_000_000).astype(np.int32) for _ in range(3)]
    s = superutils.ordered_set_int32()
    s.update(DeviceArray.from_numpy(parts[0]))
    s.update(parts[1])
    s.update(DeviceArray.from_numpy(parts[2]))
    _check(s, parts, "int32")


def test_float_keys_nan_null_select():
    from vaex_amd import superutils
    from vaex_amd.device import DeviceArray
    rng = np.random.default_rng(4)
    n = 1_500_000
    keys = np.round(rng.normal(size=n) * 1000, 1)
    keys[rng.random(n) < 0.02] = np.nan
    keys[7] = -0.0
    mask = rng.random(n) < 0.01
    s = superutils.ordered_set_float64()
    s.update(keys, mask)
    _check(s, [keys], "float64", masks=[mask])
    assert s.nan_count == int(np.isnan(keys[~mask]).sum()) and s.null_count == int(mask.sum())
    # select: only the selected rows enter the set (device mask)
    sel = rng.random(n) < 0.5
    s2 = superutils.ordered_set_float64()
    s2.update(DeviceArray.from_numpy(keys), select=DeviceArray.from_numpy(sel.astype(np.uint8)))
    ref = oracle.OrderedSet(nmaps=1)
    ref.update(keys[sel])
    np.testing.assert_array_equal(s2.key_array(), ref.key_array(np.float64))


@pytest.mark.parametrize("dtype", ["float64", "float32", "int64", "uint16", "int8"])
def test_grouper_sort_on_device(dtype):
    """Grouper(sort=True) orders the set's keys with the device argsort: ascending, NaN after
    the numbers, null last (groupby.py:137-156) -- equal to Python's sorted() on the same
    keys; counts follow their keys."""
    import vaex_amd
    from vaex_amd.groupby import Grouper
    rng = np.random.default_rng(9)
    n = 200_000
    if dtype.startswith("float"):
        keys = np.round(rng.normal(size=n) * 50).astype(dtype)
        keys[rng.random(n) < 0.01] = np.nan
        keys[3] = -0.0
    else:
        info = np.iinfo(dtype)
        keys = rng.integers(info.min, info.max, n, endpoint=True).astype(dtype)
    mask = rng.random(n) < 0.005
    df = vaex_amd.from_arrays(k=np.ma.array(keys, mask=mask))
    g = Grouper(df.k, df=df, sort=True)
    labels = g.labels()
    plain = [v for v in labels if v is not None]
    exp = sorted(plain, key=lambda v: (1, 0) if v != v else (0, v))
    got = [v for v in labels if v is not None]
    assert [(0 if v == v else 1, v if v == v else 0) for v in got] == [(0 if v == v else 1, v if v == v else 0) for v in exp]
    assert labels[-1] is None  # null last
