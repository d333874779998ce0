"""Fused hash groupby (``libvaexhip`` ``vh_hashagg_*``, ``vaex_amd/csrc/hashagg.hip``).

``groupby(key).agg(...)`` of one integer key column (any width) with count / sum / mean
aggregates over at most two numeric value columns runs as ONE hash-partitioned pass over
the data instead of the reference's two passes (ordered_set build, then
``_ordinal_values`` + ``BinnerOrdinal`` + ``AggCount``/``AggSum``; groupby.py:97-168,
484-533).  The per-key results are the same grids' central parts; groups come out sorted
by key.  :func:`try_groupby` returns ``None`` for any query outside that shape (masks,
filters, selections, other aggregators, wide keys) and the caller takes the general
grouper path; an overflowing hash table also returns ``None`` (never a partial result).
"""
import ctypes

import numpy as np

from . import _lib, hostops
from .device import DeviceArray
from .utils import label_dtype

KEY_DTYPES = {"int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64"}
VALUE_KINDS = "fiub"


class HashAggOverflow(RuntimeError):
    pass


class HashAgg:
    """Accumulates groups over one or more chunks of (key, values) rows."""

    def __init__(self, key_dtype, value_dtypes, nonnull=None):
        """nonnull[v]: the non-NaN count of value column v is needed (count(v) / mean);
        default all."""
        self.key_dtype = np.dtype(key_dtype)
        self.value_dtypes = [np.dtype(d) for d in value_dtypes]
        kcode, _ = _lib.dtype_code(self.key_dtype)
        codes = (ctypes.c_int * max(1, len(self.value_dtypes)))(*[_lib.dtype_code(d)[0] for d in self.value_dtypes])
        if nonnull is None:
            nonnull = [True] * len(self.value_dtypes)
        self.nonnull = list(nonnull)
        nnmask = sum(1 << i for i, want in enumerate(nonnull) if want)
        h = ctypes.c_void_p()
        _lib.call("vh_hashagg_create", kcode, len(self.value_dtypes), codes, nnmask, ctypes.byref(h))
        self._h = h
        self._keep = []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib().vh_hashagg_destroy(h)
            self._h = None

    def update(self, keys, values):
        n = len(keys)
        if any(len(v) != n for v in values):
            raise ValueError("key and value columns differ in length")
        cols = [keys] + list(values)
        on_device = [isinstance(c, DeviceArray) for c in cols]
        if any(on_device) and not all(on_device):
            cols = [c if isinstance(c, DeviceArray) else DeviceArray.from_numpy(c) for c in cols]
            self._keep.append(cols)
            loc = _lib.LOC_DEVICE
        elif all(on_device):
            loc = _lib.LOC_DEVICE
        else:
            cols = [np.ascontiguousarray(c) for c in cols]
            loc = _lib.LOC_HOST
        ptrs = [c.ptr if isinstance(c, DeviceArray) else c.ctypes.data for c in cols]
        vals = (ctypes.c_void_p * max(1, len(values)))(*ptrs[1:])
        rc = _lib.lib().vh_hashagg_update(self._h, ptrs[0], vals, n, loc)
        if rc != 0:
            msg = _lib.lib().vh_last_error().decode(errors="replace")
            if "overflow" in msg or "too many groups" in msg:
                raise HashAggOverflow(msg)
            _lib.check(rc)

    def order_first(self, keys):
        """After finish(): put the groups in the order their keys first appear in ``keys`` (the
        whole key column the updates saw) -- an ordered_set's ordinal order
        (hash_primitives.hpp:96-281), what ``groupby(key, assume_sparse=True)`` returns."""
        loc = _lib.LOC_DEVICE if isinstance(keys, DeviceArray) else _lib.LOC_HOST
        if loc == _lib.LOC_HOST:
            keys = np.ascontiguousarray(keys)
        ptr = keys.ptr if loc == _lib.LOC_DEVICE else keys.ctypes.data
        _lib.call("vh_hashagg_order_first", self._h, ptr, len(keys), loc)

    def finish(self, comm=None, gather=True, device_keys=False, first_order_keys=None):
        """The groups, key-sorted: (keys, counts, sums, nonnull).  With an RCCL communicator
        (``comm.device``) the ranks' groups are first exchanged by hash partition on the
        device (vh_hashagg_exchange): each rank keeps the groups it owns, or with ``gather``
        the whole result."""
        m = ctypes.c_uint64()
        _lib.call("vh_hashagg_finish", self._h, ctypes.byref(m))
        if first_order_keys is not None:
            self.order_first(first_order_keys)
        if comm is not None and comm.world > 1:
            if not comm.device:
                raise ValueError("the device exchange needs an RCCL communicator")
            _lib.call("vh_hashagg_exchange", self._h, comm.handle, int(bool(gather)))
            _lib.call("vh_hashagg_finish", self._h, ctypes.byref(m))
        return self._read(m.value, device_keys)

    def _read(self, m, device_keys=False):
        # page-locked result columns: the read-back is one fast DMA per column; keys that are
        # decoded on the device next (combined multi-key groupby keys) stay in HBM
        keys = DeviceArray.empty(m, np.int64) if device_keys else _lib.pinned_empty(m, np.int64)
        counts = _lib.pinned_empty(m, np.int64)
        sums = [_lib.pinned_empty(m, np.float64 if d.kind == "f" else (np.int64 if d.kind == "i" else np.uint64))
                for d in self.value_dtypes]
        nonnull = [_lib.pinned_empty(m, np.int64) if want else None for want in self.nonnull]
        nv = max(1, len(self.value_dtypes))
        sp = (ctypes.c_void_p * nv)(*[s.ctypes.data for s in sums])
        npp = (ctypes.c_void_p * nv)(*[c.ctypes.data if c is not None else None for c in nonnull])
        if m:
            kptr = keys.ptr if device_keys else keys.ctypes.data
            _lib.call("vh_hashagg_read", self._h, kptr, counts.ctypes.data, sp, npp)
        if self.key_dtype == np.uint64 and not device_keys:
            keys = keys.view(np.uint64)  # the library returns the key bits
        return keys, counts, sums, nonnull


def eligible_key(df, by, allow_filtered=False):
    """The key column name when ``by`` is one plain, unmasked, native integer column on an
    unfiltered frame (the fused path's key), else None.  allow_filtered: filtered frames too
    (the dense-grid route, whose aggregators take the filter as their keep mask)."""
    if isinstance(by, (list, tuple)):
        if len(by) != 1:
            return None
        by = by[0]
    if not isinstance(by, str) and type(by).__name__ != "Expression":
        return None
    by = str(by)
    if (df.filtered and not allow_filtered) or by not in df.columns or df.is_category(by):
        return None
    key = df.columns[by]
    if np.ma.isMaskedArray(key) or np.dtype(key.dtype).name not in KEY_DTYPES:
        return None
    if isinstance(key, np.ndarray) and (key.ndim != 1 or not key.dtype.isnative):
        return None
    return by


def _plan(df, by, actions, parse):
    """(key column, [(out name, op, value index)], value columns) or None if not eligible."""
    from . import agg as vagg
    by = eligible_key(df, by)
    if by is None:
        return None
    items = parse(actions, [by])
    if items is None:
        return None
    value_names, ops = [], []
    for name, a in items:
        if getattr(a, "selection", None) not in (None, False):
            return None
        if isinstance(a, vagg.AggregatorDescriptorBasic) and a.name == "AggCount" and a.expression == "*":
            ops.append((name, "count", None))
            continue
        short = getattr(a, "short_name", None)
        if not ((isinstance(a, vagg.AggregatorDescriptorBasic) and a.name in ("AggCount", "AggSum"))
                or isinstance(a, vagg.AggregatorDescriptorMean)):
            return None
        col = str(a.expression)
        if col not in df.columns or col == by:
            return None
        c = df.columns[col]
        dt = np.dtype(c.dtype)
        if np.ma.isMaskedArray(c) or dt.kind not in VALUE_KINDS or not dt.isnative:
            return None
        if isinstance(c, np.ndarray) and c.ndim != 1:
            return None
        if col not in value_names:
            value_names.append(col)
        ops.append((name, {"count": "nonnull", "sum": "sum", "mean": "mean"}[short], value_names.index(col)))
    if len(value_names) > 2 or not ops:
        return None
    return by, ops, value_names


def try_groupby(df, by, actions, parse, sort=False, row_limit=None, first_order=False):
    """The fused path of ``DataFrame.groupby(by, agg=actions)``; ``None`` = not taken.  Groups
    come out sorted by key, or with ``first_order`` in the order their keys first appear (the
    ordered_set order of ``assume_sparse=True``; single process only)."""
    from .dataframe import DataFrame, RowLimitException
    plan = _plan(df, by, actions, parse)
    if plan is None:
        return None
    by, ops, value_names = plan
    key = df.columns[by]
    distributed = getattr(df.executor, "world", 1) > 1
    if first_order and distributed:
        return None  # first appearance across row shards: the ordered_set route
    values = [df.columns[v] for v in value_names]
    nonnull = [any(op in ("nonnull", "mean") and vi == i for _, op, vi in ops) for i in range(len(values))]
    ha = HashAgg(key.dtype, [v.dtype for v in values], nonnull)
    # the executor's row range (a distributed executor: this rank's shard) in its chunks
    executor = df.executor
    start, end = executor.row_range(df)
    chunk = max(1, executor.chunk_size_for(df))
    ok = True
    try:
        for i1 in range(start, end, chunk):
            i2 = min(end, i1 + chunk)
            ha.update(key[i1:i2], [v[i1:i2] for v in values])
    except HashAggOverflow:
        ok = False
    if distributed:  # every rank takes the same route, or the collectives below would hang
        from .distributed import all_ranks_true
        ok = all_ranks_true(ok, executor.comm)
    if not ok:
        return None
    # the library's internal combined keys (groupby.py COMBINED_KEY / RECOMBINED_KEY) are
    # decoded on the device right after: keep them in HBM (single GPU, int64 keys)
    device_keys = by.startswith("__vaex_amd_") and np.dtype(key.dtype) == np.int64 and not distributed
    if distributed and executor.comm.device:  # RCCL: hash-partition exchange on the device
        keys, counts, sums, nonnull = ha.finish(executor.comm, gather=True)
    else:
        keys, counts, sums, nonnull = ha.finish(device_keys=device_keys,
                                                first_order_keys=key[start:end] if first_order else None)
        if distributed:  # CPU exchange: the same partition, merged on the host
            from .distributed import combine_groups
            keys, counts, sums, nonnull = combine_groups((keys, counts, sums, nonnull), executor.comm)
    if row_limit is not None and len(keys) > row_limit:
        raise RowLimitException(f"Resulting grouper has {len(keys):,} unique combinations, which is larger "
                                f"than the allowed row limit of {row_limit:,}")
    kdt = np.dtype(key.dtype)
    if device_keys:
        labels = keys
    else:
        labels = hostops.astype(keys, kdt)
        if len(labels):  # groupby.py:131-133
            lo, hi = hostops.minmax(labels) if first_order else (labels[0], labels[-1])
            labels = hostops.astype(labels, label_dtype(kdt, lo, hi))
    columns = {by: labels}
    for name, op, vi in ops:
        if op == "count":
            columns[name] = counts
        elif op == "nonnull":
            columns[name] = nonnull[vi]
        elif op == "sum":
            columns[name] = sums[vi]
        else:
            columns[name] = hostops.true_divide(sums[vi], nonnull[vi])
    return DataFrame(columns)
