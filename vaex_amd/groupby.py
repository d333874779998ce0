"""groupby / binby on the GPU path (``packages/vaex-core/vaex/groupby.py``).

``Grouper`` (groupby.py:97-168): pass 1 builds the GPU ordered set of the key
(``df._set``), its ``key_array`` becomes the group labels (ints down-cast with
``required_dtype_for_max``), ``sort=True`` rebuilds a sorted set (``ordered_set.create``);
pass 2 bins ``_ordinal_values(key, set)`` with a ``BinnerOrdinal`` -- which the task part
turns into the fused set-ordinal binner (hash probe inside the bin kernel, no ordinal
column materialised).  ``GrouperCategory`` (groupby.py:216-245) bins categorical columns
directly.  ``GroupBy.agg`` (groupby.py:484-533) strips the edges; with >1 key the
cartesian grid is filtered by count > 0.
"""
import copy

import numpy as np

from . import agg as vagg
from . import hostops
from .dataframe import DataFrame, Expression, RowLimitException
from .utils import extract_central_part, label_dtype


class BinnerBase:
    pass


class Grouper(BinnerBase):
    def __init__(self, expression, df=None, sort=False, pre_sort=True, row_limit=None, df_original=None):
        self.df = df if df is not None else expression.df
        df_original = df_original if df_original is not None else self.df
        self.sort = sort
        self.expression = str(expression)
        self.label = self.expression
        oset = df_original._set(self.expression, unique_limit=row_limit)
        self.bin_values = oset.key_array()
        if self.bin_values.dtype.kind == "i" and len(self.bin_values):  # groupby.py:133-135
            self.bin_values = self.bin_values.astype(
                label_dtype(self.bin_values.dtype, self.bin_values.min(), self.bin_values.max()))
        self.has_null = oset.has_null
        self.null_value = oset.null_value
        self.sort_indices = None
        if sort:
            values = self.bin_values
            nulls = np.zeros(len(values), bool)
            if oset.has_null:
                nulls[oset.null_value] = True
            # arrow-style sort: nulls last, NaN after numbers (groupby.py:137-156), as a
            # stable radix argsort on the GPU; the null slot is moved to the end
            order = _device_argsort(values)
            if oset.has_null:
                order = np.concatenate([order[order != oset.null_value], [oset.null_value]]).astype(np.int64)
            sorted_values = values[order]
            null_value = int(np.nonzero(nulls[order])[0][0]) if oset.has_null else -1
            oset = type(oset)(sorted_values.astype(oset._dtype), null_value, oset.nan_count, oset.null_count,
                              oset.fingerprint + "-sorted")
            self.bin_values = sorted_values
            self.null_value = null_value
        self.set = oset
        basename = "set_%s" % "".join(c if c.isalnum() else "_" for c in self.expression)
        self.setname = self.df.add_variable(basename, self.set, unique=True)
        self.binby_expression = "_ordinal_values(%s, %s)" % (self.expression, self.setname)
        self.N = len(self.bin_values)
        self.binner = self.df._binner_ordinal(self.binby_expression, self.N)

    def labels(self):
        vals = self.bin_values.tolist()
        if self.has_null:
            vals[self.null_value] = None
        return vals


def _device_argsort(values):
    """Stable ascending order of a key array (NaN last), computed on the GPU (vh_argsort)."""
    from . import _lib
    from .device import DeviceArray
    values = np.ascontiguousarray(values)
    if not len(values):
        return np.empty(0, np.int64)
    keys = DeviceArray.from_numpy(values)
    out = DeviceArray(len(values), np.int64)
    _lib.call("vh_argsort", len(values), keys.ptr, _lib.dtype_code(values.dtype)[0], out.ptr)
    return out.to_numpy()


# integer keys whose value range is at most this many cells are binned densely
DENSE_KEY_MAX = 1 << 24


class GrouperDense(BinnerBase):
    """Integer keys spanning a small value range: ``BinnerOrdinal(key, N = max - min + 1,
    min_value = min)``, exactly how the reference bins categoricals (GrouperCategory,
    groupby.py:216-245), after one GPU min/max pass.  This replaces the set-build pass and
    the per-row hash probe of ``_ordinal_values`` (Grouper) for dense keys; groups that do not
    occur are dropped with the count(*) grid.  Groups come out sorted by key, which is also
    the ``sort=True`` order."""

    dense = True

    def __init__(self, expression, vmin, vmax, df=None, row_limit=None, speculative=False):
        self.df = df if df is not None else expression.df
        self.expression = str(expression)
        self.label = self.expression
        self.min_value = int(vmin)
        self.N = int(vmax) - int(vmin) + 1
        self.speculative = speculative  # [vmin, vmax] guessed from a sample (_dense_range)
        dtype = self.df.data_type(self.expression)
        self.value_dtype = label_dtype(dtype, vmin, vmax)
        self._bin_values = None
        self.sort_indices = None
        self.binner = self.df._binner_ordinal(self.expression, self.N, self.min_value)
        self.key_dtype = dtype

    @property
    def bin_values(self):
        """min_value .. max (built on demand: a single-key groupby only needs the occupied ones)."""
        if self._bin_values is None:
            self._bin_values = _label_range(self.min_value, self.N, self.value_dtype)
        return self._bin_values

    def labels(self):
        return self.bin_values.tolist()


def _label_range(vmin, n, dtype, threads=True):
    """min .. min + n - 1 as `dtype` (label_dtype chose it to hold them), built in that dtype
    directly (no int64 array and cast for a 1e6-group result)."""
    dtype = np.dtype(dtype)
    if dtype.kind in "iu":
        return hostops.arange(vmin, n, dtype, threads=threads)
    return np.arange(vmin, vmin + n, dtype=np.int64).astype(dtype)


# a dense key range is guessed from this many evenly spaced rows (vh_minmax_sample) when the
# column has at least SPECULATE_MIN_ROWS rows in HBM; the guess is widened by 1/32 of its span
# (uniform keys: the sample's extremes lie ~span / 65536 inside the true ones)
SPECULATE_MIN_ROWS = 1 << 22
SPECULATE_SAMPLE = 1 << 16


class DenseRangeMiss(Exception):
    """A speculative dense range missed keys (the grid's under/overflow cells are not empty)."""


def _sampled_range(col, n, dtype):
    """(lo, hi) widened from the min / max of SPECULATE_SAMPLE evenly spaced rows, or None."""
    import ctypes

    from . import _lib
    from .device import DeviceArray
    if not isinstance(col, DeviceArray) or n < SPECULATE_MIN_ROWS or not dtype.isnative:
        return None
    lo, hi = ctypes.c_double(), ctypes.c_double()
    code, _ = _lib.dtype_code(dtype)
    _lib.call("vh_minmax_sample", col.ptr, n, code, SPECULATE_SAMPLE, ctypes.byref(lo), ctypes.byref(hi))
    if not (np.isfinite(lo.value) and np.isfinite(hi.value)):
        return None
    lo, hi = int(lo.value), int(hi.value)
    info = np.iinfo(dtype)
    room = int(info.max) - (hi - lo + 1)  # the binner's ordinal_count is a T: it must hold the span
    if room < 0:
        return None
    margin = min(max(64, (hi - lo) // 32), room // 2)
    return max(lo - margin, int(info.min)), min(hi + margin, int(info.max))


def _dense_range(df, expression, speculative=False):
    """(min, max) when an integer, unmasked key spans <= DENSE_KEY_MAX values, else None.
    speculative: a range guessed from a row sample (no full min/max pass), as a third item
    True; GroupBy.agg raises DenseRangeMiss when rows fall outside it."""
    expression = str(expression)
    col = df.columns.get(expression)
    if col is None or np.ma.isMaskedArray(col):
        return None
    dtype = np.dtype(col.dtype)
    if dtype.kind not in "iu":
        return None
    # a filtered frame: the sampled range is the unfiltered column's (a superset; the empty
    # cells of the filtered counts are dropped), the exact range the filtered min / max
    n = df.length_unfiltered()
    if n == 0:
        return None
    if speculative and (rng := _sampled_range(col, n, dtype)) is not None:
        span = rng[1] - rng[0] + 1
        if span <= DENSE_KEY_MAX and span <= 4 * n + 1024 and abs(rng[0]) < 2 ** 53 and abs(rng[1]) < 2 ** 53:
            return rng[0], rng[1], True
    vmin, vmax = df.minmax(expression)
    if not (np.isfinite(vmin) and np.isfinite(vmax)):  # no rows (an empty filter)
        return None
    if not (abs(int(vmin)) < 2 ** 53 and abs(int(vmax)) < 2 ** 53):
        return None
    span = int(vmax) - int(vmin) + 1
    # BinnerOrdinal_<T> takes ordinal_count as a T (superagg_binners.cpp:99): e.g. int8 keys
    # spanning more than 127 values take the hash route
    if span > DENSE_KEY_MAX or span > 4 * n + 1024 or span > int(np.iinfo(dtype).max):
        return None
    return int(vmin), int(vmax)


def first_appearance_order(df, key, res):
    """The key-sorted groups of a dense-range groupby result ``res`` reordered by the row each
    key first appears at in ``df[key]`` -- the ordinal order of an ordered_set built over the
    key column (hash_primitives.hpp:96-281), i.e. the Grouper route's group order
    (groupby.py:97-168) -- on the device (vh_dense_first_order: run-head prefix scan, radix
    sort of the first rows), the columns permuted by host threads."""
    import ctypes
    from . import _lib
    from .device import DeviceArray
    labels = np.asarray(res.columns[key])
    m = len(labels)
    if m < 2:
        return res
    col = df.columns[key]
    lab64 = hostops.astype(labels, np.int64)
    perm = _lib.pinned_empty(m, np.int64)
    if isinstance(col, DeviceArray):
        ptr, loc = col.ptr, _lib.LOC_DEVICE
    else:
        col = np.ascontiguousarray(col)
        ptr, loc = col.ctypes.data, _lib.LOC_HOST
    code, _ = _lib.dtype_code(np.dtype(col.dtype))
    vmin = int(lab64[0])
    span = int(lab64[-1]) - vmin + 1
    _lib.call("vh_dense_first_order", ptr, df.length_unfiltered(), loc, code, ctypes.c_int64(vmin), span,
              lab64.ctypes.data, m, perm.ctypes.data)
    names = list(res.columns)
    return DataFrame(dict(zip(names, hostops.take_columns([res.columns[k] for k in names], perm))))


COMBINE_OCCUPANCY = 10  # groupby.py:329-333: combine when rows / cells < 10
COMBINED_KEY = "__vaex_amd_combined_key"


def _key_ranges(df, by):
    """[(name, min, max)] when every key of a multi-key groupby is a plain unmasked native
    integer column of an unfiltered frame with exact (< 2**53) limits, else None."""
    if df.filtered or len(by) < 2:
        return None
    names = []
    for b in by:
        if not isinstance(b, str) and not isinstance(b, Expression):
            return None
        name = str(b)
        col = df.columns.get(name)
        if col is None or df.is_category(name) or np.ma.isMaskedArray(col) or name in names:
            return None
        dt = np.dtype(col.dtype)
        if dt.kind not in "iu" or not dt.isnative or (isinstance(col, np.ndarray) and col.ndim != 1):
            return None
        names.append(name)
    if df.length_unfiltered() == 0:
        return None
    # one min / max pass per distinct column: keys that alias one column (the h2o benchmark's
    # id1 / id2 / id4 / id5 are all df['i1_100'], groupbyh2o.py:26-36) share it
    by_col = {}
    for name in names:
        by_col.setdefault(id(df.columns[name]), name)
    promises = {k: df.minmax(name, delay=True) for k, name in by_col.items()}
    df.execute()
    out = []
    for name in names:
        vmin, vmax = (int(x) for x in promises[id(df.columns[name])].get())
        if not (abs(vmin) < 2 ** 53 and abs(vmax) < 2 ** 53):
            return None
        out.append((name, vmin, vmax))
    return out


def groupby_multikey(df, by, agg, sort=False, row_limit=None, combine="auto"):
    """Multi-key ``groupby(by=[k1, k2, ...], agg=...)`` (groupby.py:248-333).

    ``combine`` is the reference's ``assume_sparse`` (dataframe.py:6679 passes it as
    ``GroupBy(combine=...)``, groupby.py:313-333): ``True`` always combines the keys into
    one grouper, ``'auto'`` combines when rows / cells < 10, ``False`` never does (the
    caller bins the cartesian grid; this returns None).

    Integer keys: with enough rows per cell (``'auto'``) every key becomes a dense grouper
    and the cartesian grid is binned directly.  Otherwise the keys are combined on the GPU
    into one int64 key, the cartesian ordinal ``sum_j (k_j - min_j) * prod(span_{j+1..})``
    (``vh_combine_keys``, first key most significant), which takes the single-key routes
    (dense grid, fused hash pass, or the set grouper for other aggregators); the labels are
    decoded back per key.  The reference combines the per-key set ordinals instead of value
    offsets; both give the lexicographic order of ``sort=True``.  Keys that are not plain
    integer columns (floats, masked, filtered frames) are combined through their GPU set
    ordinals exactly as the reference does (:func:`_groupby_combine_sets`).

    Group order without ``sort``: whenever the keys are combined (``True``, or ``'auto'``
    below the occupancy) the combined grouper's set order, i.e. the order in which each key
    combination first appears (GrouperCombined over an ordered_set, what the reference
    produces with one thread), as the single-key ``assume_sparse=True`` route does; the
    dense cartesian route of ``'auto'`` (enough rows per cell) is sorted per key.

    Returns None when the query is not taken here (``combine=False``, or ``'auto'`` with
    keys that do not qualify): the caller takes the grouper-built cartesian GroupBy."""
    if combine is False:
        return None
    ranges = _key_ranges(df, by)
    if ranges is None:
        return _groupby_combine_sets(df, by, agg, sort=sort, row_limit=row_limit, combine=combine)
    spans = [vmax - vmin + 1 for _, vmin, vmax in ranges]
    cells = 1
    for sp in spans:
        cells *= sp
    names = [name for name, _, _ in ranges]
    # combined keys (True, or 'auto' below the occupancy): the combined grouper's set order
    # without sort, as GrouperCombined over an ordered_set gives (groupby.py:313-333)
    first_order = not sort
    if cells >= 2 ** 62:
        return _groupby_recombine(df, ranges, agg, sort=sort, row_limit=row_limit, combine=combine)
    n = df.length_unfiltered()
    if combine == "auto" and n / cells >= COMBINE_OCCUPANCY and all(sp <= DENSE_KEY_MAX for sp in spans):
        dense_ranges = {name: (vmin, vmax) for name, vmin, vmax in ranges}
        return GroupBy(df, by=names, sort=sort, row_limit=row_limit, dense_ranges=dense_ranges).agg(agg)
    return _groupby_combined(df, ranges, agg, names, sort=sort, row_limit=row_limit, first_order=first_order)


def _groupby_combined(df, ranges, agg, key_names, sort=False, row_limit=None, first_order=False):
    """Combine the integer key columns of ``ranges`` [(name, min, max)] into one int64 key
    and group by it: the single-key routes, in first-appearance order with ``first_order``
    (the ``assume_sparse=True`` single-key route), else sorted by combined key =
    lexicographic.  Returns {key name: labels (decoded per key), aggregate columns...}."""
    combined, mults = _combine_columns(df, ranges)
    # the aggregators are named against the original frame (callables expand over its
    # non-key columns), then evaluated on a copy that also holds the combined key
    actions = [(name, a) for name, a in parse_actions(df, agg, key_names)]
    tmp = df.copy()
    tmp.add_column(COMBINED_KEY, combined)
    res = tmp.groupby(COMBINED_KEY, agg=actions, sort=sort, row_limit=row_limit,
                      assume_sparse=True if first_order else "auto")
    columns = _decode_labels(df, res.columns[COMBINED_KEY], None, ranges, mults)
    for name, values in res.columns.items():
        if name != COMBINED_KEY:
            columns[name] = values
    return DataFrame(columns)


ORDINAL_KEY = "__vaex_amd_ordinal_{}"


def _groupby_combine_sets(df, by, agg, sort=False, row_limit=None, combine=True):
    """``_combine`` over per-key set groupers (groupby.py:248-288, GroupByBase combine=True
    :313-315): each key gets its GPU ordered_set (Grouper, ``sort`` orders it), every row's
    ordinal into it (``map_ordinal`` on the device for HBM columns; masked rows take the
    set's null ordinal, NaN its NaN ordinal), and the ordinal columns are combined like
    integer keys of range [0, N - 1].  Labels are the sets' keys at the decoded ordinals.
    For keys the integer route does not take (floating point, masked, filtered frames).
    ``combine='auto'`` decides from the set sizes, as the reference does (rows / cells < 10
    combines; otherwise the cartesian grid of these groupers).  Returns None for categorical
    or binner keys (the caller's cartesian GroupBy)."""
    from .device import DeviceArray
    if any(isinstance(b, BinnerBase) or not isinstance(b, (str, Expression)) or df.is_category(b) for b in by):
        return None
    names = [str(b) for b in by]
    n = df.length_unfiltered()
    work = df.copy()
    groupers, ranges = [], []
    for name in names:
        groupers.append(Grouper(work[name], df=work, sort=sort, row_limit=row_limit, df_original=df))
    cells = 1
    for g in groupers:
        cells *= g.N
    if any(g.N == 0 for g in groupers) or (combine == "auto" and n / max(cells, 1) >= COMBINE_OCCUPANCY):
        return GroupBy(work, by=groupers, sort=sort, row_limit=row_limit).agg(agg)
    for i, (name, g) in enumerate(zip(names, groupers)):
        col = df._eval_host(name, 0, n)
        mask = np.ma.getmaskarray(col) if np.ma.isMaskedArray(col) else None
        if np.ma.isMaskedArray(col):
            col = col.data
        ords = g.set.map_ordinal(col if isinstance(col, DeviceArray) else np.ascontiguousarray(col))
        if mask is not None and mask.any():
            ords = np.array(ords, copy=True)
            ords[mask] = g.null_value
        key = ORDINAL_KEY.format(i)
        work.add_column(key, ords)
        ranges.append((key, 0, g.N - 1))
    actions = [(name, a) for name, a in parse_actions(df, agg, names)]
    if cells >= 2 ** 62:
        res = _groupby_recombine(work, ranges, actions, sort=sort, row_limit=row_limit, combine=True,
                                 key_names=names)
    else:
        res = _groupby_combined(work, ranges, actions, names, sort=sort, row_limit=row_limit, first_order=not sort)
    columns = {}
    for name, g, (key, _, _) in zip(names, groupers, ranges):
        ords = res.columns[key]
        ords = ords.to_numpy() if isinstance(ords, DeviceArray) else np.asarray(ords)
        ords = ords.astype(np.int64)
        vals = np.asarray(g.bin_values)[ords]
        if getattr(g, "has_null", False):  # the null group's label is masked (Grouper.labels: None)
            vals = np.ma.masked_array(vals, mask=ords == g.null_value)
        columns[name] = vals
    for name, values in res.columns.items():
        if not name.startswith("__vaex_amd_ordinal_"):
            columns[name] = values
    return DataFrame(columns)


def _combine_columns(df, ranges):
    """Cartesian ordinal of integer key columns on the GPU (``vh_combine_keys``): returns the
    int64 device column and the per-key multipliers (first key most significant)."""
    import ctypes
    from . import _lib
    from .device import DeviceArray
    spans = [vmax - vmin + 1 for _, vmin, vmax in ranges]
    mults = [1] * len(spans)
    for i in range(len(spans) - 2, -1, -1):
        mults[i] = mults[i + 1] * spans[i + 1]
    n = df.length_unfiltered()
    cols, keep = [], []
    for name, _, _ in ranges:
        c = df.columns[name]
        if not isinstance(c, DeviceArray):
            c = DeviceArray.from_numpy(np.ascontiguousarray(c))
            keep.append(c)
        cols.append(c)
    combined = DeviceArray.empty(n, np.int64)
    k = len(cols)
    _lib.call("vh_combine_keys", n, k, (ctypes.c_void_p * k)(*[c.ptr for c in cols]),
              (ctypes.c_int * k)(*[_lib.dtype_code(c.dtype)[0] for c in cols]),
              (ctypes.c_int64 * k)(*[vmin for _, vmin, _ in ranges]), (ctypes.c_int64 * k)(*mults), combined.ptr)
    del keep
    return combined, mults


def _decode_labels(df, ck, table, ranges, mults):
    """{key name: labels} of combined keys ``ck`` (host or HBM), decoded on the GPU
    (``vh_decode_keys``, optionally through the dense-rank ``table``), each key in its
    label dtype (groupby.py:131-133 down-casts)."""
    import ctypes
    from . import _lib
    from .device import DeviceArray
    ck = ck if isinstance(ck, DeviceArray) else DeviceArray.from_numpy(np.ascontiguousarray(ck, dtype=np.int64))
    n, k = len(ck), len(ranges)
    dtypes = []
    for name, vmin, vmax in ranges:
        kd = np.dtype(df.columns[name].dtype)
        if name.startswith("__vaex_amd_"):
            dtypes.append(np.dtype(np.int64))  # an internal key decoded again next: int64 in HBM
        else:
            dtypes.append(np.dtype(label_dtype(kd, vmin, vmax)) if n else kd)
    if ck.dtype != np.int64:
        raise TypeError("combined keys must be int64")
    outs = [DeviceArray.empty(n, dt) for dt in dtypes]
    if n:
        _lib.call("vh_decode_keys", n, ck.ptr, table.ptr if table is not None else None, k,
                  (ctypes.c_int64 * k)(*[vmin for _, vmin, _ in ranges]), (ctypes.c_int64 * k)(*mults),
                  (ctypes.c_int64 * k)(*[vmax - vmin + 1 for _, vmin, vmax in ranges]),
                  (ctypes.c_int * k)(*[dt.itemsize for dt in dtypes]), (ctypes.c_void_p * k)(*[o.ptr for o in outs]))
    # labels of the library's internal recombined keys stay in HBM: the next _decode_labels
    # (_groupby_recombine) reads them there
    return {name: (o if name.startswith("__vaex_amd_") else o.to_numpy(pinned=True)) if n else np.empty(0, dt)
            for (name, _, _), o, dt in zip(ranges, outs, dtypes)}


RECOMBINED_KEY = "__vaex_amd_recombined_key_{}"


def _groupby_recombine(df, ranges, agg, sort=False, row_limit=None, combine="auto", key_names=None):
    """Multi-key groupby whose cartesian span reaches 2**62: the reference's ``_combine``
    recursion (groupby.py:248-288).  The leading keys whose span product stays below 2**62
    are combined on the GPU into one int64 value, that value is replaced by its dense rank
    (``vh_dense_rank_i64``: radix sort, run heads, scan; the reference builds an ordered
    set of it instead, GrouperCombined + ``ordered_set::create`` hash_primitives.hpp:468-516;
    sorted ranks keep the lexicographic key order), and the rank column (span = number of
    distinct combinations) replaces those keys; the remaining keys are combined with it the same way
    (recursing while the spans still overflow).  Labels are decoded back per key."""
    import ctypes
    from . import _lib
    from .device import DeviceArray
    spans = [vmax - vmin + 1 for _, vmin, vmax in ranges]
    take, prod = 1, spans[0]
    while take < len(spans) and prod * spans[take] < 2 ** 62:
        prod *= spans[take]
        take += 1
    if take < 2:
        return None  # two keys alone overflow 62 bits: not combinable here
    head, rest = ranges[:take], ranges[take:]
    names = key_names or [name for name, _, _ in ranges]
    actions = [(name, a) for name, a in parse_actions(df, agg, names)]
    combined, mults = _combine_columns(df, head)
    n = len(combined)
    ordinal = DeviceArray.empty(n, np.int32)
    distinct_dev = DeviceArray.empty(max(n, 1), np.int64)
    m = ctypes.c_uint64()
    _lib.call("vh_dense_rank_i64", n, combined.ptr, ordinal.ptr, distinct_dev.ptr, ctypes.byref(m))
    del combined
    depth = 0
    while RECOMBINED_KEY.format(depth) in df.columns:
        depth += 1
    key = RECOMBINED_KEY.format(depth)
    tmp = df.copy()
    tmp.add_column(key, ordinal)
    by = [key] + [name for name, _, _ in rest]
    res = tmp.groupby(by, agg=actions, sort=sort, row_limit=row_limit, assume_sparse=combine)
    columns = _decode_labels(df, res.columns[key], distinct_dev, head, mults)
    del distinct_dev
    for name, values in res.columns.items():
        if name != key:
            columns[name] = values
    return DataFrame(columns)


class GrouperCategory(BinnerBase):
    """groupby.py:216-245: categorical column -> BinnerOrdinal(min_value, N)."""

    def __init__(self, expression, df=None, sort=False, row_limit=None):
        self.df = df if df is not None else expression.df
        self.expression = str(expression)
        self.label = self.expression
        cat = self.df._categories[self.expression]
        self.bin_values = np.asarray(cat["labels"], dtype=object)
        self.N = cat["N"]
        self.min_value = cat["min_value"]
        self.sort_indices = None
        self.binner = self.df._binner_ordinal(self.expression, self.N, self.min_value)
        if row_limit is not None and self.N > row_limit:
            raise RowLimitException(f"Resulting grouper has {self.N:,} unique combinations, which is larger "
                                    f"than the allowed row limit of {row_limit:,}")

    def labels(self):
        return list(self.bin_values)


class GroupByBase:
    def __init__(self, df, by, sort=False, row_limit=None, dense=True, dense_ranges=None, first_order=False):
        df_original = df
        df = df.copy()
        self.df = df
        self.sort = sort
        # groups in the order their keys first appear (the ordered_set grouper's order without
        # sort): a dense single key finishes on the device (vh_dense_first_take)
        self.first_order = first_order
        self.key_df = df_original
        self.row_limit = row_limit
        if not isinstance(by, (list, tuple)):
            by = [by]
        self.by = []
        for by_value in by:
            if isinstance(by_value, BinnerBase):
                self.by.append(by_value)
            elif df.is_category(by_value):
                self.by.append(GrouperCategory(df[str(by_value)], df=df, sort=sort, row_limit=row_limit))
            elif dense and (rng := (dense_ranges or {}).get(str(by_value)) or _dense_range(df, by_value)) is not None:
                self.by.append(GrouperDense(df[str(by_value)], rng[0], rng[1], df=df, row_limit=row_limit,
                                            speculative=len(rng) > 2 and rng[2]))
            else:
                self.by.append(Grouper(df[str(by_value)], df=df, sort=sort, row_limit=row_limit,
                                       df_original=df_original))
        self.groupby_expression = [str(b.expression) for b in self.by]
        self.binners = tuple(b.binner for b in self.by)
        self.shape = [b.N for b in self.by]
        self.dims = self.groupby_expression[:]

    def _agg(self, actions):
        """groupby.py:345-402: every aggregate gets edges=True on the grouper binners."""
        df = self.df
        grids = {}
        self.counts = None
        self.count_desc = None
        dense1 = len(self.by) == 1 and isinstance(self.by[0], GrouperDense)
        parsed = parse_actions(df, actions, self.groupby_expression)
        # first-appearance order on the device: every aggregate a plain superagg grid (count /
        # sum / min / max of a native column, no selection), so its HBM grid is gathered in
        # that order and read back once (instead of the whole grid plus a host gather)
        key_col = self.key_df.columns.get(str(self.by[0].expression)) if dense1 else None
        self.device_finish = self.first_order and dense1 and key_col is not None and \
            not np.ma.isMaskedArray(key_col) and np.dtype(key_col.dtype).kind in "iu" and all(
            type(a) is vagg.AggregatorDescriptorBasic and a.name in ("AggCount", "AggSum", "AggMin", "AggMax")
            and a.selection in (None, False) for _, a in parsed)
        self.descs = {}
        for column_name, aggregate in parsed:
            # per-query flags go on a copy: a user's descriptor object may be reused by later
            # or concurrent queries (occupancy / keep_device are this query's state)
            aggregate = copy.copy(aggregate)
            self.descs[column_name] = aggregate
            aggregate.edges = True
            aggregate.keep_device = self.device_finish
            is_count = isinstance(aggregate, vagg.AggregatorDescriptorBasic) and aggregate.name == "AggCount" \
                and aggregate.expression == "*" and aggregate.selection in (None, False)
            if is_count and dense1 and self.counts is None:
                aggregate.want_occupancy = True  # the occupied range, found on the device
                self.count_desc = aggregate
            values = df._agg(aggregate, self.binners, delay=True)
            grids[column_name] = values
            if is_count:
                self.counts = values
        return grids


def parse_actions(df, actions, groupby_expression):
    """The agg= argument as [(output column name, aggregator descriptor)] (groupby.py:345-402)."""
    if isinstance(actions, dict):
        actions = list(actions.items())
    elif not isinstance(actions, (list, tuple)) or isinstance(actions, str):
        actions = [actions]
    out = []

    def add(aggregate, column_name=None, override_name=None):
        if column_name is None or override_name is not None:
            column_name = aggregate.pretty_name(override_name, df)
        out.append((column_name, aggregate))

    for item in actions:
        override_name = None
        if isinstance(item, tuple):
            name, aggregates = item
        else:
            aggregates, name = item, None
        if not isinstance(aggregates, (list, tuple)) or isinstance(aggregates, str):
            aggregates = [aggregates]
        elif name is not None:
            override_name = name
        for aggregate in aggregates:
            if isinstance(aggregate, str) and aggregate == "count":
                add(vagg.count(), "count" if name is None else name)
            else:
                if isinstance(aggregate, str):
                    aggregate = vagg.aggregates[aggregate]
                if callable(aggregate):
                    if name is None:
                        for column_name in df.get_column_names():
                            if column_name not in groupby_expression:
                                add(aggregate(column_name), override_name=override_name)
                    else:
                        add(aggregate(name), name, override_name=override_name)
                else:
                    add(aggregate, name, override_name=override_name)
    return out


class GroupBy(GroupByBase):
    def agg(self, actions):
        """groupby.py:484-533."""
        arrays = self._agg(actions)
        has_non_existing_pairs = len(self.by) > 1 or any(getattr(b, "dense", False) for b in self.by)
        counts = self.counts
        if has_non_existing_pairs and counts is None:
            desc = vagg.count(edges=True)
            if len(self.by) == 1 and isinstance(self.by[0], GrouperDense):
                desc.want_occupancy = True
                # an internal count(*): only its occupancy is needed when every cell of the
                # occupied range holds a group, so its grid stays in HBM (read back only for
                # the compaction mask)
                desc.keep_device = True
                self.count_desc = desc
            counts = self.df._agg(desc, self.binners, delay=True)
        if len(self.by) == 1 and isinstance(self.by[0], GrouperDense):
            return self._agg_dense(arrays, counts)
        self.df.execute()
        arrays = {k: extract_central_part(np.asarray(v.get())) for k, v in arrays.items()}
        columns = {}
        if has_non_existing_pairs:
            counts_edges = np.asarray(counts.get())
            counts = extract_central_part(counts_edges)
            mask = counts > 0
            if self.row_limit is not None and any(getattr(b, "dense", False) for b in self.by):
                groups = int(np.count_nonzero(mask))
                if groups > self.row_limit:  # what the set build of Grouper raises (groupby.py:125)
                    raise RowLimitException(f"Resulting grouper has {groups:,} unique combinations, which is "
                                            f"larger than the allowed row limit of {self.row_limit:,}")
            every = bool(mask.all())  # every cell occupied: no compaction
            coords = [c[mask] for c in np.meshgrid(*[np.asarray(b.bin_values) for b in self.by], indexing="ij")]
            for b, coord in zip(self.by, coords):
                columns[b.label] = coord
            for k, v in arrays.items():
                columns[k] = v if every and v.ndim == 1 else v[mask]
        else:
            columns[self.by[0].label] = np.asarray(self.by[0].bin_values)
            for k, v in arrays.items():
                assert v.ndim == 1
                columns[k] = v
        return DataFrame(columns)


    def _agg_dense(self, arrays, counts):
        """One dense integer key (GrouperDense): the occupied range of the count(*) grid is
        found by host threads (count_nonzero per chunk, no mask array when every cell of it is
        occupied), and the label range is built on the host pool while the GPU bins (labels
        sliced to the occupied cells afterwards) -- groupby.py:484-533's result: groups in key
        order, empty cells dropped."""
        g = self.by[0]
        dtype0 = np.dtype(g.value_dtype)
        # a range of up to 4 Mi labels is built while the GPU bins (larger ones only for the
        # occupied cells, afterwards)
        labels = hostops.submit(_label_range, g.min_value, g.N, dtype0, False) if g.N <= (1 << 22) else None
        try:
            self.df.execute()
        finally:
            labels = labels.result() if labels is not None else None
        if self.device_finish:
            from .taskparts import DeviceResult
            if isinstance(counts.get(), DeviceResult) and all(isinstance(v.get(), DeviceResult) for v in arrays.values()):
                return self._agg_dense_device(arrays, counts)
            # a part handed a host result back (keep_device not honoured): key order on the
            # host, and the caller applies the first-appearance order itself
            self.device_finish = False
        from .taskparts import DeviceResult
        arrays = {k: extract_central_part(np.asarray(v.get())) for k, v in arrays.items()}
        cres = counts.get()
        occ = getattr(self.count_desc, "occupancy", None)
        if isinstance(cres, DeviceResult) and occ is not None:
            # the internal count(*) grid is still in HBM: the edge cells and the occupied range
            # come from the device, the grid itself only when the range has empty cells
            cagg, central = cres.agg, None
            L = cagg.grid.length1d
            nnz, first, last = occ
            if g.speculative and (cagg.occupancy(1, 2)[0] or cagg.occupancy(L - 1, L)[0] or nnz == 0):
                raise DenseRangeMiss(g.expression)
        else:
            counts_edges = np.asarray(cres)
            central = extract_central_part(counts_edges)
            nnz, first, last = occ if occ is not None else hostops.occupancy(central)
            # keys outside the guessed range sit in the under / overflow cells
            if g.speculative and (counts_edges[1] or counts_edges[-1] or nnz == 0):
                raise DenseRangeMiss(g.expression)
        if g.speculative:
            g.value_dtype = label_dtype(g.key_dtype, g.min_value + first, g.min_value + last)
        if self.row_limit is not None and nnz > self.row_limit:  # what Grouper's set build raises (groupby.py:125)
            raise RowLimitException(f"Resulting grouper has {nnz:,} unique combinations, which is "
                                    f"larger than the allowed row limit of {self.row_limit:,}")
        if nnz == 0:
            first, last = 0, -1
        sl = slice(first, last + 1)
        every = nnz == last - first + 1  # the occupied range has no empty cell: no compaction
        if every:
            lab = labels[sl] if labels is not None and np.dtype(g.value_dtype) == dtype0 else \
                _label_range(g.min_value + first, nnz, g.value_dtype)
            columns = {g.label: lab}
            for k, v in arrays.items():
                columns[k] = v[sl]
            return DataFrame(columns)
        if central is None:
            central = extract_central_part(np.asarray(cres))
        mask = central[sl] > 0
        columns = {g.label: (np.flatnonzero(mask) + (g.min_value + first)).astype(g.value_dtype)}
        for k, v in arrays.items():
            columns[k] = v[sl][mask]
        return DataFrame(columns)


    def _agg_dense_device(self, arrays, counts):
        """_agg_dense for the first-appearance order with the grids still in HBM: the occupied
        range from the device occupancy of the count(*) grid, then vh_dense_first_take gathers
        every grid's occupied cells in the order their keys first appear in the key column and
        reads them back (the result of Grouper(sort=False)'s ordered_set order, groupby.py:
        97-168, 484-533)."""
        import ctypes
        from . import _lib
        from .device import DeviceArray
        g = self.by[0]
        aggs = {k: v.get().agg for k, v in arrays.items()}
        cagg = counts.get().agg
        L = cagg.grid.length1d
        nnz, first, last = self.count_desc.occupancy
        if g.speculative:
            # keys outside the guessed range sit in the under / overflow cells
            if cagg.occupancy(1, 2)[0] or cagg.occupancy(L - 1, L)[0] or nnz == 0:
                raise DenseRangeMiss(g.expression)
            g.value_dtype = label_dtype(g.key_dtype, g.min_value + first, g.min_value + last)
        if self.row_limit is not None and nnz > self.row_limit:
            raise RowLimitException(f"Resulting grouper has {nnz:,} unique combinations, which is "
                                    f"larger than the allowed row limit of {self.row_limit:,}")
        label_dt = np.dtype(g.value_dtype)
        if nnz == 0:
            columns = {g.label: np.empty(0, label_dt)}
            for k, a in aggs.items():
                columns[k] = np.empty(0, self.descs[k].dtype_out if k in self.descs else a._grid_dtype)
            return DataFrame(columns)
        names = list(aggs)
        outs = [_lib.pinned_empty(nnz, aggs[k]._grid_dtype) for k in names]
        lab = _lib.pinned_empty(nnz, label_dt)
        off = 2 + first  # central part starts at cell 2 (extract_central_part)
        srcs = [aggs[k].device_grid_ptr() + off * aggs[k]._grid_dtype.itemsize for k in names]
        cisz = cagg._grid_dtype.itemsize
        key = self.key_df.columns[g.expression]
        if isinstance(key, DeviceArray):
            kptr, kloc = key.ptr, _lib.LOC_DEVICE
        else:
            key = np.ascontiguousarray(key)
            kptr, kloc = key.ctypes.data, _lib.LOC_HOST
        k = len(names)
        _lib.call("vh_dense_first_take", kptr, self.key_df.length_unfiltered(), kloc, _lib.dtype_code(np.dtype(key.dtype))[0],
                  ctypes.c_int64(g.min_value + first), last - first + 1, cagg.device_grid_ptr() + off * cisz, cisz, nnz, k,
                  (ctypes.c_void_p * max(k, 1))(*srcs), (ctypes.c_int * max(k, 1))(*[aggs[n]._grid_dtype.itemsize for n in names]),
                  (ctypes.c_void_p * max(k, 1))(*[o.ctypes.data for o in outs]), label_dt.itemsize, lab.ctypes.data)
        columns = {g.label: lab}
        for name, o in zip(names, outs):
            # the grid's dtype is the binned one (datetime64 / timedelta64 bin as 64-bit
            # integers): the result column takes the descriptor's output dtype, as
            # TaskPartAggregation.get_result does (cpu.py:592-605)
            dtype_out = np.dtype(self.descs[name].dtype_out) if name in self.descs else o.dtype
            if dtype_out != o.dtype and dtype_out.itemsize == o.dtype.itemsize:
                o = o.view(dtype_out.newbyteorder("=") if dtype_out.byteorder not in "<=|" else dtype_out)
            columns[name] = o
        return DataFrame(columns)


class GroupByDeferred:
    """``df.groupby(by)`` without aggregators (dataframe.py:6622-6683 returns a GroupBy whose
    groupers are built up front).  Here ``.agg(actions)`` is ``df.groupby(by, agg=actions)``,
    so it takes the same GPU routes (multi-key combine, dense grid, fused hash pass); any
    other attribute builds the grouper-based :class:`GroupBy` on first use."""

    def __init__(self, df, by, sort=False, assume_sparse="auto", row_limit=None):
        self._df, self._by = df, by
        self._kw = dict(sort=sort, assume_sparse=assume_sparse, row_limit=row_limit)
        self._real = None

    def agg(self, actions):
        return self._df.groupby(self._by, agg=actions, **self._kw)

    def _groupby(self):
        if self._real is None:
            kw = self._kw
            self._real = GroupBy(self._df, by=self._by, sort=kw["sort"], row_limit=kw["row_limit"],
                                 dense=kw["assume_sparse"] != True)  # noqa: E712
        return self._real

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._groupby(), name)


class _Coord:
    def __init__(self, values):
        self.values = np.asarray(values)


class BinByResult:
    """The xarray.DataArray the reference returns, reduced to data / dims / coords."""

    def __init__(self, data, dims, coords):
        self.data = data
        self.dims = tuple(dims)
        self.coords = {k: _Coord(v) for k, v in coords.items()}


class BinBy(GroupByBase):
    def agg(self, actions):
        arrays = self._agg(actions)
        self.df.execute()
        arrays = {k: extract_central_part(np.asarray(v.get())) for k, v in arrays.items()}
        keys = list(arrays)
        coords = {b.label: list(b.bin_values) for b in self.by}
        if len(arrays) == 1 and not isinstance(actions, dict):
            return BinByResult(arrays[keys[0]], self.dims, coords)
        final = np.stack([arrays[k] for k in keys])
        coords = dict(coords)
        coords["statistic"] = keys
        return BinByResult(final, ["statistic"] + self.dims, coords)
