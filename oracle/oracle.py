"""CPU oracle for the binned-statistics / groupby path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the *checker*.  The product
(``vaex_amd``) never imports it and fails loudly when its HIP library is
missing.

It wraps ``liboracle.so`` (``superagg_oracle.c``, a plain-C restatement of the
reference's superagg C++; each function there cites the reference file:line it
follows) and adds:

* :func:`grid_shape`, :func:`bin_indices`, :func:`aggregate` -- the Grid/Binner/
  Agg semantics of ``packages/vaex-core/src/agg.hpp:50-143``,
  ``superagg_binners.cpp`` and ``superagg.cpp`` on whole columns.
* :class:`OrderedSet` -- a pure-Python restatement of ``ordered_set``
  (``packages/vaex-core/src/hash_primitives.hpp:417-583``) including the
  NaN/null special ordinals (``:436-450``) and ``nmaps`` partitioning.
* :func:`groupby_reference` -- key -> (sum, count) maps as
  ``groupby.py:97-168,484-533`` computes them.

Pinning: ``tests/test_oracle_kats.py`` checks this oracle against every KAT in
``tests/golden/kats.json`` (transcribed from the reference's own tests).
"""
import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

DTYPES = ["float64", "float32", "int64", "int32", "int16", "int8",
          "uint64", "uint32", "uint16", "uint8", "bool"]
DTYPE_CODE = {name: i for i, name in enumerate(DTYPES)}

# upcast<T> (superagg.cpp:289-346)
UPCAST = {"float64": "float64", "float32": "float64", "bool": "int64",
          "int8": "int64", "int16": "int64", "int32": "int64", "int64": "int64",
          "uint8": "uint64", "uint16": "uint64", "uint32": "uint64", "uint64": "uint64"}

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, u64, i32, dbl = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
        L.or_binner_scalar.argtypes = [i32, i32, vp, vp, u64, dbl, dbl, u64, u64, vp]
        L.or_binner_ordinal.argtypes = [i32, i32, vp, vp, u64, u64, u64, u64, vp]
        L.or_agg_count.argtypes = [i32, i32, vp, vp, vp, u64, vp]
        L.or_agg_sum.argtypes = [i32, i32, vp, vp, vp, u64, vp]
        L.or_agg_minmax.argtypes = [i32, i32, i32, vp, vp, vp, u64, vp]
        L.or_agg_first.argtypes = [i32, i32, vp, vp, vp, u64, vp, vp]
        L.or_agg_sum_moment.argtypes = [i32, i32, vp, vp, vp, u64, ctypes.c_uint32, vp]
        L.or_hash64.argtypes = [u64]
        L.or_hash64.restype = u64
        L.or_set_create.argtypes = [i32]
        L.or_set_create.restype = vp
        L.or_set_destroy.argtypes = [vp]
        L.or_set_update.argtypes = [vp, vp, u64]
        L.or_set_length.argtypes = [vp]
        L.or_set_length.restype = u64
        L.or_set_key_array.argtypes = [vp, vp]
        L.or_set_map_ordinal.argtypes = [vp, vp, u64, vp]
        L.or_minmax_f64.argtypes = [vp, u64, vp, vp]
        L.or_bench_grid2d.argtypes = [vp, vp, vp, u64, dbl, dbl, dbl, dbl, u64, i32, i32, u64, vp, vp]
        L.or_bench_grid2d.restype = i32
        L.or_bench_count1d.argtypes = [vp, u64, i32, u64, i32, vp, vp]
        L.or_bench_count1d.restype = i32
        L.or_bench_groupby_i32.argtypes = [vp, vp, u64, i32, i32, u64, ctypes.c_int64, vp, vp, vp]
        L.or_bench_groupby_i32.restype = ctypes.c_int64
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def _dtype_info(ar):
    """(dtype name, flip) -- non-native byte order => flip (find_type_from_dtype, utils.py:879-903)."""
    dt = ar.dtype
    flip = dt.byteorder not in ("<", "=", "|")
    name = dt.newbyteorder("=").name if flip else dt.name
    if dt.kind in "mM":
        name = "int64"
    return name, int(flip)


def as_u64_bits(value, dtype=None):
    """A BinnerOrdinal_<T> ctor argument: pybind11 casts the Python value to T
    (py::init<std::string, T, T>, superagg_binners.cpp:191; bool via truthiness), then the
    C++ ctor converts T to uint64_t (:99): integers sign-extend / wrap modulo 2**64, floats
    truncate toward zero (x86-64 cvttsd2si)."""
    dt = np.dtype(dtype) if dtype is not None else None
    if dt is not None and dt.kind == "b":
        return int(bool(value))
    if isinstance(value, (float, np.floating)) or (dt is not None and dt.kind == "f"):
        return int(math.trunc(float(value))) & (2 ** 64 - 1)
    v = int(value)
    if dt is not None and dt.kind in "iu":
        bits = dt.itemsize * 8
        v &= (1 << bits) - 1
        if dt.kind == "i" and v >= 1 << (bits - 1):
            v -= 1 << bits
    return v & (2 ** 64 - 1)


class Binner:
    """Spec of a scalar or ordinal binner (superagg_binners.cpp:5-184)."""

    def __init__(self, kind, data, vmin=None, vmax=None, bins=None, ordinal_count=None,
                 min_value=0, mask=None):
        self.kind = kind
        self.data = np.ascontiguousarray(data)
        self.mask = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self.vmin, self.vmax, self.bins = vmin, vmax, bins
        self.ordinal_count, self.min_value = ordinal_count, min_value

    def shape(self):
        if self.kind == "scalar":
            return self.bins + 3
        return as_u64_bits(self.ordinal_count, _dtype_info(self.data)[0]) + 3


def grid_shape(binners):
    return tuple(b.shape() for b in binners)


def grid_strides(binners):
    """strides[0] = 1, strides[d] = strides[d-1]*shape[d-1] (agg.hpp:60-69)."""
    strides, s = [], 1
    for b in binners:
        strides.append(s)
        s *= b.shape()
    return strides


def bin_indices(binners, n):
    """indices1d for n rows (agg.hpp:106-136; superagg_binners.cpp:14-56,104-142)."""
    L = lib()
    out = np.zeros(n, dtype=np.uint64)
    for b, stride in zip(binners, grid_strides(binners)):
        name, flip = _dtype_info(b.data)
        code = DTYPE_CODE[name]
        if b.kind == "scalar":
            rc = L.or_binner_scalar(code, flip, _ptr(b.data), _ptr(b.mask), n, float(b.vmin),
                                    float(b.vmax), int(b.bins), stride, _ptr(out))
        else:
            rc = L.or_binner_ordinal(code, flip, _ptr(b.data), _ptr(b.mask), n,
                                     as_u64_bits(b.ordinal_count, name), as_u64_bits(b.min_value, name),
                                     stride, _ptr(out))
        assert rc == 0
    return out


def _fortran_view(flat, shape):
    return flat.reshape(shape, order="F") if shape else flat.reshape(())


def new_grid(kind, dtype, shape):
    """Zero/initial grid for an aggregator, as the AggXxx ctors fill it (superagg.cpp)."""
    length = int(np.prod(shape)) if shape else 1
    if kind == "count":
        return np.zeros(length, np.int64), None
    if kind in ("sum", "sum_moment"):
        return np.zeros(length, UPCAST[dtype]), None
    np_dt = np.dtype(dtype)
    if kind in ("min", "max"):
        if np_dt.kind == "f":
            fill = np.inf if kind == "min" else -np.inf
        elif np_dt.kind == "b":
            fill = kind == "min"
        else:
            info = np.iinfo(np_dt)
            fill = info.max if kind == "min" else info.min
        return np.full(length, fill, np_dt), None
    if kind == "first":
        if np_dt.kind == "f":
            omax = np.finfo(np_dt).max
        elif np_dt.kind == "b":
            omax = True
        else:
            omax = np.iinfo(np_dt).max
        return np.zeros(length, np_dt), np.full(length, omax, np_dt)
    raise ValueError(kind)


def aggregate(kind, idx, grid, data=None, data2=None, mask=None, moment=2, grid2=None, dtype=None):
    """Apply one aggregator over all rows in row order (superagg.cpp:168-505)."""
    L = lib()
    n = len(idx)
    idx = np.ascontiguousarray(idx, dtype=np.uint64)
    mask = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    if data is not None:
        data = np.ascontiguousarray(data)
        name, flip = _dtype_info(data)
    else:
        name, flip = (dtype or "int64"), 0
    code = DTYPE_CODE[name]
    if kind == "count":
        rc = L.or_agg_count(code, flip, _ptr(data), _ptr(mask), _ptr(idx), n, _ptr(grid))
    elif kind == "sum":
        rc = L.or_agg_sum(code, flip, _ptr(data), _ptr(mask), _ptr(idx), n, _ptr(grid))
    elif kind in ("min", "max"):
        rc = L.or_agg_minmax(int(kind == "max"), code, flip, _ptr(data), _ptr(mask), _ptr(idx), n,
                             _ptr(grid))
    elif kind == "first":
        data2 = np.ascontiguousarray(data2)
        rc = L.or_agg_first(code, flip, _ptr(data), _ptr(data2), _ptr(idx), n, _ptr(grid),
                            _ptr(grid2))
    elif kind == "sum_moment":
        rc = L.or_agg_sum_moment(code, flip, _ptr(data), _ptr(mask), _ptr(idx), n, moment,
                                 _ptr(grid))
    else:
        raise ValueError(kind)
    assert rc == 0


def reduce_grids(kind, grids, grids2=None):
    """Aggregator::reduce, parts[0].reduce(parts[1:]) (superagg.cpp:160-167,205-212,252-259,
    354-361,470-480)."""
    out = grids[0].copy()
    out2 = None if grids2 is None else grids2[0].copy()
    for k in range(1, len(grids)):
        o = grids[k]
        if kind in ("count", "sum", "sum_moment"):
            out = out + o
        elif kind == "max":
            out = np.where(out < o, o, out)
        elif kind == "min":
            out = np.where(o < out, o, out)
        elif kind == "first":
            take = grids2[k] < out2
            out = np.where(take, o, out)
            out2 = np.where(take, grids2[k], out2)
    return out, out2


def compute_grid(binners, kind, data=None, data2=None, mask=None, n=None, dtype=None, moment=2):
    """Full Grid + one Agg, returned as the F-ordered numpy view with edges."""
    if n is None:
        n = len(binners[0].data) if binners else len(data)
    shape = grid_shape(binners)
    idx = bin_indices(binners, n) if binners else np.zeros(n, np.uint64)
    dname = dtype
    if data is not None:
        dname = _dtype_info(np.asarray(data))[0]
    grid, grid2 = new_grid(kind, dname or "int64", shape)
    aggregate(kind, idx, grid, data=data, data2=data2, mask=mask, moment=moment, grid2=grid2,
              dtype=dname)
    return _fortran_view(grid, shape)


def nunique_grid(binners, data, mask=None, selection=False, dropmissing=False, dropnan=False, n=None):
    """AggNUnique over all rows (agg_hash_primitive.cpp:24-60 with the counter's count(),
    hash.hpp:208-222): per cell  distinct + (nulls > 0) + (nans > 0), minus the null / nan
    ROW counts when dropmissing / dropnan (the reference subtracts counts, not presence).
    mask: aggregator data mask (1 = keep); selection: a selection mask was set, so rows
    with mask 0 are outside it and not seen.  Values compare with == (-0.0 == 0.0)."""
    data = np.asarray(data)
    if n is None:
        n = len(data)
    shape = grid_shape(binners)
    length = int(np.prod(shape)) if shape else 1
    idx = (bin_indices(binners, n) if binners else np.zeros(n, np.uint64)).astype(np.int64)
    name, flip = _dtype_info(data)
    vals = data.byteswap().view(data.dtype.newbyteorder()) if flip else data
    keep = np.ones(n, bool) if mask is None else np.asarray(mask).astype(bool)
    seen = keep if selection else np.ones(n, bool)
    nulls = np.bincount(idx[seen & ~keep], minlength=length)
    v = vals[keep & seen]
    c = idx[keep & seen]
    if v.dtype.kind == "f":
        isnan = np.isnan(v)
        nans = np.bincount(c[isnan], minlength=length)
        v, c = v[~isnan].astype(np.float64), c[~isnan]
        v = np.where(v == 0, 0.0, v)  # -0.0 and 0.0 are one key
        bits = v.view(np.int64)
    else:
        nans = np.zeros(length, np.int64)
        bits = v.astype(np.int64)
    pairs = np.unique(np.stack([c, bits], axis=1), axis=0) if len(c) else np.zeros((0, 2), np.int64)
    distinct = np.bincount(pairs[:, 0], minlength=length)
    out = distinct + (nulls > 0) + (nans > 0)
    if dropmissing:
        out = out - nulls
    if dropnan:
        out = out - nans
    return _fortran_view(out.astype(np.int64), shape)


def var_grid(binners, data, mask=None, n=None):
    """AggregatorDescriptorVar (agg.py:196-224): the expression is cast to float64
    (``expression.astype('float64')``, :197-198), then _sum_moment(2), sum and count of
    the cast values on the same binners; finish = sum_moment/count - (sum/count)**2
    (0/0 -> nan, divide and invalid ignored)."""
    x = np.asarray(data).astype(np.float64)
    sm = compute_grid(binners, "sum_moment", data=x, mask=mask, n=n, moment=2)
    s = compute_grid(binners, "sum", data=x, mask=mask, n=n)
    c = compute_grid(binners, "count", data=x, mask=mask, n=n)
    with np.errstate(divide="ignore", invalid="ignore"):
        mean = s / c
        return np.asarray(sm, dtype=np.float64) / c - mean ** 2


def extract_central_part(ar):
    """utils.py:919-920."""
    return ar[(slice(2, -1),) * ar.ndim]


def hash64(x):
    return int(lib().or_hash64(int(x) & (2 ** 64 - 1)))


class OrderedSet:
    """Restatement of ordered_set<T> (hash_primitives.hpp:417-583, hash.hpp:124-257).

    Keys are processed in the given row order, as ``_update`` does for one
    thread: keys are bucketed per map (``hash % nmaps``), maps are flushed in
    map order (so within a map insertion order == row order), then null and
    NaN rows go to map 0 (``:248-274``).
    """

    def __init__(self, nmaps=1):
        self.nmaps = nmaps
        self.maps = [dict() for _ in range(nmaps)]
        self.nan_count = 0
        self.null_count = 0
        self.nan_value = 0x7FFFFFFF
        self.null_value = 0x7FFFFFFF
        self._offset_null_nan = 0

    @staticmethod
    def _hash_key(key, dtype):
        if np.dtype(dtype).kind == "f":
            bits = np.array([key], dtype=np.float64 if np.dtype(dtype).itemsize == 8 else np.float32)
            if bits.dtype == np.float32:
                return hash64(int(bits.view(np.uint32)[0]))  # float hash: zero-extended bits
            return hash64(int(bits.view(np.uint64)[0]))
        return hash64(int(key))  # int32/int64 sign-extend, unsigned zero-extend

    @staticmethod
    def _ident(key, dtype):
        """Map identity of a key: floats by bit pattern (hash<double> hashes the bits,
        hash.hpp:69-85, so -0.0 and 0.0 land in different buckets and stay distinct keys;
        a Python dict would merge them), integers by value."""
        if np.dtype(dtype).kind == "f":
            return ("f", int(np.array([key], dtype=dtype).view(np.uint64 if np.dtype(dtype).itemsize == 8
                                                              else np.uint32)[0]), float(key))
        return key.item()

    def update(self, keys, mask=None, return_values=False):
        """``_update`` (hash_primitives.hpp:96-281).  With ``return_values`` (the offsets path)
        null rows are flushed before NaN rows, otherwise NaN before null (:248-274)."""
        keys = np.asarray(keys)
        buckets = [[] for _ in range(self.nmaps)]
        nulls, nans = [], []
        for i, k in enumerate(keys):
            if mask is not None and mask[i]:
                nulls.append(i)
            elif keys.dtype.kind == "f" and k != k:
                nans.append(i)
            else:
                buckets[self._hash_key(k, keys.dtype) % self.nmaps].append(self._ident(k, keys.dtype))
        for m, bucket in enumerate(buckets):
            for k in bucket:
                mp = self.maps[m]
                if k not in mp:
                    ordinal = len(mp) + (self._offset_null_nan if m == 0 else 0)
                    mp[k] = ordinal
        def add_nan():
            self.nan_count += 1
            if self.nan_count == 1:
                self.nan_value = len(self.maps[0]) + self._offset_null_nan
                self._offset_null_nan += 1

        def add_null():
            self.null_count += 1
            if self.null_count == 1:
                self.null_value = len(self.maps[0]) + self._offset_null_nan
                self._offset_null_nan += 1
        if return_values:
            for _ in nulls:
                add_null()
            for _ in nans:
                add_nan()
        else:
            for _ in nans:
                add_nan()
            for _ in nulls:
                add_null()

    def offsets(self):
        out, off = [], 0
        for i, m in enumerate(self.maps):
            out.append(off)
            off += len(m)
            if i == 0:
                off += int(self.null_count > 0) + int(self.nan_count > 0)
        return out

    def __len__(self):
        return sum(len(m) for m in self.maps) + int(self.null_count > 0) + int(self.nan_count > 0)

    def key_array(self, dtype):
        out = np.zeros(len(self), dtype=dtype)
        for m, off in zip(self.maps, self.offsets()):
            for k, v in m.items():
                out[v + off] = k[2] if isinstance(k, tuple) else k
        if self.nan_count:
            out[self.nan_value] = np.nan
        if self.null_count:
            out[self.null_value] = -1
        return out

    def map_ordinal(self, keys):
        keys = np.asarray(keys)
        n = len(self)
        out_dtype = np.int8 if n < 2 ** 7 else np.int16 if n < 2 ** 15 else np.int32 if n < 2 ** 31 else np.int64
        offs = self.offsets()
        out = np.empty(len(keys), dtype=out_dtype)
        for i, k in enumerate(keys):
            if keys.dtype.kind == "f" and k != k:
                out[i] = self.nan_value
                continue
            m = self._hash_key(k, keys.dtype) % self.nmaps
            v = self.maps[m].get(self._ident(k, keys.dtype))
            out[i] = -1 if v is None else v + offs[m]
        return out


def groupby_reference(keys, values):
    """key -> (sum, count) map with sums accumulated in row order, as the reference's
    single-threaded groupby(...).agg({v: [sum, count]}) produces them (NaN values are
    skipped by AggSum and by count(v); superagg.cpp:171-184,380-386)."""
    keys = np.asarray(keys)
    values = np.asarray(values, dtype=np.float64)
    uniq, inverse = np.unique(keys, return_inverse=True)
    ok = ~np.isnan(values)
    counts = np.bincount(inverse[ok], minlength=len(uniq)).astype(np.int64)
    sums = np.bincount(inverse[ok], weights=values[ok], minlength=len(uniq))
    return uniq, sums, counts


def minmax_f64(x):
    lo, hi = ctypes.c_double(), ctypes.c_double()
    x = np.ascontiguousarray(x, dtype=np.float64)
    lib().or_minmax_f64(_ptr(x), len(x), ctypes.addressof(lo), ctypes.addressof(hi))
    return lo.value, hi.value


# ---- multi-key / multi-aggregate groupby (groupby.py) -------------------------------------
def _grouper(values, sort=True):
    """Grouper of one key column with sort=True (groupby.py:97-168): the set's keys sorted
    (NaN after the numbers, groupby.py:137-156), each row's ordinal into them.  Returns
    (labels, ordinal per row)."""
    values = np.asarray(values)
    if values.dtype.kind == "f":
        nan = np.isnan(values)
        labels = np.unique(values[~nan])
        ordinal = np.searchsorted(labels, values).astype(np.int64)
        if nan.any():
            ordinal[nan] = len(labels)
            labels = np.append(labels, np.nan)
        return labels, ordinal
    labels, ordinal = np.unique(values, return_inverse=True)
    return labels, ordinal.astype(np.int64)


def _combine(ordinals, counts):
    """_combine (groupby.py:248-288): the cartesian ordinal of as many leading groupers as
    fit below 2**63 (first grouper most significant, cumulative_counts multipliers), made
    into one GrouperCombined whose bins are the combined values that occur (a set, sorted);
    the remaining groupers are combined with it recursively.  Returns (ordinal per row,
    [per grouper: its ordinal of each combined group])."""
    ords, ns = list(ordinals), list(counts)
    take, prod = 1, ns[0]
    while take < len(ns) and prod * ns[take] < 2 ** 63 - 1:
        prod *= ns[take]
        take += 1
    cum = [1]
    for nk in reversed(ns[1:take]):
        cum.insert(0, cum[0] * nk)
    combined = np.zeros(len(ords[0]), np.int64)
    for o, m in zip(ords[:take], cum):
        combined += o * np.int64(m)
    bins, ordinal = np.unique(combined, return_inverse=True)
    parts = [(bins // np.int64(m)) % np.int64(nk) for nk, m in zip(ns[:take], cum)]
    if take == len(ns):
        return ordinal.astype(np.int64), parts
    inner, inner_parts = _combine([ordinal.astype(np.int64)] + ords[take:], [len(bins)] + ns[take:])
    first = inner_parts[0]
    return inner, [p[first] for p in parts] + inner_parts[1:]


def groupby_agg(columns, by, aggs, combine="auto"):
    """``df.groupby(by, sort=True, combine=combine).agg(...)`` restated on numpy
    (groupby.py:97-168 Grouper, :248-288 _combine, :313-333 combine='auto', :484-533 agg):
    groups in the lexicographic order of the sorted key labels, only the key combinations
    that occur; aggregates per group as the superagg grids compute them in row order --
    count(*) of every row, count(v) of the non-NaN rows, sum(v) upcast (float64 / int64 /
    uint64, NaN skipped), mean = sum / count(v), min / max ignoring NaN (an all-NaN group
    keeps the AggMin/AggMax fill, superagg.cpp:199-204,246-251).

    columns: {name: numpy array}; by: key names; aggs: [(out_name, op, column or None)] with
    op in count / sum / mean / min / max.  Returns {name: numpy array} with the key labels
    first."""
    by = [by] if isinstance(by, str) else list(by)
    n = len(columns[by[0]])
    groupers = [_grouper(columns[b]) for b in by]
    counts = [len(g[0]) for g in groupers]
    cells = int(np.prod([float(c) for c in counts]))
    if len(by) >= 2 and (combine is True or (combine == "auto" and n / max(cells, 1) < 10)):
        ordinal, parts = _combine([g[1] for g in groupers], counts)
        ngroups = len(parts[0])
        labels = [g[0][p] for g, p in zip(groupers, parts)]
        keep = None
    else:
        # cartesian grid (C order of the ordinals = meshgrid 'ij'), empty cells dropped
        ordinal = np.zeros(n, np.int64)
        for g, c in zip(groupers, counts):
            ordinal = ordinal * c + g[1]
        ngroups = int(np.prod(counts))
        present = np.bincount(ordinal, minlength=ngroups) > 0 if len(by) > 1 else np.ones(ngroups, bool)
        keep = np.flatnonzero(present)
        idx = np.unravel_index(keep, counts)
        labels = [g[0][i] for g, i in zip(groupers, idx)]
    out = {b: lab for b, lab in zip(by, labels)}
    cnt_all = np.bincount(ordinal, minlength=ngroups)
    for name, op, col in aggs:
        if op == "count" and col is None:
            r = cnt_all
        else:
            v = np.asarray(columns[col])
            ok = ~np.isnan(v) if v.dtype.kind == "f" else np.ones(n, bool)
            cnt = np.bincount(ordinal[ok], minlength=ngroups).astype(np.int64)
            if op == "count":
                r = cnt
            elif op in ("sum", "mean"):
                up = np.float64 if v.dtype.kind == "f" else (np.uint64 if v.dtype.kind in "ub" else np.int64)
                s = np.zeros(ngroups, up)
                np.add.at(s, ordinal[ok], v[ok].astype(up))
                if op == "sum":
                    r = s
                else:
                    with np.errstate(divide="ignore", invalid="ignore"):
                        r = s.astype(np.float64) / cnt
            elif op in ("min", "max"):
                g, _ = new_grid(op, v.dtype.name, (ngroups,))
                (np.minimum if op == "min" else np.maximum).at(g, ordinal[ok], v[ok])
                r = g
            else:
                raise ValueError(op)
        out[name] = r if keep is None else r[keep]
    return out
