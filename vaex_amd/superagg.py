"""``vaex.superagg``-compatible module surface over libvaexhip (HIP, MI355X).

Same class names, constructor signatures, methods and error behaviour as the
reference's pybind11 module (``packages/vaex-core/src/superagg.cpp:586-626``,
``superagg_binners.cpp:186-303``), so task-part code written against
``vaex.superagg`` drives the GPU unchanged:

* ``Grid(binners)``, ``.bin(aggs[, length])``, ``.binners`` (``agg.hpp:50-143``)
* ``BinnerScalar_<dtype>[_non_native](expression, vmin, vmax, bins)``
* ``BinnerOrdinal_<dtype>[_non_native](expression, ordinal_count, min_value)``
* ``Agg{Count,Sum,Min,Max,First}_<dtype>[_non_native](grid)``,
  ``AggSumMoment_<dtype>[_non_native](grid, moment)`` with ``set_data(ar, index)``,
  ``set_data_mask``, ``clear_data_mask``, ``reduce``, ``__sizeof__``, ``.grid``
  and a live, writable, Fortran-ordered array view (``np.asarray(agg)``).

Differences forced by the device boundary (documented in DESIGN.md): the grid lives in
HBM and the array view is a host image kept coherent around ``bin``/``reduce``; input
buffers may be numpy arrays (staged to HBM per chunk) or :class:`DeviceArray` (read in
place).  ``BinnerSetOrdinal`` is an extension: ``BinnerOrdinal`` over
``_ordinal_values(key, set)`` with the hash lookup fused into the bin kernel.
"""
import ctypes

import numpy as np

from . import _lib
from .device import DeviceArray

DTYPES = _lib.DTYPES


def _column(ar):
    """(ptr, length, itemsize, ndim, loc, keepalive) of a buffer handed to set_data."""
    if isinstance(ar, DeviceArray):
        return ar.ptr, len(ar), ar.itemsize, 1, _lib.LOC_DEVICE, ar
    a = np.asarray(ar)
    if a.ndim == 1 and not a.flags.c_contiguous:
        a = np.ascontiguousarray(a)
    length = len(a) if a.ndim >= 1 else a.size
    _lib.host_register(a)
    return a.ctypes.data, length, a.itemsize, a.ndim, _lib.LOC_HOST, a


def _u64_of(value, dtype):
    """A T ctor argument converted to uint64_t the way C++ converts it
    (superagg_binners.cpp:99): ints via T (wrap, sign-extend), floats truncated."""
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return int(np.trunc(float(value))) & (2 ** 64 - 1)
    if dt.kind == "b":
        return int(bool(value))
    v = int(value)
    bits = dt.itemsize * 8
    v &= (1 << bits) - 1
    if dt.kind == "i" and v >= 1 << (bits - 1):
        v -= 1 << bits
    return v & (2 ** 64 - 1)


class Binner:
    """Base class of all binners (``py::class_<Binner>``, superagg.cpp:594)."""

    _handle = None

    def _set(self, name, ar, *extra):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        return ptr, length, itemsize, ndim, loc, keep

    def set_data(self, ar):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        _lib.call("vh_binner_set_data", self._handle, ptr, length, itemsize, ndim, loc)
        self._data_ref = keep

    def set_data_mask(self, ar):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        if loc == _lib.LOC_HOST:
            keep = np.ascontiguousarray(keep, dtype=np.uint8) if keep.dtype != np.uint8 else keep
            ptr = keep.ctypes.data
        _lib.call("vh_binner_set_data_mask", self._handle, ptr, length, ndim, loc)
        self._mask_ref = keep

    def clear_data_mask(self):
        _lib.call("vh_binner_clear_data_mask", self._handle)
        self._mask_ref = None

    def _copy_from(self, other):
        h = ctypes.c_void_p()
        _lib.call("vh_binner_copy", other._handle, ctypes.byref(h))
        self._handle = h.value
        self._data_ref = getattr(other, "_data_ref", None)
        self._mask_ref = getattr(other, "_mask_ref", None)

    def copy(self):
        b = type(self).__new__(type(self))
        b.__dict__.update(self.__dict__)
        b._copy_from(self)
        return b

    def shape(self):
        s = ctypes.c_uint64()
        _lib.call("vh_binner_shape", self._handle, ctypes.byref(s))
        return s.value

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h:
            try:
                _lib.call("vh_binner_destroy", h)
            except Exception:
                pass
            self._handle = None


class _BinnerScalarBase(Binner):
    """BinnerScalar<T, u64, FlipEndian> (superagg_binners.cpp:5-93)."""

    _dtype = "float64"
    _flip = 0

    def __init__(self, expression, vmin, vmax, bins):
        self._expression = str(expression)
        self._vmin, self._vmax, self._bins = float(vmin), float(vmax), int(bins)
        h = ctypes.c_void_p()
        code = _lib.DTYPE_CODE[self._dtype]
        _lib.call("vh_binner_scalar_create", self._expression.encode(), code, self._flip, self._vmin, self._vmax,
                  self._bins, ctypes.byref(h))
        self._handle = h.value

    expression = property(lambda self: self._expression)
    bins = property(lambda self: self._bins)
    vmin = property(lambda self: self._vmin)
    vmax = property(lambda self: self._vmax)

    def __reduce__(self):
        return (type(self), (self._expression, self._vmin, self._vmax, self._bins))


class _BinnerOrdinalBase(Binner):
    """BinnerOrdinal<T, u64, FlipEndian> (superagg_binners.cpp:95-184)."""

    _dtype = "int64"
    _flip = 0

    def __init__(self, expression, ordinal_count, min_value=0):
        self._expression = str(expression)
        self._ordinal_count = _u64_of(ordinal_count, self._dtype)
        self._min_value = _u64_of(min_value, self._dtype)
        h = ctypes.c_void_p()
        code = _lib.DTYPE_CODE[self._dtype]
        _lib.call("vh_binner_ordinal_create", self._expression.encode(), code, self._flip, self._ordinal_count,
                  self._min_value, ctypes.byref(h))
        self._handle = h.value

    expression = property(lambda self: self._expression)
    ordinal_count = property(lambda self: self._ordinal_count)
    min_value = property(lambda self: self._min_value)

    def __reduce__(self):
        return (type(self), (self._expression, self._ordinal_count, self._min_value))


class BinnerSetOrdinal(Binner):
    """BinnerOrdinal over ``_ordinal_values(key, set)`` (functions.py:2441-2448) with the
    ``map_ordinal`` hash probe fused into the bin kernel: ``set_data`` takes the raw key
    column, ``set_data_mask`` its null mask (null keys -> the set's null ordinal)."""

    def __init__(self, expression, ordered_set, ordinal_count):
        self._expression = str(expression)
        self._set = ordered_set
        self._ordinal_count = int(ordinal_count)
        h = ctypes.c_void_p()
        _lib.call("vh_binner_set_ordinal_create", self._expression.encode(), ordered_set._handle,
                  self._ordinal_count, ctypes.byref(h))
        self._handle = h.value

    expression = property(lambda self: self._expression)
    ordinal_count = property(lambda self: self._ordinal_count)
    min_value = property(lambda self: 0)


class Grid:
    """Grid<> (agg.hpp:50-143): strides[0] = 1, the first binner varies fastest."""

    def __init__(self, binners):
        self._binners = list(binners)
        arr = (ctypes.c_void_p * max(1, len(self._binners)))(*[b._handle for b in self._binners])
        h = ctypes.c_void_p()
        _lib.call("vh_grid_create", arr, len(self._binners), ctypes.byref(h))
        self._handle = h.value
        dims = ctypes.c_int()
        n = max(1, len(self._binners))
        shapes = (ctypes.c_uint64 * n)()
        strides = (ctypes.c_uint64 * n)()
        length1d = ctypes.c_uint64()
        _lib.call("vh_grid_info", self._handle, ctypes.byref(dims), shapes, strides, ctypes.byref(length1d))
        self.dimensions = dims.value
        self.shapes = tuple(shapes[i] for i in range(self.dimensions))
        self.strides = tuple(strides[i] for i in range(self.dimensions))
        self.length1d = length1d.value

    @property
    def binners(self):
        return list(self._binners)

    def bin(self, aggs, length=None):
        aggs = list(aggs)
        for a in aggs:
            a._before_device_use()
        arr = (ctypes.c_void_p * max(1, len(aggs)))(*[a._handle for a in aggs])
        has_length = length is not None
        _lib.call("vh_grid_bin", self._handle, arr, len(aggs), int(length) if has_length else 0, int(has_length))
        for a in aggs:
            a._after_device_write()

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h:
            try:
                _lib.call("vh_grid_destroy", h)
            except Exception:
                pass
            self._handle = None


class Aggregator:
    """Base of all aggregators (``py::class_<Aggregator>``, superagg.cpp:590-593)."""

    _kind = None
    _dtype = "float64"
    _flip = 0

    def __init__(self, grid, *args):
        self._grid = grid  # keep_alive<1, 2>
        moment = int(args[0]) if args else 0
        h = ctypes.c_void_p()
        _lib.call("vh_agg_create", grid._handle, _lib.AGG_KIND[self._kind], _lib.DTYPE_CODE[self._dtype],
                  self._flip, moment, ctypes.byref(h))
        self._handle = h.value
        self._moment = moment
        nbytes, gdt, isz = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64()
        _lib.call("vh_agg_info", self._handle, ctypes.byref(nbytes), ctypes.byref(gdt), ctypes.byref(isz))
        self._nbytes = nbytes.value
        self._grid_dtype = np.dtype(DTYPES[gdt.value] if DTYPES[gdt.value] != "bool" else "bool")
        self._host = None        # host image of the grid (array view target)
        self._exposed = False    # a view was handed out: the host image may be written by the user
        self._device_newer = True
        self._refs = {}

    # ---- data ----------------------------------------------------------------
    def set_data(self, ar, index=0):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        _lib.call("vh_agg_set_data", self._handle, ptr, length, itemsize, ndim, int(index), loc)
        self._refs[("data", int(index) if self._kind == "AggFirst" else 0)] = keep

    def set_data_mask(self, ar):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        if loc == _lib.LOC_HOST and keep.dtype != np.uint8:
            keep = np.ascontiguousarray(keep, dtype=np.uint8)
            ptr = keep.ctypes.data
        _lib.call("vh_agg_set_data_mask", self._handle, ptr, length, ndim, loc)
        self._refs["mask"] = keep

    def clear_data_mask(self):
        _lib.call("vh_agg_clear_data_mask", self._handle)
        self._refs.pop("mask", None)

    @property
    def grid(self):
        return self._grid

    def __sizeof__(self):
        return self._nbytes

    # ---- host image / device coherence --------------------------------------
    def _release_host(self):
        """The current host image now belongs to a result array (which keeps this object,
        and so the image, alive through its base): later reads get a fresh image."""
        self._released = self._host
        self._host = None
        self._exposed = False
        self._device_newer = True

    def _ensure_host(self):
        if self._host is None:
            self._host = _lib.pinned_empty(self._grid.length1d, self._grid_dtype)
            self._device_newer = True
        if self._device_newer:
            _lib.call("vh_agg_download", self._handle, self._host.ctypes.data, self._nbytes)
            self._device_newer = False

    def _before_device_use(self):
        if self._exposed:  # the user may have written through the view
            _lib.call("vh_agg_upload", self._handle, self._host.ctypes.data, self._nbytes)

    def _after_device_write(self):
        self._device_newer = True
        if self._exposed:
            self._ensure_host()

    @property
    def __array_interface__(self):
        """Live writable view of the grid, shape = binner shapes, Fortran strides (agg.hpp:166-179)."""
        self._ensure_host()
        self._exposed = True
        g = self._grid
        isz = self._grid_dtype.itemsize
        return {
            "shape": tuple(g.shapes),
            "typestr": self._grid_dtype.str,
            "data": (self._host.ctypes.data, False),
            "strides": tuple(s * isz for s in g.strides) if g.dimensions else None,
            "version": 3,
        }

    def device_grid_ptr(self):
        """HBM address of the grid (length1d items of the grid dtype)."""
        p, p2 = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("vh_agg_device_ptr", self._handle, ctypes.byref(p), ctypes.byref(p2))
        return p.value

    def occupancy(self, begin=0, end=None):
        """(nonzero count, first, last) of grid items [begin, end) relative to begin, found on
        the device ((0, -1, -1) when none): a dense groupby's occupied cells without a scan of
        the host image."""
        end = self._grid.length1d if end is None else end
        self._before_device_use()
        out = (ctypes.c_int64 * 3)()
        _lib.call("vh_agg_occupancy", self._handle, int(begin), int(end), out)
        return int(out[0]), int(out[1]), int(out[2])

    def device_order_ptr(self):
        """HBM address of AggFirst's order grid."""
        p, p2 = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("vh_agg_device_ptr", self._handle, ctypes.byref(p), ctypes.byref(p2))
        return p2.value

    def order_grid(self):
        """AggFirst's order grid (host copy, same layout as the value grid)."""
        out = np.empty(self._grid.length1d, self._grid_dtype)
        _lib.call("vh_agg_download_order", self._handle, out.ctypes.data, self._nbytes)
        g = self._grid
        return out.reshape(g.shapes, order="F") if g.dimensions else out.reshape(())

    def reduce(self, others):
        """Aggregator::reduce (superagg.cpp:160-167, 205-212, 252-259, 354-361, 470-480)."""
        others = list(others)
        self._before_device_use()
        for o in others:
            o._before_device_use()
        arr = (ctypes.c_void_p * max(1, len(others)))(*[o._handle for o in others])
        _lib.call("vh_agg_reduce", self._handle, arr, len(others))
        self._after_device_write()

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h:
            try:
                _lib.call("vh_agg_destroy", h)
            except Exception:
                pass
            self._handle = None


class _AggNUniqueBase(Aggregator):
    """AggNUnique_<t>(grid, dropmissing, dropnan) (agg_hash_primitive.cpp:6-102,
    superagg.cpp add_agg): distinct values per cell, an int64 grid derived from the
    (cell, value) pairs kept in HBM."""

    _kind = "AggNUnique"

    def __init__(self, grid, dropmissing=False, dropnan=False):
        super().__init__(grid, (1 if dropmissing else 0) | (2 if dropnan else 0))
        self.dropmissing, self.dropnan = bool(dropmissing), bool(dropnan)

    def set_selection_mask(self, ar):
        ptr, length, itemsize, ndim, loc, keep = _column(ar)
        _lib.call("vh_agg_set_selection_mask", self._handle, ptr, length, ndim, loc)
        self._refs["selection"] = keep

    def _before_device_use(self):
        pass  # the grid is derived from the pairs: writes through a view do not feed back


def _register():
    ns = globals()
    for dtype in DTYPES:
        for flip in (0, 1):
            postfix = dtype + ("_non_native" if flip else "")
            attrs = {"_dtype": dtype, "_flip": flip, "__module__": __name__}
            ns["BinnerScalar_" + postfix] = type("BinnerScalar_" + postfix, (_BinnerScalarBase,), dict(attrs))
            ns["BinnerOrdinal_" + postfix] = type("BinnerOrdinal_" + postfix, (_BinnerOrdinalBase,), dict(attrs))
            for kind in ("AggCount", "AggSum", "AggMin", "AggMax", "AggFirst", "AggSumMoment"):
                name = kind + "_" + postfix
                ns[name] = type(name, (Aggregator,), dict(attrs, _kind=kind))
            ns["AggNUnique_" + postfix] = type("AggNUnique_" + postfix, (_AggNUniqueBase,), dict(attrs))


_register()
