"""``vaex.superutils.ordered_set_<dtype>`` over the GPU hash set of libvaexhip.

Mirrors ``ordered_set`` (``packages/vaex-core/src/hash_primitives.hpp:417-621``;
bindings ``hash_primitives.cpp:26-73``): ``update``, ``key_array``, ``map_ordinal``,
``isin``, ``merge``, ``seal``, ``nan_count``/``null_count``/``has_nan``/``has_null``,
``nan_value``/``null_value``, ``fingerprint``, ``len()``, the ``create`` constructor
``ordered_set_<t>(keys, null_value, nan_count, null_count, fingerprint)`` and
``flatten_values``.

Ordinals are assigned in first-appearance order over all ``update`` calls -- what a
single-threaded reference ``update`` with ``nmaps = 1`` produces.  (With threads the
reference's order depends on interleaving and ``nmaps``; groupby results are compared
as key -> value maps)
"""
import ctypes

import numpy as np

from . import _lib
from .device import DeviceArray
from .superagg import _column

DTYPES = _lib.DTYPES


class _OrderedSetBase:
    _dtype = "int64"

    def __init__(self, *args):
        h = ctypes.c_void_p()
        _lib.call("vh_set_create", _lib.DTYPE_CODE[self._dtype], ctypes.byref(h))
        self._handle = h.value
        self.fingerprint = ""
        self.sealed = False
        if len(args) >= 4:
            # ordered_set::create(keys, null_value, nan_count, null_count, fingerprint)
            # (hash_primitives.hpp:468-516): keys in order get ordinals 0..n-1
            keys, null_value, nan_count, null_count = args[:4]
            keys = np.asarray(keys, dtype=self._dtype)
            mask = None
            if null_count:
                mask = np.zeros(len(keys), np.uint8)
                mask[int(null_value)] = 1
            self.update(keys, mask)
            if len(self) != len(keys):
                raise RuntimeError(f"key array of length {len(keys)} does not match expected length of {len(self)}")
            if bool(nan_count) != self.has_nan:
                raise RuntimeError("NaN found in data, while claiming there should be none" if self.has_nan
                                   else "no NaN found in data, while claiming there should be")
            if len(args) >= 5 and args[4] is not None:
                self.fingerprint = args[4]
            self.sealed = True

    # ---- building --------------------------------------------------------------
    def update(self, ar, *args, **kwargs):
        """update(keys[, mask], start_index=0, chunk_size=..., bucket_size=..., return_values=False)"""
        mask = None
        rest = list(args)
        if rest and (isinstance(rest[0], (np.ndarray, list, DeviceArray)) or rest[0] is None):
            mask = rest.pop(0)
        mask = kwargs.pop("mask", mask)
        # select (this build): only rows where select != 0 enter the set (a filtered or
        # selected chunk, evaluated on the device, without compacting it)
        select = kwargs.pop("select", None)
        return_values = kwargs.get("return_values", False)
        if np.ma.isMaskedArray(ar):
            m = np.ma.getmaskarray(ar)
            mask = m if mask is None else (np.asarray(mask, bool) | m)
            ar = ar.data
        if not isinstance(ar, DeviceArray):
            ar = np.ascontiguousarray(ar, dtype=self._dtype)
        kptr, n, _, _, loc, keep = _column(ar)
        mptr = None
        mkeep = None
        if mask is not None:
            mkeep = np.ascontiguousarray(mask, dtype=np.uint8) if not isinstance(mask, DeviceArray) else mask
            mptr = mkeep.ctypes.data if isinstance(mkeep, np.ndarray) else mkeep.ptr
        if select is not None:
            skeep = select if isinstance(select, DeviceArray) else np.ascontiguousarray(select, dtype=np.uint8)
            sptr = skeep.ptr if isinstance(skeep, DeviceArray) else skeep.ctypes.data
            _lib.call("vh_set_update_selected", self._handle, kptr, mptr, sptr, n, loc)
        else:
            _lib.call("vh_set_update", self._handle, kptr, mptr, n, loc)
        if return_values:
            ordinals = self.map_ordinal(ar).astype(np.int64)
            if mask is not None:
                ordinals[np.asarray(mask, bool)] = self.null_value
            return ordinals, np.zeros(len(ordinals), np.int16)
        return None

    def merge(self, others):
        if self.sealed:
            raise RuntimeError("hashmap is sealed, cannot merge")
        for o in others:
            keys = o.key_array()
            mask = None
            if o.has_null:
                mask = np.zeros(len(keys), np.uint8)
                mask[o.null_value] = 1
            self.update(keys, mask)

    def seal(self):
        self.sealed = True

    # ---- reading ---------------------------------------------------------------
    def _info(self):
        vals = [ctypes.c_int64() for _ in range(5)]
        _lib.call("vh_set_info", self._handle, *[ctypes.byref(v) for v in vals])
        return [v.value for v in vals]

    def __len__(self):
        return self._info()[0]

    def length(self):
        return len(self)

    nan_count = property(lambda self: self._info()[1])
    null_count = property(lambda self: self._info()[2])
    nan_value = property(lambda self: self._info()[3])
    null_value = property(lambda self: self._info()[4])
    has_nan = property(lambda self: self._info()[1] > 0)
    has_null = property(lambda self: self._info()[2] > 0)

    def key_array(self):
        n = len(self)
        out = np.empty(n, dtype=self._dtype)
        if n:
            _lib.call("vh_set_key_array", self._handle, out.ctypes.data)
        return out

    def keys(self):
        ka = self.key_array().tolist()
        if self.has_null:
            ka[self.null_value] = None
        return ka

    def _ordinal_dtype(self):
        n = len(self)
        return np.int8 if n < 2 ** 7 else np.int16 if n < 2 ** 15 else np.int32 if n < 2 ** 31 else np.int64

    def map_ordinal(self, keys):
        """key -> ordinal, -1 for unknown keys; dtype sized by len(set) (hash_primitives.hpp:543-583)."""
        out_dtype = np.dtype(self._ordinal_dtype())
        if isinstance(keys, DeviceArray):
            out = DeviceArray(len(keys), out_dtype)
            _lib.call("vh_set_map_ordinal", self._handle, keys.ptr, len(keys), _lib.LOC_DEVICE, out.ptr,
                      out_dtype.itemsize, _lib.LOC_DEVICE)
            return out
        if np.ma.isMaskedArray(keys):
            keys = keys.data
        keys = np.ascontiguousarray(keys, dtype=self._dtype)
        out = np.empty(len(keys), out_dtype)
        if len(keys):
            _lib.call("vh_set_map_ordinal", self._handle, keys.ctypes.data, len(keys), _lib.LOC_HOST,
                      out.ctypes.data, out_dtype.itemsize, _lib.LOC_HOST)
        return out

    def isin(self, values):
        return self.map_ordinal(np.asarray(values, dtype=self._dtype)) >= 0

    def flatten_values(self, values, map_index, out):
        out[:] = values  # one map: offsets are all 0 (hash_common::flatten_values)
        return out

    def __sizeof__(self):
        return len(self) * 16

    def __reduce__(self):
        keys = self.key_array()
        return (type(self), (keys, self.null_value, self.nan_count, self.null_count, self.fingerprint))

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h:
            try:
                _lib.call("vh_set_destroy", h)
            except Exception:
                pass
            self._handle = None


def _register():
    ns = globals()
    for dtype in DTYPES:
        name = "ordered_set_" + dtype
        ns[name] = type(name, (_OrderedSetBase,), {"_dtype": dtype, "__module__": __name__})


_register()


def ordered_set_type_from_dtype(dtype):
    """vaex.hash.ordered_set_type_from_dtype for primitive dtypes."""
    dt = np.dtype(dtype)
    if dt.kind in "mM":
        name = "int64"
    else:
        name = dt.newbyteorder("=").name
    return globals()["ordered_set_" + name]
