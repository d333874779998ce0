"""HBM-resident columns.

A :class:`DeviceArray` is a 1-d column living in the MI355X's HBM (allocated by
``libvaexhip``).  DataFrames built from DeviceArrays are binned in place: the
executor hands the device pointers straight to ``vh_grid_bin`` (no host staging),
which is how the 1e9-row benchmark columns stay resident.
"""
import ctypes

import numpy as np

from . import _lib


class DeviceArray:
    def __init__(self, length, dtype, _ptr=None, _owner=None):
        self.dtype = np.dtype(dtype)
        self.length = int(length)
        self._owner = _owner
        if _ptr is None:
            p = ctypes.c_void_p()
            _lib.call("vh_malloc", ctypes.byref(p), max(1, self.nbytes))
            self.ptr = p.value
            self._owns = True
        else:
            self.ptr = _ptr
            self._owns = False

    # ---- construction -------------------------------------------------------
    @classmethod
    def empty(cls, length, dtype):
        return cls(length, dtype)

    @classmethod
    def from_numpy(cls, ar):
        ar = np.ascontiguousarray(ar)
        if ar.ndim != 1:
            raise ValueError("Expected a 1d array")
        d = cls(len(ar), ar.dtype)
        if d.nbytes:
            _lib.call("vh_memcpy_htod", d.ptr, ar.ctypes.data, d.nbytes)
        return d

    @classmethod
    def random(cls, length, dist="normal", seed=0, a=0.0, b=1.0, dtype="float64"):
        """Synthetic column generated in HBM: dist 'uniform' [a, b), 'normal' (mean a, sd b),
        'randint' [a, b) (int32/int64), or the sorted layouts 'sorted_normal' (ascending normal
        quantiles, mean a, sd b) and 'sorted_int' ([a, b) in equal consecutive runs)."""
        d = cls(length, dtype)
        code = {"uniform": 0, "normal": 1, "randint": 2, "sorted_normal": 3, "sorted_int": 4}[dist]
        dcode, _ = _lib.dtype_code(d.dtype)
        _lib.call("vh_fill_random", d.ptr, d.length, dcode, code, seed, float(a), float(b))
        return d

    # ---- views / copies -----------------------------------------------------
    @property
    def nbytes(self):
        return self.length * self.dtype.itemsize

    @property
    def itemsize(self):
        return self.dtype.itemsize

    @property
    def ndim(self):
        return 1

    @property
    def shape(self):
        return (self.length,)

    def __len__(self):
        return self.length

    def __getitem__(self, item):
        if not isinstance(item, slice):
            raise TypeError("DeviceArray only supports contiguous slices")
        start, stop, step = item.indices(self.length)
        if step != 1:
            raise TypeError("DeviceArray only supports contiguous slices")
        stop = max(start, stop)
        return DeviceArray(stop - start, self.dtype, _ptr=self.ptr + start * self.itemsize,
                           _owner=self if self._owner is None else self._owner)

    def to_numpy(self, pinned=False):
        """A host copy; pinned: into page-locked memory from the library's block cache (read
        back by the copy kernel at the link rate; a pageable copy runs at ~17 GB/s)."""
        if pinned:
            from .hostops import _empty
            out = _empty(self.length, self.dtype)
        else:
            out = np.empty(self.length, self.dtype)
        if self.nbytes:
            _lib.call("vh_memcpy_dtoh", out.ctypes.data, self.ptr, self.nbytes)
        return out

    def __array__(self, dtype=None, copy=None):
        a = self.to_numpy()
        return a if dtype is None else a.astype(dtype)

    def __del__(self):
        if getattr(self, "_owns", False) and self.ptr:
            try:
                _lib.call("vh_free", self.ptr)
            except Exception:
                pass
            self.ptr = None

    def __repr__(self):
        return f"DeviceArray(length={self.length}, dtype={self.dtype})"


def is_device_array(x):
    return isinstance(x, DeviceArray)
