"""Helpers restated from ``packages/vaex-core/vaex/utils.py`` for the binning path."""
import numpy as np


def find_type_from_dtype(namespace, prefix, dtype, transient=True, support_non_native=True):
    """utils.py:879-903: prefix + dtype name (+ '_non_native'); datetime/timedelta -> int64."""
    dt = np.dtype(dtype)
    postfix = str(dt.newbyteorder("=") if dt.byteorder not in "<=|" else dt)
    if dt.kind in "mM":
        postfix = "int64"
    if support_non_native and dt.kind != "O" and dt.byteorder not in ("<", "=", "|"):
        postfix += "_non_native"
    name = prefix + postfix
    if hasattr(namespace, name):
        return getattr(namespace, name)
    raise ValueError("Could not find a class (%s), seems %s is not supported" % (name, dt))


def extract_central_part(ar):
    """utils.py:919-920 -- strip the nan/underflow/overflow cells [2:-1] of every axis."""
    return ar[(slice(2, -1),) * ar.ndim]


def required_dtype_for_max(N, signed=True):
    """utils.py:947-956."""
    dtypes = [np.int8, np.int16, np.int32, np.int64] if signed else [np.uint8, np.uint16, np.uint32, np.uint64]
    for dtype in dtypes:
        if N <= np.iinfo(dtype).max:
            return np.dtype(dtype)
    raise ValueError(f"Cannot store a max value on {N} inside an uint64/int64")


def label_dtype(key_dtype, vmin, vmax):
    """dtype of groupby labels for an integer key spanning [vmin, vmax]: signed keys are
    down-cast to ``required_dtype_for_max(max)`` (groupby.py:131-133), unsigned keep their
    dtype.  Unlike the reference, a minimum below that dtype's range widens it instead of
    wrapping (the reference's astype would wrap e.g. int32 -1000 into int8)."""
    key_dtype = np.dtype(key_dtype)
    if key_dtype.kind != "i":
        return key_dtype
    dt = required_dtype_for_max(int(vmax))
    while int(vmin) < np.iinfo(dt).min:
        dt = required_dtype_for_max(np.iinfo(dt).max + 1)
    return dt


def _expand_shape(shape, dimension):
    """utils.py:793-798."""
    if isinstance(shape, (tuple, list)):
        assert len(shape) == dimension, "wants to expand shape %r to dimension %d" % (shape, dimension)
        return tuple(shape)
    return (shape,) * dimension


def _expand_limits(limits, dimension):
    """utils.py:801-807."""
    if isinstance(limits, (tuple, list, np.ndarray)) and \
            (isinstance(limits[0], (tuple, list, np.ndarray)) or isinstance(limits[0], str) or limits[0] is None):
        assert len(limits) == dimension, "wants to expand shape %r to dimension %d" % (limits, dimension)
        return tuple(limits)
    return (limits,) * dimension


def listify(*args):
    """utils.py listify: (waslist, [lists...])."""
    if isinstance(args[0], (list, tuple)):
        return True, [list(a) if isinstance(a, (list, tuple)) else [a] for a in args]
    return False, [[a] for a in args]


def unlistify(waslist, *args):
    if waslist:
        return args[0] if len(args) == 1 else args
    values = [a[0] for a in args]
    return values[0] if len(values) == 1 else values


def div_ceil(n, d):
    return (n + d - 1) // d


def as_contiguous(ar):
    return ar if ar.flags["C_CONTIGUOUS"] else ar.copy()
