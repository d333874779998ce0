"""ctypes binding of ``libvaexhip.so`` (C-ABI declared in ``include/vaexhip.h``).

The product path has no fallback: if the HIP library is missing this module raises
``ImportError`` and every GPU entry point fails loudly.
"""
import ctypes
import mmap
import os
import threading
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAEX_AMD_LIB", os.path.join(HERE, "libvaexhip.so"))

DTYPES = ["float64", "float32", "int64", "int32", "int16", "int8",
          "uint64", "uint32", "uint16", "uint8", "bool"]
DTYPE_CODE = {name: i for i, name in enumerate(DTYPES)}
AGG_KIND = {"AggCount": 0, "AggSum": 1, "AggMin": 2, "AggMax": 3, "AggFirst": 4, "AggSumMoment": 5, "AggNUnique": 6}
LOC_AUTO, LOC_HOST, LOC_DEVICE = 0, 1, 2

# every symbol the header declares, with (restype, argtypes)
_vp, _u64, _i32, _i64, _dbl = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_double
_p = ctypes.POINTER
SIGNATURES = {
    "vh_last_error": (ctypes.c_char_p, []),
    "vh_abi_version": (_i32, []),
    "vh_device_count": (_i32, [_p(_i32)]),
    "vh_set_device": (_i32, [_i32]),
    "vh_get_device": (_i32, [_p(_i32)]),
    "vh_synchronize": (_i32, []),
    "vh_malloc": (_i32, [_p(_vp), _u64]),
    "vh_free": (_i32, [_vp]),
    "vh_host_alloc": (_i32, [_p(_vp), _u64]),
    "vh_host_free": (_i32, [_vp, _u64]),
    "vh_host_cache_trim": (_i32, []),
    "vh_device_cache_trim": (_i32, []),
    "vh_host_register": (_i32, [_vp, _u64]),
    "vh_host_unregister": (_i32, [_vp]),
    "vh_memcpy_htod": (_i32, [_vp, _vp, _u64]),
    "vh_memcpy_dtoh": (_i32, [_vp, _vp, _u64]),
    "vh_memcpy_dtod": (_i32, [_vp, _vp, _u64]),
    "vh_memset": (_i32, [_vp, _i32, _u64]),
    "vh_fill_random": (_i32, [_vp, _u64, _i32, _i32, _u64, _dbl, _dbl]),
    "vh_timing_enable": (_i32, [_i32]),
    "vh_timing_reset": (_i32, []),
    "vh_timing_read": (_i32, [ctypes.c_char_p, _p(_u64), _p(_dbl)]),
    "vh_stream": (_i32, [_p(_vp)]),
    "vh_stat_read": (_i32, [ctypes.c_char_p, _p(_u64), _i32]),
    "vh_binner_scalar_create": (_i32, [ctypes.c_char_p, _i32, _i32, _dbl, _dbl, _u64, _p(_vp)]),
    "vh_binner_ordinal_create": (_i32, [ctypes.c_char_p, _i32, _i32, _u64, _u64, _p(_vp)]),
    "vh_binner_set_ordinal_create": (_i32, [ctypes.c_char_p, _vp, _u64, _p(_vp)]),
    "vh_binner_copy": (_i32, [_vp, _p(_vp)]),
    "vh_binner_destroy": (_i32, [_vp]),
    "vh_binner_set_data": (_i32, [_vp, _vp, _u64, _i32, _i32, _i32]),
    "vh_binner_set_data_mask": (_i32, [_vp, _vp, _u64, _i32, _i32]),
    "vh_binner_clear_data_mask": (_i32, [_vp]),
    "vh_binner_shape": (_i32, [_vp, _p(_u64)]),
    "vh_binner_size": (_i32, [_vp, _p(_u64)]),
    "vh_grid_create": (_i32, [_p(_vp), _i32, _p(_vp)]),
    "vh_grid_destroy": (_i32, [_vp]),
    "vh_grid_info": (_i32, [_vp, _p(_i32), _p(_u64), _p(_u64), _p(_u64)]),
    "vh_grid_bin": (_i32, [_vp, _p(_vp), _i32, _u64, _i32]),
    "vh_agg_create": (_i32, [_vp, _i32, _i32, _i32, ctypes.c_uint32, _p(_vp)]),
    "vh_agg_destroy": (_i32, [_vp]),
    "vh_agg_set_data": (_i32, [_vp, _vp, _u64, _i32, _i32, _i32, _i32]),
    "vh_agg_set_data_mask": (_i32, [_vp, _vp, _u64, _i32, _i32]),
    "vh_agg_clear_data_mask": (_i32, [_vp]),
    "vh_agg_set_selection_mask": (_i32, [_vp, _vp, _u64, _i32, _i32]),
    "vh_agg_nunique_export": (_i32, [_vp, _p(_u64), _vp, _vp, _vp, _vp]),
    "vh_agg_nunique_import": (_i32, [_vp, _u64, _vp, _vp, _vp, _vp]),
    "vh_agg_info": (_i32, [_vp, _p(_u64), _p(_i32), _p(_u64)]),
    "vh_agg_download": (_i32, [_vp, _vp, _u64]),
    "vh_agg_upload": (_i32, [_vp, _vp, _u64]),
    "vh_agg_download_order": (_i32, [_vp, _vp, _u64]),
    "vh_agg_occupancy": (_i32, [_vp, _u64, _u64, _vp]),
    "vh_agg_upload_order": (_i32, [_vp, _vp, _u64]),
    "vh_agg_device_ptr": (_i32, [_vp, _p(_vp), _p(_vp)]),
    "vh_agg_reduce": (_i32, [_vp, _p(_vp), _i32]),
    "vh_set_create": (_i32, [_i32, _p(_vp)]),
    "vh_set_destroy": (_i32, [_vp]),
    "vh_set_update": (_i32, [_vp, _vp, _vp, _u64, _i32]),
    "vh_set_update_selected": (_i32, [_vp, _vp, _vp, _vp, _u64, _i32]),
    "vh_set_seal": (_i32, [_vp]),
    "vh_set_info": (_i32, [_vp, _p(_i64), _p(_i64), _p(_i64), _p(_i64), _p(_i64)]),
    "vh_set_key_array": (_i32, [_vp, _vp]),
    "vh_set_map_ordinal": (_i32, [_vp, _vp, _u64, _i32, _vp, _i32, _i32]),
    "vh_minmax": (_i32, [_vp, _u64, _i32, _i32, _vp, _i32, _p(_dbl), _p(_dbl)]),
    "vh_minmax_sample": (_i32, [_vp, _u64, _i32, _u64, _p(_dbl), _p(_dbl)]),
    "vh_hashagg_create": (_i32, [_i32, _i32, _p(_i32), ctypes.c_uint32, _p(_vp)]),
    "vh_hashagg_destroy": (_i32, [_vp]),
    "vh_hashagg_update": (_i32, [_vp, _vp, _p(_vp), _u64, _i32]),
    "vh_hashagg_finish": (_i32, [_vp, _p(_u64)]),
    "vh_hashagg_read": (_i32, [_vp, _vp, _vp, _p(_vp), _p(_vp)]),
    "vh_hashagg_order_first": (_i32, [_vp, _vp, _u64, _i32]),
    "vh_dense_first_order": (_i32, [_vp, _u64, _i32, _i32, _i64, _u64, _vp, _u64, _vp]),
    "vh_dense_first_take": (_i32, [_vp, _u64, _i32, _i32, _i64, _u64, _vp, _i32, _u64, _i32, _vp, _vp, _vp, _i32, _vp]),
    "vh_host_take": (_i32, [_i32, _vp, _vp, _vp, _vp, _u64, _i32]),
    "vh_combine_keys": (_i32, [_u64, _i32, _p(_vp), _p(_i32), _p(_i64), _p(_i64), _vp]),
    "vh_dense_rank_i64": (_i32, [_u64, _vp, _vp, _vp, _p(_u64)]),
    "vh_decode_keys": (_i32, [_u64, _vp, _vp, _i32, _p(_i64), _p(_i64), _p(_i64), _p(_i32), _p(_vp)]),
    "vh_comm_unique_id": (_i32, [_vp]),
    "vh_comm_init": (_i32, [_vp, _i32, _i32, _p(_vp)]),
    "vh_comm_loopback": (_i32, [_i32, _p(_vp)]),
    "vh_comm_destroy": (_i32, [_vp]),
    "vh_comm_allreduce": (_i32, [_vp, _vp, _u64, _i32, _i32, _i32]),
    "vh_comm_allgather": (_i32, [_vp, _vp, _vp, _u64, _i32]),
    "vh_comm_alltoallv": (_i32, [_vp, _vp, _p(_u64), _vp, _p(_u64), _i32]),
    "vh_comm_barrier": (_i32, [_vp]),
    "vh_comm_agg_allreduce": (_i32, [_vp, _vp]),
    "vh_hashagg_exchange": (_i32, [_vp, _vp, _i32]),
    "vh_argsort": (_i32, [_u64, _vp, _i32, _vp]),
    "vh_expr_eval": (_i32, [_p(ctypes.c_uint32), _i32, _p(_u64), _i32, _p(_vp), _p(_i32), _i32, _u64, _i32, _vp]),
}

_lib = None


class HipError(RuntimeError):
    """A failed libvaexhip call (the reference raises RuntimeError from its C++ too)."""


def load_library(path):
    """ctypes handle of a libvaexhip build with every C-ABI signature bound."""
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: the HIP library must be built "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C vaex_amd/csrc)")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.vh_abi_version() != 1:
        raise ImportError("libvaexhip ABI version mismatch")
    return L


def lib():
    global _lib
    if _lib is None:
        _lib = load_library(LIB_PATH)
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().vh_last_error().decode(errors="replace")
        raise HipError(msg)


_TRACE = {} if os.environ.get("VAEX_AMD_TRACE_CALLS") else None


def call(name, *args):
    if _TRACE is None:
        check(getattr(lib(), name)(*args))
        return
    import time
    t0 = time.perf_counter()
    try:
        check(getattr(lib(), name)(*args))
    finally:
        n, tot = _TRACE.get(name, (0, 0.0))
        _TRACE[name] = (n + 1, tot + time.perf_counter() - t0)


def trace_report(reset=True):
    """{C-ABI function: (calls, seconds)} since the last report (VAEX_AMD_TRACE_CALLS=1)."""
    if _TRACE is None:
        return {}
    out = dict(_TRACE)
    if reset:
        _TRACE.clear()
    return out


def dtype_code(dtype):
    """(code, flip_endian) of a numpy dtype (find_type_from_dtype, utils.py:879-903:
    datetime/timedelta bin as int64, non-native byte order -> *_non_native)."""
    dt = np.dtype(dtype)
    flip = dt.byteorder not in ("<", "=", "|")
    native = dt.newbyteorder("=") if flip else dt
    if native.kind in "mM":
        name = "int64"
    else:
        name = native.name
    if name not in DTYPE_CODE:
        raise ValueError(f"dtype {dt} is not supported")
    return DTYPE_CODE[name], int(flip)


def device_count():
    n = ctypes.c_int(0)
    check(lib().vh_device_count(ctypes.byref(n)))
    return n.value


def synchronize():
    call("vh_synchronize")


def stat_read(name, reset=True):
    """An engine statistic (vh_stat_read), e.g. "tile_overflow_rows"."""
    v = ctypes.c_uint64()
    call("vh_stat_read", name.encode(), ctypes.byref(v), int(bool(reset)))
    return v.value


def timing_enable(on=True):
    call("vh_timing_enable", int(bool(on)))


def timing_reset():
    call("vh_timing_reset")


def timing_read(kernel):
    n, ms = ctypes.c_uint64(), ctypes.c_double()
    call("vh_timing_read", kernel.encode(), ctypes.byref(n), ctypes.byref(ms))
    return n.value, ms.value


class _PinnedBlock:
    """A page-locked host block (vh_host_alloc) that numpy arrays view; returned to the
    library's block cache when the last array over it is gone."""

    def __init__(self, n, dtype):
        dtype = np.dtype(dtype)
        self.nbytes = max(1, n * dtype.itemsize)
        p = ctypes.c_void_p()
        call("vh_host_alloc", ctypes.byref(p), self.nbytes)
        self.ptr = p.value
        self.__array_interface__ = {"shape": (n,), "typestr": dtype.str, "data": (self.ptr, False), "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().vh_host_free(self.ptr, self.nbytes)
            self.ptr = None


# ---- file mappings registered for direct DMA (vh_host_register) ------------------------
_REG_LOCK = threading.RLock()  # re-entrant: a finalizer may run from GC inside the lock
_MAPS = {}   # id(mmap) -> [address, live column count]
_ROOTS = {}  # id(root column array) -> id(mmap), or None when registration failed


def _release(key, mk):
    with _REG_LOCK:
        _ROOTS.pop(key, None)
        ent = _MAPS.get(mk)
        if ent is None:
            return
        ent[1] -= 1
        if ent[1] == 0:
            del _MAPS[mk]
            lib().vh_host_unregister(ent[0])


def host_register(a):
    """Register the file mapping under a host column (vaex_amd.open maps HDF5 columns
    with mmap) once, so the binning pipeline DMAs its chunks in place instead of copying
    them into pinned bounce buffers.  The registration lives while any column array over
    the mapping does (finalizers run before the arrays release the mapping).  A bin() call
    cannot race the unregistration: the binners / aggregators it reads hold their column
    arrays (and so the root array) until they are destroyed, and vh_host_unregister drains
    the device before it unpins.
    VH_HOST_REGISTER=0 turns this off.  Returns True when `a` lies in a registered mapping."""
    if os.environ.get("VH_HOST_REGISTER", "1") == "0" or not isinstance(a, np.ndarray) or a.nbytes < (64 << 20):
        return False
    root = a
    while isinstance(root.base, np.ndarray):
        root = root.base
    mv = root.base
    if not (isinstance(mv, memoryview) and isinstance(mv.obj, mmap.mmap)):
        return False
    key = id(root)
    with _REG_LOCK:
        if key in _ROOTS:
            return _ROOTS[key] is not None
        mm = mv.obj
        mk = id(mm)
        ent = _MAPS.get(mk)
        if ent is None:
            addr = np.frombuffer(mm, np.uint8).ctypes.data
            if lib().vh_host_register(addr, len(mm)) != 0:
                # e.g. more than the host can pin: the bounce-buffer pipeline streams it
                _ROOTS[key] = None
                weakref.finalize(root, _ROOTS.pop, key, None).atexit = False
                return False
            ent = _MAPS[mk] = [addr, 0]
        ent[1] += 1
        _ROOTS[key] = mk
        weakref.finalize(root, _release, key, mk).atexit = False
        return True


def pinned_empty(n, dtype):
    """1-d numpy array of n items in page-locked memory (fast D2H read-back target)."""
    return np.asarray(_PinnedBlock(int(n), dtype))


def trim_caches():
    """Return the library's cached blocks to the system: page-locked host blocks
    (vh_host_cache_trim) and the calling thread's device blocks (vh_device_cache_trim)."""
    call("vh_host_cache_trim")
    call("vh_device_cache_trim")
