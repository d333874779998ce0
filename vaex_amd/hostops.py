"""Host-side finishing of large results (a groupby's 1e6-group label column, a mean's
division) in page-locked, already-faulted memory, split over a few threads: numpy releases
the GIL inside ufunc loops, and a fresh 8 MB output costs ~2000 page faults on first touch.
Results are bit-identical to the single numpy call (element-wise operations)."""
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib

MIN_SPLIT = 1 << 18  # below this a single call is cheaper than the hand-off
_pool = None
_pool_lock = threading.Lock()


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(8, n, int(os.environ.get("OMP_NUM_THREADS", n))))


def _get_pool():
    global _pool
    with _pool_lock:
        if _pool is None:
            _pool = ThreadPoolExecutor(_threads(), thread_name_prefix="vaex_amd_host")
    return _pool


def submit(fn, *args):
    """fn(*args) on the host pool (a Future): host work overlapped with a GPU pass, which
    releases the GIL while the library waits on the device."""
    return _get_pool().submit(fn, *args)


def _run(fn, n, min_split=MIN_SPLIT):
    """fn(i0, i1) over [0, n) in chunks, on the pool when n is large."""
    k = min(_threads(), max(1, n // min_split))
    if k == 1:
        fn(0, n)
        return
    pool = _get_pool()
    b = [n * i // k for i in range(k + 1)]
    for f in [pool.submit(fn, b[i], b[i + 1]) for i in range(k)]:
        f.result()


def _empty(n, dtype):
    """Page-locked output from the library's block cache (faulted in already); plain memory
    where the runtime has none to give (no device: the CPU-only tests)."""
    try:
        return _lib.pinned_empty(n, dtype)
    except _lib.HipError:
        return np.empty(n, dtype)


def true_divide(a, b):
    """a / b (numpy true division, divide / invalid ignored) for 1-d arrays."""
    a, b = np.asarray(a), np.asarray(b)
    if a.ndim != 1 or b.shape != a.shape or len(a) < MIN_SPLIT:
        with np.errstate(divide="ignore", invalid="ignore"):
            return a / b
    with np.errstate(divide="ignore", invalid="ignore"):
        out = _empty(len(a), np.true_divide(a[:1], b[:1]).dtype)

    def part(i0, i1):
        with np.errstate(divide="ignore", invalid="ignore"):
            np.true_divide(a[i0:i1], b[i0:i1], out=out[i0:i1])

    _run(part, len(a))
    return out


def arange(vmin, n, dtype, threads=True):
    """vmin .. vmin + n - 1 in `dtype` (every value representable in it).  threads=False: on
    the calling thread only (a job already running on the pool must not wait on it)."""
    dtype = np.dtype(dtype)
    if n < MIN_SPLIT:
        return np.arange(vmin, vmin + n, dtype=dtype)
    out = _empty(n, dtype)

    def part(i0, i1):
        out[i0:i1] = np.arange(vmin + i0, vmin + i1, dtype=dtype)

    if threads:
        _run(part, n)
    else:
        part(0, n)
    return out


def astype(a, dtype):
    """a.astype(dtype, copy=False) for a 1-d array (a C cast, element-wise)."""
    a, dtype = np.asarray(a), np.dtype(dtype)
    if a.dtype == dtype or a.ndim != 1 or len(a) < MIN_SPLIT:
        return a.astype(dtype, copy=False)
    out = _empty(len(a), dtype)

    def part(i0, i1):
        out[i0:i1] = a[i0:i1]

    _run(part, len(a))
    return out


def take(a, idx):
    """a[idx] for a 1-d array and an int64 index array (in range)."""
    return take_columns([a], idx)[0]


def take_columns(cols, idx):
    """[c[idx] for c in cols] (1-d arrays, int64 indices in range): one call of the library's
    host gather over the host threads, each thread one index range of every column (numpy's
    take holds the interpreter lock)."""
    import ctypes
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    cols = [np.asarray(c) for c in cols]
    fast = [c.ndim == 1 and c.dtype.itemsize in (1, 2, 4, 8) and not c.dtype.hasobject for c in cols]
    out = [None] * len(cols)
    if len(idx) >= MIN_SPLIT // 8:
        todo = [i for i, f in enumerate(fast) if f]
        srcs = [np.ascontiguousarray(cols[i]) for i in todo]
        dsts = [_empty(len(idx), s.dtype) for s in srcs]
        if todo:
            k = len(todo)
            _lib.call("vh_host_take", k, (ctypes.c_void_p * k)(*[d.ctypes.data for d in dsts]),
                      (ctypes.c_void_p * k)(*[s.ctypes.data for s in srcs]), (ctypes.c_int * k)(*[s.dtype.itemsize for s in srcs]),
                      idx.ctypes.data, len(idx), _threads())
        for i, d in zip(todo, dsts):
            out[i] = d
    for i, c in enumerate(cols):
        if out[i] is None:
            out[i] = np.take(c, idx)
    return out


def variance(sum_moment, sums, counts):
    """agg.py:207-213's finish, element-wise in the same operations (bit-identical to the
    numpy expression): mean = sum / count, m2 / count - mean ** 2, over the host threads (the
    inputs may be strided views of the grids' host images; the work is split along the last
    axis)."""
    sm = np.asarray(sum_moment, dtype=np.float64)
    s = np.asarray(sums, dtype=np.float64)
    c = np.asarray(counts)
    if sm.shape != s.shape or s.shape != c.shape or sm.size < MIN_SPLIT or sm.ndim == 0:
        with np.errstate(divide="ignore", invalid="ignore"):
            mean = s / c
            return sm / c - mean ** 2
    order = "F" if sm.ndim > 1 and not sm.flags.c_contiguous else "C"
    out = np.empty(sm.shape, np.float64, order=order)

    def part(i0, i1):
        sl = (Ellipsis, slice(i0, i1))
        with np.errstate(divide="ignore", invalid="ignore"):
            mean = s[sl] / c[sl]
            np.subtract(sm[sl] / c[sl], mean * mean, out=out[sl])

    last = sm.shape[-1]
    if last >= 8:
        _run(part, last, max(1, last // 8))
    else:
        part(0, last)
    return out


def minmax(a):
    """(a.min(), a.max()) of a non-empty 1-d integer array."""
    a = np.asarray(a)
    if a.ndim != 1 or len(a) < MIN_SPLIT:
        return a.min(), a.max()
    res = {}

    def part(i0, i1):
        res[i0] = (a[i0:i1].min(), a[i0:i1].max())

    _run(part, len(a))
    return min(v[0] for v in res.values()), max(v[1] for v in res.values())


def occupancy(a):
    """(nonzero count, first nonzero index, last nonzero index) of a 1-d array ((0, -1, -1)
    when all are zero): count_nonzero per chunk on the host threads; the first / last index
    is searched only inside chunks that are not fully occupied (a dense groupby's count grid
    usually is)."""
    a = np.asarray(a)
    n = len(a)
    res = {}

    def part(i0, i1):
        c = a[i0:i1]
        nz = int(np.count_nonzero(c))
        if nz == 0:
            res[i0] = (0, -1, -1)
        elif nz == i1 - i0:
            res[i0] = (nz, i0, i1 - 1)
        else:
            idx = np.flatnonzero(c)
            res[i0] = (nz, i0 + int(idx[0]), i0 + int(idx[-1]))

    if n:
        _run(part, n, MIN_SPLIT // 8)  # a streaming count: every thread's memory bandwidth helps
    parts = [res[k] for k in sorted(res)]
    nnz = sum(p[0] for p in parts)
    firsts = [p[1] for p in parts if p[0]]
    lasts = [p[2] for p in parts if p[0]]
    return nnz, (firsts[0] if firsts else -1), (lasts[-1] if lasts else -1)
