"""Where the C2 step's grid read-back time goes: np.asarray of the two 1027^2 grids after a bin,
split into the pinned host-image allocation and the vh_agg_download copy."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 7
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
ts = {"alloc": [], "download": [], "download_again": [], "dtoh_fresh": [], "dtoh_again": [], "asarray_count": [],
      "asarray_total": []}
keep = []
for it in range(30):
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    count = superagg.AggCount_int64(grid)
    total = superagg.AggSum_float64(grid)
    total.set_data(w, 0)
    grid.bin([count, total])
    _lib.synchronize()
    t0 = time.perf_counter()
    a = np.asarray(count)
    t1 = time.perf_counter()
    b = np.asarray(total)
    t2 = time.perf_counter()
    h = _lib.pinned_empty(grid.length1d, np.float64)
    t3 = time.perf_counter()
    _lib.call("vh_agg_download", total._handle, h.ctypes.data, total._nbytes)
    t4 = time.perf_counter()
    _lib.call("vh_agg_download", total._handle, h.ctypes.data, total._nbytes)
    t5 = time.perf_counter()
    d = DeviceArray.empty(grid.length1d, np.float64)
    _lib.call("vh_memcpy_dtoh", h.ctypes.data, d.ptr, total._nbytes)
    t6 = time.perf_counter()
    _lib.call("vh_memcpy_dtoh", h.ctypes.data, d.ptr, total._nbytes)
    t7 = time.perf_counter()
    keep = [a, b, h, d]
    if it >= 5:
        ts["asarray_count"].append(t1 - t0)
        ts["asarray_total"].append(t2 - t1)
        ts["alloc"].append(t3 - t2)
        ts["download"].append(t4 - t3)
        ts["download_again"].append(t5 - t4)
        ts["dtoh_fresh"].append(t6 - t5)
        ts["dtoh_again"].append(t7 - t6)
for k, v in ts.items():
    print(f"{k:15s} median {np.median(v) * 1e6:8.1f} us  min {min(v) * 1e6:8.1f} us")
