"""Time the grid read-back (vh_agg_download into the pinned host image) of a 1e6-cell grid."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = 10_000_000
keys = DeviceArray.random(n, "randint", seed=5, a=0, b=1_000_000, dtype="int32")
if len(sys.argv) > 1:  # the bench's state first: 1e9-row C2 columns + one C2 query
    N = int(float(sys.argv[1]))
    x = DeviceArray.random(N, "normal", seed=2)
    y = DeviceArray.random(N, "normal", seed=3)
    w = DeviceArray.random(N, "uniform", seed=4)
    bx, by = superagg.BinnerScalar_float64("x", -4, 4, 1024), superagg.BinnerScalar_float64("y", -4, 4, 1024)
    bx.set_data(x)
    by.set_data(y)
    gg = superagg.Grid([bx, by])
    cc, ss = superagg.AggCount_int64(gg), superagg.AggSum_float64(gg)
    ss.set_data(w, 0)
    gg.bin([cc, ss])
    np.asarray(cc)
    print("C2 state ready", flush=True)
for it in range(5):
    b = superagg.BinnerOrdinal_int32("k", 1_000_000, 0)
    b.set_data(keys)
    g = superagg.Grid([b])
    c = superagg.AggCount_int64(g)
    g.bin([c])
    _lib.synchronize()
    t0 = time.perf_counter()
    a = np.asarray(c)
    t1 = time.perf_counter()
    h = _lib.pinned_empty(c._grid.length1d, np.int64)
    t2 = time.perf_counter()
    _lib.call("vh_agg_download", c._handle, h.ctypes.data, c._nbytes)
    t3 = time.perf_counter()
    p = np.empty(c._grid.length1d, np.int64)
    _lib.call("vh_agg_download", c._handle, p.ctypes.data, c._nbytes)
    t4 = time.perf_counter()
    print(f"asarray {1e3*(t1-t0):.3f} ms  pinned_empty {1e3*(t2-t1):.3f}  download->pinned {1e3*(t3-t2):.3f}  "
          f"download->pageable {1e3*(t4-t3):.3f}", flush=True)
    del a, h, p, c, g, b
