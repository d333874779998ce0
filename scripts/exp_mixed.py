"""C2's shape with mixed column types (float64 x, y with a float32 w; float32 x, y with a
float64 w): pass-A kernel and step times, fast mixed kernels against the generic pass A
(VH_TILE_F32=0).  usage: python scripts/exp_mixed.py [rows] [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cols = {dt: (DeviceArray.random(n, "normal", seed=2, dtype=dt), DeviceArray.random(n, "normal", seed=3, dtype=dt),
             DeviceArray.random(n, "uniform", seed=4, dtype=dt)) for dt in ("float32", "float64")}


def step(bdt, vdt):
    x, y, _ = cols[bdt]
    w = cols[vdt][2]
    bx = getattr(superagg, "BinnerScalar_" + bdt)("x", -4.0, 4.0, 1024)
    by = getattr(superagg, "BinnerScalar_" + bdt)("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    c = superagg.AggCount_int64(grid)
    s = getattr(superagg, "AggSum_" + vdt)(grid)
    s.set_data(w, 0)
    grid.bin([c, s])
    return np.asarray(c)


for bdt, vdt in (("float64", "float32"), ("float32", "float64")):
    for mode in ("1", "0"):
        os.environ["VH_TILE_F32"] = mode
        step(bdt, vdt)
        ts, ks = [], {}
        for _ in range(reps):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            step(bdt, vdt)
            _lib.synchronize()
            ts.append(time.perf_counter() - t0)
            _lib.timing_enable(False)
            for k in ("tile_scatter", "tile_scatter_mixed", "tile_reduce"):
                v = _lib.timing_read(k)[1]
                if v:
                    ks.setdefault(k, []).append(v)
        print(f"binners {bdt} sum {vdt} VH_TILE_F32={mode}: {statistics.median(ts) * 1e3:7.3f} ms  "
              + "  ".join(f"{k} {statistics.median(v):.3f}" for k, v in ks.items()), flush=True)
