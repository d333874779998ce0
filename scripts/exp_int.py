"""C2's shape on integer binby columns (int32 / int64 x, y in [0, 1024) binned over 1024 bins,
count + sum of a float64 w): fast integer pass A against the generic pass A (VH_TILE_F32=0).
usage: python scripts/exp_int.py [rows] [reps]"""
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
w = DeviceArray.random(n, "uniform", seed=4)
for dt in ("int32", "int64"):
    x = DeviceArray.random(n, "randint", seed=2, a=0, b=1024, dtype=dt)
    y = DeviceArray.random(n, "randint", seed=3, a=0, b=1024, dtype=dt)

    def step():
        bx = getattr(superagg, "BinnerScalar_" + dt)("x", 0, 1024, 1024)
        by = getattr(superagg, "BinnerScalar_" + dt)("y", 0, 1024, 1024)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        c = superagg.AggCount_int64(grid)
        s = superagg.AggSum_float64(grid)
        s.set_data(w, 0)
        grid.bin([c, s])
        return np.asarray(c)

    for mode in ("1", "0"):
        os.environ["VH_TILE_F32"] = mode
        step()
        ts, ks = [], {}
        for _ in range(reps):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            step()
            _lib.synchronize()
            ts.append(time.perf_counter() - t0)
            _lib.timing_enable(False)
            for k in ("tile_scatter", "tile_scatter_int", "tile_reduce"):
                v = _lib.timing_read(k)[1]
                if v:
                    ks.setdefault(k, []).append(v)
        print(f"binners {dt} + float64 sum, VH_TILE_F32={mode}: {statistics.median(ts) * 1e3:7.3f} ms  "
              + "  ".join(f"{k} {statistics.median(v):.3f}" for k, v in ks.items()), flush=True)
    del x, y
