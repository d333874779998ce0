"""The bench's C2 step (count + sum(w) on 1027^2 cells, grids read back) six times, with host
timestamps per phase, for a rocprofv3 kernel / copy timeline: where the step's time outside
the kernels goes.  usage: python scripts/exp_c2_steps.py [rows]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
for it in range(6):
    _lib.synchronize()
    t = [time.perf_counter()]
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    count = superagg.AggCount_int64(grid)
    total = superagg.AggSum_float64(grid)
    total.set_data(w, 0)
    t.append(time.perf_counter())
    grid.bin([count, total])
    t.append(time.perf_counter())
    a, b = np.asarray(count), np.asarray(total)
    t.append(time.perf_counter())
    del count, total, grid, a, b
    t.append(time.perf_counter())
    print(f"step {it}: setup {1e3 * (t[1] - t[0]):.3f}  bin {1e3 * (t[2] - t[1]):.3f}  read-back {1e3 * (t[3] - t[2]):.3f}  "
          f"free {1e3 * (t[4] - t[3]):.3f}  total {1e3 * (t[4] - t[0]):.3f} ms", flush=True)
