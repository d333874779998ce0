"""C-ABI call log of one C2 bench step (count + sum(w) on the 1027^2 grid, grids read back),
after warm-up: each library call's start / end relative to the step start (host clock), and
the library's own timeline of the binning call (VAEX_AMD_TRACE_CALLS-free: HIP-event kernel
times).  usage: python scripts/exp_c2_calls.py [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)


def step():
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    count = superagg.AggCount_int64(grid)
    total = superagg.AggSum_float64(grid)
    total.set_data(w, 0)
    grid.bin([count, total])
    return np.asarray(count), np.asarray(total)


for _ in range(3):
    step()
_lib.synchronize()
log = []
orig = _lib.call
T0 = [0.0]


def traced(name, *a):
    t = time.perf_counter()
    try:
        return orig(name, *a)
    finally:
        log.append((name, t - T0[0], time.perf_counter() - T0[0]))


_lib.call = traced
for rep in range(3):
    log.clear()
    _lib.synchronize()
    T0[0] = time.perf_counter()
    step()
    _lib.synchronize()
    total = time.perf_counter() - T0[0]
_lib.call = orig
print(f"step {total * 1e3:.3f} ms")
prev = 0.0
for name, a, b in log:
    print(f"{a * 1e3:8.3f} +{(a - prev) * 1e3:6.3f} host | {(b - a) * 1e3:7.3f} in call  {name}")
    prev = b
_lib.timing_reset()
_lib.timing_enable(True)
step()
_lib.synchronize()
_lib.timing_enable(False)
print({k: round(_lib.timing_read(k)[1], 4) for k in ("tile_sample", "tile_scatter_f64", "tile_reduce") if _lib.timing_read(k)[0]})
