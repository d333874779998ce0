"""C2 query then dense groupby (bench order), for a rocprofv3 kernel/copy timeline."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vaex_amd  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = 10 ** 9
if os.environ.get("WITH_C2", "1") == "1":
    x = DeviceArray.random(n, "normal", seed=2)
    y = DeviceArray.random(n, "normal", seed=3)
    w = DeviceArray.random(n, "uniform", seed=4)
    for _ in range(2):
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        c, s = superagg.AggCount_int64(grid), superagg.AggSum_float64(grid)
        s.set_data(w, 0)
        grid.bin([c, s])
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)
for it in range(4):
    _lib.synchronize()
    t0 = time.perf_counter()
    dfg = df.groupby("key", agg={"v": ["sum", "count"]})
    _lib.synchronize()
    print("auto", it, round((time.perf_counter() - t0) * 1e3, 2), "ms", flush=True)
