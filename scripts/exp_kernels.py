"""Median HIP-event kernel times of the C2 (count+sum, count-only), C3 (`auto`) and h2o q3
tile-path passes in this process, as one JSON line -- for A/Bs run as separate processes, so every
variant gets the same allocation sequence and hence the same scratch placement (two
libraries in one process own scratch at different places: a +-7 % effect on pass A,
DESIGN §5.10).  usage: [VAEX_AMD_LIB=...] [VH_...=...] python scripts/exp_kernels.py TAG [rows] [reps]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

tag = sys.argv[1]
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 9
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
df3 = vaex_amd.from_arrays(key=keys, v=x)
# h2o q3's shape: int32 key, int8 sum + float32 mean (two narrow slots packed in one stream)
v1 = DeviceArray.random(n, "randint", seed=6, a=5, b=15, dtype="int8")
v3 = DeviceArray.random(n, "normal", seed=7, dtype="float32")
dfq3 = vaex_amd.from_arrays(key=keys, v1=v1, v3=v3)


def c2(with_sum):
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    aggs = [superagg.AggCount_int64(grid)]
    if with_sum:
        s = superagg.AggSum_float64(grid)
        s.set_data(w, 0)
        aggs.append(s)
    grid.bin(aggs)
    return [np.asarray(a) for a in aggs]


out = {"tag": tag}
for name, f, ka in (("c2sum", lambda: c2(True), "tile_scatter_f64"), ("c2count", lambda: c2(False), "tile_scatter_f64"),
                    ("c3", lambda: df3.groupby("key", agg={"v": ["sum", "count"]}), "tile_scatter_ord"),
                    ("q3", lambda: dfq3.groupby("key").agg({"v1": "sum", "v3": "mean"}), "tile_scatter_ord")):
    f()
    a, b = [], []
    for _ in range(reps):
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        f()
        _lib.synchronize()
        _lib.timing_enable(False)
        a.append(_lib.timing_read(ka)[1])
        b.append(_lib.timing_read("tile_reduce")[1])
    out[name] = [round(statistics.median(a), 3), round(statistics.median(b), 3)]
print(json.dumps(out), flush=True)
