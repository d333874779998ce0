"""C2 with a row mask (a selection or filter: df.count(binby=[x, y], selection=...) sets one
keep mask on every aggregator): pass-A kernel and step times against the unmasked step.
usage: python scripts/exp_mask.py [rows] [reps]"""
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
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
keep = DeviceArray.random(n, "randint", seed=5, a=0, b=2, dtype="int8")  # 0 / 1 bytes


def step(masked, with_sum):
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
    if masked:
        for a in aggs:
            a.set_data_mask(keep)
    grid.bin(aggs)
    return [np.asarray(a) for a in aggs]


for with_sum in (True, False):
    for masked in (False, True):
        step(masked, with_sum)
        ts, ks = [], {}
        for _ in range(reps):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            out = step(masked, with_sum)
            _lib.synchronize()
            ts.append(time.perf_counter() - t0)
            _lib.timing_enable(False)
            for k in ("tile_sample", "tile_scatter", "tile_scatter_f64", "tile_reduce", "bin_fused_global", "bin_aggregate"):
                v = _lib.timing_read(k)[1]
                if v:
                    ks.setdefault(k, []).append(v)
        print(f"{'count+sum' if with_sum else 'count':9s} masked={masked!s:5s}: {statistics.median(ts) * 1e3:7.3f} ms  "
              + "  ".join(f"{k} {statistics.median(v):.3f}" for k, v in ks.items())
              + f"  count total {int(out[0].sum())}", flush=True)
