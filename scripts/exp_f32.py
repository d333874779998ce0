"""Binning of float32 columns (vaex files often store float32): the C2 shape (2-D 1024^2
count + sum) and small grids, kernel times per pass and the end-to-end step, against the
float64 columns of the same values.  usage: [F32_CASES=small] python scripts/exp_f32.py [rows] [reps]"""
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
cols = {}
for dt in ("float32", "float64"):
    cols[dt] = [DeviceArray.random(n, "normal", seed=2, dtype=dt), DeviceArray.random(n, "normal", seed=3, dtype=dt),
                DeviceArray.random(n, "uniform", seed=4, dtype=dt)]


def step(dt, bins, with_sum):
    x, y, w = cols[dt]
    cls = getattr(superagg, "BinnerScalar_" + dt)
    bx, by = cls("x", -4.0, 4.0, bins), cls("y", -4.0, 4.0, bins)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    aggs = [superagg.AggCount_int64(grid)]
    if with_sum:
        s = getattr(superagg, "AggSum_" + dt)(grid)
        s.set_data(w, 0)
        aggs.append(s)
    grid.bin(aggs)
    return [np.asarray(a) for a in aggs]


CASES = {"tile": ((1024, True), (1024, False), (256, True)), "small": ((64, True), (64, False), (128, False))}
for bins, with_sum in CASES[os.environ.get("F32_CASES", "tile")]:
    ref = None
    for dt in ("float64", "float32"):
        step(dt, bins, with_sum)
        ts, ks = [], {}
        for _ in range(reps):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            out = step(dt, bins, with_sum)
            _lib.synchronize()
            ts.append(time.perf_counter() - t0)
            _lib.timing_enable(False)
            for k in ("tile_sample", "tile_scatter", "tile_scatter_f64", "tile_scatter_f32", "tile_reduce", "bin_small_f64",
                      "bin_fused_lds", "bin_fused_global", "bin_cells", "bin_aggregate_lds", "bin_aggregate", "bin_indices", "bin_small_f32"):
                v = _lib.timing_read(k)[1]
                if v:
                    ks.setdefault(k, []).append(v)
        if ref is None:
            ref = out
        same = all(np.array_equal(a, b) for a, b in zip(out[:1], ref[:1]))
        print(f"{bins}^2 {'count+sum' if with_sum else 'count':9s} {dt}: {statistics.median(ts) * 1e3:7.3f} ms  "
              + "  ".join(f"{k} {statistics.median(v):.3f}" for k, v in ks.items()) + f"  counts == f64: {same}",
              flush=True)
