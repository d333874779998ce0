"""Experiment: per-row kernel time of the tiled pipeline vs chunk size (does the
Infinity Cache absorb the pass-A -> pass-B intermediate when a chunk's working set
fits in it?).  Prints per chunk size: kernel ms per 1e9 rows for each tile kernel."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1 << 28
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
K = ["tile_sample", "tile_scatter_f64", "tile_reduce"]
for with_sum in (False, True):
    for chunk in (1 << 21, 1 << 22, 1 << 23, 1 << 24, 1 << 25, 1 << 26, n):
        def run():
            bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
            by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
            grid = superagg.Grid([bx, by])
            aggs = [superagg.AggCount_int64(grid)]
            if with_sum:
                aggs.append(superagg.AggSum_float64(grid))
            for k in range(0, n, chunk):
                bx.set_data(x[k:k + chunk])
                by.set_data(y[k:k + chunk])
                if with_sum:
                    aggs[1].set_data(w[k:k + chunk], 0)
                grid.bin(aggs)
            return aggs
        run()
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        run()
        _lib.synchronize()
        t = time.perf_counter() - t0
        _lib.timing_enable(False)
        per = {}
        for k in K:
            c, ms = _lib.timing_read(k)
            per[k] = round(ms * 1e9 / n, 3)
        print(json.dumps({"sum": with_sum, "chunk": chunk, "wall_ms_per_1e9": round(t * 1e3 * 1e9 / n, 2),
                          "kernel_ms_per_1e9": per, "kernel_total": round(sum(per.values()), 3)}), flush=True)
