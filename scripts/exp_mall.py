"""Does the tile path's partition exchange stay in the 256 MB memory-side cache when a pass
covers few rows?  Per-row cost of pass A / pass B of the C2 count+sum (and count-only)
query at several row counts on resident columns (regions ~10 B/row for count+sum)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    x = DeviceArray.random(N, "normal", seed=2)
    y = DeviceArray.random(N, "normal", seed=3)
    w = DeviceArray.random(N, "uniform", seed=4)
    for sums in (True, False):
        for n in (2 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20, 256 << 20, N):
            if n > N:
                continue
            xs, ys, ws = x[:n], y[:n], w[:n]

            def step():
                bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
                by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
                bx.set_data(xs)
                by.set_data(ys)
                grid = superagg.Grid([bx, by])
                aggs = [superagg.AggCount_int64(grid)]
                if sums:
                    aggs.append(superagg.AggSum_float64(grid))
                    aggs[1].set_data(ws, 0)
                grid.bin(aggs)

            reps = max(3, min(50, int(2e9 // n)))
            for _ in range(2):
                step()
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            for _ in range(reps):
                step()
            _lib.synchronize()
            t = (time.perf_counter() - t0) / reps
            _lib.timing_enable(False)
            per = {}
            for k in ("tile_sample", "tile_scatter_f64", "tile_reduce"):
                c, ms = _lib.timing_read(k)
                if c:
                    per[k] = ms / c
            a = per.get("tile_scatter_f64", 0)
            b = per.get("tile_reduce", 0)
            print(f"sums={sums} n={n:>11d} step={t*1e3:8.3f} ms  A={a:8.4f} ms ({a*1e6/n:6.3f} ns/row)  "
                  f"B={b:8.4f} ms ({b*1e6/n:6.3f} ns/row)", flush=True)


if __name__ == "__main__":
    main()
