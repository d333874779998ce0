"""XCD-resident tile path vs the two-pass path: parity (counts exact, sums 1e-6) and
timing of C2 count+sum / count-only at several row counts and distributions.
Usage: python scripts/exp_resident.py [rows ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    sizes = [int(float(a)) for a in sys.argv[1:]] or [1 << 22, (1 << 24) + 4096 * 3 + 2, 100_000_000, 1_000_000_000]
    os.environ["VH_RES_MIN_ROWS"] = str(1 << 20)
    N = max(sizes)
    cols = {"normal": (DeviceArray.random(N, "normal", seed=2), DeviceArray.random(N, "normal", seed=3)),
            "uniform": (DeviceArray.random(N, "uniform", seed=5), DeviceArray.random(N, "uniform", seed=6))}
    w = DeviceArray.random(N, "uniform", seed=4)
    for dist, (x, y) in cols.items():
        lo, hi = (-4.0, 4.0) if dist == "normal" else (0.0, 1.0)
        for n in sizes:
            for sums in (True, False):
                xs, ys, ws = x[:n], y[:n], w[:n]

                def step():
                    bx = superagg.BinnerScalar_float64("x", lo, hi, 1024)
                    by = superagg.BinnerScalar_float64("y", lo, hi, 1024)
                    bx.set_data(xs)
                    by.set_data(ys)
                    grid = superagg.Grid([bx, by])
                    aggs = [superagg.AggCount_int64(grid)]
                    if sums:
                        aggs.append(superagg.AggSum_float64(grid))
                        aggs[1].set_data(ws, 0)
                    grid.bin(aggs)
                    return [np.asarray(a).copy() for a in aggs]

                res = {}
                tms = {}
                for mode in ("0", "1", "2"):
                    os.environ["VH_RESIDENT"] = mode
                    r = step()
                    reps = 5 if n >= 10**8 else 3
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
                    for k in ("tile_sample", "tile_scatter_f64", "tile_resident", "tile_reduce"):
                        c, ms = _lib.timing_read(k)
                        if c:
                            per[k] = round(ms / c, 4)
                    res[mode] = r
                    tms[mode] = (round(t * 1e3, 3), per)
                ok = True
                for mode in ("1", "2"):
                    ok &= np.array_equal(res[mode][0], res["0"][0])
                    if sums:
                        ok &= np.allclose(res[mode][1], res["0"][1], rtol=1e-9, atol=1e-9)
                print(f"{dist:8s} n={n:>11d} sums={sums!s:5s} equal={ok} tot={int(res['1'][0].sum())} "
                      f"two-pass={tms['0']} l2={tms['1']} wt={tms['2']}", flush=True)
    os.environ["VH_RESIDENT"] = "1"


if __name__ == "__main__":
    main()
