"""Same-process A/B of library builds on the C2 workload: the builds are loaded side by
side and their steps interleaved, so clock and box drift hit every build alike.

usage: python scripts/ab_inproc.py lib1.so lib2.so ... [--rows 1e9] [--rounds 12]
Prints the median step / per-kernel times per build (count+sum and count-only)."""
import argparse
import gc
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

KERNELS = ["tile_sample", "tile_scatter_f64", "tile_scatter_ord", "tile_scatter_set", "tile_scatter", "tile_reduce", "minmax", "ha_sample",
           "ha_scatter_f64", "ha_reduce", "ha_finish", "set_sample", "set_insert", "set_reduce"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--workloads", default="c2sum,c2count", help="c2sum,c2count,c2mm,c2var,c3,c3mm,c3fused,c3set")
    a = ap.parse_args()
    libs = [_lib.load_library(os.path.abspath(p)) for p in a.libs]
    _lib._lib = libs[0]
    n = int(a.rows)
    x = DeviceArray.random(n, "normal", seed=2)
    y = DeviceArray.random(n, "normal", seed=3)
    w = DeviceArray.random(n, "uniform", seed=4)
    workloads = a.workloads.split(",")
    if any(w.startswith("c3") for w in workloads):
        import vaex_amd
        keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
        df3 = vaex_amd.from_arrays(key=keys, v=x)

    def step(wl):
        if wl == "c3":
            df3.groupby("key", agg={"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v")})
            return
        if wl == "c3mm":
            df3.groupby("key", agg={"v": ["sum", "count", "min", "max"]}, assume_sparse=True)
            return
        if wl in ("c3fused", "c3fused0"):  # c3fused0: no count(v) (count(*) only)
            from vaex_amd.hashagg import HashAgg
            ha = HashAgg(keys.dtype, [x.dtype], [wl == "c3fused"])
            ha.update(keys, [x])
            ha.finish()
            return
        if wl == "c3set":
            from vaex_amd import superutils
            superutils.ordered_set_int32().update(keys)
            return
        with_sum = wl in ("c2sum", "c2mm", "c2var")
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        aggs = [superagg.AggCount_int64(grid)]
        if with_sum:
            aggs.append(superagg.AggSum_float64(grid))
            aggs[1].set_data(w, 0)
        if wl == "c2mm":
            aggs += [superagg.AggMin_float64(grid), superagg.AggMax_float64(grid)]
        if wl == "c2var":
            aggs.append(superagg.AggSumMoment_float64(grid, 2))
        for ag in aggs[2:]:
            ag.set_data(w, 0)
        grid.bin(aggs)

    res = {(i, wl): {k: [] for k in KERNELS} for i in range(len(libs)) for wl in workloads}
    for rnd in range(a.rounds + 1):
        for i, L in enumerate(libs):
            _lib._lib = L
            for ws in workloads:
                _lib.synchronize()
                _lib.timing_reset()
                _lib.timing_enable(True)
                step(ws)
                _lib.synchronize()
                _lib.timing_enable(False)
                gc.collect()
                if rnd == 0:
                    continue  # warm-up round
                for k in KERNELS:
                    c, ms = _lib.timing_read(k)
                    if c:
                        res[(i, ws)][k].append(ms / c)
        print(f"round {rnd} done", flush=True)
    _lib._lib = libs[0]
    for ws in workloads:
        print(ws)
        for i, p in enumerate(a.libs):
            med = {k: round(statistics.median(v), 3) for k, v in res[(i, ws)].items() if v}
            mn = {k: round(min(v), 3) for k, v in res[(i, ws)].items() if v}
            print(f"  {os.path.basename(p):28s} median {med}  min {mn}")


if __name__ == "__main__":
    main()
