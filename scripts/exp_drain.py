"""C2 count+sum pass A with and without draining the prefetched batch before each commit
(VH_TILE_DRAIN=1 / 0: two instantiations of one kernel in one library, same scratch),
interleaved.  usage: python scripts/exp_drain.py [rows] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)


def step():
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    c, s = superagg.AggCount_int64(grid), superagg.AggSum_float64(grid)
    s.set_data(w, 0)
    grid.bin([c, s])


res = {"0": [], "1": []}
for r in range(rounds + 1):
    for m in (("0", "1") if r % 2 else ("1", "0")):
        os.environ["VH_TILE_DRAIN"] = m
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        step()
        _lib.synchronize()
        _lib.timing_enable(False)
        if r:
            res[m].append(_lib.timing_read("tile_scatter_f64")[1])
for m, v in res.items():
    print(f"drain={m}: pass A median {statistics.median(v):.3f} ms  min {min(v):.3f}  all {[round(t, 3) for t in v]}", flush=True)
