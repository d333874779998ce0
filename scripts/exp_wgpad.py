"""C2 count+sum pass A against the spacing of the pass-A workgroups' streams (VH_TILE_WGPAD
extra entries between consecutive streams; one scratch, the largest first), interleaved:
do the 256 write fronts, spaced one stream apart, alias in the memory channels?
usage: python scripts/exp_wgpad.py [rows] [rounds] [pads...]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pads = sys.argv[3:] or ["65536", "4104", "1032", "264", "136", "8", "0"]
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


res = {p: [] for p in pads}
for r in range(rounds + 1):
    for p in (pads if r % 2 == 0 else pads[::-1]):
        os.environ["VH_TILE_WGPAD"] = p
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        step()
        _lib.synchronize()
        _lib.timing_enable(False)
        if r:
            res[p].append(_lib.timing_read("tile_scatter_f64")[1])
for p in pads:
    v = res[p]
    print(f"wgpad {int(p):6d} entries: pass A median {statistics.median(v):.3f} ms  min {min(v):.3f}", flush=True)
