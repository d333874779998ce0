"""Does where the tile path's region scratch lands in HBM move C2 pass A?  Allocates a dummy
block of `gb` GB before the first C2 step (so the ~10 GB of regions the step allocates land
elsewhere), then times 6 C2 count+sum steps (HIP-event pass A / pass B ms).
usage: python scripts/exp_placement.py gb [rows]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

gb = float(sys.argv[1])
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 9
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
dummy = DeviceArray.empty(int(gb * 1e9 / 8), np.float64) if gb > 0 else None


def step():
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    count = superagg.AggCount_int64(grid)
    total = superagg.AggSum_float64(grid)
    total.set_data(w, 0)
    grid.bin([count, total])
    return count


step()
res = []
for _ in range(6):
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    step()
    _lib.synchronize()
    _lib.timing_enable(False)
    res.append((_lib.timing_read("tile_scatter_f64")[1], _lib.timing_read("tile_reduce")[1]))
a = sorted(r[0] for r in res)
b = sorted(r[1] for r in res)
print(f"dummy {gb:5.1f} GB  pass A min {a[0]:.3f} med {a[len(a) // 2]:.3f} ms   pass B min {b[0]:.3f} med {b[len(b) // 2]:.3f} ms", flush=True)
