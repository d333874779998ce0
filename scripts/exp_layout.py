"""C2 pass A against the layout of its region scratch, in one process (one allocation):
VH_TILE_WGPAD (entries between workgroup blocks), VH_TILE_EOFF / VH_TILE_VOFF (entry / value
array start offsets), rotated over two rounds; HIP-event ms.  usage: python scripts/exp_layout.py [dummy_gb]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
n = 10 ** 9
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


combos = [(0, 0, 0), (8, 0, 0), (64, 0, 0), (256, 0, 0), (1024, 0, 0), (8200, 0, 0), (0, 0, 32), (0, 0, 256),
          (0, 0, 4096), (0, 0, 262144), (0, 128, 0), (0, 2048, 0), (0, 2048, 262144 + 256)]
# the largest padding first: the scratch is allocated once, at its largest
os.environ["VH_TILE_WGPAD"], os.environ["VH_TILE_EOFF"], os.environ["VH_TILE_VOFF"] = "8200", "2048", str(262144 + 256)
step()
res = {}
for rnd in range(2):
    for c in (combos if rnd == 0 else combos[::-1]):
        os.environ["VH_TILE_WGPAD"], os.environ["VH_TILE_EOFF"], os.environ["VH_TILE_VOFF"] = (str(v) for v in c)
        step()
        for _ in range(2):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            step()
            _lib.synchronize()
            _lib.timing_enable(False)
            res.setdefault(c, []).append(_lib.timing_read("tile_scatter_f64")[1])
print(f"dummy {gb} GB")
for c in combos:
    print("wgpad %6d eoff %5d voff %7d  pass A min %.3f max %.3f ms" % (c + (min(res[c]), max(res[c]))), flush=True)
