"""Experiment: time the tiled-path kernels under VH_TILE_DEBUG switches (1: no region
stores, 2: no batch_commit, 4: no LDS rank) on the C2 workload."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the switches exist only in the ablation build (make -C vaex_amd/csrc ablation)
os.environ.setdefault("VAEX_AMD_LIB", os.path.join(ROOT, "vaex_amd", "libvaexhip_ablation.so"))
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)


def run(with_sum, reps=5):
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    aggs = [superagg.AggCount_int64(grid)]
    if with_sum:
        aggs.append(superagg.AggSum_float64(grid))
        aggs[1].set_data(w, 0)
    grid.bin(aggs)
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(reps):
        grid.bin(aggs)
    _lib.timing_enable(False)
    out = {}
    for k in ("tile_scatter_f64", "tile_scatter", "tile_reduce", "tile_sample"):
        c, ms = _lib.timing_read(k)
        if c:
            out[k] = round(ms / c, 3)
    return out


for dbg in os.environ.get("EXP_DEBUG", "0,1,2,4,6").split(","):
    os.environ["VH_TILE_DEBUG"] = dbg
    for ws in (False, True):
        print(f"debug={dbg} sum={ws}", run(ws), flush=True)
