"""Where C2 pass A's time goes, one process (ablation build; results wrong by design): the
count+sum step with VH_TILE_DEBUG bits, interleaved over rounds -- 0 full, 128 no stream /
region stores, 32 no commit (loads, cell math, ranking), 96 no commit and no ranking.
usage: VAEX_AMD_LIB=vaex_amd/libvaexhip_ablation.so python scripts/exp_ablate_inproc.py [rows] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
modes = os.environ.get("DBGS", "0 128 32 96").split()


def step(with_sum):
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    grid = superagg.Grid([bx, by])
    aggs = [superagg.AggCount_int64(grid)]
    if with_sum:
        s = superagg.AggSum_float64(grid)
        s.set_data(w, 0)
        aggs.append(s)
    grid.bin(aggs)


res = {}
for r in range(rounds + 1):
    for ws in (True, False):
        for m in modes:
            os.environ["VH_TILE_DEBUG"] = m
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            step(ws)
            _lib.synchronize()
            _lib.timing_enable(False)
            if r:
                res.setdefault((ws, m), []).append(_lib.timing_read("tile_scatter_f64")[1])
for (ws, m), v in sorted(res.items()):
    print(f"{'count+sum' if ws else 'count-only':10s} VH_TILE_DEBUG={m:4s} pass A median {statistics.median(v):.3f} ms  min {min(v):.3f}", flush=True)
