"""Interleaved comparison of VH_TILE_CHUNK_ROWS settings (pass A + pass B per row chunk,
so a chunk's regions can stay in the memory-side cache) on the C2 workload.
usage: python scripts/exp_chunkrows.py 0 16777216 33554432 ... [--rounds 8]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("chunks", nargs="+")
ap.add_argument("--rows", type=float, default=1e9)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
n = int(a.rows)
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)


def step(with_sum):
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


res = {}
for rnd in range(a.rounds + 1):
    for c in a.chunks:
        os.environ["VH_TILE_CHUNK_ROWS"] = c
        for ws in (True, False):
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            step(ws)
            _lib.synchronize()
            t = time.perf_counter() - t0
            _lib.timing_enable(False)
            if rnd == 0:
                continue
            kern = {k: _lib.timing_read(k)[1] for k in ("tile_scatter_f64", "tile_reduce")}
            r = res.setdefault((c, ws), {"wall": [], "A": [], "B": []})
            r["wall"].append(t * 1e3)
            r["A"].append(kern["tile_scatter_f64"])
            r["B"].append(kern["tile_reduce"])
    print(f"round {rnd}", flush=True)
for (c, ws), r in sorted(res.items(), key=lambda kv: (not kv[0][1], int(kv[0][0]))):
    print(f"{'count+sum' if ws else 'count'} chunk={c:>12}: wall {statistics.median(r['wall']):.3f} ms  "
          f"passA {statistics.median(r['A']):.3f}  passB {statistics.median(r['B']):.3f}")
