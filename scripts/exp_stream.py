"""Stream layout vs per-tile regions for the tile path (VH_TILE_STREAM=1 / 0), same process,
interleaved: C2 count-only and count+sum (1027^2, 1e9 rows) and C3 dense groupby pass A / B
by HIP events, and the two layouts' grids compared (counts exact, sums 1e-9 relative).
usage: python scripts/exp_stream.py [rows] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)


def c2(with_sum):
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
    return [np.asarray(a).copy() for a in aggs]


def timed(f, kernels):
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    r = f()
    _lib.synchronize()
    t = time.perf_counter() - t0
    _lib.timing_enable(False)
    return r, t * 1e3, {k: _lib.timing_read(k)[1] for k in kernels}


def c2var():
    df = vaex_amd.from_arrays(x=x, y=y, w=w)
    return [np.asarray(df.var("w", binby=["x", "y"], limits=[[-4.0, 4.0], [-4.0, 4.0]], shape=1024))]


K = ["tile_scatter_f64", "tile_reduce"]
only = os.environ.get("EXP_ONLY", "")
res = {}
for name, f in (("count", lambda: c2(False)), ("count+sum", lambda: c2(True)), ("var", c2var)):
    if only and only != name:
        continue
    out = {"0": [], "1": []}
    grids = {}
    for rep in range(reps + 1):
        for mode in ("1", "0") if rep % 2 else ("0", "1"):
            os.environ["VH_TILE_STREAM"] = mode
            r, ms, per = timed(f, K)
            if rep:
                out[mode].append((ms, per["tile_scatter_f64"], per["tile_reduce"]))
            grids[mode] = r
    same = all(np.array_equal(a, b) if a.dtype.kind in "iu" else np.allclose(a, b, rtol=1e-9, atol=0, equal_nan=True)
               for a, b in zip(grids["0"], grids["1"]))
    for mode in ("0", "1"):
        a = np.array(out[mode])
        print(f"{name:10s} stream={mode}  step {np.median(a[:, 0]):7.3f} ms  pass A {np.median(a[:, 1]):6.3f} "
              f"(min {a[:, 1].min():6.3f})  pass B {np.median(a[:, 2]):6.3f}", flush=True)
    print(f"{name:10s} grids equal across layouts: {same}", flush=True)

# C3 dense groupby (auto route)
if only and only != "c3":
    sys.exit(0)
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)
KO = ["tile_scatter_ord", "tile_reduce"]
out = {"0": [], "1": []}
got = {}
for rep in range(reps + 1):
    for mode in ("1", "0") if rep % 2 else ("0", "1"):
        os.environ["VH_TILE_STREAM"] = mode
        r, ms, per = timed(lambda: df.groupby("key", agg={"v": ["sum", "count"]}), KO)
        if rep:
            out[mode].append((ms, per["tile_scatter_ord"], per["tile_reduce"]))
        got[mode] = (r["key"].to_numpy(), r["v"].to_numpy(), r["v_sum"].to_numpy())
for mode in ("0", "1"):
    a = np.array(out[mode])
    print(f"C3 auto    stream={mode}  query {np.median(a[:, 0]):7.3f} ms  pass A {np.median(a[:, 1]):6.3f}  "
          f"pass B {np.median(a[:, 2]):6.3f}", flush=True)
print("C3 equal across layouts:", bool(np.array_equal(got["0"][0], got["1"][0]) and np.array_equal(got["0"][1], got["1"][1])
                                       and np.allclose(got["0"][2], got["1"][2], rtol=1e-9, atol=1e-12)), flush=True)
