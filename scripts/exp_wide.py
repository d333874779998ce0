"""A/B of the tile path's pass-A stream-out modes in one process (VH_TILE_WIDE: 0 = per-entry
stores, bit 0 = wide 16-byte stores of 8-aligned padded runs, bit 1 = non-temporal cell
stores, bit 2 = non-temporal value stores).  C2 count+sum, C2 count-only and the C3 dense
ordinal grid at 1e9 rows; per-kernel HIP-event milliseconds, modes rotated over rounds."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
modes = [int(m) for m in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "5", "7", "3"])]
x = DeviceArray.random(n, "normal", seed=2)
y = DeviceArray.random(n, "normal", seed=3)
w = DeviceArray.random(n, "uniform", seed=4)
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)


def c2(with_sum):
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
    bx.set_data(x)
    by.set_data(y)
    g = superagg.Grid([bx, by])
    c = superagg.AggCount_int64(g)
    aggs = [c]
    if with_sum:
        s = superagg.AggSum_float64(g)
        s.set_data(w, 0)
        aggs.append(s)
    g.bin(aggs)
    return [np.asarray(a).copy() for a in aggs]


def c3():
    b = superagg.BinnerOrdinal_int32("k", 1_000_000, 5)
    b.set_data(keys)
    g = superagg.Grid([b])
    c = superagg.AggCount_int64(g)
    s = superagg.AggSum_float64(g)
    s.set_data(v, 0)
    g.bin([c, s])
    return [np.asarray(c).copy(), np.asarray(s).copy()]


legs = {"c2_count_sum": lambda: c2(True), "c2_count": lambda: c2(False), "c3_dense": c3}
ref = {}
res = {}
for rnd in range(2):
    for m in (modes if rnd == 0 else modes[::-1]):
        os.environ["VH_TILE_WIDE"] = str(m)
        for name, f in legs.items():
            out = f()
            _lib.synchronize()
            if name not in ref:
                ref[name] = out
            same = all(np.array_equal(a, b) if a.dtype.kind in "iu" else np.allclose(a, b, rtol=1e-9, atol=0)
                       for a, b in zip(out, ref[name]))
            _lib.timing_reset()
            _lib.timing_enable(True)
            t0 = time.perf_counter()
            for _ in range(5):
                f()
            _lib.synchronize()
            t = (time.perf_counter() - t0) / 5
            _lib.timing_enable(False)
            per = {}
            for k in ("tile_sample", "tile_scatter_f64", "tile_scatter_ord", "tile_reduce"):
                c, ms = _lib.timing_read(k)
                if c:
                    per[k] = round(ms / c, 3)
            res.setdefault((name, m), []).append((round(t * 1e3, 3), per, same))
            print(rnd, name, "mode", m, "step_ms", round(t * 1e3, 3), per, "same_as_first", same, flush=True)
print("summary (best of rounds): leg mode step_ms passA passB")
for (name, m), rs in sorted(res.items()):
    best = min(rs, key=lambda r: r[0])
    pa = min(r[1].get("tile_scatter_f64", r[1].get("tile_scatter_ord", 0)) for r in rs)
    pb = min(r[1].get("tile_reduce", 0) for r in rs)
    print(f"{name:14s} {m}  {best[0]:7.3f}  A {pa:6.3f}  B {pb:6.3f}  same {all(r[2] for r in rs)}")
