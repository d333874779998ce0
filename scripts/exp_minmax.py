"""groupby(int32 key, 1e6 keys, assume_sparse=True).agg(v: sum, count, min, max) on 1e9 resident
rows, random and sorted keys: end-to-end ms (best of 3) and the tile kernels' HIP-event ms, plus
a C-ABI call trace of one query (host time between calls).  usage: python scripts/exp_minmax.py [rows]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
v = DeviceArray.random(n, "normal", seed=6)
names = ["tile_sample", "tile_scatter_ord", "tile_reduce", "dense_first", "minmax"]
for layout in ("random", "sorted"):
    if layout == "sorted":
        keys = DeviceArray.random(n, "sorted_int", a=5, b=5 + 1_000_000, dtype="int32")
    else:
        keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
    df = vaex_amd.from_arrays(key=keys, v=v)

    def q():
        r = df.groupby("key", agg={"v": ["sum", "count", "min", "max"]}, assume_sparse=True)
        return [r[c].to_numpy() for c in r.get_column_names()]

    q()
    ts = []
    for _ in range(3):
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        q()
        _lib.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        _lib.timing_enable(False)
    per = {k: round(_lib.timing_read(k)[1], 3) for k in names if _lib.timing_read(k)[0]}
    print(layout, "ms", [round(t, 3) for t in ts], per, flush=True)
    # call trace of one more query
    log = []
    orig = _lib.call

    def traced(name, *a):
        t0 = time.perf_counter()
        try:
            return orig(name, *a)
        finally:
            log.append((name, t0, time.perf_counter()))
    _lib.call = traced
    _lib.synchronize()
    T0 = time.perf_counter()
    q()
    _lib.synchronize()
    _lib.call = orig
    tot = time.perf_counter() - T0
    big = [(nm, round((a - T0) * 1e3, 3), round((b - a) * 1e3, 3)) for nm, a, b in log if b - a > 1e-4]
    prev, gaps = T0, []
    for nm, a, b in log:
        if a - prev > 1e-4:
            gaps.append((nm, round((a - prev) * 1e3, 3)))
        prev = b
    print(layout, "trace total", round(tot * 1e3, 3), "calls > 0.1 ms", big, "host gaps > 0.1 ms before", gaps, flush=True)
    del df, keys
