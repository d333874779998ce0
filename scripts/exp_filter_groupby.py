"""The C3 groupby (int32 key over 1e6 values, sum + count of a float64 column) on a filtered
HBM frame (df[df.v > 0]: one keep mask on every aggregator) against the unfiltered frame:
end-to-end ms and the tile kernels.  usage: python scripts/exp_filter_groupby.py [rows] [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
v = DeviceArray.random(n, "normal", seed=2)
df = vaex_amd.from_arrays(key=keys, v=v)
dff = df[df.v > 0]
for name, frame in (("unfiltered", df), ("filtered v > 0", dff)):
    q = lambda: frame.groupby("key", agg={"v": ["sum", "count"]})  # noqa: E731
    r = q()
    ts, ks = [], {}
    for _ in range(reps):
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        r = q()
        _lib.synchronize()
        ts.append(time.perf_counter() - t0)
        _lib.timing_enable(False)
        for k in ("tile_sample", "tile_scatter", "tile_scatter_ord", "tile_reduce", "expr_eval", "ha_scatter_f64"):
            c, ms = _lib.timing_read(k)
            if c:
                ks.setdefault(k, []).append(ms)
    print(f"{name:16s}: {statistics.median(ts) * 1e3:8.3f} ms  groups {len(r)}  "
          + "  ".join(f"{k} {statistics.median(x):.3f}" for k, x in ks.items()), flush=True)
