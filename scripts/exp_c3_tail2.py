"""Where the host part of the C3 `auto` query goes (after the GPU pass): pinned vs plain memory
count_nonzero rates, hostops.occupancy on the 1e6-cell count grid, and a timed replay of
GroupBy._agg_dense's pieces.  usage: python scripts/exp_c3_tail2.py [rows]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib, groupby, hostops  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402


def best(f, k=7):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 4)


m = 1_000_003
pin = _lib.pinned_empty(m, np.int64)
pin[:] = 3
plain = np.full(m, 3, np.int64)
print("count_nonzero 8 MB: pinned", best(lambda: np.count_nonzero(pin)), "ms  plain", best(lambda: np.count_nonzero(plain)), "ms")
print("occupancy: pinned", best(lambda: hostops.occupancy(pin)), "ms  plain", best(lambda: hostops.occupancy(plain)), "ms")
print("threads", hostops._threads(), "MIN_SPLIT", hostops.MIN_SPLIT)

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)
T = {}
orig_occ, orig_dense, orig_exec = hostops.occupancy, groupby.GroupBy._agg_dense, df.executor.execute


def wrap(name, f):
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[name] = T.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
    return g


hostops.occupancy = wrap("occupancy", orig_occ)
groupby.GroupBy._agg_dense = wrap("_agg_dense", orig_dense)
df.executor.execute = wrap("execute", orig_exec)
for rep in range(4):
    T.clear()
    _lib.synchronize()
    t0 = time.perf_counter()
    r = df.groupby("key", agg={"v": ["sum", "count"]})
    t1 = time.perf_counter()
    cols = [r[c].to_numpy() for c in r.get_column_names()]
    t2 = time.perf_counter()
    print(rep, "groupby", round((t1 - t0) * 1e3, 3), "to_numpy", round((t2 - t1) * 1e3, 3), {k: round(x, 3) for k, x in T.items()})
