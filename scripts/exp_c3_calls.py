"""C-ABI call log of one C3 `auto` query (after warm-up): each library call's start and end
relative to the query start (host clock), so host time between calls and time blocked inside
calls are visible.  usage: python scripts/exp_c3_calls.py [rows] [mode: auto|hash|fused_api]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
mode = sys.argv[2] if len(sys.argv) > 2 else "auto"
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)


def q():
    if mode == "hash_minmax":
        r = df.groupby("key", agg={"v": ["sum", "count", "min", "max"]}, assume_sparse=True)
        return [r[c].to_numpy() for c in r.get_column_names()]
    elif mode == "var":
        return df.var("v", binby=["key"], limits=[5, 5 + 10 ** 6], shape=10 ** 6)
    else:
        r = df.groupby("key", agg={"v": ["sum", "count"]}, assume_sparse="auto" if mode == "auto" else True)
    return r["key"].to_numpy(), r["v"].to_numpy(), r["v_sum"].to_numpy()


for _ in range(3):
    q()
_lib.synchronize()
log = []
orig = _lib.call
T0 = [0.0]


def traced(name, *a):
    t = time.perf_counter()
    try:
        return orig(name, *a)
    finally:
        log.append((name, t - T0[0], time.perf_counter() - T0[0]))


_lib.call = traced
for rep in range(3):
    log.clear()
    _lib.synchronize()
    T0[0] = time.perf_counter()
    q()
    _lib.synchronize()
    total = time.perf_counter() - T0[0]
print(f"query {total * 1e3:.3f} ms")
prev = 0.0
for name, a, b in log:
    print(f"{a * 1e3:8.3f} +{(a - prev) * 1e3:6.3f} host | {(b - a) * 1e3:7.3f} in call  {name}")
    prev = b
print(f"after last call: {(total - prev) * 1e3:.3f} ms")
