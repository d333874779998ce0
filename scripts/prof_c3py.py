"""Python-side profile of the C3 `auto` groupby (1e9 rows, after warm-up): cProfile of three
queries, sorted by total time, plus the wall time of each.  usage: python scripts/prof_c3py.py [rows]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)


def q():
    r = df.groupby("key", agg={"v": ["sum", "count"]})
    return r["key"].to_numpy(), r["v"].to_numpy(), r["v_sum"].to_numpy()


for _ in range(3):
    q()
_lib.synchronize()
pr = cProfile.Profile()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    pr.enable()
    q()
    pr.disable()
    ts.append((time.perf_counter() - t0) * 1e3)
print("query ms", [round(t, 3) for t in ts])
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
