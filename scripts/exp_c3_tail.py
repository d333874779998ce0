"""Where the host time of a dense groupby's tail goes (after the GPU pass): wraps the pieces
of GroupBy._agg_dense with timers over a few C3 `auto` queries (1e9 rows)."""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vaex_amd  # noqa: E402
from vaex_amd import _lib, groupby, hostops, dataframe, taskparts, execution  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)
acc = defaultdict(float)


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[f"{mod.__name__}.{name}"] += time.perf_counter() - t0
    setattr(mod, name, g)


for mod, name in ((hostops, "occupancy"), (groupby, "_label_range"), (groupby, "extract_central_part"),
                  (groupby, "_dense_range"), (groupby, "parse_actions")):
    wrap(mod, name)
for cls, name in ((groupby.GroupBy, "_agg"), (groupby.GroupBy, "_agg_dense"), (dataframe.DataFrame, "execute"),
                  (taskparts.TaskPartAggregation, "get_result"), (taskparts.TaskPartAggregation, "process"),
                  (dataframe.DataFrame, "__init__")):
    f = getattr(cls, name)

    def mk(f, key):
        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[key] += time.perf_counter() - t0
        return g
    setattr(cls, name, mk(f, f"{cls.__name__}.{name}"))

q = lambda: df.groupby("key", agg={"v": ["sum", "count"]})  # noqa: E731
for _ in range(3):
    q()
acc.clear()
reps = 5
_lib.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    r = q()
_lib.synchronize()
tot = (time.perf_counter() - t0) / reps
print(f"query {tot * 1e3:.3f} ms")
for k, val in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:45s} {val / reps * 1e3:8.3f} ms")
