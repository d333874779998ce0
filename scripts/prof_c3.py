"""cProfile of the C3 dense groupby route's host side (bench.py's groupby 'auto' leg)."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=2)
df = vaex_amd.from_arrays(key=keys, v=v)
q = lambda: df.groupby("key", agg={"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v")})  # noqa: E731
for _ in range(3):
    q()
_lib.synchronize()
pr = cProfile.Profile()
pr.enable()
q()
_lib.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:7000])
if _lib._TRACE is not None:
    _lib.trace_report()
    import time
    t0 = time.perf_counter()
    q()
    _lib.synchronize()
    t1 = time.perf_counter()
    print(f"query {1e3 * (t1 - t0):.3f} ms; C-ABI calls (calls, ms):")
    for k, (c, s) in sorted(_lib.trace_report().items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:32s} {c:4d} {1e3 * s:8.3f}")
