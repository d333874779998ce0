"""Where C3's end-to-end groupby time goes beyond its kernels: groupby('key').agg(sum, count)
on HBM columns (1e9 rows, 1e6 keys), timed per phase with cProfile after warm-up.
usage: python scripts/exp_c3_overhead.py [rows]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=2)
df = vaex_amd.from_arrays(key=keys, v=v)


def q():
    return df.groupby("key", agg={"v_sum": vaex_amd.agg.sum("v"), "v_count": vaex_amd.agg.count("v")})


for _ in range(3):
    q()
_lib.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    q()
_lib.synchronize()
print(f"end to end {1e3 * (time.perf_counter() - t0) / 5:.2f} ms per query", flush=True)
_lib.timing_reset()
_lib.timing_enable(True)
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    q()
_lib.synchronize()
pr.disable()
_lib.timing_enable(False)
for k in ("minmax", "tile_sample", "tile_scatter_ord", "tile_reduce"):
    c, ms = _lib.timing_read(k)
    if c:
        print(f"kernel {k}: {ms / 5:.3f} ms per query")
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
