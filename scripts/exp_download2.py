"""The bench's auto groupby step with per-call timing of the read-back (C3, 1e9 rows)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import vaex_amd  # noqa: E402
from vaex_amd import _lib, superagg  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
v = DeviceArray.random(n, "normal", seed=6)
orig = superagg.Aggregator._ensure_host
log = []


def timed(self):
    _lib.synchronize()
    t0 = time.perf_counter()
    orig(self)
    log.append((time.perf_counter() - t0) * 1e3)


if not os.environ.get("NO_SYNC"):
    superagg.Aggregator._ensure_host = timed
df = vaex_amd.from_arrays(key=keys, v=v)
for it in range(4):
    log.clear()
    t0 = time.perf_counter()
    g = df.groupby("key", agg={"v": ["sum", "count"]})
    t = time.perf_counter() - t0
    rep = {k: (c, round(s * 1e3, 3)) for k, (c, s) in _lib.trace_report().items() if s > 1e-4}
    print(f"step {1e3 * t:.2f} ms, read-backs {[round(x, 3) for x in log]} calls {rep}", flush=True)
# the same grid read again after an idle moment
