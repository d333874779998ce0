"""Where C1's per-query time goes: df.count(binby='x', shape=256) on 1e7
rows resident in HBM, with limits given (bin only) and with the minmax pass.  Prints the
median wall time, the C-ABI calls (VAEX_AMD_TRACE_CALLS=1) and the top Python frames."""
import cProfile
import os
import pstats
import sys
import time

os.environ["VAEX_AMD_TRACE_CALLS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
x = DeviceArray.random(n, "normal", seed=1)
df = vaex_amd.from_arrays(x=x)
for name, lim in (("bin", [-5.0, 5.0]), ("minmax+bin", None)):
    for _ in range(20):
        df.count(binby="x", shape=256, limits=lim)
    _lib.synchronize()
    _lib.trace_report()
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        df.count(binby="x", shape=256, limits=lim)
        ts.append(time.perf_counter() - t0)
    calls = _lib.trace_report()
    print(f"{name}: median {np.median(ts) * 1e3:.4f} ms, min {min(ts) * 1e3:.4f} ms")
    for k, (c, t) in sorted(calls.items(), key=lambda kv: -kv[1][1]):
        print(f"   {k:28s} {c / 200:5.1f} calls/query  {t / 200 * 1e3:.4f} ms/query")
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(50):
        df.count(binby="x", shape=256, limits=lim)
    _lib.synchronize()
    _lib.timing_enable(False)
    for k in ("minmax", "bin_cells", "bin_aggregate_lds", "bin_fused_lds", "bin_fused_global", "bin_reduce0", "bin_small_f64"):
        c, ms = _lib.timing_read(k)
        if c:
            print(f"   kernel {k:20s} {c / 50:4.1f}/query {ms / c * 1e3:8.2f} us")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        df.count(binby="x", shape=256, limits=lim)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)
