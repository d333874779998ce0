"""AggFirst on the C2 grid (1e9 rows resident): per-kernel HIP-event times of the tiled engine
(first.hip), median of 4 after a warm-up.  usage: python scripts/exp_first.py [rows] [shape]
(ablation: VAEX_AMD_LIB=vaex_amd/libvaexhip_ablation.so VH_FIRST_DEBUG=1 -> no stream
reservation atomics, results wrong by design)"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
shape = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
df = vaex_amd.from_arrays(x=DeviceArray.random(n, "normal", seed=2), y=DeviceArray.random(n, "normal", seed=3),
                          w=DeviceArray.random(n, "uniform", seed=4), o=DeviceArray.random(n, "uniform", seed=9))
lim = [[-4, 4], [-4, 4]]
res = {}
for rep in range(5):
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    r = df.first("w", "o", binby=["x", "y"], limits=lim, shape=shape)
    _lib.synchronize()
    t = time.perf_counter() - t0
    _lib.timing_enable(False)
    if rep == 0:
        continue
    res.setdefault("end_to_end", []).append(t * 1e3)
    for k in ("first_sample", "first_scatter", "first_reduce"):
        c, ms = _lib.timing_read(k)
        if c:
            res.setdefault(k, []).append(ms / c)
print("shape", shape, {k: round(statistics.median(v), 3) for k, v in res.items()}, "finite", int(np.isfinite(np.asarray(r)).sum()))
