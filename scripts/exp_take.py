"""Host gather of groupby result columns (hostops.take_columns -> vh_host_take) on this box:
5 columns x 1e6 groups, a random and an identity-like permutation, pinned vs plain sources,
against numpy take.  usage: python scripts/exp_take.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaex_amd import _lib, hostops  # noqa: E402


def best(f, k=7):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 3), round(float(np.median(ts)) * 1e3, 3)


m = 1_000_000
rng = np.random.default_rng(1)
perm = rng.permutation(m).astype(np.int64)
near = np.arange(m, dtype=np.int64)
near[1::2], near[::2] = near[::2].copy(), near[1::2].copy()
plain = [rng.random(m) for _ in range(5)]
pinned = []
for c in plain:
    p = _lib.pinned_empty(m, np.float64)
    p[:] = c
    pinned.append(p)
print("threads", hostops._threads(), "cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for name, idx in (("random", perm), ("near-identity", near)):
    print(name, "take_columns pinned", best(lambda: hostops.take_columns(pinned, idx)),
          "plain", best(lambda: hostops.take_columns(plain, idx)),
          "numpy x5", best(lambda: [np.take(c, idx) for c in plain]))
