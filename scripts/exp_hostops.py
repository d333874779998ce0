"""Host-side finishing costs on this box: the pieces of a dense 1e6-group groupby's tail
(occupancy of the count grid, label range, permutation take, casts), each timed alone."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from vaex_amd import _lib, hostops  # noqa: E402

m = 1_000_000


def t(name, f, k=10):
    f()
    t0 = time.perf_counter()
    for _ in range(k):
        f()
    print(f"{name:40s} {(time.perf_counter() - t0) / k * 1e3:8.3f} ms", flush=True)


print("threads", hostops._threads(), "affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())
counts = _lib.pinned_empty(m + 3, np.int64)
counts[:] = np.random.default_rng(0).integers(1, 2000, m + 3)
sums = _lib.pinned_empty(m + 3, np.float64)
sums[:] = 1.0
perm = np.random.default_rng(1).permutation(m).astype(np.int64)
t("occupancy (threads)", lambda: hostops.occupancy(counts[2:-1]))
t("count_nonzero single", lambda: np.count_nonzero(counts[2:-1]))
t("counts > 0 single", lambda: counts[2:-1] > 0)
t("arange int32 threads", lambda: hostops.arange(5, m, np.int32))
t("arange int32 single", lambda: hostops.arange(5, m, np.int32, threads=False))
t("astype int32->int64 threads", lambda: hostops.astype(np.arange(m, dtype=np.int32), np.int64))
t("take f64 threads", lambda: hostops.take(sums[2:-1], perm))
t("take f64 single clip", lambda: np.take(sums[2:-1], perm, mode="clip"))
t("pinned_empty 8MB", lambda: _lib.pinned_empty(m, np.int64))
t("np.empty 8MB + touch", lambda: np.empty(m, np.int64).fill(0))
