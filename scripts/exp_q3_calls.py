"""Host timeline of one h2o query: every C-ABI call in order with its start offset and
duration (the GPU waits show as long calls, host work as the gaps between them).
usage: python scripts/exp_q3_calls.py [rows] [query]"""
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
q = sys.argv[2] if len(sys.argv) > 2 else "q3"
rng = np.random.default_rng(0)
cols = dict(id3=rng.integers(5, 1_000_005, n).astype(np.int32), v1=rng.integers(5, 15, n).astype(np.int8),
            v2=rng.integers(5, 15, n).astype(np.int8), v3=rng.normal(size=n).astype(np.float32))
df = vaex_amd.from_arrays(**{k: DeviceArray.from_numpy(v) for k, v in cols.items()})
del cols
Q = {"q3": lambda: df.groupby(["id3"]).agg({"v1": "sum", "v3": "mean"}),
     "q5": lambda: df.groupby(["id3"]).agg({"v1": "sum", "v2": "sum", "v3": "sum"}),
     "q7": lambda: df.groupby(["id3"]).agg({"v1": "max", "v2": "min"})}
seq = []
orig = _lib.call


def traced(name, *args):
    t0 = time.perf_counter()
    try:
        return orig(name, *args)
    finally:
        seq.append((name, t0, time.perf_counter()))


for it in range(4):
    _lib.synchronize()
    seq.clear()
    _lib.call = traced
    t0 = time.perf_counter()
    Q[q]()
    _lib.synchronize()
    t1 = time.perf_counter()
    _lib.call = orig
print(f"{q}: {(t1 - t0) * 1e3:.3f} ms (last of 4)")
prev = t0
for name, a, b in seq:
    print(f"  {(a - t0) * 1e3:8.3f} ms  gap {(a - prev) * 1e3:7.3f}  call {(b - a) * 1e3:7.3f}  {name}")
    prev = b
print(f"  end gap {(t1 - prev) * 1e3:.3f} ms")
