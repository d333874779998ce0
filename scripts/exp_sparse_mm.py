"""Time assume_sparse groupby routes: count/sum (fused hash aggregation) vs min/max/first
(set-ordinal binner).  Usage: python scripts/exp_sparse_mm.py [rows]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 10 ** 6, dtype="int32")
v = DeviceArray.random(n, "normal", seed=2)
df = vaex_amd.from_arrays(key=keys, v=v)
A = vaex_amd.agg
cases = {
    "count+sum": {"c": A.count("v"), "s": A.sum("v")},
    "min": {"m": A.min("v")},
    "max": {"M": A.max("v")},
    "min+max+sum": {"m": A.min("v"), "M": A.max("v"), "s": A.sum("v")},
    "first": {"f": A.first("v", order_expression="v")},
}
for name, agg in cases.items():
    ts = []
    for _ in range(4):
        _lib.synchronize()
        t0 = time.perf_counter()
        r = df.groupby("key", agg=agg, assume_sparse=True)
        _lib.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"{name:12s} rows={n:.0e} groups={len(r)} best={min(ts[1:]) * 1e3:.2f} ms", flush=True)
