"""h2o q10 on bench.py's HBM-generated h2o frame (h2o_frame): per-call C-ABI times of warm
queries, to compare with scripts/exp_h2o.py's host-generated columns.
usage: VAEX_AMD_TRACE_CALLS=1 python scripts/exp_q10_bench_data.py [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vaex_amd import _lib  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
df = bench.h2o_frame(n)
q10 = bench.h2o_queries(df)["q10"]
for it in range(3):
    _lib.synchronize()
    _lib.trace_report()
    t0 = time.perf_counter()
    r = q10()
    _lib.synchronize()
    t = time.perf_counter() - t0
    top = sorted(_lib.trace_report().items(), key=lambda kv: -kv[1][1])[:6]
    print(f"q10 run {it}: {t * 1e3:.1f} ms  groups {len(r)}  " + "  ".join(f"{k} {1e3 * v[1]:.1f}" for k, v in top), flush=True)
    r = None
