"""h2o groupby G1 (benchmarks/groupbyh2o.py:15-93 with fixtures.py:38-70's columns) on HBM
columns: q1-q5, q7, q10 timed end to end.  usage: python scripts/exp_h2o.py [rows] [q...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 8
which = sys.argv[2:] or ["q1", "q2", "q3", "q4", "q5", "q7", "q10"]
rng = np.random.default_rng(0)
i1_100 = rng.integers(5, 105, n).astype(np.int8)
i4_1M = rng.integers(5, 1_000_005, n).astype(np.int32)
i1_10 = rng.integers(5, 15, n).astype(np.int8)
x4 = rng.normal(size=n).astype(np.float32)
d = {k: DeviceArray.from_numpy(v) for k, v in dict(i1_100=i1_100, i4_1M=i4_1M, i1_10=i1_10, x4=x4).items()}
df = vaex_amd.from_arrays(**d)
for a, b in [("id1", "i1_100"), ("id2", "i1_100"), ("id3", "i4_1M"), ("id4", "i1_100"), ("id5", "i1_100"),
             ("id6", "i4_1M"), ("v1", "i1_10"), ("v2", "i1_10"), ("v3", "x4")]:
    df.columns[a] = df.columns[b]  # the benchmark's aliases (df['id1'] = df['i1_100'])
Q = {
    "q1": lambda: df.groupby(["id1"]).agg({"v1": "sum"}),
    "q2": lambda: df.groupby(["id1", "id2"]).agg({"v1": "sum"}),
    "q3": lambda: df.groupby(["id3"]).agg({"v1": "sum", "v3": "mean"}),
    "q4": lambda: df.groupby(["id4"]).agg({"v1": "mean", "v2": "mean", "v3": "mean"}),
    "q5": lambda: df.groupby(["id6"]).agg({"v1": "sum", "v2": "sum", "v3": "sum"}),
    "q7": lambda: df.groupby(["id3"]).agg({"v1": "max", "v2": "min"}),
    "q10": lambda: df.groupby(["id1", "id2", "id3", "id4", "id5", "id6"]).agg({"v3": "sum", "v1": "count"}),
}
for q in which:
    for it in range(int(os.environ.get("H2O_REPS", "3"))):
        _lib.synchronize()
        if os.environ.get("H2O_CPROF_EACH"):
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        t0 = time.perf_counter()
        r = Q[q]()
        _lib.synchronize()
        t = time.perf_counter() - t0
        if os.environ.get("H2O_CPROF_EACH"):
            pr.disable()
            if t > 1.0:
                pstats.Stats(pr).sort_stats("tottime").print_stats(12)
        if os.environ.get("H2O_EACH"):
            top = sorted(_lib.trace_report().items(), key=lambda kv: -kv[1][1])[:4]
            print(f"  {q} run {it}: {t * 1e3:.2f} ms", "  ".join(f"{k} {1e3 * v[1]:.1f}" for k, v in top), flush=True)
    print(f"{q}: {t * 1e3:.2f} ms  {n / t / 1e9:.2f} G rows/s  groups {len(r)}", flush=True)
if os.environ.get("H2O_PROFILE"):  # host-side breakdown of the last query: Python frames + C-ABI calls
    import cProfile
    import pstats
    os.environ["VAEX_AMD_TRACE_CALLS"] = "1"
    for q in which:
        _lib.trace_report()
        pr = cProfile.Profile()
        pr.enable()
        Q[q]()
        _lib.synchronize()
        pr.disable()
        print("== profile", q)
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)
        for k, (c, sec) in sorted(_lib.trace_report().items(), key=lambda kv: -kv[1][1])[:15]:
            print(f"  {k:32s} {c:5d} {1e3 * sec:10.3f} ms")
