"""The fused hash groupby (hashagg.hip, HashAgg API) on C3's columns with shuffled and sorted
int32 keys (1e9 rows, 1e6 keys): per-kernel HIP-event ms, for rocprofv3 PMC passes of
k_ha_scatter_k4's RUNS / plain variants.  usage: python scripts/exp_hash_sorted.py [rows] [layouts] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402
from vaex_amd.hashagg import HashAgg  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
layouts = sys.argv[2].split(",") if len(sys.argv) > 2 else ["random", "sorted"]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
v = DeviceArray.random(n, "normal", seed=6)
for layout in layouts:
    if layout == "sorted":
        keys = DeviceArray.random(n, "sorted_int", a=5, b=5 + 1_000_000, dtype="int32")
    else:
        keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
    for rep in range(reps + 1):
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        ha = HashAgg(keys.dtype, [v.dtype], [False])
        ha.update(keys, [v])
        k, c, s, _ = ha.finish()
        _lib.synchronize()
        _lib.timing_enable(False)
        per = {}
        for name in ("ha_sample", "ha_scatter", "ha_scatter_f64", "ha_reduce", "ha_finish"):
            cnt, ms = _lib.timing_read(name)
            if cnt:
                per[name] = round(ms / cnt, 3)
        if rep:
            print(layout, rep, per, "groups", len(k), "count_ok", int(np.asarray(c).sum()) == n, flush=True)
    del keys
