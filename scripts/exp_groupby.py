"""Time one groupby mode (C3 shape): python scripts/exp_groupby.py auto|hash [rows]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

mode = sys.argv[1]
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 9
card = int(float(sys.argv[3])) if len(sys.argv) > 3 else 10 ** 6
keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + card, dtype=os.environ.get("KEYDT", "int32"))
v = DeviceArray.random(n, "normal", seed=6)
df = vaex_amd.from_arrays(key=keys, v=v)
sparse = {"auto": "auto", "hash": True, "fused": None}[mode]
K = ["tile_scatter_ord", "ha_sample", "ha_scatter", "ha_scatter_f64", "ha_reduce", "ha_direct", "ha_finish", "minmax", "tile_sample", "tile_scatter", "tile_reduce"]
import cProfile
import os
import pstats
prof = cProfile.Profile() if os.environ.get("PROF") else None
for it in range(3):
    if prof is not None and it == 2:
        prof.enable()
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    if mode == "fused":  # the hash path on the same (dense) keys, bypassing the routing
        from vaex_amd.hashagg import HashAgg
        ha = HashAgg(keys.dtype, [v.dtype], [False])
        ha.update(keys, [v])
        out = ha.finish()
        dfg = {"key": DeviceArray.from_numpy(out[0])}
    else:
        dfg = df.groupby("key", agg={"v": ["sum", "count"]}, assume_sparse=sparse)
    _lib.synchronize()
    t = time.perf_counter() - t0
    if prof is not None and it == 2:
        prof.disable()
    _lib.timing_enable(False)
    per = {k: round(_lib.timing_read(k)[1], 3) for k in K if _lib.timing_read(k)[0]}
    print(mode, it, "seconds", round(t, 4), "groups", len(dfg["key"].to_numpy()), per, flush=True)
if prof is not None:
    pstats.Stats(prof).sort_stats("cumulative").print_stats(40)
