"""Where h2o q3's pass A (k_tile_scatter_ord, int32 key + int8 / float32 packed narrow slots)
spends its time, one process (ablation build; results wrong by design): VH_TILE_DEBUG bits
interleaved over rounds -- 0 full, 128 no stream stores, 32 no commit (loads, cell math,
ranking), 96 no commit and no ranking.  Also times the C3 shape (int32 key + float64) for
comparison.
usage: VAEX_AMD_LIB=vaex_amd/libvaexhip_ablation.so python scripts/exp_q3_ablate.py [rows] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(0)
cols = dict(id3=rng.integers(5, 1_000_005, n).astype(np.int32), v1=rng.integers(5, 15, n).astype(np.int8),
            v3=rng.normal(size=n).astype(np.float32))
d = {k: DeviceArray.from_numpy(v) for k, v in cols.items()}
del cols
d["w"] = DeviceArray.random(n, "normal", seed=4)
df = vaex_amd.from_arrays(**d)
shapes = {"q3": lambda: df.groupby(["id3"]).agg({"v1": "sum", "v3": "mean"}),
          "c3": lambda: df.groupby(["id3"]).agg({"w": "sum"})}
modes = os.environ.get("DBGS", "0 128 32 96").split()
res = {}
for r in range(rounds + 1):
    for name, q in shapes.items():
        for m in modes:
            os.environ["VH_TILE_DEBUG"] = m
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            q()
            _lib.synchronize()
            _lib.timing_enable(False)
            if r:
                for k in ("tile_scatter_ord", "tile_reduce"):
                    res.setdefault((name, m, k), []).append(_lib.timing_read(k)[1])
for (name, m, k), v in sorted(res.items()):
    print(f"{name} VH_TILE_DEBUG={m:4s} {k:17s} median {statistics.median(v):.3f} ms  min {min(v):.3f}", flush=True)
