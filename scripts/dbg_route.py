"""Which kernels a groupby query runs (HIP-event timer names): usage dbg_route.py [rows] [q...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["tile_sample", "tile_scatter", "tile_scatter_f64", "tile_scatter_ord", "tile_scatter_set", "tile_reduce",
         "bin_fused_global", "bin_fused_lds", "bin_aggregate", "bin_indices", "ha_scatter_f64", "ha_scatter",
         "ha_reduce", "ha_direct", "minmax"]
sys.argv = [sys.argv[0], sys.argv[1] if len(sys.argv) > 1 else "1e7"] + (sys.argv[2:] or ["q3", "q5", "q7"])
src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "exp_h2o.py")).read()
g = {"__name__": "dbg", "__file__": __file__}
exec(compile(src.split("for q in which:")[0], "exp_h2o.py", "exec"), g)
_lib = g["_lib"]
for q in g["which"]:
    _lib.timing_reset()
    _lib.timing_enable(True)
    g["Q"][q]()
    _lib.synchronize()
    _lib.timing_enable(False)
    print(q, {k: (_lib.timing_read(k)[0], round(_lib.timing_read(k)[1], 3)) for k in NAMES if _lib.timing_read(k)[0]}, flush=True)
