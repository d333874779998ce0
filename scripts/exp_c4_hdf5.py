"""C4 shape on one GPU: mean(w, binby=[x, y], shape=1024) over float64 columns memory-mapped
from a vaex HDF5 file (export_hdf5 -> vaex_amd.open), i.e. the host -> HBM streaming path
(pinned double-buffered H2D pipeline) instead of HBM-resident columns.

usage: python scripts/exp_c4_hdf5.py [rows] [dir]   (rows default 2e8 = 4.8 GB of columns)
Prints one JSON line: end-to-end rows/s and host GB/s of the timed passes (page cache warm
after the first pass), and whether the result equals the same query on HBM columns."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "c4_columns.hdf5")
    cols = {"x": DeviceArray.random(n, "normal", seed=2), "y": DeviceArray.random(n, "normal", seed=3),
            "w": DeviceArray.random(n, "uniform", seed=4)}
    host = {k: v.to_numpy() for k, v in cols.items()}
    t0 = time.perf_counter()
    vaex_amd.from_arrays(**host).export_hdf5(path)
    t_write = time.perf_counter() - t0
    del host
    q = dict(binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024)
    ref = np.asarray(vaex_amd.from_arrays(**cols).mean("w", **q))
    df = vaex_amd.open(path)
    times = []
    for _ in range(3):
        _lib.synchronize()
        t0 = time.perf_counter()
        got = np.asarray(df.mean("w", **q))
        _lib.synchronize()
        times.append(time.perf_counter() - t0)
    t = min(times[1:])
    equal = bool(np.allclose(got, ref, rtol=1e-9, atol=0, equal_nan=True))
    print(json.dumps({"workload": "C4 shape: mean(w, binby=[x,y], shape=1024) over mmap'd HDF5 float64 columns",
                      "rows": n, "seconds": t, "first_pass_seconds": times[0], "rows_per_s": n / t,
                      "host_GBps": 24 * n / t / 1e9, "write_seconds": t_write, "matches_hbm_result": equal}))
    os.remove(path)


if __name__ == "__main__":
    main()
