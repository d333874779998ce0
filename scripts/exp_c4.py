"""C4 host-link sweep (not part of the library): mean(w, binby=[x, y], shape=1024) over a
mapped HDF5 file of `rows` rows, for task pass sizes x host-pipeline modes.
run: python scripts/exp_c4.py [rows]"""
import os
import sys
import time

import numpy as np

import vaex_amd
from vaex_amd import execution
from vaex_amd.device import DeviceArray

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 2_000_000_000
path = f"/dev/shm/exp_c4_{os.getpid()}.hdf5"
cols = {"x": DeviceArray.random(rows, "normal", seed=12), "y": DeviceArray.random(rows, "normal", seed=13),
        "w": DeviceArray.random(rows, "uniform", seed=14)}
vaex_amd.from_arrays(**cols).export_hdf5(path)
del cols
try:
    df = vaex_amd.open(path)
    lim = [[-4.0, 4.0], [-4.0, 4.0]]
    fast = os.environ.get("EXP_C4_FAST")  # one configuration (profiling)
    for reg, pipe in ((("1", "0"),) if fast else (("1", "0"), ("0", "0"))):
        os.environ["VH_HOST_REGISTER"], os.environ["VH_HOST_PIPE"] = reg, pipe
        for ps in ((1 << 28,) if fast else (1 << 26, 1 << 28, 1 << 29, 1 << 30, 1 << 31)):
            execution.CHUNK_SIZE_HOST = ps
            df.mean("w", binby=["x", "y"], limits=lim, shape=1024)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                df.mean("w", binby=["x", "y"], limits=lim, shape=1024)
                ts.append(time.perf_counter() - t0)
            t = min(ts)
            if os.environ.get("EXP_C4_PROFILE"):
                import cProfile
                import pstats
                pr = cProfile.Profile()
                pr.enable()
                df.mean("w", binby=["x", "y"], limits=lim, shape=1024)
                pr.disable()
                pstats.Stats(pr).sort_stats("tottime").print_stats(8)
                from vaex_amd import _lib
                orig, acc = _lib.call, {}

                def timed(name, *a):
                    t = time.perf_counter()
                    try:
                        return orig(name, *a)
                    finally:
                        e = acc.setdefault(name, [0, 0.0])
                        e[0] += 1
                        e[1] += time.perf_counter() - t

                _lib.call = timed
                t = time.perf_counter()
                df.mean("w", binby=["x", "y"], limits=lim, shape=1024)
                print("query", round(time.perf_counter() - t, 4))
                _lib.call = orig
                for k, (c, tt) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
                    print(f"  {k:32s} {c:4d} {tt * 1e3:9.2f} ms")
            print(f"register={reg} pipe={pipe} pass=2^{ps.bit_length() - 1}: {t:.4f} s  {24 * rows / t / 1e9:6.2f} GB/s", flush=True)
finally:
    os.remove(path)
