"""Why the bench's host -> HBM copies ran at ~30 GB/s where a fresh process reaches ~57:
the same 1 GiB library copy before and after the steps the bench takes first (HBM
allocations, an HDF5 export to /dev/shm).  run: python scripts/h2d_lib_probe.py"""
import os
import time

import numpy as np

from vaex_amd import _lib
from vaex_amd.device import DeviceArray

GiB = 1 << 30
d = DeviceArray(GiB, np.uint8)
h = _lib.pinned_empty(GiB, np.uint8)
h[:] = 1
p = np.ones(GiB, np.uint8)


def show(tag):
    for name, src in (("pinned", h), ("pageable", p)):
        best = 1e30
        for _ in range(4):
            t0 = time.perf_counter()
            _lib.call("vh_memcpy_htod", d.ptr, src.ctypes.data, GiB)
            best = min(best, time.perf_counter() - t0)
        print(f"{tag:28s} {name:8s} {GiB / best / 1e9:6.2f} GB/s", flush=True)


show("fresh")
h2 = _lib.pinned_empty(GiB, np.uint8)
h2[:] = 1
h, h2 = h2, h
show("second pinned block")
cols = [DeviceArray.random(2_000_000_000, "normal", seed=s) for s in range(3)]
show("after 48 GB in HBM")
big = _lib.pinned_empty(8 * GiB, np.uint8)
big[:] = 1
h = big[:GiB]
show("8 GiB pinned block")
import vaex_amd
path = f"/dev/shm/h2d_probe_{os.getpid()}.hdf5"
try:
    vaex_amd.from_arrays(x=cols[0], y=cols[1], w=cols[2]).export_hdf5(path)
    show("after 48 GB export")
    h3 = _lib.pinned_empty(GiB, np.uint8)
    h3[:] = 1
    h = h3
    show("pinned after export")
finally:
    os.remove(path)
