"""vaex_amd -- vaex-core's binned-statistics and groupby hot path on the AMD MI355X.

The product path is ``libvaexhip.so`` (hand-written HIP kernels for gfx950 behind the
C-ABI of ``include/vaexhip.h``); this package is the host-side mirror of the
reference's plugin surface for that path:

* :mod:`vaex_amd.superagg`   -- ``vaex.superagg`` (Grid, Binner*, Agg*)
* :mod:`vaex_amd.superutils` -- ``vaex.superutils.ordered_set_*``
* :mod:`vaex_amd.agg`        -- ``vaex.agg`` descriptors
* :mod:`vaex_amd.execution`  -- ``ExecutorLocal`` (chunk loop feeding the GPU)
* :mod:`vaex_amd.dataframe`  -- ``DataFrame.count/sum/mean/.../groupby``
* :mod:`vaex_amd.distributed` -- row sharding over GPUs + RCCL grid reduce
* :mod:`vaex_amd.hdf5`       -- memory-mapped vaex HDF5 files (read + export), no h5py
* :mod:`vaex_amd.expr`       -- expressions / selections / filters evaluated on the GPU
"""
from . import _lib  # noqa: F401  (fails loudly if the HIP library is missing)
from . import agg, superagg, superutils  # noqa: F401
from .dataframe import DataFrame, Expression, RowLimitException, from_arrays, from_dict  # noqa: F401
from .device import DeviceArray  # noqa: F401
from .execution import ExecutorLocal, default_executor  # noqa: F401

__version__ = "0.1.0"


def open(path):
    """vaex.open (vaex/__init__.py open): HDF5 files are memory-mapped column by column
    (hdf5.py); Arrow IPC / Feather files are memory-mapped through pyarrow; the columns
    are host arrays that binning streams to HBM chunk by chunk."""
    p = str(path)
    low = p.lower()
    if low.endswith((".hdf5", ".h5")):
        from .hdf5 import open as open_hdf5
        return open_hdf5(p)
    if low.endswith((".arrow", ".feather", ".ipc")):
        import numpy as np
        import pyarrow as pa
        src = pa.memory_map(p, "r")
        try:
            table = pa.ipc.open_file(src).read_all()
        except pa.ArrowInvalid:
            table = pa.ipc.open_stream(pa.memory_map(p, "r")).read_all()
        cols = {}
        for name in table.column_names:
            ch = table.column(name).combine_chunks()
            if ch.null_count:
                cols[name] = np.ma.array(ch.to_numpy(zero_copy_only=False), mask=ch.is_null().to_numpy(zero_copy_only=False))
            else:
                cols[name] = ch.to_numpy(zero_copy_only=False)
        return DataFrame(cols)
    raise ValueError(f"cannot open {p!r}: only .hdf5/.h5 and .arrow/.feather files are supported")

_lib.lib()  # load now: the product has no CPU fallback
