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
"""
from . import _lib  # noqa: F401  (fails loudly if the HIP library is missing)
from . import agg, superagg, superutils  # noqa: F401
from .dataframe import DataFrame, Expression, RowLimitException, from_arrays, from_dict  # noqa: F401
from .device import DeviceArray  # noqa: F401
from .execution import ExecutorLocal, default_executor  # noqa: F401

__version__ = "0.1.0"

_lib.lib()  # load now: the product has no CPU fallback
