"""Multi-GPU binning: one process per GPU, rows sharded by range, dense grids merged with
one collective.

The reference has no multi-process path (its ``reduce`` merges per-thread private grids,
``superagg.cpp:160-167``); here every rank bins its own row range into its own HBM grids,
then the grids are combined with an all-reduce over RCCL (``torch.distributed`` backend
"nccl" on ROCm, xGMI between the GPUs of a node): SUM for count/sum/moment grids, MIN/MAX
for min/max grids.  AggFirst needs the (order, value) pair and is combined by an
all-gather + the AggFirst reduce rule (``superagg.cpp:470-480``).  torch is plumbing here:
it aliases the library's HBM grid through ``__cuda_array_interface__`` (no copy).

The grid-combine rules are written against plain arrays (:func:`combine_grids`) so the
same code runs on CPU with the gloo backend in the tests.
"""
import numpy as np

_NP_TO_TORCH = None


def shard_range(n, rank, world):
    """Contiguous row range [i1, i2) of ``rank`` out of ``world``."""
    return n * rank // world, n * (rank + 1) // world


def _torch_dtype(np_dtype):
    import torch
    return {np.dtype("int64"): torch.int64, np.dtype("uint64"): torch.int64, np.dtype("float64"): torch.float64,
            np.dtype("float32"): torch.float32, np.dtype("int32"): torch.int32, np.dtype("int16"): torch.int16,
            np.dtype("int8"): torch.int8, np.dtype("uint8"): torch.uint8, np.dtype("bool"): torch.bool}[np.dtype(np_dtype)]


def combine_grids(kind, tensor, order_tensor=None, group=None):
    """In-place all-reduce of one flattened grid tensor by aggregator kind."""
    import torch
    import torch.distributed as dist
    if kind in ("AggCount", "AggSum", "AggSumMoment"):
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group)
    elif kind == "AggMin":
        dist.all_reduce(tensor, op=dist.ReduceOp.MIN, group=group)
    elif kind == "AggMax":
        dist.all_reduce(tensor, op=dist.ReduceOp.MAX, group=group)
    elif kind == "AggFirst":
        world = dist.get_world_size(group)
        vals = [torch.empty_like(tensor) for _ in range(world)]
        ords = [torch.empty_like(order_tensor) for _ in range(world)]
        dist.all_gather(vals, tensor, group=group)
        dist.all_gather(ords, order_tensor, group=group)
        v, o = vals[0].clone(), ords[0].clone()
        for r in range(1, world):
            take = ords[r] < o
            v = torch.where(take, vals[r], v)
            o = torch.where(take, ords[r], o)
        tensor.copy_(v)
        order_tensor.copy_(o)
    else:
        raise ValueError(kind)


def allreduce_aggs(aggs, group=None):
    """All-reduce the HBM grids of superagg aggregators across the ranks (RCCL)."""
    import torch
    from .device import DeviceArray
    for agg in aggs:
        agg._before_device_use()
        length = agg.grid.length1d
        dev = DeviceArray(length, agg._grid_dtype, _ptr=agg.device_grid_ptr(), _owner=agg)
        t = torch.as_tensor(dev, device="cuda")
        if agg._grid_dtype == np.dtype("uint64"):
            t = t.view(torch.int64)
        order = None
        if agg._kind == "AggFirst":
            odev = DeviceArray(length, agg._grid_dtype, _ptr=agg.device_order_ptr(), _owner=agg)
            order = torch.as_tensor(odev, device="cuda")
        combine_grids(agg._kind, t, order, group=group)
        torch.cuda.synchronize()
        agg._after_device_write()
