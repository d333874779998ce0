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

from .execution import ExecutorLocal


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


# ---------------------------------------------------------------------------------------
# Distributed execution: every task pass of a DataFrame runs on each rank's row shard and
# the reduced task parts are combined across ranks before the results are fulfilled, so
# df.count/sum/mean/minmax/groupby/binby work unchanged on top.
# ---------------------------------------------------------------------------------------

def _reduce_op_for(kind):
    return {"AggCount": "sum", "AggSum": "sum", "AggSumMoment": "sum", "AggMin": "min", "AggMax": "max",
            "AggFirst": "first"}[kind]


def combine_minmax(vmin, vmax, group=None):
    """NaN-ignoring global (min, max) of per-rank limits (tasks.py:173-185 across ranks)."""
    import torch
    import torch.distributed as dist
    lo = torch.tensor([np.inf if np.isnan(vmin) else float(vmin)], dtype=torch.float64)
    hi = torch.tensor([-np.inf if np.isnan(vmax) else float(vmax)], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        lo, hi = lo.cuda(), hi.cuda()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo, hi = float(lo.item()), float(hi.item())
    return (np.nan if np.isinf(lo) and lo > 0 else lo), (np.nan if np.isinf(hi) and hi < 0 else hi)


def merge_key_arrays(gathered, make_set):
    """Global ordered set from the ranks' key arrays: rank r's keys are inserted after
    those of ranks < r, each rank's in its own ordinal order, so with contiguous row shards
    the ordinals are first-appearance order over the whole column (what one update pass
    over all rows gives, ``ordered_set::merge`` semantics, hash_primitives.hpp:96-281).
    ``gathered``: per rank (keys, null_index or -1); ``make_set()``: an empty set with
    ``update(keys, mask)``."""
    merged = make_set()
    for keys, null_index in gathered:
        keys = np.asarray(keys)
        if not len(keys):
            continue
        mask = None
        if null_index is not None and null_index >= 0:
            mask = np.zeros(len(keys), np.uint8)
            mask[int(null_index)] = 1
        merged.update(keys, mask)
    return merged


def _host_allreduce(arr, op, group):
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(arr).view(np.int64) if arr.dtype == np.uint64 else
                         np.ascontiguousarray(arr))
    dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op],
                    group=group)
    out = t.numpy()
    return out.view(np.uint64) if arr.dtype == np.uint64 else out


def combine_aggs_host(aggs, group=None):
    """All-reduce aggregator grids through host memory (gloo): download, combine, upload."""
    from . import _lib
    import torch
    import torch.distributed as dist
    for agg in aggs:
        agg._before_device_use()
        grid = np.empty(agg.grid.length1d, agg._grid_dtype)
        _lib.call("vh_agg_download", agg._handle, grid.ctypes.data, agg._nbytes)
        op = _reduce_op_for(agg._kind)
        if op == "first":
            order = np.empty(agg.grid.length1d, agg._grid_dtype)
            _lib.call("vh_agg_download_order", agg._handle, order.ctypes.data, agg._nbytes)
            world = dist.get_world_size(group)
            vals = [torch.empty_like(torch.from_numpy(grid)) for _ in range(world)]
            ords = [torch.empty_like(torch.from_numpy(order)) for _ in range(world)]
            dist.all_gather(vals, torch.from_numpy(grid), group=group)
            dist.all_gather(ords, torch.from_numpy(order), group=group)
            v, o = vals[0].numpy().copy(), ords[0].numpy().copy()
            for r in range(1, world):
                take = ords[r].numpy() < o
                v[take] = vals[r].numpy()[take]
                o[take] = ords[r].numpy()[take]
            grid, order = v, o
            _lib.call("vh_agg_upload_order", agg._handle, np.ascontiguousarray(order).ctypes.data, agg._nbytes)
        else:
            grid = _host_allreduce(grid, op, group)
        grid = np.ascontiguousarray(grid)
        _lib.call("vh_agg_upload", agg._handle, grid.ctypes.data, agg._nbytes)
        agg._after_device_write()


def nunique_state(agg):
    """(cells, values, nulls, nans) of an AggNUnique as host arrays (deduplicated pairs)."""
    import ctypes
    from . import _lib
    n = ctypes.c_uint64()
    _lib.call("vh_agg_nunique_export", agg._handle, ctypes.byref(n), None, None, None, None)
    L = agg.grid.length1d
    cells, vals = np.empty(n.value, np.uint64), np.empty(n.value, np.uint64)
    nulls, nans = np.empty(L, np.uint64), np.empty(L, np.uint64)
    _lib.call("vh_agg_nunique_export", agg._handle, ctypes.byref(n), cells.ctypes.data, vals.ctypes.data,
              nulls.ctypes.data, nans.ctypes.data)
    return cells, vals, nulls, nans


def combine_nunique(agg, group=None):
    """AggNUnique across ranks: every rank gathers the others' (cell, value) pairs and
    missing / NaN counts and merges them into its own (counter::merge,
    hash_primitives.hpp:393-415); distinct values are not additive, so no grid all-reduce."""
    import torch.distributed as dist
    from . import _lib
    mine = nunique_state(agg)
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine, group=group)
    me = dist.get_rank(group)
    for r, (cells, vals, nulls, nans) in enumerate(gathered):
        if r == me:
            continue
        cells, vals = np.ascontiguousarray(cells, np.uint64), np.ascontiguousarray(vals, np.uint64)
        nulls, nans = np.ascontiguousarray(nulls, np.uint64), np.ascontiguousarray(nans, np.uint64)
        _lib.call("vh_agg_nunique_import", agg._handle, len(cells), cells.ctypes.data, vals.ctypes.data,
                  nulls.ctypes.data, nans.ctypes.data)
    agg._after_device_write()


class ExecutorDistributed(ExecutorLocal):
    """ExecutorLocal over this rank's row shard, combining task parts across ranks.

    One process per GPU (``torch.distributed``): with ``shard_rows`` every rank holds the
    same (e.g. memory-mapped) DataFrame and processes rows ``shard_range(n, rank, world)``;
    without it each rank's DataFrame already is its shard.  After the local parts are
    reduced: aggregator grids are all-reduced (RCCL on HBM grids with backend "nccl",
    through host memory with "gloo"), min/max limits are reduced, and ordered sets are
    merged from all ranks' key arrays (:func:`merge_key_arrays`) so every rank bins with
    the same global ordinals.
    """

    def __init__(self, group=None, shard_rows=True, device_collectives=None, chunk_size=None):
        import torch.distributed as dist
        super().__init__(chunk_size)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.shard_rows = shard_rows
        self.device_collectives = (dist.get_backend(group) == "nccl") if device_collectives is None \
            else device_collectives

    def row_range(self, df):
        n = df.length_unfiltered()
        return shard_range(n, self.rank, self.world) if self.shard_rows else (0, n)

    def chunk_size_for(self, df):
        if self.chunk_size is None and df.is_device_resident():
            i1, i2 = self.row_range(df)
            return max(1, i2 - i1)
        return super().chunk_size_for(df)

    def combine_parts(self, parts):
        from .taskparts import TaskPartAggregation, TaskPartMinMax, TaskPartSetCreate
        for p in parts:
            if isinstance(p, TaskPartAggregation):
                aggs = p.get_aggregators()
                for agg in [a for a in aggs if a._kind == "AggNUnique"]:
                    combine_nunique(agg, group=self.group)
                aggs = [a for a in aggs if a._kind != "AggNUnique"]
                if self.device_collectives:
                    allreduce_aggs(aggs, group=self.group)
                else:
                    combine_aggs_host(aggs, group=self.group)
            elif isinstance(p, TaskPartMinMax):
                p.vmin, p.vmax = combine_minmax(p.vmin, p.vmax, group=self.group)
            elif isinstance(p, TaskPartSetCreate):
                p.set = combine_sets(p.set, group=self.group)


def all_ranks_true(flag, group=None):
    """Logical AND of a per-rank flag (a MIN all-reduce)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def merge_groups(parts):
    """Merge per-rank fused-groupby results ``(keys, counts, sums, nonnull)`` (each sorted by
    key, hashagg.py) into one key-sorted result: counts and integer sums add exactly, float
    sums add in rank order.  ``nonnull`` entries may be None (not requested)."""
    parts = [p for p in parts if len(p[0])]
    if not parts:
        return None
    nv = len(parts[0][2])
    keys = np.concatenate([p[0] for p in parts])
    uniq, inv = np.unique(keys, return_inverse=True)
    m = len(uniq)
    counts = np.zeros(m, np.int64)
    np.add.at(counts, inv, np.concatenate([p[1] for p in parts]))
    sums, nonnull = [], []
    for v in range(nv):
        cat = np.concatenate([p[2][v] for p in parts])
        out = np.zeros(m, cat.dtype)
        np.add.at(out, inv, cat)
        sums.append(out)
        if parts[0][3][v] is None:
            nonnull.append(None)
        else:
            nn = np.zeros(m, np.int64)
            np.add.at(nn, inv, np.concatenate([p[3][v] for p in parts]))
            nonnull.append(nn)
    return uniq, counts, sums, nonnull


def group_owner(keys, world):
    """Owner rank of each group key: splitmix64 of the key's 64-bit pattern modulo the world
    size (SURVEY.md §8e hash partition).  ``keys``: int64 / uint64 array."""
    z = np.ascontiguousarray(keys).view(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world)).astype(np.int64)


def _pack_groups(keys, counts, sums, nonnull):
    """Rows of 64-bit words [key, count, sum_0.., nonnull_v..] (bit patterns, int64)."""
    cols = [np.ascontiguousarray(keys).view(np.int64), np.ascontiguousarray(counts, np.int64)]
    cols += [np.ascontiguousarray(s).view(np.int64) for s in sums]
    cols += [np.ascontiguousarray(c, np.int64) for c in nonnull if c is not None]
    return np.stack(cols, axis=1) if cols[0].size else np.empty((0, len(cols)), np.int64)


def _unpack_groups(mat, key_dtype, sum_dtypes, has_nonnull):
    mat = np.ascontiguousarray(mat)
    keys = mat[:, 0].copy().view(key_dtype)
    counts = mat[:, 1].copy()
    sums = [mat[:, 2 + v].copy().view(dt) for v, dt in enumerate(sum_dtypes)]
    nonnull, c = [], 2 + len(sum_dtypes)
    for want in has_nonnull:
        nonnull.append(mat[:, c].copy() if want else None)
        c += int(bool(want))
    return keys, counts, sums, nonnull


def _exchange(mat, send_counts, group, device):
    """All-to-all of packed group rows (rows already ordered by destination rank)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ncol = mat.shape[1]
    sc = torch.tensor(send_counts, dtype=torch.int64, device=device)
    rc = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(r) for r in rc.cpu()]
    src = torch.from_numpy(np.ascontiguousarray(mat).reshape(-1)).to(device)
    dst = torch.empty(sum(recv_counts) * ncol, dtype=torch.int64, device=device)
    dist.all_to_all_single(dst, src, [r * ncol for r in recv_counts], [s * ncol for s in send_counts],
                           group=group)
    return dst.cpu().numpy().reshape(-1, ncol), recv_counts


def _all_gather_rows(mat, group, device):
    """All-gather of a variable number of packed rows per rank (sizes first, then padded)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ncol = mat.shape[1]
    n = torch.tensor([mat.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s) for s in torch.cat(sizes).cpu()]
    top = max(sizes)
    buf = np.zeros((top, ncol), np.int64)
    buf[:mat.shape[0]] = mat
    t = torch.from_numpy(buf.reshape(-1)).to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [o.cpu().numpy().reshape(top, ncol)[:s] for o, s in zip(outs, sizes)]


def combine_groups(local, group=None):
    """Merge every rank's fused-groupby result by hash partition: each group
    row goes to its owner rank (:func:`group_owner`) in one all-to-all, owners merge what
    they received (:func:`merge_groups`, senders in rank order, so float sums add in the
    same order as a merge of all ranks' parts), and the disjoint owner results are
    all-gathered so every rank holds the whole key-sorted result.  Each group crosses the
    links twice (to its owner, then to every rank) instead of every rank receiving every
    other rank's full table.  Over "nccl" the exchanges run on HBM tensors (RCCL / xGMI),
    over "gloo" through host memory."""
    import torch.distributed as dist
    keys, counts, sums, nonnull = local
    keys = np.asarray(keys)
    key_dtype = keys.dtype if keys.dtype == np.uint64 else np.dtype(np.int64)
    sums = [np.asarray(s) for s in sums]
    sum_dtypes = [s.dtype for s in sums]
    has_nn = [c is not None for c in nonnull]
    world = dist.get_world_size(group)
    device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    mat = _pack_groups(keys.astype(key_dtype, copy=False), counts, sums, nonnull)
    owner = group_owner(mat[:, 0], world)
    order = np.argsort(owner, kind="stable")  # keeps each destination's rows key-sorted
    send_counts = np.bincount(owner, minlength=world).tolist()
    recv, recv_counts = _exchange(mat[order], send_counts, group, device)
    parts, at = [], 0
    for r in recv_counts:
        parts.append(_unpack_groups(recv[at:at + r], key_dtype, sum_dtypes, has_nn))
        at += r
    merged = merge_groups(parts)
    if merged is None:
        merged = _unpack_groups(np.empty((0, mat.shape[1]), np.int64), key_dtype, sum_dtypes, has_nn)
    owned = _pack_groups(*merged)
    gathered = np.concatenate(_all_gather_rows(owned, group, device), axis=0)
    out = _unpack_groups(gathered, key_dtype, sum_dtypes, has_nn)
    order = np.argsort(out[0], kind="stable")
    return (out[0][order], out[1][order], [s[order] for s in out[2]],
            [None if c is None else c[order] for c in out[3]])


def combine_sets(local_set, group=None):
    """Replace a rank's ordered set by the global one (all-gather of key arrays)."""
    import torch.distributed as dist
    keys = local_set.key_array()
    null_index = int(local_set.null_value) if local_set.has_null else -1
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, (keys, null_index), group=group)
    return merge_key_arrays(gathered, lambda: type(local_set)())
