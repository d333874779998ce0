"""Multi-GPU binning and groupby: one process per GPU, rows sharded by range, results
combined with one exchange step.  No PyTorch: the collectives are RCCL
bound by libvaexhip (:class:`vaex_amd.comm.RcclComm`), or the CPU exchange
(:class:`vaex_amd.comm.HostComm`) on which the multi-process tests run the same code.

The reference has no multi-process path (its ``reduce`` merges per-thread private grids,
``superagg.cpp:160-167``); here every rank bins its own row range into its own HBM grids,
then:

* dense grids are all-reduced in place on HBM (``vh_comm_agg_allreduce``): SUM for
  count / sum / moment grids, MIN / MAX for min / max grids, AggFirst by (order, rank) on
  the device (``superagg.cpp:470-480``);
* fused-groupby results are exchanged by hash partition on the device
  (``vh_hashagg_exchange``): every group row to owner ``splitmix64(key) % world``, owners
  fold equal keys in rank order;
* limits (min/max), flags, ordered-set key arrays and AggNUnique value sets are small and
  travel through the communicator's host path.

Over :class:`HostComm` the same combines run through host memory (grids downloaded,
folded in rank order, uploaded; groups merged with numpy) -- the rules are written against
plain arrays (:func:`combine_grids`, :func:`combine_groups`) so they run without a GPU.
"""
import ctypes

import numpy as np

from . import comm as vcomm
from .execution import ExecutorLocal


def shard_range(n, rank, world):
    """Contiguous row range [i1, i2) of ``rank`` out of ``world``."""
    return n * rank // world, n * (rank + 1) // world


def _comm(comm):
    return comm if comm is not None else vcomm.get()


def _reduce_op_for(kind):
    return {"AggCount": "sum", "AggSum": "sum", "AggSumMoment": "sum", "AggMin": "min", "AggMax": "max",
            "AggFirst": "first"}[kind]


def combine_grids(kind, grid, order=None, comm=None):
    """One flattened grid (numpy) combined over the ranks by aggregator kind: returns
    (grid, order).  AggFirst keeps the value of the smallest order, the lower rank on ties
    (superagg.cpp:470-480 applied to the ranks' parts in rank order)."""
    comm = _comm(comm)
    op = _reduce_op_for(kind)
    if op != "first":
        return comm.allreduce(grid, op), None
    parts = comm.allgather((np.asarray(grid), np.asarray(order)))
    v, o = parts[0][0].copy(), parts[0][1].copy()
    for gv, go in parts[1:]:
        take = go < o
        v = np.where(take, gv, v)
        o = np.where(take, go, o)
    return v, o


def allreduce_aggs(aggs, comm=None):
    """Combine superagg aggregators' grids across the ranks: in place on HBM over RCCL, or
    through host memory over the CPU exchange."""
    comm = _comm(comm)
    from . import _lib
    for agg in aggs:
        agg._before_device_use()
        if comm.device:
            comm.agg_allreduce(agg)
        else:
            grid = np.empty(agg.grid.length1d, agg._grid_dtype)
            _lib.call("vh_agg_download", agg._handle, grid.ctypes.data, agg._nbytes)
            order = None
            if agg._kind == "AggFirst":
                order = np.empty(agg.grid.length1d, agg._grid_dtype)
                _lib.call("vh_agg_download_order", agg._handle, order.ctypes.data, agg._nbytes)
            grid, order = combine_grids(agg._kind, grid, order, comm)
            if order is not None:
                order = np.ascontiguousarray(order)
                _lib.call("vh_agg_upload_order", agg._handle, order.ctypes.data, agg._nbytes)
            grid = np.ascontiguousarray(grid)
            _lib.call("vh_agg_upload", agg._handle, grid.ctypes.data, agg._nbytes)
        agg._after_device_write()


def allreduce_scalar(value, op="sum", comm=None):
    """A Python float reduced over the ranks."""
    return float(_comm(comm).allreduce(np.array([float(value)]), op)[0])


def barrier(comm=None):
    _comm(comm).barrier()


def shutdown():
    vcomm.shutdown()


def combine_minmax(vmin, vmax, comm=None):
    """NaN-ignoring global (min, max) of per-rank limits (tasks.py:173-185 across ranks)."""
    lo = np.inf if np.isnan(vmin) else float(vmin)
    hi = -np.inf if np.isnan(vmax) else float(vmax)
    comm = _comm(comm)
    lo = float(comm.allreduce(np.array([lo]), "min")[0])
    hi = float(comm.allreduce(np.array([hi]), "max")[0])
    return (np.nan if np.isinf(lo) and lo > 0 else lo), (np.nan if np.isinf(hi) and hi < 0 else hi)


def all_ranks_true(flag, comm=None):
    """Logical AND of a per-rank flag (a MIN all-reduce)."""
    return bool(_comm(comm).allreduce(np.array([1 if flag else 0], np.int64), "min")[0])


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


def combine_sets(local_set, comm=None):
    """Replace a rank's ordered set by the global one (all-gather of key arrays)."""
    keys = local_set.key_array()
    null_index = int(local_set.null_value) if local_set.has_null else -1
    gathered = _comm(comm).allgather((keys, null_index))
    return merge_key_arrays(gathered, lambda: type(local_set)())


def nunique_state(agg):
    """(cells, values, nulls, nans) of an AggNUnique as host arrays (deduplicated pairs)."""
    from . import _lib
    n = ctypes.c_uint64()
    _lib.call("vh_agg_nunique_export", agg._handle, ctypes.byref(n), None, None, None, None)
    L = agg.grid.length1d
    cells, vals = np.empty(n.value, np.uint64), np.empty(n.value, np.uint64)
    nulls, nans = np.empty(L, np.uint64), np.empty(L, np.uint64)
    _lib.call("vh_agg_nunique_export", agg._handle, ctypes.byref(n), cells.ctypes.data, vals.ctypes.data,
              nulls.ctypes.data, nans.ctypes.data)
    return cells, vals, nulls, nans


def combine_nunique(agg, comm=None):
    """AggNUnique across ranks: every rank gathers the others' (cell, value) pairs and
    missing / NaN counts and merges them into its own (counter::merge,
    hash_primitives.hpp:393-415); distinct values are not additive, so no grid all-reduce."""
    from . import _lib
    comm = _comm(comm)
    gathered = comm.allgather(nunique_state(agg))
    for r, (cells, vals, nulls, nans) in enumerate(gathered):
        if r == comm.rank:
            continue
        cells, vals = np.ascontiguousarray(cells, np.uint64), np.ascontiguousarray(vals, np.uint64)
        nulls, nans = np.ascontiguousarray(nulls, np.uint64), np.ascontiguousarray(nans, np.uint64)
        _lib.call("vh_agg_nunique_import", agg._handle, len(cells), cells.ctypes.data, vals.ctypes.data,
                  nulls.ctypes.data, nans.ctypes.data)
    agg._after_device_write()


class ExecutorDistributed(ExecutorLocal):
    """ExecutorLocal over this rank's row shard, combining task parts across ranks.

    One process per GPU: with ``shard_rows`` every rank holds the same (e.g. memory-mapped)
    DataFrame and processes rows ``shard_range(n, rank, world)``; without it each rank's
    DataFrame already is its shard.  After the local parts are reduced: aggregator grids
    are combined (:func:`allreduce_aggs`), min/max limits are reduced, and ordered sets are
    merged from all ranks' key arrays (:func:`merge_key_arrays`) so every rank bins with
    the same global ordinals.
    """

    def __init__(self, comm=None, shard_rows=True, chunk_size=None):
        super().__init__(chunk_size)
        self.comm = _comm(comm)
        self.rank = self.comm.rank
        self.world = self.comm.world
        self.shard_rows = shard_rows

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
                    combine_nunique(agg, self.comm)
                allreduce_aggs([a for a in aggs if a._kind != "AggNUnique"], self.comm)
            elif isinstance(p, TaskPartMinMax):
                p.vmin, p.vmax = combine_minmax(p.vmin, p.vmax, self.comm)
            elif isinstance(p, TaskPartSetCreate):
                p.set = combine_sets(p.set, self.comm)


# ---- groupby results ------------------------------------------------------------------
def merge_groups(parts):
    """Merge per-rank fused-groupby results ``(keys, counts, sums, nonnull)`` (each sorted by
    key, hashagg.py) into one key-sorted result: counts and integer sums add exactly, float
    sums add in rank order.  ``nonnull`` entries may be None (not requested)."""
    parts = [p for p in parts if len(p[0])]
    if not parts:
        return None
    nv = len(parts[0][2])
    keys = np.concatenate([p[0] for p in parts])
    order = np.argsort(keys, kind="stable")  # equal keys stay in rank order
    keys = keys[order]
    heads = np.flatnonzero(np.r_[True, keys[1:] != keys[:-1]])
    uniq = keys[heads]

    def fold(cat):
        cat = cat[order]
        if cat.dtype.kind == "f":  # sequential adds in rank order within a key
            out = cat[heads].copy()
            run = np.diff(np.r_[heads, len(keys)])
            for k in range(1, int(run.max()) if len(run) else 1):
                sel = run > k
                out[sel] = out[sel] + cat[heads[sel] + k]
            return out
        return np.add.reduceat(cat, heads).astype(cat.dtype, copy=False)

    counts = fold(np.concatenate([p[1] for p in parts]).astype(np.int64))
    sums = [fold(np.concatenate([p[2][v] for p in parts])) for v in range(nv)]
    nonnull = [None if parts[0][3][v] is None else fold(np.concatenate([p[3][v] for p in parts]).astype(np.int64))
               for v in range(nv)]
    return uniq, counts, sums, nonnull


def group_owner(keys, world):
    """Owner rank of each group key: splitmix64 of the key's 64-bit pattern modulo the world
    size (SURVEY.md §8e hash partition; the device exchange uses the same function).
    ``keys``: int64 / uint64 array."""
    z = np.ascontiguousarray(keys).view(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world)).astype(np.int64)


def combine_groups(local, comm=None):
    """Merge every rank's fused-groupby result by hash partition (host path): each group row
    goes to its owner rank (:func:`group_owner`) in one all-to-all, owners merge what they
    received (:func:`merge_groups`, senders in rank order), and the disjoint owner results
    are all-gathered so every rank holds the whole key-sorted result.  The device path is
    ``HashAgg.exchange`` (vh_hashagg_exchange), same partition and fold order."""
    comm = _comm(comm)
    keys, counts, sums, nonnull = local
    keys = np.asarray(keys)
    key_dtype = keys.dtype if keys.dtype == np.uint64 else np.dtype(np.int64)
    keys = keys.astype(key_dtype, copy=False)
    sums = [np.asarray(s) for s in sums]
    owner = group_owner(keys, comm.world)
    out = []
    for d in range(comm.world):
        sel = owner == d  # keeps each destination's rows key-sorted
        out.append((keys[sel], np.asarray(counts)[sel], [s[sel] for s in sums],
                    [None if c is None else np.asarray(c)[sel] for c in nonnull]))
    recv = comm.alltoall(out)
    merged = merge_groups([(k, c, list(s), list(nn)) for k, c, s, nn in recv])
    if merged is None:
        merged = (np.empty(0, key_dtype), np.empty(0, np.int64), [s[:0] for s in sums],
                  [None if c is None else np.empty(0, np.int64) for c in nonnull])
    owned = comm.allgather(merged)
    keys = np.concatenate([o[0] for o in owned]).astype(key_dtype, copy=False)
    order = np.argsort(keys, kind="stable")
    counts = np.concatenate([o[1] for o in owned])[order]
    sums = [np.concatenate([o[2][v] for o in owned])[order] for v in range(len(sums))]
    nonnull = [None if nonnull[v] is None else np.concatenate([o[3][v] for o in owned])[order]
               for v in range(len(nonnull))]
    return keys[order], counts, sums, nonnull
