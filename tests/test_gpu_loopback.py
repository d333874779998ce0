"""Multi-rank device code on one GPU: the library's loopback communicator
(``vh_comm_loopback``) hosts N virtual ranks in this process, one thread each, behind the
same C-ABI as RCCL.  What runs here with N ranks' data is the device code around the
collectives that a world-1 RCCL run reduces to a self-copy:

* the rank-order device fold of an all-reduce (``k_fold_ranks``, every dtype and op);
* ``vh_comm_agg_allreduce``: count / sum / moment / min / max grids and AggFirst's
  (value, order) rule across ranks, ties to the lower rank (``k_first_ranks``;
  reference rule ``superagg.cpp:470-480`` applied to the parts in rank order,
  ``execution.py:279-289``);
* ``vh_hashagg_exchange``: owner hash, device pack, the all-to-all segment sizes, the
  sort-and-fold of received groups (``k_xo_*``), and the padded all-gather;
* ``ExecutorDistributed`` end to end: the C4 query ``mean(w, binby=[x, y], shape=1024)``
  with rows sharded, and the C3 / C5 hash groupby through the device exchange.

Every result is compared with the single-process oracle on the whole data.
"""
import concurrent.futures as cf
import ctypes

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

WORLDS = [2, 3, 8]


def run_ranks(world, fn, *args):
    """fn(comm, *args) on `world` loopback ranks (one thread each); results in rank order."""
    from vaex_amd import comm as vcomm
    comms = vcomm.loopback_group(world)
    try:
        with cf.ThreadPoolExecutor(world) as ex:
            futs = [ex.submit(fn, c, *args) for c in comms]
            return [f.result(timeout=300) for f in futs]
    finally:
        for c in comms:
            c.close()


def shard(n, rank, world):
    from vaex_amd.distributed import shard_range
    return slice(*shard_range(n, rank, world))


# ---- raw collectives ----------------------------------------------------------------------
NUMERIC = ["float64", "float32", "int64", "int32", "int16", "int8", "uint64", "uint32", "uint16", "uint8", "bool"]


def _rank_data(dtype, rank, n):
    rng = np.random.default_rng(100 + rank)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        a = rng.normal(scale=1e3, size=n).astype(dt)
        a[::17] = -0.0
    elif dt.kind == "b":
        a = rng.integers(0, 2, n).astype(bool)
    else:
        info = np.iinfo(dt)
        a = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    return a


def _allreduce_rank(c, n):
    from vaex_amd.comm import reduce_arrays
    from vaex_amd.device import DeviceArray
    out = {}
    for dtype in NUMERIC:
        for op in ("sum", "min", "max"):
            if dtype == "bool" and op == "sum":
                continue
            mine = _rank_data(dtype, c.rank, n)
            d = DeviceArray.from_numpy(mine)
            c.allreduce_device(d.ptr, n, np.dtype(dtype), op)
            got_dev = d.to_numpy()
            got_host = c.allreduce(mine, op)  # host buffer: staged through HBM
            want = reduce_arrays([_rank_data(dtype, r, n) for r in range(c.world)], op)
            out[(dtype, op)] = (got_dev, got_host, want)
    return out


@pytest.mark.parametrize("world", WORLDS)
def test_loopback_allreduce_every_dtype_and_op(world):
    n = 1031
    for res in run_ranks(world, _allreduce_rank, n):
        for (dtype, op), (got_dev, got_host, want) in res.items():
            # rank-order fold == the serial merge order: bit-exact, floats included
            np.testing.assert_array_equal(got_dev.view(np.uint8), want.view(np.uint8), err_msg=f"{dtype} {op}")
            np.testing.assert_array_equal(got_host.view(np.uint8), want.view(np.uint8), err_msg=f"{dtype} {op} host")


def _gather_a2a_rank(c, sizes):
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    W, r = c.world, c.rank
    # all-gather of 40 bytes per rank
    send = np.full(40, r + 1, np.uint8)
    ds, dr = DeviceArray.from_numpy(send), DeviceArray.empty(40 * W, np.uint8)
    _lib.call("vh_comm_allgather", c.handle, ds.ptr, dr.ptr, 40, _lib.LOC_DEVICE)
    gathered = dr.to_numpy()
    # all-to-all: rank s sends sizes[s][d] bytes valued (s * 16 + d) to rank d
    sb = np.array(sizes[r], np.uint64)
    rb = np.array([sizes[s][r] for s in range(W)], np.uint64)
    payload = np.concatenate([np.full(int(sizes[r][d]), r * 16 + d, np.uint8) for d in range(W)])
    dsend = DeviceArray.from_numpy(payload if len(payload) else np.zeros(1, np.uint8))
    drecv = DeviceArray.empty(max(1, int(rb.sum())), np.uint8)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    _lib.call("vh_comm_alltoallv", c.handle, dsend.ptr, sb.ctypes.data_as(u64p), drecv.ptr, rb.ctypes.data_as(u64p),
              _lib.LOC_DEVICE)
    recv = drecv.to_numpy()[:int(rb.sum())]
    c.barrier()
    return gathered, recv


@pytest.mark.parametrize("world", WORLDS)
def test_loopback_allgather_and_alltoallv_segments(world):
    rng = np.random.default_rng(world)
    sizes = rng.integers(0, 300, (world, world))
    sizes[0, :] = 0  # a rank that sends nothing
    sizes[:, world - 1] = 0  # a rank that receives nothing
    res = run_ranks(world, _gather_a2a_rank, sizes.tolist())
    for r, (gathered, recv) in enumerate(res):
        np.testing.assert_array_equal(gathered, np.repeat(np.arange(1, world + 1, dtype=np.uint8), 40))
        want = np.concatenate([np.full(sizes[s][r], s * 16 + r, np.uint8) for s in range(world)])
        np.testing.assert_array_equal(recv, want)


def _mismatch_rank(c):
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    d = DeviceArray.empty(16, np.uint8)
    try:
        if c.rank == 0:
            _lib.call("vh_comm_allgather", c.handle, d.ptr, d.ptr, 8, _lib.LOC_DEVICE)
        else:
            z = np.zeros(c.world, np.uint64)
            u64p = ctypes.POINTER(ctypes.c_uint64)
            _lib.call("vh_comm_alltoallv", c.handle, d.ptr, z.ctypes.data_as(u64p), d.ptr, z.ctypes.data_as(u64p),
                      _lib.LOC_DEVICE)
    except _lib.HipError as e:
        return str(e)
    return None


def test_loopback_mismatched_collectives_fail_every_rank():
    msgs = run_ranks(2, _mismatch_rank)
    assert all(m is not None and "different collectives" in m for m in msgs), msgs


# ---- aggregator grids across ranks --------------------------------------------------------
def _agg_data(n):
    rng = np.random.default_rng(7)
    x = rng.normal(size=n)
    x[::101] = np.nan
    w = rng.normal(size=n)
    w[::37] = np.nan
    # order values with many ties, across rank boundaries too: AggFirst keeps the earliest
    # row, i.e. the lower rank
    o = rng.integers(0, 40, n).astype(np.float64)
    i16 = rng.integers(-30000, 30000, n).astype(np.int16)
    u64 = rng.integers(0, 2 ** 62, n, dtype=np.uint64)
    f32 = rng.normal(size=n).astype(np.float32)
    return x, w, o, i16, u64, f32


def _agg_rank(c, n):
    from vaex_amd import superagg
    from vaex_amd.distributed import allreduce_aggs
    x, w, o, i16, u64, f32 = (a[shard(n, c.rank, c.world)] for a in _agg_data(n))
    b = superagg.BinnerScalar_float64("x", -3, 3, 61)
    b.set_data(x)
    grid = superagg.Grid([b])
    aggs = {"count": superagg.AggCount_float64(grid), "countw": superagg.AggCount_float64(grid),
            "sum": superagg.AggSum_float64(grid), "min": superagg.AggMin_float64(grid),
            "max": superagg.AggMax_float64(grid), "first": superagg.AggFirst_float64(grid),
            "min16": superagg.AggMin_int16(grid), "max16": superagg.AggMax_int16(grid),
            "sum16": superagg.AggSum_int16(grid), "sumu64": superagg.AggSum_uint64(grid),
            "mom2": superagg.AggSumMoment_float64(grid, 2), "minf32": superagg.AggMin_float32(grid),
            "firstf32": superagg.AggFirst_float32(grid)}
    for k in ("countw", "sum", "min", "max", "mom2"):
        aggs[k].set_data(w, 0)
    aggs["first"].set_data(w, 0)
    aggs["first"].set_data(o, 1)
    for k in ("min16", "max16", "sum16"):
        aggs[k].set_data(i16, 0)
    aggs["sumu64"].set_data(u64, 0)
    aggs["minf32"].set_data(f32, 0)
    aggs["firstf32"].set_data(f32, 0)
    aggs["firstf32"].set_data(o.astype(np.float32), 1)
    grid.bin(list(aggs.values()))
    allreduce_aggs(list(aggs.values()), c)
    out = {k: np.asarray(a).copy() for k, a in aggs.items()}
    out["first_order"] = np.asarray(aggs["first"].order_grid()).copy()
    return out


@pytest.mark.parametrize("world", WORLDS)
def test_loopback_agg_allreduce_matches_oracle(world):
    n = 400_009
    x, w, o, i16, u64, f32 = _agg_data(n)
    spec = [oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=61)]
    want = {"count": oracle.compute_grid(spec, "count"), "countw": oracle.compute_grid(spec, "count", data=w),
            "sum": oracle.compute_grid(spec, "sum", data=w), "min": oracle.compute_grid(spec, "min", data=w),
            "max": oracle.compute_grid(spec, "max", data=w), "first": oracle.compute_grid(spec, "first", data=w, data2=o),
            "min16": oracle.compute_grid(spec, "min", data=i16), "max16": oracle.compute_grid(spec, "max", data=i16),
            "sum16": oracle.compute_grid(spec, "sum", data=i16), "sumu64": oracle.compute_grid(spec, "sum", data=u64),
            "mom2": oracle.compute_grid(spec, "sum_moment", data=w, moment=2),
            "minf32": oracle.compute_grid(spec, "min", data=f32),
            "firstf32": oracle.compute_grid(spec, "first", data=f32, data2=o.astype(np.float32))}
    # the order grid AggFirst keeps: the smallest order per cell
    idx = oracle.bin_indices(spec, n)
    og, _ = oracle.new_grid("first", "float64", oracle.grid_shape(spec))
    og2 = np.full_like(og, np.finfo(np.float64).max)
    oracle.aggregate("first", idx, og, data=w, data2=o, grid2=og2)
    for r, got in enumerate(run_ranks(world, _agg_rank, n)):
        for k, v in want.items():
            if k in ("sum", "mom2"):
                np.testing.assert_allclose(got[k], v, rtol=1e-9, atol=1e-9, err_msg=f"rank {r} {k}")
            else:
                np.testing.assert_array_equal(got[k], v, err_msg=f"rank {r} {k}")
        np.testing.assert_array_equal(got["first_order"].ravel(order="F"), og2, err_msg=f"rank {r} first order")


# ---- C4: mean(w, binby=[x, y], shape=1024), rows sharded ----------------------------------
def _c4_data(n):
    rng = np.random.default_rng(44)
    x, y, w = rng.normal(size=n), rng.normal(size=n), rng.random(n)
    w[::1000] = np.nan
    return x, y, w


def _c4_rank(c, n):
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.distributed import ExecutorDistributed
    x, y, w = _c4_data(n)
    df = DataFrame({"x": x, "y": y, "w": w}, executor=ExecutorDistributed(c, shard_rows=True))
    mean = np.asarray(df.mean("w", binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024))
    count = np.asarray(df.count(binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024))
    return mean, count


@pytest.mark.parametrize("world", WORLDS)
def test_loopback_c4_mean_rows_sharded(world):
    n = 3_000_017
    x, y, w = _c4_data(n)
    spec = [oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024), oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)]
    s = oracle.extract_central_part(oracle.compute_grid(spec, "sum", data=w))
    cw = oracle.extract_central_part(oracle.compute_grid(spec, "count", data=w))
    cnt = oracle.extract_central_part(oracle.compute_grid(spec, "count"))
    with np.errstate(divide="ignore", invalid="ignore"):
        want = s / cw
    for mean, count in run_ranks(world, _c4_rank, n):
        np.testing.assert_array_equal(count, cnt)
        np.testing.assert_allclose(mean, want, rtol=1e-9, atol=1e-12, equal_nan=True)


# ---- groupby partition exchange -----------------------------------------------------------
def _gb_data(n, kind):
    rng = np.random.default_rng(9)
    if kind == "int64":
        keys = (rng.integers(-10 ** 5, 10 ** 5, n) * 7919).astype(np.int64)
    elif kind == "uint64":
        keys = (rng.integers(0, 50_000, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))  # above 2^63 too
    else:
        keys = rng.integers(-40_000, 40_000, n).astype(np.int32)
    v = rng.normal(size=n)
    v[::13] = np.nan
    u = rng.integers(0, 200, n).astype(np.uint8)
    return keys, v, u


def _exchange_rank(c, n, kind, gather):
    from vaex_amd.hashagg import HashAgg
    keys, v, u = (a[shard(n, c.rank, c.world)] for a in _gb_data(n, kind))
    ha = HashAgg(keys.dtype, [v.dtype, u.dtype], [True, False])
    ha.update(keys, [v, u])
    k, cnt, sums, nonnull = ha.finish(c, gather=gather)
    return np.array(k), np.array(cnt), np.array(sums[0]), np.array(sums[1]), np.array(nonnull[0])


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("kind", ["int32", "int64", "uint64"])
@pytest.mark.parametrize("gather", [True, False])
def test_loopback_hashagg_exchange_matches_oracle(world, kind, gather):
    from vaex_amd.distributed import group_owner
    n = 600_011
    keys, v, u = _gb_data(n, kind)
    uk, s, nn = oracle.groupby_reference(keys, v)
    cnt = np.unique(keys, return_counts=True)[1]
    su = np.bincount(np.unique(keys, return_inverse=True)[1], weights=u.astype(np.float64)).astype(np.uint64)
    res = run_ranks(world, _exchange_rank, n, kind, gather)
    if gather:
        parts = res
    else:
        # each rank keeps exactly the groups it owns
        for r, (k, *_rest) in enumerate(res):
            kb = k.view(np.uint64) if kind == "uint64" else k.astype(np.int64)
            assert np.all(group_owner(kb, world) == r), r
        allk = np.concatenate([p[0] for p in res])
        order = np.argsort(allk.view(np.uint64) if kind == "uint64" else allk, kind="stable")
        parts = [tuple(np.concatenate([p[i] for p in res])[order] for i in range(5))]
    for k, c, s1, s2, n1 in parts:
        k = k.view(np.uint64) if kind == "uint64" else k.astype(keys.dtype)
        np.testing.assert_array_equal(k, uk)
        np.testing.assert_array_equal(c, cnt)
        np.testing.assert_array_equal(n1, nn)
        np.testing.assert_array_equal(s2, su)
        np.testing.assert_allclose(s1, s, rtol=1e-9, atol=1e-9)


def _queries_rank(c):
    from test_gpu_distributed import _data, _queries
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.distributed import ExecutorDistributed
    return _queries(DataFrame(_data(), executor=ExecutorDistributed(c, shard_rows=True)))


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_executor_queries_match_single_process(world):
    """The whole distributed query set (grids, limits, first, dense / hash / nunique / fused
    groupby) with the device exchange, every rank's result against one process's and against
    the oracle."""
    import vaex_amd
    from test_gpu_distributed import _check_vs_oracle, _compare, _data, _queries
    ref = _queries(vaex_amd.from_arrays(**_data()))
    _check_vs_oracle(ref)
    for got in run_ranks(world, _queries_rank):
        _compare(got, ref)
        _check_vs_oracle(got)
