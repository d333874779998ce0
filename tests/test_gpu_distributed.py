"""ExecutorDistributed on the GPU.

* Two ranks (processes) share the box's GPU: each bins its row shard with the HIP library,
  the task parts are combined over the CPU exchange (RCCL refuses two ranks on one
  device), and every query must equal the single-process result.
* One rank over RCCL (libvaexhip's own communicator, vh_comm_*): the in-place HBM grid
  all-reduce for every aggregator kind (count / sum / min / max / first, 16-bit min/max
  through the all-gather fold), and the device hash-partition exchange of groupby results
  (vh_hashagg_exchange) behind DataFrame.groupby -- results equal the single-process ones
  bit for bit.  (The box has one GPU: world > 1 over RCCL runs at round end on 8 GPUs.)
"""
import multiprocessing as mp
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    rng = np.random.default_rng(11)
    n = 300_003
    x = rng.normal(size=n)
    y = rng.normal(size=n)
    w = rng.random(n)
    x[::997] = np.nan
    key = rng.integers(0, 5000, n).astype(np.int32) * 7 - 300
    # sparse keys (value span >> rows): DataFrame.groupby takes the fused hash path
    skey = (rng.integers(0, 20000, n).astype(np.int64) * 104729 - 10 ** 9).astype(np.int32)
    c = rng.integers(0, 40, n).astype(np.int16)
    return dict(x=x, y=y, w=w, key=key, skey=skey, c=c)


def _queries(df):
    import vaex_amd
    out = {}
    out["count"] = np.asarray(df.count(binby=["x", "y"], limits=[[-3, 3], [-3, 3]], shape=64))
    out["sum"] = np.asarray(df.sum("w", binby=["x", "y"], limits=[[-3, 3], [-3, 3]], shape=64))
    out["mean"] = np.asarray(df.mean("w", binby=["x"], limits=[-3, 3], shape=100))
    out["minmax"] = np.asarray(df.minmax("x"))
    out["count_minmax"] = np.asarray(df.count(binby=["x"], limits="minmax", shape=32))
    out["cmax"] = np.asarray(df.max("c", binby=["x"], limits=[-3, 3], shape=40))
    out["first"] = np.asarray(df.first("w", "y", binby=["x"], limits=[-3, 3], shape=20))
    for mode, sparse in (("dense", "auto"), ("hash", True)):
        g = df.groupby("key", agg={"v_sum": vaex_amd.agg.sum("w"), "n": "count"}, sort=True, assume_sparse=sparse)
        out[f"gb_{mode}_key"] = np.asarray(g["key"].to_numpy())
        out[f"gb_{mode}_sum"] = np.asarray(g["v_sum"].to_numpy())
        out[f"gb_{mode}_n"] = np.asarray(g["n"].to_numpy())
    g = df.groupby("key", agg={"nu": vaex_amd.agg.nunique("c"), "nu_sel": vaex_amd.agg.nunique("c", selection="x > 0")},
                   sort=True)
    out["gb_nunique"] = np.asarray(g["nu"].to_numpy())
    out["gb_nunique_sel"] = np.asarray(g["nu_sel"].to_numpy())
    g = df.groupby("skey", agg={"w": ["sum", "count", "mean"]})
    for c in g.get_column_names():
        out[f"gb_fused_{c}"] = np.asarray(g[c].to_numpy())
    return out


def _check_vs_oracle(got):
    """The query set's grids and groupbys against the oracle (not only against another run of
    the product): 2-d count / sum, 1-d mean, max of an int16 column, first, and the dense /
    hash / fused groupby sums and counts (map comparison for the unsorted fused result)."""
    d = _data()
    x, y, w, c = d["x"], d["y"], d["w"], d["c"]
    sx = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=64)
    sy = oracle.Binner("scalar", y, vmin=-3, vmax=3, bins=64)
    np.testing.assert_array_equal(got["count"], oracle.extract_central_part(oracle.compute_grid([sx, sy], "count")))
    np.testing.assert_allclose(got["sum"], oracle.extract_central_part(oracle.compute_grid([sx, sy], "sum", data=w)),
                               rtol=1e-9, atol=1e-12)
    s1 = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=100)
    cs = oracle.extract_central_part(oracle.compute_grid([s1], "sum", data=w))
    cc = oracle.extract_central_part(oracle.compute_grid([s1], "count", data=w))
    with np.errstate(invalid="ignore", divide="ignore"):
        np.testing.assert_allclose(got["mean"], cs / cc, rtol=1e-9, atol=1e-12)
    s40 = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=40)
    np.testing.assert_array_equal(got["cmax"], oracle.extract_central_part(oracle.compute_grid([s40], "max", data=c)))
    s20 = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=20)
    np.testing.assert_array_equal(got["first"], oracle.extract_central_part(oracle.compute_grid([s20], "first", data=w, data2=y)))
    uk, us, un = oracle.groupby_reference(d["key"], w)
    for mode in ("dense", "hash"):
        np.testing.assert_array_equal(got[f"gb_{mode}_key"], uk)
        np.testing.assert_array_equal(got[f"gb_{mode}_n"], un)
        np.testing.assert_allclose(got[f"gb_{mode}_sum"], us, rtol=1e-9, atol=1e-9)
    fk, fs, fn = oracle.groupby_reference(d["skey"], w)
    keys = got["gb_fused_skey"]
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(keys[order], fk)
    cols = [k for k in got if k.startswith("gb_fused_") and k != "gb_fused_skey"]
    assert len(cols) == 3, cols
    for k in cols:  # count(*) (named after the column, groupby.py's naming), sum, mean
        v = got[k][order]
        if v.dtype.kind in "iu":
            np.testing.assert_array_equal(v, fn, err_msg=k)
        elif "mean" in k:
            np.testing.assert_allclose(v, fs / fn, rtol=1e-9, atol=1e-12, err_msg=k)
        else:
            np.testing.assert_allclose(v, fs, rtol=1e-9, atol=1e-9, err_msg=k)


def _compare(got, ref):
    for k, v in ref.items():
        if k.endswith("sum") or k.endswith("mean") or k == "mean":
            np.testing.assert_allclose(got[k], v, rtol=1e-9, atol=1e-12, err_msg=k)
        else:
            np.testing.assert_array_equal(got[k], v, err_msg=k)


def _worker(rank, world, path, port):
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd import comm
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.distributed import ExecutorDistributed
    c = comm.init("host", rank=rank, world=world, addr="127.0.0.1", port=port, timeout=120)
    df = DataFrame(_data(), executor=ExecutorDistributed(c, shard_rows=True))
    out = _queries(df)
    if rank == 0:
        np.savez(path, **out)
    c.barrier()
    c.close()


def test_two_rank_executor_matches_single_process():
    import vaex_amd
    port = _free_port()
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.npz")
        procs = [ctx.Process(target=_worker, args=(r, 2, path, port)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        got = dict(np.load(path))
    _compare(got, _queries(vaex_amd.from_arrays(**_data())))
    _check_vs_oracle(got)


def _rccl_worker(path, port):
    import sys
    sys.path.insert(0, ROOT)
    import vaex_amd
    from vaex_amd import comm, superagg
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.distributed import ExecutorDistributed, allreduce_aggs
    c = comm.init("rccl", rank=0, world=1, addr="127.0.0.1", port=port, timeout=60)
    assert c.device and c.backend == "rccl"
    rng = np.random.default_rng(5)
    n = 500_000
    x = rng.normal(size=n)
    w = rng.normal(size=n)
    o = rng.permutation(n).astype(np.float64)
    i16 = rng.integers(-30000, 30000, n).astype(np.int16)
    u64 = rng.integers(0, 2 ** 60, n, dtype=np.uint64)
    out = {}
    b = superagg.BinnerScalar_float64("x", -3, 3, 77)
    b.set_data(x)
    grid = superagg.Grid([b])
    aggs = {"count": superagg.AggCount_float64(grid), "sum": superagg.AggSum_float64(grid),
            "min": superagg.AggMin_float64(grid), "max": superagg.AggMax_float64(grid),
            "first": superagg.AggFirst_float64(grid), "min16": superagg.AggMin_int16(grid),
            "sumu64": superagg.AggSum_uint64(grid)}
    for k in ("sum", "min", "max"):
        aggs[k].set_data(w, 0)
    aggs["first"].set_data(w, 0)
    aggs["first"].set_data(o, 1)
    aggs["min16"].set_data(i16, 0)
    aggs["sumu64"].set_data(u64, 0)
    grid.bin(list(aggs.values()))
    before = {k: np.asarray(a).copy() for k, a in aggs.items()}
    before["first_order"] = np.asarray(aggs["first"].order_grid()).copy()
    allreduce_aggs(list(aggs.values()), c)
    for k, a in aggs.items():
        out[k] = np.asarray(a).copy()
        out[k + "_before"] = before[k]
    out["first_order"] = np.asarray(aggs["first"].order_grid()).copy()
    out["first_order_before"] = before["first_order"]
    df = DataFrame(_data(), executor=ExecutorDistributed(c, shard_rows=True))
    for k, v in _queries(df).items():
        out["q_" + k] = v
    out["scalar"] = np.array([c.allreduce(np.array([2.5]), "sum")[0]])
    c.barrier()
    np.savez(path, **out)
    c.close()


def test_rccl_single_rank_grids_and_groupby_exchange():
    import vaex_amd
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "r.npz")
        p = ctx.Process(target=_rccl_worker, args=(path, _free_port()))
        p.start()
        p.join(300)
        assert p.exitcode == 0
        got = dict(np.load(path))
    for k in ("count", "sum", "min", "max", "first", "min16", "sumu64", "first_order"):
        np.testing.assert_array_equal(got[k], got[k + "_before"], err_msg=k)
    assert got["scalar"][0] == 2.5
    ref = _queries(vaex_amd.from_arrays(**_data()))
    _compare({k[2:]: v for k, v in got.items() if k.startswith("q_")}, ref)
    # the grids themselves against the oracle (the all-reduce kept them intact)
    rng = np.random.default_rng(5)
    n = 500_000
    x, w = rng.normal(size=n), rng.normal(size=n)
    spec = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=77)
    np.testing.assert_array_equal(got["count"], oracle.compute_grid([spec], "count"))
    np.testing.assert_allclose(got["sum"], oracle.compute_grid([spec], "sum", data=w), rtol=1e-9, atol=1e-12)


def _exchange_worker(path, port):
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd import comm
    from vaex_amd.hashagg import HashAgg
    c = comm.init("rccl", rank=0, world=1, addr="127.0.0.1", port=port, timeout=60)
    rng = np.random.default_rng(3)
    keys = (rng.integers(-10 ** 6, 10 ** 6, 400_000) * 7919).astype(np.int64)
    v = rng.normal(size=len(keys))
    v[::13] = np.nan
    u = rng.integers(0, 100, len(keys)).astype(np.uint8)
    ha = HashAgg(keys.dtype, [v.dtype, u.dtype], [True, False])
    ha.update(keys, [v, u])
    # world 1: the exchange path (owner, pack, all-to-all, fold, gather) must hand back the
    # same groups it was given
    k1, c1, s1, n1 = ha.finish()
    ha2 = HashAgg(keys.dtype, [v.dtype, u.dtype], [True, False])
    ha2.update(keys, [v, u])
    # HashAgg.finish skips the exchange at world 1: drive the C-ABI directly
    from vaex_amd import _lib
    import ctypes
    m = ctypes.c_uint64()
    _lib.call("vh_hashagg_finish", ha2._h, ctypes.byref(m))
    _lib.call("vh_hashagg_exchange", ha2._h, c.handle, 1)
    _lib.call("vh_hashagg_finish", ha2._h, ctypes.byref(m))
    k2, c2, s2, n2 = ha2._read(m.value)
    np.savez(path, k1=k1, c1=c1, s1a=s1[0], s1b=s1[1], n1=n1[0], k2=k2, c2=c2, s2a=s2[0], s2b=s2[1], n2=n2[0],
             keys=keys, v=v)
    c.close()


def test_rccl_hashagg_exchange_roundtrip():
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "x.npz")
        p = ctx.Process(target=_exchange_worker, args=(path, _free_port()))
        p.start()
        p.join(300)
        assert p.exitcode == 0
        got = np.load(path)
    for a, b in (("k1", "k2"), ("c1", "c2"), ("s1b", "s2b"), ("n1", "n2")):
        np.testing.assert_array_equal(got[a], got[b], err_msg=a)
    # two independent updates: float sums in different atomic orders
    np.testing.assert_allclose(got["s1a"], got["s2a"], rtol=1e-12, atol=1e-15)
    uk, s, cnt = oracle.groupby_reference(got["keys"], got["v"])
    np.testing.assert_array_equal(got["k2"], uk)
    np.testing.assert_array_equal(got["n2"], cnt)
    np.testing.assert_allclose(got["s2a"], s, rtol=1e-9, atol=1e-9)
