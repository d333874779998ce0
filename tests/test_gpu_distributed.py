"""ExecutorDistributed on the GPU: two ranks (processes) share the box's GPU, each bins its
row shard with the HIP library, task parts are combined over gloo (host-memory path; the
RCCL path runs the same combine on HBM grids), and every query must equal the
single-process result: counts / groupby keys exact, float sums within 1e-9 relative."""
import os
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


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
    out = {}
    out["count"] = np.asarray(df.count(binby=["x", "y"], limits=[[-3, 3], [-3, 3]], shape=64))
    out["sum"] = np.asarray(df.sum("w", binby=["x", "y"], limits=[[-3, 3], [-3, 3]], shape=64))
    out["mean"] = np.asarray(df.mean("w", binby=["x"], limits=[-3, 3], shape=100))
    out["minmax"] = np.asarray(df.minmax("x"))
    out["count_minmax"] = np.asarray(df.count(binby=["x"], limits="minmax", shape=32))
    for mode, sparse in (("dense", "auto"), ("hash", True)):
        g = df.groupby("key", agg={"v_sum": __import__("vaex_amd").agg.sum("w"), "n": "count"}, sort=True,
                       assume_sparse=sparse)
        out[f"gb_{mode}_key"] = np.asarray(g["key"].to_numpy())
        out[f"gb_{mode}_sum"] = np.asarray(g["v_sum"].to_numpy())
        out[f"gb_{mode}_n"] = np.asarray(g["n"].to_numpy())
    g = df.groupby("key", agg={"nu": __import__("vaex_amd").agg.nunique("c"),
                               "nu_sel": __import__("vaex_amd").agg.nunique("c", selection="x > 0")}, sort=True)
    out["gb_nunique"] = np.asarray(g["nu"].to_numpy())
    out["gb_nunique_sel"] = np.asarray(g["nu_sel"].to_numpy())
    g = df.groupby("skey", agg={"w": ["sum", "count", "mean"]})
    for c in g.get_column_names():
        out[f"gb_fused_{c}"] = np.asarray(g[c].to_numpy())
    return out


def _worker(rank, world, path):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.distributed import ExecutorDistributed
    df = DataFrame(_data(), executor=ExecutorDistributed(shard_rows=True))
    out = _queries(df)
    if rank == 0:
        np.savez(path, **out)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_executor_matches_single_process():
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    import vaex_amd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(31500 + os.getpid() % 1000)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.npz")
        mp.spawn(_worker, args=(2, path), nprocs=2, join=True)
        got = dict(np.load(path))
    ref = _queries(vaex_amd.from_arrays(**_data()))
    for k, v in ref.items():
        if k.endswith("sum") or k.endswith("mean") or k == "mean":
            np.testing.assert_allclose(got[k], v, rtol=1e-9, atol=1e-12, err_msg=k)
        else:
            np.testing.assert_array_equal(got[k], v, err_msg=k)


def _nccl_groups_worker(rank, world, path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    from vaex_amd.distributed import combine_groups
    rng = np.random.default_rng(3)
    keys = np.unique(rng.integers(-10 ** 12, 10 ** 12, 70_000))
    counts = rng.integers(1, 9, len(keys)).astype(np.int64)
    sums = rng.normal(size=len(keys))
    nn = rng.integers(0, 9, len(keys)).astype(np.int64)
    gk, gc, gs, gn = combine_groups((keys, counts, [sums], [nn]))
    np.savez(path, keys=keys, counts=counts, sums=sums, nn=nn, gk=gk, gc=gc, gs=gs[0], gn=gn[0])
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_group_exchange_single_rank():
    """The hash-partition all-to-all + all-gather of groupby results on HBM tensors over RCCL
    (one rank on the box's GPU): the exchange must hand back every group bit-exactly."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(34500 + os.getpid() % 1000)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "g.npz")
        mp.spawn(_nccl_groups_worker, args=(1, path), nprocs=1, join=True)
        got = np.load(path)
    for a, b in (("keys", "gk"), ("counts", "gc"), ("sums", "gs"), ("nn", "gn")):
        np.testing.assert_array_equal(got[a], got[b], err_msg=a)
