"""Multi-rank combine (vaex_amd/distributed.py) on CPU: several processes joined by the
CPU exchange (vaex_amd.comm.HostComm, the fake of the RCCL communicator), world 2 and 3.

Each rank bins its row shard with the oracle, the grids / groups / sets are combined with
the same exchange code the GPU path runs (over RCCL there), and the result must equal the
whole column processed at once: counts exact, sums within 1e-9 relative, min/max/first
exact.  No torch: the processes rendezvous through MASTER_ADDR / VAEX_AMD_COMM_PORT."""
import multiprocessing as mp
import os
import socket
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(target, world, path):
    """Run target(rank, world, path, port) in `world` fresh processes; every one must exit 0."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=target, args=(r, world, path, port)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _comm(rank, world, port):
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd import comm
    return comm.init("host", rank=rank, world=world, addr="127.0.0.1", port=port, timeout=60)


def _data():
    rng = np.random.default_rng(42)
    n = 60001
    x = rng.normal(size=n)
    w = rng.normal(size=n)
    o = rng.permutation(n).astype("f8")
    return x, w, o


def _grids(x, w, o):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle
    b = [oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=50)]
    return {
        "AggCount": (oracle.compute_grid(b, "count").ravel(order="F"), None),
        "AggSum": (oracle.compute_grid(b, "sum", data=w).ravel(order="F"), None),
        "AggMin": (oracle.compute_grid(b, "min", data=w).ravel(order="F"), None),
        "AggMax": (oracle.compute_grid(b, "max", data=w).ravel(order="F"), None),
        "AggFirst": _first(oracle, b, w, o),
    }


def _first(oracle, b, w, o):
    idx = oracle.bin_indices(b, len(w))
    g, g2 = oracle.new_grid("first", "float64", oracle.grid_shape(b))
    oracle.aggregate("first", idx, g, data=w, data2=o, grid2=g2)
    return g, g2


def _worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    from vaex_amd.distributed import combine_grids, shard_range
    x, w, o = _data()
    i1, i2 = shard_range(len(x), rank, world)
    out = {}
    for kind, (g, g2) in _grids(x[i1:i2], w[i1:i2], o[i1:i2]).items():
        g, g2 = combine_grids(kind, np.ascontiguousarray(g), None if g2 is None else np.ascontiguousarray(g2), comm)
        out[kind] = g
        if g2 is not None:
            out[kind + "_order"] = g2
    if rank == 0:
        np.savez(path, **out)
    comm.barrier()
    comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_grid_combine(world):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.npz")
        _spawn(_worker, world, path)
        got = np.load(path)
        x, w, o = _data()
        ref = _grids(x, w, o)
        np.testing.assert_array_equal(got["AggCount"], ref["AggCount"][0])
        np.testing.assert_allclose(got["AggSum"], ref["AggSum"][0], rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(got["AggMin"], ref["AggMin"][0])
        np.testing.assert_array_equal(got["AggMax"], ref["AggMax"][0])
        np.testing.assert_array_equal(got["AggFirst"], ref["AggFirst"][0])
        np.testing.assert_array_equal(got["AggFirst_order"], ref["AggFirst"][1])


def test_shard_range_covers_rows():
    from vaex_amd.distributed import shard_range
    for n in (0, 1, 7, 1000003):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def _keys():
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 500, 20001).astype("f8")
    keys[rng.integers(0, len(keys), 40)] = np.nan
    mask = np.zeros(len(keys), bool)
    mask[rng.integers(0, len(keys), 30)] = True
    return keys, mask


def _set_worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    from oracle import oracle
    from vaex_amd.distributed import combine_minmax, merge_key_arrays, shard_range
    keys, mask = _keys()
    i1, i2 = shard_range(len(keys), rank, world)
    local = oracle.OrderedSet(1)
    local.update(keys[i1:i2], mask[i1:i2])
    ka = local.key_array(np.float64)
    gathered = comm.allgather((ka, local.null_value if local.null_count else -1))
    merged = merge_key_arrays(gathered, lambda: oracle.OrderedSet(1))
    shard = keys[i1:i2]
    lo, hi = combine_minmax(np.nanmin(shard), np.nanmax(shard), comm)
    empty_lo, empty_hi = combine_minmax(np.nan if rank == 0 else 3.0, np.nan if rank == 0 else 4.0, comm)
    if rank == 0:
        np.savez(path, keys=merged.key_array(np.float64), null_value=merged.null_value, nan_value=merged.nan_value,
                 minmax=np.array([lo, hi, empty_lo, empty_hi]))
    comm.barrier()
    comm.close()


def test_two_rank_set_merge_and_minmax():
    """Global ordered set from two ranks' key arrays == one set updated shard by shard
    (ordinals in first-appearance order; NaN / null at the end of the update call that
    first saw them), and NaN-ignoring min/max across ranks."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle
    from vaex_amd.distributed import shard_range
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "set.npz")
        _spawn(_set_worker, 2, path)
        got = np.load(path)
        keys, mask = _keys()
        ref = oracle.OrderedSet(1)
        for r in range(2):
            i1, i2 = shard_range(len(keys), r, 2)
            ref.update(keys[i1:i2], mask[i1:i2])
        np.testing.assert_array_equal(got["keys"], ref.key_array(np.float64))
        assert int(got["null_value"]) == ref.null_value and int(got["nan_value"]) == ref.nan_value
        np.testing.assert_array_equal(got["minmax"], [np.nanmin(keys), np.nanmax(keys), 3.0, 4.0])


def _groups_worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    from oracle import oracle
    from vaex_amd.distributed import all_ranks_true, combine_groups, shard_range
    keys, v, w = _group_data()
    i1, i2 = shard_range(len(keys), rank, world)
    # the per-rank fused-groupby result (what HashAgg.finish returns), from the oracle
    uk, s, c = oracle.groupby_reference(keys[i1:i2], v[i1:i2])
    counts = np.bincount(np.searchsorted(uk, keys[i1:i2]), minlength=len(uk)).astype(np.int64)
    wsum = np.zeros(len(uk), np.int64)
    np.add.at(wsum, np.searchsorted(uk, keys[i1:i2]), w[i1:i2].astype(np.int64))
    local = (uk.astype(np.int64), counts, [s, wsum], [c, None])
    gk, gc, gs, gn = combine_groups(local, comm)
    flags = [all_ranks_true(True, comm), all_ranks_true(rank == 0, comm)]
    if rank == 0:
        np.savez(path, keys=gk, counts=gc, s=gs[0], w=gs[1], nn=gn[0], flags=np.array(flags))
    comm.barrier()
    comm.close()


def _group_data():
    rng = np.random.default_rng(21)
    n = 50_001
    keys = (rng.integers(0, 3000, n) * 7919 - 10 ** 6).astype(np.int64)
    v = rng.normal(size=n)
    v[::17] = np.nan
    w = rng.integers(-5, 6, n).astype(np.int8)
    return keys, v, w


@pytest.mark.parametrize("world", [2, 3])
def test_two_rank_fused_groupby_merge(world):
    """Per-rank fused-groupby results (keys sorted, counts, float and int sums, non-NaN
    counts) merged across ranks by the hash-partition all-to-all == the whole-column
    result; and the all-ranks flag used to keep every rank on the same groupby route."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "groups.npz")
        _spawn(_groups_worker, world, path)
        got = np.load(path)
        keys, v, w = _group_data()
        uk, s, c = oracle.groupby_reference(keys, v)
        np.testing.assert_array_equal(got["keys"], uk)
        np.testing.assert_array_equal(got["counts"], np.bincount(np.searchsorted(uk, keys)))
        np.testing.assert_array_equal(got["nn"], c)
        np.testing.assert_allclose(got["s"], s, rtol=1e-12, atol=1e-12)
        ew = np.zeros(len(uk), np.int64)
        np.add.at(ew, np.searchsorted(uk, keys), w.astype(np.int64))
        np.testing.assert_array_equal(got["w"], ew)
        assert got["flags"].tolist() == [True, False]


def _u64_groups_worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    from vaex_amd.distributed import combine_groups, shard_range
    keys = _u64_keys()
    i1, i2 = shard_range(len(keys), rank, world)
    uk, inv = np.unique(keys[i1:i2], return_inverse=True)
    counts = np.bincount(inv, minlength=len(uk)).astype(np.int64)
    usum = np.zeros(len(uk), np.uint64)
    np.add.at(usum, inv, (keys[i1:i2] >> np.uint64(40)))
    gk, gc, gs, gn = combine_groups((uk, counts, [usum], [None]), comm)
    if rank == world - 1:
        np.savez(path, keys=gk, counts=gc, s=gs[0], nn_none=np.array([gn[0] is None]))
    comm.barrier()
    comm.close()


def _u64_keys():
    rng = np.random.default_rng(5)
    base = rng.integers(0, 2 ** 63, 400, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    return base[rng.integers(0, 400, 20_000)]


def test_hash_partition_merge_uint64_keys():
    """uint64 keys above 2**63 keep unsigned order and exact unsigned sums through the
    all-to-all (three ranks, one of them may own no group); owners are in range."""
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd.distributed import group_owner
    keys = _u64_keys()
    own = group_owner(keys, 3)
    assert own.min() >= 0 and own.max() < 3
    np.testing.assert_array_equal(own, group_owner(keys.copy(), 3))
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "u64.npz")
        _spawn(_u64_groups_worker, 3, path)
        got = np.load(path)
        uk, inv = np.unique(keys, return_inverse=True)
        assert got["keys"].dtype == np.uint64
        np.testing.assert_array_equal(got["keys"], uk)
        np.testing.assert_array_equal(got["counts"], np.bincount(inv))
        es = np.zeros(len(uk), np.uint64)
        np.add.at(es, inv, keys >> np.uint64(40))
        np.testing.assert_array_equal(got["s"], es)
        assert bool(got["nn_none"][0])


def _empty_rank_worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    from vaex_amd.distributed import combine_groups
    if rank == 1:  # an empty shard: no groups at all
        local = (np.empty(0, np.int64), np.empty(0, np.int64), [np.empty(0, np.float64)], [np.empty(0, np.int64)])
    else:
        keys = np.array([-7, 3, 10 ** 12], np.int64) + rank
        local = (keys, np.array([1, 2, 3], np.int64), [np.array([0.5, 1.5, 2.5])], [np.array([1, 1, 3], np.int64)])
    gk, gc, gs, gn = combine_groups(local, comm)
    if rank == 1:
        np.savez(path, keys=gk, counts=gc, s=gs[0], nn=gn[0])
    comm.barrier()
    comm.close()


def test_hash_partition_merge_with_an_empty_rank():
    """A rank with no groups (empty row shard) still takes part in both exchanges and ends
    with the whole merged, key-sorted result."""
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "e.npz")
        _spawn(_empty_rank_worker, 3, path)
        got = np.load(path)
    base = np.array([-7, 3, 10 ** 12], np.int64)
    keys = np.concatenate([base, base + 2])
    order = np.argsort(keys)
    np.testing.assert_array_equal(got["keys"], keys[order])
    np.testing.assert_array_equal(got["counts"], np.array([1, 2, 3, 1, 2, 3])[order])
    np.testing.assert_array_equal(got["s"], np.array([0.5, 1.5, 2.5, 0.5, 1.5, 2.5])[order])
    np.testing.assert_array_equal(got["nn"], np.array([1, 1, 3, 1, 1, 3])[order])


def test_message_codec_roundtrip():
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd.comm import decode, encode
    objs = [None, True, -5, 2 ** 62, 1.5, "x", b"\x00\xff", np.arange(7, dtype=np.int16),
            np.zeros((2, 3), ">f8"), np.array([], np.uint64), [1, (2.0, None)], {"a": [np.ones(3)]}]
    for o in objs:
        got = decode(encode(o))
        if isinstance(o, np.ndarray):
            assert got.dtype == o.dtype and got.shape == o.shape and np.array_equal(got, o)
        elif isinstance(o, dict):
            np.testing.assert_array_equal(got["a"][0], o["a"][0])
        else:
            assert got == o
    with pytest.raises(TypeError):
        encode(object())


def _prim_worker(rank, world, path, port):
    comm = _comm(rank, world, port)
    a = comm.allreduce(np.array([rank + 1.5, -rank], np.float64), "sum")
    mn = comm.allreduce(np.array([rank, 10 - rank], np.int64), "min")
    got = comm.alltoall([(rank, d, np.full(d + 1, rank, np.int32)) for d in range(world)])
    ok = all(g[0] == s and g[1] == rank and np.array_equal(g[2], np.full(rank + 1, s, np.int32))
             for s, g in enumerate(got))
    ag = comm.allgather(rank * 10)
    if rank == world - 1:
        np.savez(path, a=a, mn=mn, ok=np.array([ok]), ag=np.array(ag))
    comm.barrier()
    comm.close()


def test_host_comm_primitives():
    world = 3
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "p.npz")
        _spawn(_prim_worker, world, path)
        got = np.load(path)
    np.testing.assert_array_equal(got["a"], [1.5 + 2.5 + 3.5, -3.0])
    np.testing.assert_array_equal(got["mn"], [0, 8])
    assert bool(got["ok"][0])
    np.testing.assert_array_equal(got["ag"], [0, 10, 20])


def test_thread_comm_primitives_and_group_merge():
    """ThreadComm (the object channel of a loopback group): the same primitives and results
    as HostComm, every rank a thread; combine_groups over it equals the one-rank merge."""
    import concurrent.futures as cf
    import sys
    sys.path.insert(0, ROOT)
    from vaex_amd.comm import ThreadComm
    from vaex_amd.distributed import combine_groups, merge_groups
    world = 4
    group = ThreadComm.Group(world)
    rng = np.random.default_rng(1)
    keys = [np.unique(rng.integers(-50, 50, 30)).astype(np.int64) for _ in range(world)]
    locs = [(k, np.ones(len(k), np.int64), [k.astype(np.float64) * 0.5], [np.ones(len(k), np.int64)]) for k in keys]

    def rank(r):
        c = ThreadComm(r, group)
        a = c.allreduce(np.array([r + 1.5, -r], np.float64), "sum")
        mn = c.allreduce(np.array([r, 10 - r], np.int64), "min")
        got = c.alltoall([(r, d) for d in range(world)])
        ok = all(g == (s, r) for s, g in enumerate(got))
        g0 = c.gather(r)
        b = c.bcast("x" if r == 0 else None)
        merged = combine_groups(locs[r], c)
        c.barrier()
        return a, mn, ok, g0, b, merged

    with cf.ThreadPoolExecutor(world) as ex:
        res = [f.result(timeout=60) for f in [ex.submit(rank, r) for r in range(world)]]
    want = merge_groups(locs)
    for r, (a, mn, ok, g0, b, merged) in enumerate(res):
        np.testing.assert_array_equal(a, [1.5 + 2.5 + 3.5 + 4.5, -6.0])
        np.testing.assert_array_equal(mn, [0, 7])
        assert ok and b == "x"
        assert g0 == (list(range(world)) if r == 0 else None)
        np.testing.assert_array_equal(merged[0], want[0])
        np.testing.assert_array_equal(merged[1], want[1])
        np.testing.assert_array_equal(merged[2][0], want[2][0])
