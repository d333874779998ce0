"""The reference's threading contract at the boundary (SURVEY.md §8b "Threading"):

* ``ordered_set.update`` is called concurrently on ONE shared set by every worker thread
  (``cpu.py:147-195``; per-map mutexes, ``hash_primitives.hpp:242-247``);
* different task parts bin their own grids concurrently (``execution.py:214-235,358-375``);
* an executor is entered from many threads at once (``tests/execution_test.py:79-101``:
  100 ``df.count`` calls from a 4-thread pool, every result equal to the serial one).

Concurrent updates may assign ordinals in any order (the reference's depend on thread
interleaving), so the set is checked as a key set plus a consistent key <-> ordinal map.
"""
import concurrent.futures
import threading

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def test_concurrent_set_update_one_set():
    from vaex_amd import superutils
    rng = np.random.default_rng(21)
    n, nthreads = 2_000_000, 8
    keys = rng.integers(-50_000, 50_000, n).astype(np.int32)
    keys[rng.random(n) < 0.001] = np.iinfo(np.int32).max
    chunks = np.array_split(keys, 64)
    shared = superutils.ordered_set_int32()
    barrier = threading.Barrier(nthreads)

    def work(t):
        barrier.wait()
        for c in chunks[t::nthreads]:
            shared.update(c)

    with concurrent.futures.ThreadPoolExecutor(nthreads) as tpe:
        list(tpe.map(work, range(nthreads)))
    serial = superutils.ordered_set_int32()
    for c in chunks:
        serial.update(c)
    ka, ks = shared.key_array(), serial.key_array()
    assert len(shared) == len(serial) == len(np.unique(keys))
    np.testing.assert_array_equal(np.sort(ka), np.sort(ks))
    # a bijection key <-> ordinal, and map_ordinal consistent with key_array
    ords = shared.map_ordinal(keys).astype(np.int64)
    assert ords.min() == 0 and ords.max() == len(shared) - 1
    np.testing.assert_array_equal(ka[ords], keys)
    # one thread: exactly the reference's single-threaded ordinals
    exp = oracle.OrderedSet(nmaps=1)
    small = keys[:20000]
    exp.update(small)
    one = superutils.ordered_set_int32()
    one.update(small)
    np.testing.assert_array_equal(one.key_array(), exp.key_array(np.int32))


def test_concurrent_grids_bin():
    """Task parts of one pass bin their own grids at the same time (GIL released in the
    C call): every part's grid equals the oracle's."""
    from vaex_amd import superagg
    rng = np.random.default_rng(22)
    n, nthreads = 3_000_000, 6
    data = [(rng.normal(size=n), rng.normal(size=n), rng.random(n)) for _ in range(nthreads)]
    out = [None] * nthreads
    barrier = threading.Barrier(nthreads)

    def work(t):
        x, y, w = data[t]
        bx = superagg.BinnerScalar_float64("x", -3, 3, 200)
        by = superagg.BinnerScalar_float64("y", -3, 3, 100 + t)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        cnt = superagg.AggCount_float64(grid)
        sm = superagg.AggSum_float64(grid)
        sm.set_data(w, 0)
        barrier.wait()
        grid.bin([cnt, sm])
        out[t] = (np.asarray(cnt).copy(), np.asarray(sm).copy())

    ths = [threading.Thread(target=work, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for t in range(nthreads):
        x, y, w = data[t]
        bx = oracle.Binner("scalar", x, vmin=-3, vmax=3, bins=200)
        by = oracle.Binner("scalar", y, vmin=-3, vmax=3, bins=100 + t)
        np.testing.assert_array_equal(out[t][0], oracle.compute_grid([bx, by], "count"))
        np.testing.assert_allclose(out[t][1], oracle.compute_grid([bx, by], "sum", data=w), rtol=1e-6, atol=1e-12)


def test_executor_thread_safe(monkeypatch):
    """tests/execution_test.py:79-101 with small_buffer: 100 counts from a 4-thread pool."""
    import vaex_amd
    rng = np.random.default_rng(23)
    x = rng.normal(size=10_000)
    x[::97] = np.nan
    df = vaex_amd.from_arrays(x=x)
    count = df.count(df.x)
    passes = df.executor.passes
    monkeypatch.setenv("VAEX_CHUNK_SIZE", "1000")
    N = 100
    with concurrent.futures.ThreadPoolExecutor(4) as tpe:
        futures = [tpe.submit(lambda: df.count(df.x)) for _ in range(N)]
        done, _ = concurrent.futures.wait(futures, return_when=concurrent.futures.FIRST_EXCEPTION)
    assert len(done) == N
    for f in done:
        assert f.result() == count
    assert df.executor.passes <= passes + N
    # binned counts from threads too
    exp = df.count(binby="x", limits=[-3, 3], shape=32)
    with concurrent.futures.ThreadPoolExecutor(4) as tpe:
        res = list(tpe.map(lambda _: df.count(binby="x", limits=[-3, 3], shape=32), range(16)))
    for r in res:
        np.testing.assert_array_equal(r, exp)
