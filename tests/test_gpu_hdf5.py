"""Binning straight from a memory-mapped HDF5 file: the mapped columns are
host arrays, streamed to HBM by the library's pinned double-buffered pipeline in 16 Mi-row
chunks, so the file is never loaded whole.  Results equal the oracle on the same arrays."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def test_count_sum_from_mapped_file(tmp_path):
    import vaex_amd
    rng = np.random.default_rng(11)
    n = (1 << 24) + 4321  # more than one staging chunk
    cols = {"x": rng.normal(size=n), "y": rng.normal(size=n), "w": rng.random(n)}
    path = tmp_path / "c2.hdf5"
    vaex_amd.from_arrays(**cols).export_hdf5(path)
    df = vaex_amd.open(path)
    assert not df.columns["x"].flags.owndata
    got_c = df.count(binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=256)
    got_s = df.sum("w", binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=256)
    bx = oracle.Binner("scalar", cols["x"], vmin=-4, vmax=4, bins=256)
    by = oracle.Binner("scalar", cols["y"], vmin=-4, vmax=4, bins=256)
    np.testing.assert_array_equal(got_c, oracle.extract_central_part(oracle.compute_grid([bx, by], "count")))
    np.testing.assert_allclose(got_s, oracle.extract_central_part(oracle.compute_grid([bx, by], "sum", data=cols["w"])),
                               rtol=1e-6, atol=1e-12)


def test_groupby_from_mapped_file(tmp_path):
    import vaex_amd
    rng = np.random.default_rng(12)
    n = 3_000_000
    key = (rng.integers(0, 5000, n) * 7919).astype(np.int32)
    v = rng.normal(size=n)
    path = tmp_path / "g.hdf5"
    vaex_amd.from_arrays(key=key, v=v).export_hdf5(path)
    df = vaex_amd.open(path)
    g = df.groupby("key", agg={"s": vaex_amd.agg.sum("v"), "n": "count"})
    uk, s, c = oracle.groupby_reference(key, v)
    order = np.argsort(g["key"].to_numpy())
    np.testing.assert_array_equal(g["key"].to_numpy()[order], uk)
    np.testing.assert_array_equal(g["n"].to_numpy()[order], c)
    np.testing.assert_allclose(g["s"].to_numpy()[order], s, rtol=1e-6, atol=1e-9)


def test_c4_mean_1024_from_mapped_file(tmp_path, monkeypatch):
    """C4's query shape (BASELINE configs[3]) on one GPU: mean(w, binby=[x, y], shape=1024)
    over a memory-mapped vaex HDF5 file, streamed through three 16 Mi-row staging chunks of
    the double-buffered pipeline in one bin() call (so buffer reuse is exercised), equal to
    the oracle's sum / count (agg.py:158-188)."""
    import vaex_amd
    from vaex_amd import execution
    monkeypatch.setattr(execution, "CHUNK_SIZE_HOST", 1 << 26)  # one host chunk -> 3 pipe chunks
    rng = np.random.default_rng(13)
    n = (1 << 25) + 12345
    cols = {"x": rng.normal(size=n), "y": rng.normal(size=n), "w": rng.random(n)}
    cols["w"][::1009] = np.nan
    path = tmp_path / "c4.hdf5"
    vaex_amd.from_arrays(**cols).export_hdf5(path)
    del cols
    df = vaex_amd.open(path)
    x, y, w = (np.asarray(df.columns[c]) for c in ("x", "y", "w"))
    lim = [[-4, 4], [-4, 4]]
    got = df.mean("w", binby=["x", "y"], limits=lim, shape=1024)
    bx = oracle.Binner("scalar", x, vmin=-4, vmax=4, bins=1024)
    by = oracle.Binner("scalar", y, vmin=-4, vmax=4, bins=1024)
    s = oracle.extract_central_part(oracle.compute_grid([bx, by], "sum", data=w))
    c = oracle.extract_central_part(oracle.compute_grid([bx, by], "count", data=w))
    with np.errstate(invalid="ignore", divide="ignore"):
        exp = s / c
    assert got.shape == (1024, 1024)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(exp))
    np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("reg,pipe", [("1", "0"), ("0", "0"), ("0", "1"), ("0", "2")])
def test_host_pipe_modes(tmp_path, monkeypatch, reg, pipe):
    """Every way a mapped column chunk reaches the DMA engine gives the oracle's answer:
    the file mapping registered once (default), the pinned bounce buffer, per-chunk
    registration, the runtime's pageable path.  The registration is dropped with the
    last column array over the mapping."""
    import gc
    import vaex_amd
    from vaex_amd import _lib, execution
    monkeypatch.setattr(execution, "CHUNK_SIZE_HOST", 1 << 26)
    monkeypatch.setenv("VH_HOST_REGISTER", reg)
    monkeypatch.setenv("VH_HOST_PIPE", pipe)
    rng = np.random.default_rng(14)
    n = 9_000_017  # > 64 MiB per column, one partial pipe chunk
    cols = {"x": rng.normal(size=n), "y": rng.normal(size=n), "w": rng.random(n)}
    path = tmp_path / "modes.hdf5"
    vaex_amd.from_arrays(**cols).export_hdf5(path)
    df = vaex_amd.open(path)
    lim = [[-4, 4], [-4, 4]]
    got_s = df.sum("w", binby=["x", "y"], limits=lim, shape=300)
    got_c = df.count(binby=["x", "y"], limits=lim, shape=300)
    assert (len(_lib._MAPS) == 1) == (reg == "1")
    bx = oracle.Binner("scalar", cols["x"], vmin=-4, vmax=4, bins=300)
    by = oracle.Binner("scalar", cols["y"], vmin=-4, vmax=4, bins=300)
    np.testing.assert_array_equal(got_c, oracle.extract_central_part(oracle.compute_grid([bx, by], "count")))
    np.testing.assert_allclose(got_s, oracle.extract_central_part(oracle.compute_grid([bx, by], "sum", data=cols["w"])),
                               rtol=1e-9, atol=1e-12)
    del df
    gc.collect()
    assert not _lib._MAPS and not _lib._ROOTS
