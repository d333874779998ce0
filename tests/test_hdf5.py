"""vaex HDF5 files without h5py (vaex_amd/hdf5.py), on CPU.

Pinned by: the reference's own fixture tests/data/with_alias.hdf5 and its test
(tests/hdf5_test.py:8-13: columns 'X-1' = [1], '#' = [2] through 'alias' attributes);
vaex-ml's iris / titanic datasets (the reference's ml tests load them) against their
well-known contents (150 rows, 50 per class, sepal length summing to 876.5; 1309
passengers, 500 survivors, 263 missing ages); a file written by libhdf5 itself
(tests/golden/make_hdf5.py, h5py: every numeric dtype, big-endian, bool, alias, mask,
column_order) against the arrays it was written from; and this build's writer read back
by the reader and, when the image's h5py is present, by libhdf5."""
import json
import os
import subprocess

import numpy as np
import pytest

import vaex_amd
from vaex_amd import hdf5

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "hdf5")
CONDA_PY = "/opt/conda/bin/python3.9"
CONDA_SITE = "/opt/conda/lib/python3.9/site-packages"


def test_reference_alias_fixture():
    df = vaex_amd.open(os.path.join(GOLDEN, "with_alias.hdf5"))  # hdf5_test.py:8-13
    assert df.columns["X-1"].tolist() == [1]
    assert df.columns["#"].tolist() == [2]


def test_iris_and_titanic():
    iris = vaex_amd.open(os.path.join(GOLDEN, "iris.hdf5"))
    assert iris.get_column_names() == ["sepal_length", "sepal_width", "petal_length", "petal_width", "class_"]
    assert len(iris) == 150 and np.bincount(iris.columns["class_"]).tolist() == [50, 50, 50]
    assert round(float(iris.columns["sepal_length"].sum()), 6) == 876.5
    t = vaex_amd.open(os.path.join(GOLDEN, "titanic.hdf5"))
    assert len(t) == 1309 and int(t.columns["survived"].sum()) == 500
    assert int(np.isnan(t.columns["age"]).sum()) == 263
    assert {"name", "sex", "ticket"} <= set(t._skipped_columns)  # string columns: out of scope


def test_h5py_written_file():
    cols, skipped = hdf5.read_columns(os.path.join(GOLDEN, "h5py_v2.hdf5"))
    exp = np.load(os.path.join(GOLDEN, "h5py_v2.npz"))
    order = [str(s) for s in exp["__order"]]
    assert list(cols) == order and not skipped
    for name in order:
        if name == "masked":
            np.testing.assert_array_equal(np.ma.getmaskarray(cols[name]), exp["masked__mask"])
            np.testing.assert_array_equal(cols[name].data, exp["masked"])
            continue
        e = exp[name.replace("-", "_minus_")]
        assert cols[name].dtype == e.dtype, name
        np.testing.assert_array_equal(cols[name], e)
    assert not cols["x"].flags.owndata  # mapped from the file, not read into memory


def _frame(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    return {"x": rng.normal(size=n), "f32": rng.random(n).astype(np.float32),
            "i8": rng.integers(-100, 100, n).astype(np.int8), "u64": rng.integers(0, 2**63, n, dtype=np.uint64),
            "b": rng.random(n) > 0.5, "X-1": np.arange(n), "#": -np.arange(n, dtype=np.int32)}


def test_export_round_trip(tmp_path):
    cols = _frame()
    df = vaex_amd.from_arrays(**cols)
    df["z"] = df.x * 2  # a virtual column is evaluated (host frame: numpy)
    path = tmp_path / "out.hdf5"
    df.export_hdf5(path)
    back = vaex_amd.open(path)
    assert back.get_column_names() == list(cols) + ["z"]
    for k, v in cols.items():
        assert back.columns[k].dtype == v.dtype
        np.testing.assert_array_equal(back.columns[k], v)
    np.testing.assert_array_equal(back.columns["z"], cols["x"] * 2)
    for k in cols:  # 4 KiB-aligned contiguous data
        assert back.columns[k].__array_interface__["data"][0] % 4096 == 0


@pytest.mark.skipif(not os.path.exists(CONDA_PY), reason="no h5py in this image")
def test_export_read_by_libhdf5(tmp_path):
    cols = _frame(3000, 1)
    path = tmp_path / "out.hdf5"
    vaex_amd.from_arrays(**cols).export_hdf5(path)
    env = dict(os.environ, PYTHONPATH=CONDA_SITE)
    out = subprocess.run([CONDA_PY, os.path.join(os.path.dirname(GOLDEN), "make_hdf5.py"), "check", str(path)],
                         capture_output=True, text=True, env=env, timeout=120)
    if out.returncode != 0 and "No module named" in out.stderr:
        pytest.skip("h5py not importable")
    assert out.returncode == 0, out.stderr
    seen = json.loads(out.stdout)
    assert seen["__order"] == ",".join(cols)
    for k, v in cols.items():
        assert seen[k]["n"] == len(v) and seen[k]["offset"], k
        assert seen[k]["sum"] == float(np.asarray(v, np.float64).sum()), k


def test_arrow_round_trip(tmp_path):
    cols = _frame(1000, 2)
    cols.pop("u64")
    path = tmp_path / "out.arrow"
    vaex_amd.from_arrays(**cols).export_arrow(path)
    back = vaex_amd.open(path)
    for k, v in cols.items():
        np.testing.assert_array_equal(back.columns[k], v)


def test_unsupported_files(tmp_path):
    p = tmp_path / "x.hdf5"
    p.write_bytes(b"not hdf5" * 100)
    with pytest.raises(hdf5.HDF5Error):
        vaex_amd.open(p)
