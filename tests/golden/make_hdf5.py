"""Golden HDF5 fixtures written by libhdf5 itself (h5py), in vaex's layout version 2
(/table/columns/<name>/data, 'mask' datasets, 'alias' attributes, a 'column_order' string
attribute -- the structure vaex/hdf5/export.py writes), for tests/test_hdf5.py.

Run with an interpreter that has h5py (this image: /opt/conda/bin/python3.9 with
PYTHONPATH=/opt/conda/lib/python3.9/site-packages); writes tests/golden/hdf5/h5py_v2.hdf5
and h5py_v2.npz (the same columns as plain arrays, the expected values).  Also provides
`check(path)`: h5py's view of a file as {name: array}, used to validate this build's
writer."""
import json
import os
import sys

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def write():
    rng = np.random.default_rng(123)
    n = 1000
    cols = {
        "x": rng.normal(size=n), "f32": rng.normal(size=n).astype(np.float32),
        "i64": rng.integers(-2**40, 2**40, n), "i32": rng.integers(-1000, 1000, n).astype(np.int32),
        "i8": rng.integers(-100, 100, n).astype(np.int8), "u16": rng.integers(0, 60000, n).astype(np.uint16),
        "u64": rng.integers(0, 2**63, n, dtype=np.uint64), "b": rng.random(n) > 0.5,
        "big": rng.normal(size=n).astype(">f8"), "X-1": np.arange(n),
    }
    mask = rng.random(n) > 0.8
    path = os.path.join(HERE, "hdf5", "h5py_v2.hdf5")
    with h5py.File(path, "w") as f:
        columns = f.require_group("/table/columns")
        order = []
        for name, ar in cols.items():
            safe = name.replace("-", "_")
            g = columns.require_group(safe)
            g.create_dataset("data", data=ar)
            if safe != name:
                g.attrs["alias"] = name
            order.append(name)
        g = columns.require_group("masked")
        g.create_dataset("data", data=cols["x"] * 2)
        g.create_dataset("mask", data=mask)
        order.append("masked")
        columns.attrs["column_order"] = ",".join(order)
    exp = dict(cols)
    exp["masked"] = cols["x"] * 2
    exp["masked__mask"] = mask
    np.savez(os.path.join(HERE, "hdf5", "h5py_v2.npz"), **{k.replace("-", "_minus_"): v for k, v in exp.items()},
             __order=np.array(order))


def check(path):
    out = {}
    with h5py.File(path, "r") as f:
        cols = f["/table/columns"]
        for name in cols:
            ds = cols[name]["data"]
            label = cols[name].attrs.get("alias", name)
            if isinstance(label, bytes):
                label = label.decode()
            out[label] = {"dtype": str(ds.dtype), "sum": float(np.asarray(ds[()], dtype=np.float64).sum()),
                          "first": float(ds[0]) if len(ds) else None, "n": len(ds),
                          "offset": ds.id.get_offset() is not None}
        order = cols.attrs.get("column_order")
        out["__order"] = order.decode() if isinstance(order, bytes) else order
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "check":
        print(json.dumps(check(sys.argv[2])))
    else:
        write()
