"""The C-ABI library loads and exports every entry point include/vaexhip.h declares
(no compute calls: these run without a GPU)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "vaexhip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(vh_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_are_exported():
    from vaex_amd import _lib
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 45
    for s in syms:
        assert hasattr(L, s), s
    # the ctypes signature table covers the whole header
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_abi_version_and_errors():
    from vaex_amd import _lib
    L = _lib.lib()
    assert L.vh_abi_version() == 1
    n = ctypes.c_int(-1)
    assert L.vh_device_count(ctypes.byref(n)) == 0 and n.value >= 0
    # creating host-side binner descriptors needs no device
    h = ctypes.c_void_p()
    assert L.vh_binner_scalar_create(b"x", 0, 0, 0.0, 1.0, 10, ctypes.byref(h)) == 0
    shape = ctypes.c_uint64()
    assert L.vh_binner_shape(h, ctypes.byref(shape)) == 0 and shape.value == 13
    # set_data validation happens before any device work (superagg_binners.cpp:63-73)
    buf = np.zeros(4, np.float32)
    rc = L.vh_binner_set_data(h, buf.ctypes.data, 4, 4, 1, 1)
    assert rc == 1 and b"Itemsize of data and binner are not equal" in L.vh_last_error()
    rc = L.vh_binner_set_data(h, buf.ctypes.data, 4, 8, 2, 1)
    assert rc == 1 and b"Expected a 1d array" in L.vh_last_error()
    assert L.vh_binner_destroy(h) == 0
    # unknown dtype codes are argument errors
    assert L.vh_binner_scalar_create(b"x", 99, 0, 0.0, 1.0, 10, ctypes.byref(h)) == 4


def test_grid_strides_host_only():
    """Grid strides/shapes (agg.hpp:54-69) are computed on the host."""
    from vaex_amd import superagg
    b1 = superagg.BinnerScalar_float64("x", 0, 1, 10)
    b2 = superagg.BinnerOrdinal_int32("y", 5, 0)
    g = superagg.Grid([b1, b2])
    assert g.shapes == (13, 8)
    assert g.strides == (1, 13)
    assert g.length1d == 13 * 8
    g0 = superagg.Grid([])
    assert g0.length1d == 1 and g0.dimensions == 0
