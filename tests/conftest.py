import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def kat_array(spec):
    """Build the (possibly big-endian / strided) numpy column a KAT binner describes."""
    data = np.array(spec["data"], dtype=spec["dtype"])
    stride = spec.get("stride", 1)
    if stride != 1:
        base = np.zeros(len(data) * stride, dtype=data.dtype)
        view = base[::stride]
        view[:] = data
        return view
    return data


@pytest.fixture(scope="session")
def kats():
    return load_kats()
