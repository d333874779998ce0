"""h2o groupby G1 (C5; benchmarks/groupbyh2o.py:15-93 with benchmarks/fixtures.py:38-70's
columns and the benchmark's aliases: id1/id2/id4/id5 one int8 column in [5, 105), id3/id6
one int32 column in [5, 1e6 + 5), v1/v2 one int8 column in [5, 15), v3 float32) -- every
query the benchmark times, through DataFrame.groupby(...).agg(...) exactly as it writes
them, checked against the oracle's groupby restatement (oracle.groupby_agg, pinned by the
reference's groupby KATs): labels, counts, integer sums, min / max bit-exact, float sums /
means within 1e-6 relative."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

QUERIES = {
    "q1": (["id1"], {"v1": "sum"}),
    "q2": (["id1", "id2"], {"v1": "sum"}),
    "q3": (["id3"], {"v1": "sum", "v3": "mean"}),
    "q4": (["id4"], {"v1": "mean", "v2": "mean", "v3": "mean"}),
    "q5": (["id6"], {"v1": "sum", "v2": "sum", "v3": "sum"}),
    "q7": (["id3"], {"v1": "max", "v2": "min"}),
    "q10": (["id1", "id2", "id3", "id4", "id5", "id6"], {"v3": "sum", "v1": "count"}),
}
ALIAS = [("id1", "i1_100"), ("id2", "i1_100"), ("id3", "i4_1M"), ("id4", "i1_100"), ("id5", "i1_100"),
         ("id6", "i4_1M"), ("v1", "i1_10"), ("v2", "i1_10"), ("v3", "x4")]


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    base = dict(i1_100=rng.integers(5, 105, n).astype(np.int8), i4_1M=rng.integers(5, 1_000_005, n).astype(np.int32),
                i1_10=rng.integers(5, 15, n).astype(np.int8), x4=rng.normal(size=n).astype(np.float32))
    base["x4"][::97] = np.nan
    return base


def _frame(base, device):
    import vaex_amd
    from vaex_amd.device import DeviceArray
    cols = {k: (DeviceArray.from_numpy(v) if device else v) for k, v in base.items()}
    df = vaex_amd.from_arrays(**cols)
    for a, b in ALIAS:
        df.columns[a] = df.columns[b]  # df['id1'] = df['i1_100'] (groupbyh2o.py:26-36)
    return df


@pytest.mark.parametrize("device", [True, False])
@pytest.mark.parametrize("q", list(QUERIES))
def test_h2o_query_matches_oracle(q, device):
    n = 3_000_017 if q != "q10" else 600_011
    base = _data(n)
    df = _frame(base, device)
    by, agg = QUERIES[q]
    res = df.groupby(by).agg(agg)
    cols = {a: base[b] for a, b in ALIAS}
    spec = [(name, "count" if op == "count" else op, None if op == "count" else name) for name, op in agg.items()]
    want = oracle.groupby_agg(cols, by, spec)
    got = {c: res[c].to_numpy() for c in by + list(agg)}
    # result order: the reference's unsorted order depends on its thread interleaving; groups
    # are compared in lexicographic label order
    order = np.lexsort([got[b] for b in by][::-1])
    for b in by:
        np.testing.assert_array_equal(got[b][order], want[b], err_msg=f"{q} {b}")
    for name, op in agg.items():
        g, w = got[name][order], want[name]
        if w.dtype.kind == "f" and op in ("sum", "mean"):
            np.testing.assert_allclose(g, w, rtol=1e-6, atol=1e-9, err_msg=f"{q} {name}")
        else:
            np.testing.assert_array_equal(g, w, err_msg=f"{q} {name}")
