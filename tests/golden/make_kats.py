"""Writes tests/golden/kats.json: known-answer tests transcribed from the reference's own
test-suite (inputs and expected outputs only; SURVEY.md §8c lists them).  Run:

    python tests/golden/make_kats.py

Each entry cites the reference test it was transcribed from.  Expected outputs are the
reference tests' literal assertions, except where noted in ``note``.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

INT64_MIN = -(2 ** 63)
INT64_MAX = 2 ** 63 - 1

superagg = [
    # tests/internal/superagg_tests.py:23-32
    dict(name="count_1d_scalar", cite="tests/internal/superagg_tests.py:23-32",
         binners=[dict(kind="scalar", dtype="float64", data=[-1, -2, 0.5, 1.5, 4.5, 5], vmin=0, vmax=5, bins=5)],
         agg=dict(kind="count"), expected=[0, 2, 1, 1, 0, 0, 1, 1]),
    # :50-59
    dict(name="count_1d_scalar_int64", cite="tests/internal/superagg_tests.py:50-59",
         binners=[dict(kind="scalar", dtype="int64", data=[-1, -2, 0, 1, 4, 5], vmin=0, vmax=5, bins=5)],
         agg=dict(kind="count"), expected=[0, 2, 1, 1, 0, 0, 1, 1],
         note="the test builds the int64 array from [-1,-2,0.5,1.5,4.5,5]; numpy truncates to [-1,-2,0,1,4,5]"),
    # :61-70
    dict(name="count_1d_ordinal", cite="tests/internal/superagg_tests.py:61-70",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -2, 0, 1, 4, 6, 10], ordinal_count=5, min_value=0)],
         agg=dict(kind="count"), expected=[0, 2, 1, 1, 0, 0, 1, 2]),
    # :72-84 -- the diagonal of the 2d grid
    dict(name="count_2d_ordinal_diagonal", cite="tests/internal/superagg_tests.py:72-84",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -2, 0, 1, 4, 6, 10], ordinal_count=5, min_value=0),
                  dict(kind="ordinal", dtype="int64", data=[-1, -2, 0, 1, 4, 6, 10], ordinal_count=5, min_value=0)],
         agg=dict(kind="count"), expected_diagonal=[0, 2, 1, 1, 0, 0, 1, 2]),
    # :86-106.  The reference test pre-mutates the grid (-=100 / +=100) and expects untouched
    # cells to read -100/100, which contradicts AggMax/AggMin's ctor fill with
    # numeric_limits<int64>::min()/max() (superagg.cpp:199-204,246-251); that file is named
    # *_tests.py so pytest never collects it.  We pin the touched cells literally and the
    # untouched cells to the ctor fill value the source defines.
    dict(name="max_1d_ordinal", cite="tests/internal/superagg_tests.py:86-98",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -1, 0, 0, 4, 6, 10], ordinal_count=5, min_value=0)],
         agg=dict(kind="max", dtype="int64", data=[-1, 2, 4, 1, 9, 6, 10]),
         expected=[INT64_MIN, 2, 4, INT64_MIN, INT64_MIN, INT64_MIN, 9, 10],
         note="untouched cells = AggMax ctor fill (superagg.cpp:199-204), see make_kats.py"),
    dict(name="min_1d_ordinal", cite="tests/internal/superagg_tests.py:100-106",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -1, 0, 0, 4, 6, 10], ordinal_count=5, min_value=0)],
         agg=dict(kind="min", dtype="int64", data=[-1, 2, 4, 1, 9, 6, 10]),
         expected=[INT64_MAX, -1, 1, INT64_MAX, INT64_MAX, INT64_MAX, 9, 6],
         note="untouched cells = AggMin ctor fill (superagg.cpp:246-251), see make_kats.py"),
    # :108-119
    dict(name="sum_1d_ordinal", cite="tests/internal/superagg_tests.py:108-119",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -1, 0, 0, 4, 6, 10], ordinal_count=5, min_value=0)],
         agg=dict(kind="sum", dtype="int64", data=[-1, 2, 4, 1, 9, 6, 10]),
         expected=[0, 1, 5, 0, 0, 0, 9, 16]),
    # tests/agg_test.py:257-262 big-endian x and y
    dict(name="big_endian_binning", cite="tests/agg_test.py:257-262",
         binners=[dict(kind="scalar", dtype=">f8", data=list(range(10)), vmin=-0.5, vmax=9.5, bins=10),
                  dict(kind="scalar", dtype=">f8", data=[0] * 10, vmin=-0.5, vmax=0.5, bins=1)],
         agg=dict(kind="count"), expected_central=[[1]] * 10),
    # tests/agg_test.py:265-272 big-endian, non-contiguous
    dict(name="big_endian_binning_non_contiguous", cite="tests/agg_test.py:265-272",
         binners=[dict(kind="scalar", dtype=">f8", data=list(range(10)), vmin=-0.5, vmax=9.5, bins=10, stride=2),
                  dict(kind="scalar", dtype=">f8", data=list(range(10)), vmin=-0.5, vmax=9.5, bins=10, stride=2)],
         agg=dict(kind="count"), expected_central_diagonal=[1] * 10),
    # tests/agg_test.py:275-281 strided
    dict(name="strides", cite="tests/agg_test.py:275-281",
         binners=[dict(kind="scalar", dtype="float64", data=list(range(10)), vmin=-0.5, vmax=9.5, bins=10, stride=2)],
         agg=dict(kind="count"), expected_central=[1] * 10),
    # tests/agg_test.py:108-147 (2d and 3d all-ones)
    dict(name="count_basics_2d", cite="tests/agg_test.py:136-140",
         binners=[dict(kind="scalar", dtype="int64", data=[0, 1, 0, 1], vmin=0., vmax=2., bins=2),
                  dict(kind="scalar", dtype="int64", data=[0, 0, 1, 1], vmin=0., vmax=2., bins=2)],
         agg=dict(kind="count"), expected_central=[[1, 1], [1, 1]]),
    dict(name="count_basics_3d", cite="tests/agg_test.py:142-147",
         binners=[dict(kind="scalar", dtype="int64", data=[0, 1, 0, 1, 0, 1, 0, 1], vmin=0., vmax=2., bins=2),
                  dict(kind="scalar", dtype="int64", data=[0, 0, 1, 1, 0, 0, 1, 1], vmin=0., vmax=2., bins=2),
                  dict(kind="scalar", dtype="int64", data=[0, 0, 0, 0, 1, 1, 1, 1], vmin=0., vmax=2., bins=2)],
         agg=dict(kind="count"), expected_central=[[[1, 1], [1, 1]], [[1, 1], [1, 1]]]),
    # tests/agg_test.py:171-181
    dict(name="count_1d_ordinal_api", cite="tests/agg_test.py:171-181",
         binners=[dict(kind="ordinal", dtype="int64", data=[-1, -2, 0, 1, 4, 5], ordinal_count=5, min_value=0)],
         agg=dict(kind="count"), expected=[0, 2, 1, 1, 0, 0, 1, 1]),
]

# DataFrame-level KATs.  The `df` fixture of tests/agg_test.py / first_test.py is the
# 21-row base frame (tests/common.py:312-380) filtered to 0 <= x < 10, so x = 0..9, y = x**2.
api = [
    dict(name="mean_basics", cite="tests/agg_test.py:184-192",
         columns=dict(x=list(range(10)), y=[i * i for i in range(10)]),
         calls=[dict(op="mean", expression="x", expected=4.5),
                dict(op="mean", expression="y", expected=28.5),
                dict(op="mean", expression="x", selection="x < 3", expected=1.0),
                dict(op="mean", expression="y", selection="x < 3", expected=5 / 3)]),
    dict(name="count_basics_1d", cite="tests/agg_test.py:108-133",
         columns=dict(x=list(range(10)), y=[i * i for i in range(10)]),
         calls=[dict(op="count", binby="x", limits=[0, 10], shape=10, expected=[1] * 10),
                dict(op="sum", expression="y", binby="x", limits=[0, 10], shape=10,
                     expected=[i * i for i in range(10)]),
                dict(op="count", expression="x", binby="x", limits=[0, 10], shape=10, selection="x < 5",
                     expected=[1] * 5 + [0] * 5),
                dict(op="sum", expression="y", binby="x", limits=[0, 10], shape=10, selection="x < 5",
                     expected=[0, 1, 4, 9, 16, 0, 0, 0, 0, 0])]),
    dict(name="first", cite="tests/first_test.py:4-12",
         columns=dict(x=list(range(10)), y=[i * i for i in range(10)]),
         calls=[dict(op="first", expression="y", order="x", expected=0),
                dict(op="first", expression="y", order="x", binby="x", limits=[0, 10], shape=2, expected=[0, 25]),
                dict(op="first", expression="y", order="-x", binby="x", limits=[0, 10], shape=2, expected=[16, 81])]),
    dict(name="groupby_1d", cite="tests/groupby_test.py:103-109",
         columns=dict(g=[0, 0, 0, 0, 1, 1, 1, 1, 2, 2]),
         calls=[dict(op="groupby_count", by="g", sort=True, expected_keys=[0, 1, 2], expected_count=[4, 4, 2])]),
    dict(name="groupby_1d_nan", cite="tests/groupby_test.py:149-155",
         columns=dict(g=[0, 0, 0, 0, 1, 1, 1, float("nan"), 2, 2]),
         calls=[dict(op="groupby_count", by="g", sort=True, expected_keys=[0, 1, 2, "nan"],
                     expected_count=[4, 3, 2, 1])]),
    dict(name="groupby_2d", cite="tests/groupby_test.py:199-207",
         columns=dict(g=[0, 0, 0, 0, 1, 1, 1, 1, 2, 2], h=[5, 5, 5, 6, 5, 5, 5, 5, 6, 6]),
         calls=[dict(op="groupby_count", by=["g", "h"], sort=True, expected_keys=[[0, 0, 1, 2], [5, 6, 5, 6]],
                     expected_count=[3, 1, 4, 2])]),
    dict(name="binby_2d", cite="tests/groupby_test.py:181-196",
         columns=dict(g=[0, 0, 0, 0, 1, 1, 1, 1, 2, 2], h=[5, 5, 5, 6, 5, 5, 5, 5, 6, 6]),
         calls=[dict(op="binby_count", by=["g", "h"], sort=True, expected=[[3, 1], [4, 0], [0, 2]])]),
]

# ordered_set KAT (tests/internal/hash_test.py:54-126): keys [3,2,1,0] float64 with an
# optional NaN at row 1 and a missing value at row 2, nmaps 1..3: taking key_array at each
# row's ordinal reproduces the input; map_ordinal(key_array) == arange(4) (null aside).
hash_sets = [
    dict(name="set_float", cite="tests/internal/hash_test.py:54-126",
         keys=[3.0, 2.0, 1.0, 0.0], nan_row=1, null_row=2, nmaps=[1, 2, 3],
         expected_map_ordinal_dtype="int8"),
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(dict(superagg=superagg, api=api, hash_sets=hash_sets), f, indent=1)
    print("wrote", os.path.join(HERE, "kats.json"))
