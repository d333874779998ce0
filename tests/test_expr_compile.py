"""Host side of the device expression evaluator (vaex_amd/expr.py), no GPU: the compiled
program's result dtype is numpy 2's for every expression (NEP 50 weak scalars, float32
rounding, narrow-int wrap), unsupported syntax is refused, and a small numpy model of the
stack machine run on the program reproduces numpy's own evaluation bit for bit."""
import numpy as np
import pytest

import vaex_amd
from vaex_amd import expr

OP = expr.OP
INV = {v: k for k, v in OP.items()}


def _frame():
    rng = np.random.default_rng(0)
    n = 257
    return vaex_amd.from_arrays(
        x=rng.normal(size=n), y=rng.normal(size=n) + 2, f=rng.normal(size=n).astype(np.float32),
        i=rng.integers(-50, 50, n).astype(np.int64), i32=rng.integers(-1000, 1000, n).astype(np.int32),
        i8=rng.integers(-100, 100, n).astype(np.int8), u8=rng.integers(0, 255, n).astype(np.uint8),
        b=rng.random(n) > 0.5)


def _run(prog, df):
    """numpy model of csrc/expr.hip's stack machine (64-bit slots as uint64 bit patterns)."""
    n = df.length_unfiltered()
    st = []
    f = lambda u: u.view(np.float64)  # noqa: E731
    g = lambda d: np.asarray(d, np.float64).view(np.uint64)  # noqa: E731
    i = lambda u: u.view(np.int64)  # noqa: E731
    h = lambda v: np.asarray(v, np.int64).view(np.uint64)  # noqa: E731
    with np.errstate(all="ignore"):
        for ins in prog.code:
            op, arg = INV[ins & 0xFF], ins >> 8
            if op == "COL":
                c = np.asarray(df.columns[prog.columns[arg]])
                st.append(g(c.astype(np.float64)) if c.dtype.kind == "f" else h(c.astype(np.int64)))
            elif op == "CONST":
                st.append(np.full(n, prog.consts[arg], np.uint64))
            elif op == "F2I":
                st.append(h(f(st.pop()).astype(np.int64)))
            elif op in ("I2F", "U2F"):
                st.append(g(i(st.pop()).astype(np.float64) if op == "I2F" else st.pop().astype(np.float64)))
            elif op == "ROUND_F32":
                st.append(g(f(st.pop()).astype(np.float32).astype(np.float64)))
            elif op == "WRAP":
                bits, sgn = arg & 0xFF, arg >> 8
                dt = np.dtype(f"{'i' if sgn else 'u'}{bits // 8}")
                st.append(h(i(st.pop()).astype(dt).astype(np.int64)))
            elif op == "NOT_B":
                st.append((st.pop() == 0).astype(np.uint64))
            elif op in ("NEG_F", "ABS_F", "SQRT", "EXP", "LOG", "SIN", "FLOOR", "ISNAN"):
                fn = {"NEG_F": np.negative, "ABS_F": np.abs, "SQRT": np.sqrt, "EXP": np.exp, "LOG": np.log,
                      "SIN": np.sin, "FLOOR": np.floor}.get(op)
                v = f(st.pop())
                st.append(np.isnan(v).astype(np.uint64) if op == "ISNAN" else g(fn(v)))
            elif op in ("NEG_I", "INV_I"):
                v = i(st.pop())
                st.append(h(-v if op == "NEG_I" else ~v))
            elif op == "WHERE":
                b_, a_, c_ = st.pop(), st.pop(), st.pop()
                st.append(np.where(c_ != 0, a_, b_))
            else:
                b_, a_ = st.pop(), st.pop()
                base, kind = op.rsplit("_", 1) if op.count("_") else (op, "")
                if kind == "F":
                    fn = {"ADD": np.add, "SUB": np.subtract, "MUL": np.multiply, "DIV": np.true_divide,
                          "FLOORDIV": np.floor_divide, "MOD": np.remainder, "POW": np.power,
                          "MIN": np.minimum, "MAX": np.maximum}.get(base)
                    cmp = {"LT": np.less, "LE": np.less_equal, "GT": np.greater, "GE": np.greater_equal,
                           "EQ": np.equal, "NE": np.not_equal}.get(base)
                    st.append(g(fn(f(a_), f(b_))) if fn else cmp(f(a_), f(b_)).astype(np.uint64))
                else:
                    fn = {"ADD": np.add, "SUB": np.subtract, "MUL": np.multiply, "FLOORDIV": np.floor_divide,
                          "MOD": np.remainder, "AND": np.bitwise_and, "OR": np.bitwise_or, "XOR": np.bitwise_xor,
                          "SHL": np.left_shift, "MIN": np.minimum, "MAX": np.maximum}.get(base)
                    cmp = {"LT": np.less, "LE": np.less_equal, "GT": np.greater, "GE": np.greater_equal,
                           "EQ": np.equal, "NE": np.not_equal}.get(base)
                    st.append(h(fn(i(a_), i(b_))) if fn else cmp(i(a_), i(b_)).astype(np.uint64))
    assert len(st) == 1
    v = st[0]
    if prog.dtype.kind == "b":
        return v != 0
    if prog.dtype.kind == "f":
        return f(v).astype(prog.dtype)
    return i(v).astype(prog.dtype)


EXPRESSIONS = [
    "x + y", "x * 2 - y / 3", "(x > 0) & (y < 2.5)", "x ** 2 + sqrt(abs(y))", "i % 7", "i // 3", "-i", "~b",
    "where(x > 0, x, -x)", "i8 + i8", "i8 * 3", "f * 2.5 + f", "i32 / 2", "x // 0.7", "x % -1.3",
    "minimum(x, y)", "u8 + 1", "i << 2", "x ** 3 - x ** 0.5", "b & (i > 3)", "f + i8", "f + i32", "i32 + i8",
    "np.floor(x) + 1", "isnan(log(x))", "u8 > 200", "i == 3", "b | ~b", "x + 1 - 1", "where(b, i8, i32)",
    "astype(i32, 'float64')", "astype(i, 'float64') ** 2", "astype(x * 100, 'int32')", "astype(i32, 'int8')",
    "astype(f, 'float64') + x", "astype(x, 'float32')", "astype(u8, 'int16') - 300", "astype(x, 'float64')",
]


@pytest.mark.parametrize("e", EXPRESSIONS)
def test_program_matches_numpy(e):
    df = _frame()
    prog = expr.compile_expression(df, e)
    ns = dict(np=np, sqrt=np.sqrt, abs=np.abs, where=np.where, minimum=np.minimum, isnan=np.isnan, log=np.log,
              astype=lambda a, d: np.asarray(a).astype(d))
    ns.update({k: np.asarray(v) for k, v in df.columns.items()})
    with np.errstate(all="ignore"):
        expected = np.asarray(eval(e, {"__builtins__": {}}, ns))  # noqa: S307
    assert prog.dtype == expected.dtype, (e, prog.dtype, expected.dtype)
    got = _run(prog, df)
    np.testing.assert_array_equal(got, expected)


@pytest.mark.parametrize("e", ["x.mean()", "[x]", "lambda: 1", "unknown + 1", "x if y else 1", "sum(x)", "x @ y"])
def test_unsupported_is_refused(e):
    with pytest.raises(expr.UnsupportedExpression):
        expr.Program(_frame(), e)


def test_virtual_columns_and_variables_inline():
    df = _frame()
    df["z"] = df.x + df.y
    df.variables["k"] = 3
    prog = expr.compile_expression(df, "z * k")
    assert prog.columns == ["x", "y"] and prog.dtype == np.float64
    np.testing.assert_array_equal(_run(prog, df), (np.asarray(df.columns["x"]) + np.asarray(df.columns["y"])) * 3)


def test_stack_depth_limit():
    deep = "x" + "".join(f" + (y * (x - {k}" for k in range(9)) + ")" * 18
    with pytest.raises(expr.UnsupportedExpression):
        expr.Program(_frame(), deep)


def test_chained_comparison_is_a_conjunction():
    df = _frame()
    x = np.asarray(df.columns["x"])
    np.testing.assert_array_equal(_run(expr.compile_expression(df, "0 < x < 1"), df), (0 < x) & (x < 1))
