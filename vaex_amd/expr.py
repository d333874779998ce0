"""Device evaluation of vaex expressions over HBM columns (``vh_expr_eval``, csrc/expr.hip).

The reference evaluates virtual columns, selections and filters with numpy, chunk by chunk
(``dataframe.py`` ``evaluate``, ``cpu.py:542-581``, ``execution.py:337-341``).  For a
DataFrame whose columns live in HBM this module compiles the expression once into a small
stack program and evaluates it with one HIP kernel per chunk, writing a new HBM column
(or a uint8 mask for selections / filters) -- no host round trip.

Semantics follow numpy 2: the result dtype of every node is numpy's own (found by running
the numpy operation on empty arrays / Python scalars, so NEP 50 weak scalars hold), float32
nodes are rounded to float32 after each operation and narrow integer nodes wrap, like
numpy's.  Supported: columns, virtual columns, variables, Python int / float / bool
constants, ``+ - * / // % **``, unary ``- ~``, comparisons (chained too), ``& | ^ << >>``,
``and / or / not`` on booleans, and the functions in :data:`FUNCTIONS` (also as ``np.f``).
Anything else raises :class:`UnsupportedExpression`, which callers turn into the host path
or an error (there is no silent fallback for HBM columns).
"""
import ast
import ctypes

import numpy as np

from . import _lib

# opcodes (csrc/expr.hip)
OP = dict(COL=0, CONST=1, I2F=2, F2I=3, ROUND_F32=4, WRAP=5, U2F=6,
          ADD_F=10, SUB_F=11, MUL_F=12, DIV_F=13, FLOORDIV_F=14, MOD_F=15, POW_F=16, NEG_F=17, ABS_F=18,
          MIN_F=19, MAX_F=20, ARCTAN2=21,
          ADD_I=30, SUB_I=31, MUL_I=32, FLOORDIV_I=33, MOD_I=34, NEG_I=35, ABS_I=36, AND_I=37, OR_I=38,
          XOR_I=39, INV_I=40, MIN_I=41, MAX_I=42, SHL_I=43, SHR_I=44, POW_I=45,
          LT_F=50, LE_F=51, GT_F=52, GE_F=53, EQ_F=54, NE_F=55,
          LT_I=60, LE_I=61, GT_I=62, GE_I=63, EQ_I=64, NE_I=65, LT_U=66, LE_U=67, GT_U=68, GE_U=69,
          NOT_B=70,
          SQRT=80, EXP=81, LOG=82, LOG10=83, SIN=84, COS=85, TAN=86, ARCSIN=87, ARCCOS=88, ARCTAN=89,
          SINH=90, COSH=91, TANH=92, FLOOR=93, CEIL=94, ISNAN=95, ISFINITE=96, ISINF=97, LOG1P=98, EXPM1=99,
          LOG2=100, EXP2=101, TRUNC=102, RINT=103,
          WHERE=110)
MAX_CODE, MAX_CONST, MAX_COLS, MAX_DEPTH = 128, 32, 16, 8

# float -> float functions (numpy ufunc, opcode)
FUNCTIONS = {
    "sqrt": (np.sqrt, "SQRT"), "exp": (np.exp, "EXP"), "log": (np.log, "LOG"), "log10": (np.log10, "LOG10"),
    "log2": (np.log2, "LOG2"), "exp2": (np.exp2, "EXP2"), "log1p": (np.log1p, "LOG1P"),
    "expm1": (np.expm1, "EXPM1"), "sin": (np.sin, "SIN"), "cos": (np.cos, "COS"), "tan": (np.tan, "TAN"),
    "arcsin": (np.arcsin, "ARCSIN"), "arccos": (np.arccos, "ARCCOS"), "arctan": (np.arctan, "ARCTAN"),
    "sinh": (np.sinh, "SINH"), "cosh": (np.cosh, "COSH"), "tanh": (np.tanh, "TANH"),
    "floor": (np.floor, "FLOOR"), "ceil": (np.ceil, "CEIL"), "trunc": (np.trunc, "TRUNC"), "rint": (np.rint, "RINT"),
}
PREDICATES = {"isnan": (np.isnan, "ISNAN"), "isfinite": (np.isfinite, "ISFINITE"), "isinf": (np.isinf, "ISINF")}


class UnsupportedExpression(ValueError):
    pass


class _Typed:
    """A compiled sub-expression: its code and numpy dtype (or a Python scalar for a
    constant, which numpy 2 promotes as a weak scalar)."""

    def __init__(self, code, dtype, scalar=None):
        self.code = code
        self.dtype = np.dtype(dtype)
        self.scalar = scalar  # the Python value of a constant leaf

    @property
    def proto(self):
        """What numpy sees for type resolution: the Python scalar or an empty array."""
        return self.scalar if self.scalar is not None else np.empty(0, self.dtype)


def _kind(dt):
    return "f" if dt.kind == "f" else ("u" if dt.kind == "u" else ("b" if dt.kind == "b" else "i"))


class Compiler:
    def __init__(self, df):
        self.df = df
        self.columns = []      # column names in slot order
        self.consts = []       # uint64 bit patterns
        self._depth = 0

    # ---- leaves -------------------------------------------------------------------
    def _const(self, value):
        if isinstance(value, bool):
            bits, dt = int(value), np.bool_
        elif isinstance(value, (int, np.integer)):
            value = int(value)
            if not -(1 << 63) <= value < (1 << 64):
                raise UnsupportedExpression("integer constant out of 64-bit range")
            bits, dt = value & 0xFFFFFFFFFFFFFFFF, np.int64
        elif isinstance(value, (float, np.floating)):
            bits, dt = int(np.array(float(value)).view(np.uint64)), np.float64
        else:
            raise UnsupportedExpression(f"constant {value!r}")
        if len(self.consts) >= MAX_CONST:
            raise UnsupportedExpression("too many constants")
        self.consts.append(bits)
        idx = len(self.consts) - 1
        return _Typed([OP["CONST"] | idx << 8], dt, scalar=value if not isinstance(value, np.generic) else value.item())

    def _column(self, name):
        col = self.df.columns[name]
        dt = np.dtype(col.dtype)
        if dt.kind not in "biuf" or not dt.isnative:
            raise UnsupportedExpression(f"column {name!r} of dtype {dt}")
        if np.ma.isMaskedArray(col):
            raise UnsupportedExpression(f"masked column {name!r}")
        if name not in self.columns:
            if len(self.columns) >= MAX_COLS:
                raise UnsupportedExpression("too many columns")
            self.columns.append(name)
        return _Typed([OP["COL"] | self.columns.index(name) << 8], dt)

    # ---- conversions -----------------------------------------------------------------
    @staticmethod
    def _to_float(t):
        """code leaving t's value as float64 bits."""
        k = _kind(t.dtype)
        if k == "f":
            return list(t.code)
        if t.scalar is not None and not isinstance(t.scalar, bool):
            return list(t.code) + [OP["I2F"]]
        return list(t.code) + [OP["U2F"] if (k == "u" and t.dtype.itemsize == 8) else OP["I2F"]]

    @staticmethod
    def _finish(code, dtype):
        """the node's own rounding / wrap-around (numpy computes in the result dtype)."""
        dtype = np.dtype(dtype)
        if dtype == np.float32:
            return code + [OP["ROUND_F32"]]
        if dtype.kind in "iu" and dtype.itemsize < 8:
            return code + [OP["WRAP"] | ((dtype.itemsize * 8) | ((dtype.kind == "i") << 8)) << 8]
        return code

    # ---- nodes ---------------------------------------------------------------------
    def visit(self, node):
        m = getattr(self, "v_" + type(node).__name__, None)
        if m is None:
            raise UnsupportedExpression(f"unsupported syntax {type(node).__name__}")
        return m(node)

    def v_Expression(self, node):
        return self.visit(node.body)

    def v_Constant(self, node):
        return self._const(node.value)

    def v_Name(self, node):
        name = node.id
        if name in self.df.columns:
            return self._column(name)
        if name in self.df.virtual_columns:
            return self.visit(ast.parse(self.df.virtual_columns[name], mode="eval"))
        if name in self.df.variables:
            v = self.df.variables[name]
            if isinstance(v, (bool, int, float, np.integer, np.floating, np.bool_)):
                return self._const(v.item() if isinstance(v, np.generic) else v)
            raise UnsupportedExpression(f"variable {name!r} is not a scalar")
        if name in ("True", "False"):
            return self._const(name == "True")
        if name in ("nan", "inf"):
            return self._const(float(name))
        raise UnsupportedExpression(f"unknown name {name!r}")

    def v_Attribute(self, node):
        # np.nan, np.inf, np.pi, np.e
        if isinstance(node.value, ast.Name) and node.value.id in ("np", "numpy"):
            if node.attr in ("nan", "inf", "pi", "e"):
                return self._const(float(getattr(np, node.attr)))
        raise UnsupportedExpression("attribute access")

    def _arith(self, opname, a, b):
        ufunc = {"+": np.add, "-": np.subtract, "*": np.multiply, "/": np.true_divide, "//": np.floor_divide,
                 "%": np.remainder, "**": np.power}[opname]
        with np.errstate(all="ignore"):
            try:
                dt = np.result_type(ufunc(a.proto, b.proto))
            except TypeError as e:
                raise UnsupportedExpression(str(e))
        if a.scalar is not None and b.scalar is not None:
            with np.errstate(all="ignore"):
                v = ufunc(a.scalar, b.scalar)
            return self._const(v.item() if isinstance(v, np.generic) else v)
        if dt.kind == "b":  # numpy: bool + bool = or, bool * bool = and
            if opname in ("+", "*"):
                return _Typed(a.code + b.code + [OP["OR_I" if opname == "+" else "AND_I"]], dt)
            raise UnsupportedExpression(f"boolean {opname}")
        if dt.kind == "f" and opname == "**" and b.scalar is not None and a.scalar is None \
                and not isinstance(b.scalar, bool) and b.scalar in (2, 0.5, -1, 1):
            # numpy's fast_scalar_power: x**2 = square, x**0.5 = sqrt, x**-1 = reciprocal
            x = self._to_float(a)
            if b.scalar == 2:
                code = x + x + [OP["MUL_F"]]
            elif b.scalar == 0.5:
                code = x + [OP["SQRT"]]
            elif b.scalar == -1:
                code = self._const(1.0).code + x + [OP["DIV_F"]]
            else:
                code = x
        elif dt.kind == "f":
            code = self._to_float(a) + self._to_float(b)
            code.append(OP[{"+": "ADD_F", "-": "SUB_F", "*": "MUL_F", "/": "DIV_F", "//": "FLOORDIV_F",
                            "%": "MOD_F", "**": "POW_F"}[opname]])
        else:
            if opname == "**" and b.scalar is not None and b.scalar < 0:
                raise UnsupportedExpression("integers to negative integer powers")
            code = a.code + b.code
            code.append(OP[{"+": "ADD_I", "-": "SUB_I", "*": "MUL_I", "//": "FLOORDIV_I", "%": "MOD_I",
                            "**": "POW_I"}[opname]])
        return _Typed(self._finish(code, dt), dt)

    def _bitwise(self, opname, a, b):
        ufunc = {"&": np.bitwise_and, "|": np.bitwise_or, "^": np.bitwise_xor,
                 "<<": np.left_shift, ">>": np.right_shift}[opname]
        try:
            dt = np.result_type(ufunc(a.proto, b.proto))
        except TypeError as e:
            raise UnsupportedExpression(str(e))
        op = {"&": "AND_I", "|": "OR_I", "^": "XOR_I", "<<": "SHL_I", ">>": "SHR_I"}[opname]
        return _Typed(self._finish(a.code + b.code + [OP[op]], dt), dt)

    def v_BinOp(self, node):
        a, b = self.visit(node.left), self.visit(node.right)
        sym = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/", ast.FloorDiv: "//", ast.Mod: "%",
               ast.Pow: "**", ast.BitAnd: "&", ast.BitOr: "|", ast.BitXor: "^", ast.LShift: "<<",
               ast.RShift: ">>"}.get(type(node.op))
        if sym is None:
            raise UnsupportedExpression(f"operator {type(node.op).__name__}")
        if sym in ("&", "|", "^", "<<", ">>"):
            return self._bitwise(sym, a, b)
        return self._arith(sym, a, b)

    def v_UnaryOp(self, node):
        a = self.visit(node.operand)
        if isinstance(node.op, ast.USub):
            if a.scalar is not None:
                return self._const(-a.scalar)
            if a.dtype.kind == "b":
                raise UnsupportedExpression("negation of a boolean")
            if a.dtype.kind == "f":
                return _Typed(self._finish(a.code + [OP["NEG_F"]], a.dtype), a.dtype)
            return _Typed(self._finish(a.code + [OP["NEG_I"]], a.dtype), a.dtype)
        if isinstance(node.op, ast.UAdd):
            return a
        if isinstance(node.op, (ast.Invert, ast.Not)):
            if a.dtype.kind == "b":
                return _Typed(a.code + [OP["NOT_B"]], np.bool_)
            if isinstance(node.op, ast.Not) or a.dtype.kind == "f":
                raise UnsupportedExpression("not / ~ of a non-boolean float")
            return _Typed(self._finish(a.code + [OP["INV_I"]], a.dtype), a.dtype)
        raise UnsupportedExpression("unary operator")

    def _compare(self, op, a, b):
        dt = np.result_type(a.proto, b.proto)
        sym = {ast.Lt: "LT", ast.LtE: "LE", ast.Gt: "GT", ast.GtE: "GE", ast.Eq: "EQ", ast.NotEq: "NE"}.get(type(op))
        if sym is None:
            raise UnsupportedExpression("comparison operator")
        if dt.kind == "f":
            return _Typed(self._to_float(a) + self._to_float(b) + [OP[sym + "_F"]], np.bool_)
        unsigned = dt.kind == "u" and dt.itemsize == 8 and sym not in ("EQ", "NE")
        return _Typed(a.code + b.code + [OP[sym + ("_U" if unsigned else "_I")]], np.bool_)

    def v_Compare(self, node):
        left = self.visit(node.left)
        out = None
        for op, comp in zip(node.ops, node.comparators):
            right = self.visit(comp)
            t = self._compare(op, left, right)
            out = t if out is None else _Typed(out.code + t.code + [OP["AND_I"]], np.bool_)
            left = right
        return out

    def v_BoolOp(self, node):
        vals = [self.visit(v) for v in node.values]
        if any(v.dtype.kind != "b" for v in vals):
            raise UnsupportedExpression("and / or of non-booleans")
        op = OP["AND_I"] if isinstance(node.op, ast.And) else OP["OR_I"]
        code = list(vals[0].code)
        for v in vals[1:]:
            code += v.code + [op]
        return _Typed(code, np.bool_)

    def v_Call(self, node):
        f = node.func
        if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id in ("np", "numpy"):
            name = f.attr
        elif isinstance(f, ast.Name):
            name = f.id
        else:
            raise UnsupportedExpression("call")
        if node.keywords:
            raise UnsupportedExpression("keyword arguments")
        if name == "astype" and len(node.args) == 2:
            return self._astype(node.args[0], node.args[1])
        args = [self.visit(a) for a in node.args]
        if name in FUNCTIONS and len(args) == 1:
            ufunc, op = FUNCTIONS[name]
            a = args[0]
            dt = np.result_type(ufunc(a.proto))
            if dt.kind != "f":
                raise UnsupportedExpression(f"{name} of {a.dtype}")
            return _Typed(self._finish(self._to_float(a) + [OP[op]], dt), dt)
        if name in PREDICATES and len(args) == 1:
            a = args[0]
            if a.dtype.kind != "f":  # integers are never nan / inf: a constant column
                return _Typed(self._const(name == "isfinite").code, np.bool_)
            return _Typed(a.code + [OP[PREDICATES[name][1]]], np.bool_)
        if name in ("abs", "absolute", "fabs") and len(args) == 1:
            a = args[0]
            if a.dtype.kind == "f" or name == "fabs":
                dt = np.result_type(np.fabs(a.proto)) if name == "fabs" else a.dtype
                return _Typed(self._finish(self._to_float(a) + [OP["ABS_F"]], dt), dt)
            return _Typed(self._finish(a.code + [OP["ABS_I"]], a.dtype), a.dtype)
        if name in ("minimum", "maximum", "fmin", "fmax", "arctan2") and len(args) == 2:
            a, b = args
            ufunc = getattr(np, name)
            dt = np.result_type(ufunc(a.proto, b.proto))
            if name in ("fmin", "fmax"):
                raise UnsupportedExpression(name)
            if dt.kind == "f":
                op = {"minimum": "MIN_F", "maximum": "MAX_F", "arctan2": "ARCTAN2"}[name]
                return _Typed(self._finish(self._to_float(a) + self._to_float(b) + [OP[op]], dt), dt)
            op = {"minimum": "MIN_I", "maximum": "MAX_I"}[name]
            return _Typed(self._finish(a.code + b.code + [OP[op]], dt), dt)
        if name == "where" and len(args) == 3:
            c, a, b = args
            if c.dtype.kind != "b":
                raise UnsupportedExpression("where condition must be boolean")
            dt = np.result_type(np.where(np.empty(0, bool), a.proto, b.proto))
            if dt.kind == "f":
                code = c.code + self._to_float(a) + self._to_float(b) + [OP["WHERE"]]
            else:
                code = c.code + a.code + b.code + [OP["WHERE"]]
            return _Typed(self._finish(code, dt), dt)
        raise UnsupportedExpression(f"function {name}")

    def _astype(self, value_node, dtype_node):
        """``astype(x, 'dtype')`` (the reference's ``Expression.astype``, expression.py;
        ``agg.py:197-201`` casts var/std inputs this way): numpy ``ndarray.astype``
        semantics -- float -> int truncates toward zero, integers wrap."""
        if not (isinstance(dtype_node, ast.Constant) and isinstance(dtype_node.value, str)):
            raise UnsupportedExpression("astype needs a constant dtype string")
        try:
            dt = np.dtype(dtype_node.value)
        except TypeError as e:
            raise UnsupportedExpression(str(e))
        if dt.kind not in "biuf" or dt.itemsize > 8:
            raise UnsupportedExpression(f"astype to {dt}")
        a = self.visit(value_node)
        if a.dtype == dt and a.scalar is None:
            return a
        if a.scalar is not None:
            with np.errstate(all="ignore"):
                return self._const(np.array(a.scalar).astype(dt).item())
        if dt.kind == "f":
            return _Typed(self._finish(self._to_float(a), dt), dt)
        if dt.kind == "b":
            if a.dtype.kind == "f":
                code = self._to_float(a) + self._const(0.0).code + [OP["NE_F"]]
            else:
                code = a.code + self._const(0).code + [OP["NE_I"]]
            return _Typed(code, dt)
        code = list(a.code) + ([OP["F2I"]] if a.dtype.kind == "f" else [])
        return _Typed(self._finish(code, dt), dt)


def _stack_depth(code):
    binary = set(range(10, 22)) - {17, 18} | (set(range(30, 46)) - {35, 36, 40}) | set(range(50, 70))
    d = m = 0
    for ins in code:
        op = ins & 0xFF
        if op in (OP["COL"], OP["CONST"]):
            d += 1
        elif op == OP["WHERE"]:
            d -= 2
        elif op in binary:
            d -= 1
        m = max(m, d)
    return m


class Program:
    """A compiled expression: evaluate(df, i1, i2) -> DeviceArray of ``dtype``."""

    def __init__(self, df, expression):
        self.expression = str(expression)
        c = Compiler(df)
        try:
            tree = ast.parse(self.expression, mode="eval")
        except SyntaxError as e:
            raise UnsupportedExpression(str(e))
        t = c.visit(tree)
        code = list(t.code)  # a constant expression is broadcast by the kernel
        if len(code) > MAX_CODE:
            raise UnsupportedExpression("expression too long for the device program")
        if _stack_depth(code) > MAX_DEPTH:
            raise UnsupportedExpression("expression too deeply nested")
        self.code = code
        self.consts = list(c.consts)
        self.columns = list(c.columns)
        self.dtype = t.dtype  # bool results are 0 / 1 bytes (numpy bool)
        self.is_bool = t.dtype.kind == "b"

    def evaluate(self, df, i1, i2, out=None):
        from .device import DeviceArray
        n = i2 - i1
        cols = []
        keep = []
        for name in self.columns:
            col = df.columns[name]
            if not isinstance(col, DeviceArray):
                col = DeviceArray.from_numpy(np.ascontiguousarray(col[i1:i2]))
                keep.append(col)
            else:
                col = col[i1:i2]
            cols.append(col)
        if out is None:
            out = DeviceArray.empty(n, self.dtype)
        k = max(1, len(cols))
        code = (ctypes.c_uint32 * len(self.code))(*self.code)
        consts = (ctypes.c_uint64 * max(1, len(self.consts)))(*self.consts)
        ptrs = (ctypes.c_void_p * k)(*[c.ptr for c in cols])
        dts = (ctypes.c_int * k)(*[_lib.dtype_code(c.dtype)[0] for c in cols])
        _lib.call("vh_expr_eval", code, len(self.code), consts, len(self.consts), ptrs, dts, len(cols), n,
                  _lib.dtype_code(self.dtype)[0], out.ptr)
        if keep:
            _lib.synchronize()  # the staged columns are freed on return
        return out


_CACHE = {}


def compile_expression(df, expression):
    """The Program of ``expression`` on ``df`` (cached per frame structure)."""
    key = (id(df), str(expression), tuple(sorted(df.virtual_columns.items())),
           tuple(sorted((k, repr(v)) for k, v in df.variables.items() if np.isscalar(v))),
           tuple((k, str(getattr(v, "dtype", ""))) for k, v in df.columns.items()))
    p = _CACHE.get(key)
    if p is None:
        p = Program(df, expression)
        if len(_CACHE) > 256:
            _CACHE.clear()
        _CACHE[key] = p
    return p
