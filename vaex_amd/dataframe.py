"""A DataFrame exposing the reference's binned-statistics API on the GPU path.

Restates the parts of ``packages/vaex-core/vaex/dataframe.py`` that drive this hot
path -- ``count/sum/mean/min/max/std/var/first`` (``:741-1000``), ``minmax``
(``:1276-1333``), ``limits`` (``:1617+``), ``_binner*``/``_create_binners``
(``:5251-5295``), ``_agg``, ``_set`` (``:474``), ``categorize`` (``:5487-5533``),
``groupby``/``binby`` (``:6622-6683``) and the binner specs ``BinnerScalar`` /
``BinnerOrdinal`` (``:6737-6800``) -- over columns that are numpy arrays (staged to
HBM per chunk) or :class:`~vaex_amd.device.DeviceArray` (HBM-resident).

The reference's lazy expression engine is out of scope: expressions
here are column names, or numpy expressions over host columns evaluated per chunk.
"""
import ast
import re

import numpy as np

from . import agg as vagg
from .device import DeviceArray
from .execution import default_executor
from .promise import Promise, delayed
from .tasks import TaskMinMax, TaskSetCreate
from .utils import _expand_limits, _expand_shape, listify, unlistify

default_shape = 128


class RowLimitException(ValueError):
    pass


def _ensure_string(e):
    return str(e) if isinstance(e, Expression) else e


def _ensure_strings(es):
    if isinstance(es, (list, tuple)):
        return [_ensure_string(e) for e in es]
    return _ensure_string(es)


class BinnerScalar:
    """Spec of a scalar binner (dataframe.py:6749-6775)."""
    kind = "scalar"

    def __init__(self, expression, minimum, maximum, count, dtype):
        self.expression = str(expression)
        self.minimum = minimum
        self.maximum = maximum
        self.count = count
        self.dtype = np.dtype(dtype)

    def __hash__(self):
        return hash((self.kind, self.expression, self.minimum, self.maximum, self.count, self.dtype))

    def __eq__(self, rhs):
        return isinstance(rhs, BinnerScalar) and (self.expression, self.minimum, self.maximum, self.count,
                                                  self.dtype) == (rhs.expression, rhs.minimum, rhs.maximum,
                                                                  rhs.count, rhs.dtype)


class BinnerOrdinal:
    """Spec of an ordinal binner (dataframe.py:6778-6800)."""
    kind = "ordinal"

    def __init__(self, expression, minimum, count, dtype):
        self.expression = str(expression)
        self.minimum = minimum
        self.count = count
        self.dtype = np.dtype(dtype)

    def __hash__(self):
        return hash((self.kind, self.expression, self.minimum, self.count, self.dtype))

    def __eq__(self, rhs):
        return isinstance(rhs, BinnerOrdinal) and (self.expression, self.minimum, self.count, self.dtype) == (
            rhs.expression, rhs.minimum, rhs.count, rhs.dtype)


class Expression:
    """A column reference or host numpy expression bound to a DataFrame."""

    def __init__(self, df, expression):
        self.df = df
        self.expression = str(expression)

    def __str__(self):
        return self.expression

    def __repr__(self):
        return f"Expression({self.expression!r})"

    def _binop(self, other, op, reverse=False):
        o = other.expression if isinstance(other, Expression) else repr(other)
        s = f"({o} {op} {self.expression})" if reverse else f"({self.expression} {op} {o})"
        return Expression(self.df, s)

    def __add__(self, o): return self._binop(o, "+")
    def __radd__(self, o): return self._binop(o, "+", True)
    def __sub__(self, o): return self._binop(o, "-")
    def __rsub__(self, o): return self._binop(o, "-", True)
    def __mul__(self, o): return self._binop(o, "*")
    def __rmul__(self, o): return self._binop(o, "*", True)
    def __truediv__(self, o): return self._binop(o, "/")
    def __pow__(self, o): return self._binop(o, "**")
    def __lt__(self, o): return self._binop(o, "<")
    def __le__(self, o): return self._binop(o, "<=")
    def __gt__(self, o): return self._binop(o, ">")
    def __ge__(self, o): return self._binop(o, ">=")
    def __eq__(self, o): return self._binop(o, "==")
    def __ne__(self, o): return self._binop(o, "!=")
    def __and__(self, o): return self._binop(o, "&")
    def __or__(self, o): return self._binop(o, "|")
    def __neg__(self): return Expression(self.df, f"(-{self.expression})")
    def __invert__(self): return Expression(self.df, f"(~{self.expression})")
    __hash__ = object.__hash__

    def astype(self, data_type):
        """expression.py ``Expression.astype``: the expression ``astype(x, 'dtype')``."""
        return Expression(self.df, f"astype({self.expression}, {str(np.dtype(data_type))!r})")

    @property
    def dtype(self):
        return self.df.data_type(self.expression)

    @property
    def values(self):
        return self.df.evaluate(self.expression)

    def to_numpy(self):
        v = self.values
        if isinstance(v, DeviceArray):
            return v.to_numpy()
        return v if np.ma.isMaskedArray(v) else np.asarray(v)  # masked columns stay masked

    def tolist(self):
        return self.to_numpy().tolist()

    def sum(self, *args, **kw): return self.df.sum(self.expression, *args, **kw)
    def count(self, *args, **kw): return self.df.count(self.expression, *args, **kw)
    def mean(self, *args, **kw): return self.df.mean(self.expression, *args, **kw)
    def min(self, *args, **kw): return self.df.min(self.expression, *args, **kw)
    def max(self, *args, **kw): return self.df.max(self.expression, *args, **kw)
    def std(self, *args, **kw): return self.df.std(self.expression, *args, **kw)
    def var(self, *args, **kw): return self.df.var(self.expression, *args, **kw)
    def minmax(self, *args, **kw): return self.df.minmax(self.expression, *args, **kw)


def _ordinal_values(x, ordered_set):
    """functions.py:2441-2448 (host evaluation; the bin kernel fuses it instead)."""
    return ordered_set.map_ordinal(x)


def _astype(x, data_type):
    """functions.py ``astype`` on host chunks (numpy ``ndarray.astype``)."""
    return np.asarray(x).astype(data_type) if not np.ma.isMaskedArray(x) else x.astype(data_type)


class DataFrame:
    def __init__(self, columns, executor=None):
        self.columns = dict(columns)
        self.variables = {}
        self.virtual_columns = {}
        self._categories = {}
        self.selection_expressions = {}
        self._filter = None
        self.executor = executor or default_executor
        lengths = {len(v) for v in self.columns.values()}
        if len(lengths) > 1:
            raise ValueError(f"columns have different lengths: {lengths}")
        self._length = lengths.pop() if lengths else 0

    # ---- structure ---------------------------------------------------------------
    def __len__(self):
        if self._filter is None:
            return self._length
        return int(self.count())

    def length_unfiltered(self):
        return self._length

    @property
    def filtered(self):
        return self._filter is not None

    def is_device_resident(self):
        return any(isinstance(c, DeviceArray) for c in self.columns.values())

    def get_column_names(self):
        return list(self.columns) + list(self.virtual_columns)

    def copy(self):
        df = DataFrame(self.columns, executor=self.executor)
        df.variables = dict(self.variables)
        df.virtual_columns = dict(self.virtual_columns)
        df._categories = dict(self._categories)
        df.selection_expressions = dict(self.selection_expressions)
        df._filter = self._filter
        # copies share the filter-mask cache (its keys hold the filter and the columns, so a
        # copy that changes either misses; groupby works on a copy)
        df._filter_mask_cache = self.__dict__.setdefault("_filter_mask_cache", {})
        return df

    def add_column(self, name, data):
        if len(data) != self._length and self.columns:
            raise ValueError("column length mismatch")
        self.columns[name] = data
        if not self._length:
            self._length = len(data)

    def __setitem__(self, name, value):
        if isinstance(value, Expression):
            self.virtual_columns[name] = value.expression
        else:
            self.add_column(name, value)

    def add_virtual_column(self, name, expression):
        self.virtual_columns[name] = str(expression)

    def add_variable(self, name, value, unique=False):
        if unique:
            base, i = name, 0
            while name in self.variables:
                i += 1
                name = f"{base}_{i}"
        self.variables[name] = value
        return name

    def __getitem__(self, item):
        if isinstance(item, Expression) and str(item) not in self.columns and \
                str(item) not in self.virtual_columns and self.data_type(item).kind == "b":
            return self.filter(item)  # df[df.x > 0] (dataframe.py __getitem__: boolean expression = filter)
        if isinstance(item, (str, Expression)):
            return Expression(self, str(item))
        raise TypeError(item)

    def __getattr__(self, name):
        if name.startswith("_") or name in ("columns", "variables", "virtual_columns"):
            raise AttributeError(name)
        if name in self.__dict__.get("columns", {}) or name in self.__dict__.get("virtual_columns", {}):
            return Expression(self, name)
        raise AttributeError(name)

    def filter(self, expression):
        df = self.copy()
        e = str(expression)
        df._filter = e if self._filter is None else f"({self._filter}) & ({e})"
        return df

    def is_category(self, expression):
        return str(expression) in self._categories

    def categorize(self, column, min_value=0, max_value=None, labels=None, inplace=False):
        """dataframe.py:5487-5533: mark an integer column as categorical with N labels."""
        df = self if inplace else self.copy()
        column = str(column)
        if labels is None:
            vmin, vmax = df.minmax(column)
            min_value = int(vmin) if min_value is None else min_value
            max_value = int(vmax) if max_value is None else max_value
            labels = list(range(min_value, max_value + 1))
        N = len(labels)
        df._categories[column] = dict(labels=labels, N=N, min_value=min_value)
        return df

    def category_labels(self, column):
        return self._categories[str(column)]["labels"]

    # ---- evaluation --------------------------------------------------------------
    def _namespace(self, i1, i2, filter_mask=None):
        ns = {"np": np, "_ordinal_values": _ordinal_values, "astype": _astype}
        for name, col in self.columns.items():
            ns[name] = col
        ns.update(self.variables)
        return ns

    def _eval_host(self, expression, i1, i2, filter_mask=None):
        expression = str(expression)
        if isinstance(filter_mask, DeviceArray):
            # HBM frame: chunks stay whole, the parts apply the filter as a row mask
            filter_mask = None
        if expression in self.columns:
            col = self.columns[expression]
            if isinstance(col, DeviceArray):
                if filter_mask is not None:
                    raise NotImplementedError("filtered DataFrames need host columns")
                return col[i1:i2]
            block = col[i1:i2]
            return block[filter_mask] if filter_mask is not None else block
        if self.is_device_resident():
            return self._eval_device(expression, i1, i2)
        if expression in self.virtual_columns:
            return self._eval_host(self.virtual_columns[expression], i1, i2, filter_mask)
        ns = {"np": np, "_ordinal_values": _ordinal_values, "astype": _astype}
        ns.update(self.variables)
        for name, col in self.columns.items():
            if name in expression:
                if isinstance(col, DeviceArray):
                    raise NotImplementedError(
                        f"expression {expression!r} over an HBM column: only plain columns bin in place")
                ns[name] = col[i1:i2]
        for name, vexpr in self.virtual_columns.items():
            if name in expression:
                ns[name] = self._eval_host(vexpr, i1, i2, None)
        with np.errstate(all="ignore"):
            value = eval(expression, {"__builtins__": {}}, ns)  # noqa: S307 (host-side expressions)
        if np.isscalar(value):
            value = np.full(i2 - i1, value)
        value = np.asarray(value) if not np.ma.isMaskedArray(value) else value
        return value[filter_mask] if filter_mask is not None else value

    def _eval_device(self, expression, i1, i2):
        """An expression over HBM columns, evaluated by the device expression kernel into
        a new HBM column (expr.py); unsupported syntax raises rather than leaving the GPU."""
        from .expr import UnsupportedExpression, compile_expression
        try:
            return compile_expression(self, expression).evaluate(self, i1, i2)
        except UnsupportedExpression as e:
            raise NotImplementedError(f"expression {expression!r} over HBM columns: {e}") from None

    def evaluate_chunk(self, expression, i1, i2, filter_mask=None):
        return self._eval_host(expression, i1, i2, filter_mask)

    def evaluate(self, expression, i1=None, i2=None, filtered=True):
        i1 = 0 if i1 is None else i1
        i2 = self._length if i2 is None else i2
        fm = self.evaluate_filter_mask(i1, i2) if (filtered and self.filtered) else None
        if isinstance(fm, DeviceArray):
            # the filtered rows of an HBM frame, read back (the compaction happens on the host)
            v = self._eval_host(expression, i1, i2)
            v = v.to_numpy() if isinstance(v, DeviceArray) else np.asarray(v)
            return v[fm.to_numpy().astype(bool)]
        return self._eval_host(expression, i1, i2, fm)

    def evaluate_filter_mask(self, i1, i2):
        if self.is_device_resident():
            # the device mask of the filter, per (i1, i2) block, kept while the frame's columns,
            # virtual columns and variables stay the same objects (the reference keeps filter
            # masks per block too: _selection_mask_caches[FILTER_SELECTION_NAME],
            # dataframe.py:4161,5967, dropped by _invalidate_selection_cache)
            return self._cached_device_mask(self._filter, i1, i2)
        return np.asarray(self._eval_host(self._filter, i1, i2), dtype=bool)

    def _cached_device_mask(self, expr, i1, i2):
        key = (expr, i1, i2,
               tuple((k, getattr(c, "ptr", id(c)), len(c)) for k, c in self.columns.items()),
               tuple(sorted(self.virtual_columns.items())), tuple((k, id(v)) for k, v in self.variables.items()))
        cache = self.__dict__.setdefault("_filter_mask_cache", {})
        m = cache.get(key)
        if m is None:
            if len(cache) >= 8:
                cache.clear()
            m = cache[key] = self._eval_device(expr, i1, i2)
        return m

    def data_type(self, expression):
        expression = str(expression)
        if expression in self.columns:
            return np.dtype(self.columns[expression].dtype)
        if self.is_device_resident():
            from .expr import UnsupportedExpression, compile_expression
            try:
                return compile_expression(self, expression).dtype
            except UnsupportedExpression as e:
                raise NotImplementedError(f"expression {expression!r} over HBM columns: {e}") from None
        v = self._eval_host(expression, 0, min(self._length, 16))
        return np.dtype(v.dtype)

    def _selection_expression(self, selection):
        if selection is True:
            selection = "default"
        if isinstance(selection, str) and selection in self.selection_expressions:
            selection = self.selection_expressions[selection]
        return str(selection)

    def device_keep_mask(self, i1, i2, selection=None, invert=False, cache=False):
        """HBM frame: one device mask of the rows a part takes (filter & selection), or its
        complement (invert: the skip mask of the min/max kernel); None = every row.  cache:
        kept per block like the filter mask (the reference's aggregation parts ask for cached
        selection masks, cpu.py:548)."""
        parts = []
        if self._filter is not None:
            parts.append(f"({self._filter})")
        if selection not in (None, False):
            parts.append(f"({self._selection_expression(selection)})")
        if not parts:
            return None
        expr = " & ".join(parts)
        expr = f"~({expr})" if invert else expr
        return self._cached_device_mask(expr, i1, i2) if cache else self._eval_device(expr, i1, i2)

    # ---- selections --------------------------------------------------------------
    def select(self, expression, name="default"):
        self.selection_expressions[name] = str(expression)

    def select_nothing(self, name="default"):
        self.selection_expressions.pop(name, None)

    def has_selection(self, name="default"):
        return name in self.selection_expressions

    def evaluate_selection_mask(self, selection, i1=0, i2=None, filter_mask=None, cache=False):
        i2 = self._length if i2 is None else i2
        if isinstance(filter_mask, DeviceArray) or (filter_mask is None and self.is_device_resident()):
            # HBM frame: the device mask of (filter &) selection over the whole chunk
            return self.device_keep_mask(i1, i2, selection, cache=cache)
        selection = self._selection_expression(selection)
        mask = self._eval_host(str(selection), i1, i2, filter_mask)
        if np.ma.isMaskedArray(mask):
            mask = mask.data & ~np.ma.getmaskarray(mask)
        return np.asarray(mask, dtype=bool)

    # ---- execution ---------------------------------------------------------------
    def execute(self):
        self.executor.execute()

    def _delay(self, delay, value):
        if delay:
            return value
        self.execute()
        return value.get() if isinstance(value, Promise) else value

    # ---- binners -----------------------------------------------------------------
    def _binner_scalar(self, expression, limits, shape):
        return BinnerScalar(expression, limits[0], limits[1], shape, self.data_type(expression))

    def _binner_ordinal(self, expression, ordinal_count, min_value=0):
        if str(expression).startswith("_ordinal_values("):
            from .taskparts import parse_ordinal_values
            key_expr, _ = parse_ordinal_values(expression)
            dtype = self.data_type(key_expr)
        else:
            dtype = self.data_type(expression)
        return BinnerOrdinal(expression, min_value, ordinal_count, dtype)

    def _binner(self, expression, limits=None, shape=None, selection=None):
        """dataframe.py:5251-5265 (limits resolved eagerly)."""
        expression = str(expression)
        if expression in self._categories:
            N = self._categories[expression]["N"]
            min_value = self._categories[expression]["min_value"]
            return self._binner_ordinal(expression, N, min_value)
        lim = self.limits(expression, limits, selection=selection)
        return self._binner_scalar(expression, lim, shape)

    def _create_binners(self, binby, limits, shape, selection=None):
        """dataframe.py:5275-5295."""
        binbys = binby if isinstance(binby, (list, tuple)) else [binby]
        binbys = [str(b) for b in _ensure_strings(binbys) if b is not None and str(b) != ""]
        limits = _expand_limits(limits, len(binbys)) if binbys else []
        shapes = _expand_shape(shape, len(binbys))
        return tuple(self._binner(b, l, s, selection) for b, l, s in zip(binbys, limits, shapes))

    # ---- limits ------------------------------------------------------------------
    def limits(self, expression, value=None, square=False, selection=None, delay=False, shape=None):
        """dataframe.py:1617-1699 for one expression: explicit [lo, hi], 'minmax' (the GPU
        min/max pre-pass) and percentages ('99.7%', '90percent'; the '%s' / 'percentsquare'
        forms too, whose square flag the reference ignores).  'Nsigma' raises like the
        reference, which calls a limits_sigma it does not define."""
        if value is None or (isinstance(value, str) and value == "minmax"):
            vmin, vmax = self.minmax(expression, selection=selection)
            return [vmin, vmax]
        if isinstance(value, str):
            match = re.match(r"([\d.]*)(\D*)", value)
            number, kind = match.groups()
            kind = kind.strip()
            if kind in ("%", "percent", "%s", "%square", "percentsquare"):
                return list(self.limits_percentage(expression, ast.literal_eval(number), selection=selection))
            if kind in ("s", "sigma", "ss", "sigmasquare"):
                raise AttributeError("'DataFrame' object has no attribute 'limits_sigma'")
            raise ValueError("limit %r not understood" % value)
        return list(value)

    def limits_percentage(self, expression, percentage=99.73, square=False, selection=False, delay=False):
        """dataframe.py:1570-1614: the range around the median holding about `percentage` %
        of the rows, read off the cumulative 16384-bin histogram over [min, max] (both
        passes on the GPU)."""
        waslist, [expressions] = listify(_ensure_strings(expression))
        sel = None if selection in (None, False) else selection
        out = []
        for expr in expressions:
            vmin, vmax = self.minmax(expr, selection=sel)
            size = 1024 * 16
            counts = np.asarray(self.count(binby=expr, shape=size, limits=[vmin, vmax], selection=selection))
            cumcounts = np.concatenate([[0], np.cumsum(counts)])
            cumcounts = cumcounts / cumcounts.max()
            f = (1 - percentage / 100.) / 2
            x = np.linspace(vmin, vmax, size + 1)
            out.append(np.interp([f, 1 - f], cumcounts, x))
        return unlistify(waslist, out)

    def minmax(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
               progress=None):
        """dataframe.py:1276-1333: NaN-ignoring min/max, cast back to the column dtype.  With
        binby, per cell of the grid (the last dimension holds [min, max]); an empty cell reads
        [inf, -inf], the OP_MIN_MAX initial values (tasks.py:173-185)."""
        if binby:
            return self._minmax_binby(expression, binby, limits, shape, selection, delay)
        expression = _ensure_strings(expression)
        waslist, [expressions] = listify(expression)
        sel = selection if selection not in (None, False) else None
        tasks = [self.executor.schedule(TaskMinMax(self, str(e), sel)) for e in expressions]
        dtype0 = self.data_type(expressions[0])

        @delayed
        def finish(*values):
            v = np.array(values)
            if dtype0.kind in "iu" and not np.isnan(v).any():
                v = v.astype(dtype0)
            return unlistify(waslist, v) if waslist else v[0]

        return self._delay(delay, finish(*tasks))

    def _minmax_binby(self, expression, binby, limits, shape, selection, delay):
        waslist, [expressions] = listify(_ensure_strings(expression))
        dtypes = [self.data_type(e) for e in expressions]
        if any(d.kind != dtypes[0].kind for d in dtypes):
            raise TypeError("cannot mix different dtypes in 1 minmax call")
        kw = dict(binby=binby, limits=limits, shape=shape, selection=selection, delay=True)
        parts = [(self.min(e, **kw), self.max(e, **kw), self.count(e, **kw)) for e in expressions]
        self.execute()
        values = []
        for mn, mx, cnt in parts:
            mn, mx, cnt = (np.asarray(p.get()) for p in (mn, mx, cnt))
            v = np.stack([mn.astype(np.float64), mx.astype(np.float64)], axis=-1)
            v[cnt == 0] = [np.inf, -np.inf]
            values.append(v)
        value = unlistify(waslist, np.array(values))
        return self._delay(delay, np.asarray(value).astype(dtypes[0]))

    # ---- aggregations ------------------------------------------------------------
    def _compute_agg(self, name, expression, binby=[], limits=None, shape=default_shape, selection=False,
                     delay=False, edges=False, progress=None, extra_expressions=None, array_type=None):
        """dataframe.py:741-827."""
        expression = _ensure_strings(expression)
        if extra_expressions:
            extra_expressions = _ensure_strings(extra_expressions)
        waslist, [expressions] = listify(expression)
        sel = None if selection is False else selection
        binners = self._create_binners(binby, limits, shape, selection=sel)
        results = []
        for expr in expressions:
            if expr in ("*", None):
                aggd = vagg.aggregates[name](selection=sel, edges=edges)
            elif extra_expressions:
                aggd = vagg.aggregates[name](expr, *extra_expressions, selection=sel, edges=edges)
            else:
                aggd = vagg.aggregates[name](expr, selection=sel, edges=edges)
            _, result = aggd.add_tasks(self, binners)
            results.append(result)

        @delayed
        def finish(*counts):
            counts = [np.asarray(c) for c in counts]
            if array_type == "list":
                return unlistify(waslist, np.asarray(counts) if waslist else counts[0]).tolist()
            return np.asarray(counts) if waslist else counts[0]

        return self._delay(delay, finish(*results))

    def count(self, expression=None, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
              edges=False, progress=None, array_type=None):
        """dataframe.py:830-853 (None or '*' counts rows, an expression counts non-NaN values)."""
        return self._compute_agg("count", "*" if expression is None else expression, binby, limits, shape, selection,
                                 delay, edges, progress, array_type=array_type)

    def sum(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
            progress=None, edges=False, array_type=None):
        return self._compute_agg("sum", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def mean(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
             progress=None, edges=False, array_type=None):
        return self._compute_agg("mean", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def min(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
            progress=None, edges=False, array_type=None):
        return self._compute_agg("min", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def max(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
            progress=None, edges=False, array_type=None):
        return self._compute_agg("max", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def std(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
            progress=None, edges=False, array_type=None):
        return self._compute_agg("std", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def var(self, expression, binby=[], limits=None, shape=default_shape, selection=False, delay=False,
            progress=None, edges=False, array_type=None):
        return self._compute_agg("var", expression, binby, limits, shape, selection, delay, edges, progress,
                                 array_type=array_type)

    def first(self, expression, order_expression, binby=[], limits=None, shape=default_shape, selection=False,
              delay=False, edges=False, progress=None, array_type=None):
        return self._compute_agg("first", expression, binby, limits, shape, selection, delay, edges, progress,
                                 extra_expressions=[order_expression], array_type=array_type)

    def _agg(self, aggregator, binners=(), delay=False, progress=None):
        """dataframe.py:5232-5249."""
        tasks, result = aggregator.add_tasks(self, binners)
        return self._delay(delay, result)

    def _set(self, expression, progress=False, selection=None, flatten=True, delay=False, unique_limit=None,
             return_inverse=False):
        """dataframe.py:474-480: the GPU ordered set of an expression's values."""
        task = self.executor.schedule(TaskSetCreate(self, str(expression), unique_limit=unique_limit,
                                                    selection=selection))
        return self._delay(delay, task)

    # ---- groupby -----------------------------------------------------------------
    def groupby(self, by=None, agg=None, sort=False, assume_sparse="auto", row_limit=None, copy=True,
                progress=None, delay=False, _speculate=True):
        """dataframe.py:6622-6683."""
        from .groupby import DenseRangeMiss, GroupBy, GroupByDeferred, _dense_range, groupby_multikey, parse_actions
        if agg is None:  # df.groupby(by).agg(...): the same routes as groupby(by, agg=...)
            return GroupByDeferred(self, by, sort=sort, assume_sparse=assume_sparse, row_limit=row_limit)
        dense_ranges = {}
        multikey = isinstance(by, (list, tuple)) and len(by) > 1
        if multikey:
            # assume_sparse is the reference's combine flag (dataframe.py:6679 ->
            # GroupBy(combine=assume_sparse), groupby.py:313-333): True combines the keys into
            # one grouper, 'auto' when rows / cells < 10, False bins the cartesian grid
            combine = True if assume_sparse is True else (False if assume_sparse is False else "auto")
            res = groupby_multikey(self, by, agg, sort=sort, row_limit=row_limit, combine=combine)
            if res is not None:
                return res
        if agg is not None and assume_sparse != True:  # noqa: E712
            # A single integer key: a dense value range bins like a categorical (min/max
            # pass + BinnerOrdinal grid, GrouperDense); otherwise count/sum/mean run as one
            # hash-partitioned pass (hashagg.py).
            from .hashagg import eligible_key, try_groupby
            # a filtered frame takes the dense route too (its groups: the occupied cells of the
            # filtered counts); the fused hash pass has no filter
            key = eligible_key(self, by, allow_filtered=True)
            if key is not None:
                rng = _dense_range(self, key, speculative=_speculate)
                if rng is not None:
                    dense_ranges[key] = rng
                elif not self.filtered:
                    res = try_groupby(self, by, agg, lambda a, g: parse_actions(self, a, g), sort=sort,
                                      row_limit=row_limit)
                    if res is not None:
                        return res
        if agg is not None and assume_sparse == True and not multikey:  # noqa: E712
            # the ordered_set grouper's result (groups in first-appearance order, or sorted).
            # count / sum / mean of an integer key: one hash-partitioned pass, the groups
            # ordered by the row their key first appears at (hashagg.order_first); other
            # aggregators over a dense key range: the BinnerOrdinal grid (tile path), then the
            # same ordering (vh_dense_first_order)
            from .groupby import first_appearance_order
            from .hashagg import eligible_key, try_groupby
            res = try_groupby(self, by, agg, lambda a, g: parse_actions(self, a, g), sort=sort, row_limit=row_limit,
                              first_order=not sort)
            if res is not None:
                return res
            key = eligible_key(self, by)
            if key is not None and getattr(self.executor, "world", 1) == 1:
                rng = _dense_range(self, key, speculative=_speculate)
                if rng is not None:
                    try:
                        gb = GroupBy(self, by=by, sort=sort, row_limit=row_limit, dense_ranges={key: rng}, first_order=not sort)
                        res = gb.agg(agg)
                    except DenseRangeMiss:
                        return self.groupby(by, agg=agg, sort=sort, assume_sparse=assume_sparse, row_limit=row_limit,
                                            _speculate=False)
                    return res if sort or gb.device_finish else first_appearance_order(self, key, res)
        groupby = GroupBy(self, by=by, sort=sort, row_limit=row_limit,
                          dense=assume_sparse != True or multikey,  # noqa: E712
                          dense_ranges=dense_ranges)
        try:
            return groupby.agg(agg)
        except DenseRangeMiss:
            # the sampled key range missed rows: the exact min / max pass decides the route
            dense_ranges.clear()
            return self.groupby(by, agg=agg, sort=sort, assume_sparse=assume_sparse, row_limit=row_limit,
                                _speculate=False)

    def export_hdf5(self, path, **kwargs):
        """dataframe.py export_hdf5: numeric columns (host or HBM) as vaex's HDF5 layout
        version 2, contiguous and 4 KiB aligned so the file maps back without copies."""
        from .hdf5 import export_hdf5
        export_hdf5(self, path)

    def export_arrow(self, path, **kwargs):
        import pyarrow as pa
        cols = {}
        for name in self.get_column_names():
            v = self.columns.get(name)
            v = v.to_numpy() if isinstance(v, DeviceArray) else np.asarray(self.evaluate(name) if v is None else v)
            cols[name] = pa.array(v)
        with pa.OSFile(str(path), "wb") as sink:
            table = pa.table(cols)
            with pa.ipc.new_file(sink, table.schema) as w:
                w.write_table(table)

    def binby(self, by=None, agg=None, sort=False, copy=True, delay=False, progress=None):
        from .groupby import BinBy
        binby = BinBy(self, by=by, sort=sort)
        if agg is None:
            return binby
        return binby.agg(agg)

    # ---- small conveniences used by tests ----------------------------------------
    def to_dict(self):
        out = {}
        for k, v in self.columns.items():
            out[k] = v.to_numpy() if isinstance(v, DeviceArray) else np.asarray(v)
        return out

    def sort(self, by, ascending=True):
        key = self.evaluate(by)
        key = key.to_numpy() if isinstance(key, DeviceArray) else np.asarray(key)
        order = np.argsort(key, kind="stable")
        if not ascending:
            order = order[::-1]
        cols = {}
        for k, v in self.columns.items():
            v = v.to_numpy() if isinstance(v, DeviceArray) else v
            cols[k] = v[order]
        return DataFrame(cols, executor=self.executor)

    def __repr__(self):
        return f"DataFrame({self._length} rows, columns={self.get_column_names()})"


def from_arrays(**arrays):
    """vaex.from_arrays: numpy arrays (host) or DeviceArray (HBM-resident) columns."""
    cols = {}
    for k, v in arrays.items():
        if isinstance(v, DeviceArray) or np.ma.isMaskedArray(v):
            cols[k] = v
        else:
            cols[k] = np.asarray(v)
    return DataFrame(cols)


def from_dict(d):
    return from_arrays(**d)
