"""``vaex.agg`` aggregator descriptors (``packages/vaex-core/vaex/agg.py``).

Same registry (``aggregates``), descriptor classes and argument meaning:
``count``, ``sum``, ``mean``, ``min``, ``max``, ``first``, ``std``, ``var``,
``_sum_moment``.  ``_create_operation`` looks up the HIP-backed class in
:mod:`vaex_amd.superagg` by name + dtype exactly as the reference does
(``agg.py:111-114``).
"""
import numpy as np

from . import superagg
from .utils import extract_central_part, find_type_from_dtype

aggregates = {}

# upcast<T> (superagg.cpp:289-346) on numpy dtypes
def _upcast(dtype):
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return np.dtype("float64")
    if dt.kind in "ib":
        return np.dtype("int64")
    if dt.kind == "u":
        return np.dtype("uint64")
    if dt.kind in "mM":
        return dt
    return dt


def register(f, name=None):
    aggregates[name or f.__name__] = f
    return f


class AggregatorDescriptor:
    def __repr__(self):
        return "vaex.agg.{}({!r})".format(self.short_name, str(self.expression))

    def pretty_name(self, id, df):
        if id is None:
            id = "_".join(map(str, self.expressions))
        return "{0}_{1}".format(id, self.short_name)

    def finish(self, value):
        return value


class AggregatorDescriptorBasic(AggregatorDescriptor):
    """agg.py:58-120."""

    def __init__(self, name, expression, short_name, multi_args=False, agg_args=[], selection=None, edges=False):
        self.name = name
        self.short_name = short_name
        self.expression = str(expression) if not multi_args else expression
        self.agg_args = agg_args
        self.edges = edges
        self.selection = selection
        if not multi_args:
            self.expressions = [] if self.expression == "*" else [self.expression]
        else:
            self.expressions = [str(e) for e in expression]

    def encode(self):
        spec = {"aggregation": self.short_name}
        if len(self.expressions) == 1:
            spec["expression"] = self.expressions[0]
        elif self.expressions:
            spec["expression"] = list(self.expressions)
        if self.selection is not None:
            spec["selection"] = str(self.selection)
        if self.edges:
            spec["edges"] = True
        if self.agg_args:
            spec["parameters"] = self.agg_args
        return spec

    def _prepare_types(self, df):
        """agg.py:90-100."""
        if self.expression == "*":
            self.dtype_in = np.dtype("int64")
            self.dtype_out = np.dtype("int64")
        else:
            self.dtype_in = df.data_type(self.expressions[0])
            self.dtype_out = self.dtype_in
            if self.short_name == "count":
                self.dtype_out = np.dtype("int64")
            if self.short_name in ["sum", "summoment", "_sum_moment"]:
                self.dtype_out = _upcast(self.dtype_in)

    def add_tasks(self, df, binners):
        from .tasks import TaskAggregation
        from .promise import delayed
        self._prepare_types(df)
        task = TaskAggregation(df, binners, self)
        task = df.executor.schedule(task)

        @delayed
        def finish(value):
            return self.finish(value)
        return [task], finish(task)

    def _create_operation(self, grid):
        """agg.py:111-114."""
        agg_op_type = find_type_from_dtype(superagg, self.name + "_", self.dtype_in)
        return agg_op_type(grid, *self.agg_args)

    def get_result(self, agg_operation):
        """agg.py:116-120.  ``want_occupancy`` (set by a dense groupby on its count(*)): the
        occupied range of the 1-d grid's central part is found on the device first."""
        if getattr(self, "want_occupancy", False) and agg_operation.grid.dimensions == 1:
            self.occupancy = agg_operation.occupancy(2, agg_operation.grid.length1d - 1)
        grid = np.asarray(agg_operation)
        if not self.edges:
            grid = extract_central_part(grid)
        return grid


class AggregatorDescriptorNUnique(AggregatorDescriptorBasic):
    """agg.py:123-144: AggNUnique_<t>(grid, dropmissing, dropnan), int64 output."""

    def __init__(self, name, expression, short_name, dropmissing, dropnan, selection=None, edges=False):
        super().__init__(name, expression, short_name, selection=selection, edges=edges)
        self.dropmissing = dropmissing
        self.dropnan = dropnan

    def encode(self):
        spec = super().encode()
        if self.dropmissing:
            spec["dropmissing"] = self.dropmissing
        if self.dropnan:
            spec["dropnan"] = self.dropnan
        return spec

    def _prepare_types(self, df):
        super()._prepare_types(df)
        self.dtype_out = np.dtype("int64")

    def _create_operation(self, grid):
        agg_op_type = find_type_from_dtype(superagg, self.name + "_", self.dtype_in)
        return agg_op_type(grid, self.dropmissing, self.dropnan)


class AggregatorDescriptorMulti(AggregatorDescriptor):
    def __init__(self, name, expression, short_name, selection=None, edges=False):
        self.name = name
        self.short_name = short_name
        self.expression = str(expression)
        self.expressions = [self.expression]
        self.selection = selection
        self.edges = edges


class AggregatorDescriptorMean(AggregatorDescriptorMulti):
    """agg.py:158-188: sum + count(expr) on the same binners (one merged pass); empty cells -> nan."""

    def __init__(self, name, expression, short_name="mean", selection=None, edges=False):
        super().__init__(name, expression, short_name, selection=selection, edges=edges)

    def add_tasks(self, df, binners):
        from . import hostops
        from .promise import delayed
        sum_agg = sum(self.expression, selection=self.selection, edges=self.edges)
        count_agg = count(self.expression, selection=self.selection, edges=self.edges)
        task_sum = sum_agg.add_tasks(df, binners)[0][0]
        task_count = count_agg.add_tasks(df, binners)[0][0]
        self.dtype_in = sum_agg.dtype_in
        self.dtype_out = sum_agg.dtype_out

        @delayed
        def finish(sum, count):
            sum = np.asarray(sum)  # a view of the grid's host image: the division makes the result
            dtype = sum.dtype
            sum_kind = sum.dtype.kind
            if sum_kind == "M":
                sum = sum.view("uint64")
                count = count.view("uint64")
            mean = hostops.true_divide(sum, count)  # sum / count, divide / invalid ignored
            if dtype.kind != mean.dtype.kind and sum_kind == "M":
                mean = mean.astype(dtype)
            return mean

        return [task_sum, task_count], finish(task_sum, task_count)


class AggregatorDescriptorVar(AggregatorDescriptorMulti):
    """agg.py:191-224: sum of squares, sum and count (float64)."""

    def __init__(self, name, expression, short_name="var", ddof=0, selection=None, edges=False):
        super().__init__(name, expression, short_name, selection=selection, edges=edges)
        self.ddof = ddof

    def add_tasks(self, df, binners):
        from .promise import delayed
        # agg.py:196-201: the moments are taken of the expression cast to float64, so
        # integer squares neither wrap nor accumulate in an int64 grid (a float64 column
        # is its own cast: the same values, no extra device pass)
        expression = str(self.expression)
        if df.data_type(expression) != np.dtype("float64"):
            expression = str(df[expression].astype("float64"))
        sum_moment = _sum_moment(expression, 2, selection=self.selection, edges=self.edges)
        sum_ = sum(expression, selection=self.selection, edges=self.edges)
        count_ = count(expression, selection=self.selection, edges=self.edges)
        task_sum_moment = sum_moment.add_tasks(df, binners)[0][0]
        task_sum = sum_.add_tasks(df, binners)[0][0]
        task_count = count_.add_tasks(df, binners)[0][0]
        self.dtype_in = sum_.dtype_in
        self.dtype_out = sum_.dtype_out

        @delayed
        def finish(sum_moment, sum, count):
            # sum_moment / count - (sum / count) ** 2 element-wise over host threads (the
            # reference's numpy expression, agg.py:207-213, bit for bit)
            from . import hostops
            return self.finish(hostops.variance(sum_moment, sum, count))

        return [task_sum_moment, task_sum, task_count], finish(task_sum_moment, task_sum, task_count)


class AggregatorDescriptorStd(AggregatorDescriptorVar):
    def finish(self, value):
        return value ** 0.5


@register
def count(expression="*", selection=None, edges=False):
    """Creates a count aggregation"""
    return AggregatorDescriptorBasic("AggCount", expression, "count", selection=selection, edges=edges)


@register
def sum(expression, selection=None, edges=False):
    """Creates a sum aggregation"""
    return AggregatorDescriptorBasic("AggSum", expression, "sum", selection=selection, edges=edges)


@register
def mean(expression, selection=None, edges=False):
    """Creates a mean aggregation"""
    return AggregatorDescriptorMean("mean", expression, "mean", selection=selection, edges=edges)


@register
def min(expression, selection=None, edges=False):
    """Creates a min aggregation"""
    return AggregatorDescriptorBasic("AggMin", expression, "min", selection=selection, edges=edges)


@register
def max(expression, selection=None, edges=False):
    """Creates a max aggregation"""
    return AggregatorDescriptorBasic("AggMax", expression, "max", selection=selection, edges=edges)


@register
def _sum_moment(expression, moment, selection=None, edges=False):
    """Creates a sum of moment aggregator"""
    return AggregatorDescriptorBasic("AggSumMoment", expression, "_sum_moment", agg_args=[moment],
                                     selection=selection, edges=edges)


@register
def first(expression, order_expression, selection=None, edges=False):
    """Creates a first aggregation (value of the row with the lowest order_expression)"""
    return AggregatorDescriptorBasic("AggFirst", [expression, order_expression], "first", multi_args=True,
                                     selection=selection, edges=edges)


@register
def std(expression, ddof=0, selection=None, edges=False):
    """Creates a standard deviation aggregation"""
    return AggregatorDescriptorStd("std", expression, "std", ddof=ddof, selection=selection, edges=edges)


@register
def var(expression, ddof=0, selection=None, edges=False):
    """Creates a variance aggregation"""
    return AggregatorDescriptorVar("var", expression, "var", ddof=ddof, selection=selection, edges=edges)


@register
def nunique(expression, dropna=False, dropnan=False, dropmissing=False, selection=None, edges=False):
    """Aggregator that calculates the number of unique items per bin (agg.py:277-288).

    :param dropmissing: do not count missing values
    :param dropnan: do not count nan values
    :param dropna: short for both"""
    if dropna:
        dropnan = True
        dropmissing = True
    return AggregatorDescriptorNUnique("AggNUnique", expression, "nunique", dropmissing, dropnan,
                                       selection=selection, edges=edges)
