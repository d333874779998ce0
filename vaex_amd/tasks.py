"""Task shapes of the binning path (``packages/vaex-core/vaex/tasks.py``).

``TaskAggregation`` / ``TaskAggregations`` (tasks.py:331-428), ``TaskSetCreate``
(tasks.py:98-118) and the min/max limits task (``TaskStatistic`` with ``OP_MIN_MAX``,
tasks.py:149-328).  Tasks are promises fulfilled by :class:`~vaex_amd.execution.ExecutorLocal`.
"""
from .promise import Promise


class Task(Promise):
    see_all = False
    cacheable = False

    def __init__(self, df, expressions, pre_filter=False):
        super().__init__()
        self.df = df
        self.expressions = list(expressions)
        self.pre_filter = pre_filter
        self.cancelled = False

    @property
    def expressions_all(self):
        return list(self.expressions)


class TaskAggregation(Task):
    """One aggregation descriptor over a tuple of binner specs (tasks.py:394-407)."""

    def __init__(self, df, binners, aggregation_description):
        expressions = [b.expression for b in binners] + list(aggregation_description.expressions)
        super().__init__(df, expressions, pre_filter=df.filtered)
        self.binners = tuple(binners)
        self.aggregation_description = aggregation_description


class TaskAggregations(Task):
    """All aggregations sharing one set of binners: one pass over the data (execution.py:47-73)."""

    def __init__(self, df, binners):
        super().__init__(df, [b.expression for b in binners], pre_filter=df.filtered)
        self.binners = tuple(binners)
        self.aggregation_descriptions = []
        self.original_tasks = []

    def add_aggregation_operation(self, descriptor):
        self.aggregation_descriptions.append(descriptor)
        for e in descriptor.expressions:
            if e not in self.expressions:
                self.expressions.append(e)


class TaskSetCreate(Task):
    """Build the ordered set of an expression's values (tasks.py:98-118); see_all: one part."""

    see_all = True

    def __init__(self, df, expression, unique_limit=None, selection=None):
        super().__init__(df, [expression], pre_filter=df.filtered)
        self.expression = expression
        self.unique_limit = unique_limit
        self.selection = selection


class TaskMinMax(Task):
    """NaN-ignoring (min, max) of one expression (OP_MIN_MAX, tasks.py:173-185)."""

    see_all = True

    def __init__(self, df, expression, selection=None):
        super().__init__(df, [expression], pre_filter=df.filtered)
        self.expression = expression
        self.selection = selection
