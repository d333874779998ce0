"""``ExecutorLocal`` for the GPU (the role of ``packages/vaex-core/vaex/execution.py:132-377``).

Same contract -- tasks are scheduled, aggregation tasks sharing binners are merged into
one ``TaskAggregations`` (one pass, ``execution.py:47-73``), the DataFrame's rows are
walked in chunks, every task part processes each chunk, parts are reduced and results
fulfilled -- but the chunk loop feeds the HIP library instead of a CPU thread pool:

* HBM-resident columns (:class:`DeviceArray`) are handed over whole (one chunk): the
  library reads them in place;
* numpy columns are handed over in host chunks (default 16 Mi rows, ``VAEX_CHUNK_SIZE``
  overrides, as ``execution.py:20-24``); the library stages each to HBM.

One task part per task: the per-thread private grids of ``ideal_splits`` exist on the CPU
to avoid write races, which device atomics already resolve.
"""
import os
import threading

import numpy as np

from .device import DeviceArray
from .tasks import TaskAggregation, TaskAggregations, TaskMinMax, TaskSetCreate
from .taskparts import TaskPartAggregation, TaskPartMinMax, TaskPartSetCreate

# rows per task pass over host (memory-mapped / numpy) columns: each pass is one bin() call,
# inside which the library double-buffers 16 Mi-row pipe chunks (copy of chunk i+1 under the
# kernels of chunk i); a pass of 16 pipe chunks leaves only its first copy exposed
CHUNK_SIZE_HOST = int(os.environ.get("VAEX_AMD_CHUNK_SIZE", 256 * 1024 * 1024))


def _env_chunk_size():
    v = os.environ.get("VAEX_CHUNK_SIZE")
    return int(v) if v not in (None, "None", "") else None


def _merge(tasks, df):
    """execution.py:47-73: aggregation tasks with equal binners -> one TaskAggregations."""
    non_mergable = [t for t in tasks if not isinstance(t, TaskAggregation)]
    per_grid = {}
    for t in tasks:
        if isinstance(t, TaskAggregation):
            per_grid.setdefault(t.binners, []).append(t)
    merged = []
    for binners, subtasks in per_grid.items():
        tm = TaskAggregations(df, binners)
        tm.original_tasks = subtasks
        for i, sub in enumerate(subtasks):
            tm.add_aggregation_operation(sub.aggregation_description)

            def assign(value, i=i, sub=sub):
                sub.fulfill(value[i])

            def fail(error, sub=sub):
                sub.reject(error)

            tm.then(assign, fail)
        merged.append(tm)
    return non_mergable + merged


class ExecutorLocal:
    def __init__(self, chunk_size=None):
        self.tasks = []
        self.chunk_size = chunk_size
        self.passes = 0
        self.local = threading.local()
        self.lock = threading.Lock()
        # passes run one at a time: a thread whose task another thread's pass took waits
        # here until that pass has fulfilled it (execution_test.py:79-101); the library
        # itself is safe for concurrent callers (per-grid / per-set locks), but one device
        # stream serialises the work anyway
        self.run_lock = threading.Lock()

    def schedule(self, task):
        with self.lock:
            self.tasks.append(task)
        return task

    def _pop_tasks(self):
        with self.lock:
            tasks, self.tasks = self.tasks, []
        return tasks

    def chunk_size_for(self, df):
        cs = self.chunk_size or _env_chunk_size()
        if cs is not None:
            return int(cs)
        if df.is_device_resident():
            return max(1, df.length_unfiltered())
        return CHUNK_SIZE_HOST

    def row_range(self, df):
        """Rows this executor processes (all of them; a distributed executor its shard)."""
        return 0, df.length_unfiltered()

    def combine_parts(self, parts):
        """Hook after the parts are reduced (a distributed executor combines across ranks)."""

    def _create_part(self, task, df):
        if isinstance(task, TaskAggregations):
            return TaskPartAggregation(df, task.binners, task.aggregation_descriptions)
        if isinstance(task, TaskSetCreate):
            return TaskPartSetCreate(df, task.expression, df.data_type(task.expression), task.unique_limit,
                                     task.selection)
        if isinstance(task, TaskMinMax):
            return TaskPartMinMax(df, task.expression, task.selection)
        raise TypeError(f"unknown task {task!r}")

    def execute(self):
        if getattr(self.local, "executing", False):
            raise RuntimeError("nested execute call")
        self.local.executing = True
        try:
            with self.run_lock:
                while True:
                    tasks = self._pop_tasks()
                    if not tasks:
                        break
                    per_df = {}
                    for t in tasks:
                        per_df.setdefault(id(t.df), (t.df, []))[1].append(t)
                    for df, df_tasks in per_df.values():
                        self._run(df, _merge(df_tasks, df))
        finally:
            self.local.executing = False

    def _run(self, df, tasks):
        self.passes += 1
        parts = []
        try:
            for t in tasks:
                parts.append(self._create_part(t, df))
        except Exception as e:
            for t in tasks:
                t.reject(e)
            raise
        expressions = []
        for p in parts:
            for e in p.expressions:
                if e not in expressions:
                    expressions.append(e)
        start, end = self.row_range(df)
        chunk_size = self.chunk_size_for(df)
        try:
            for i1 in range(start, end, chunk_size):
                i2 = min(end, i1 + chunk_size)
                filter_mask = df.evaluate_filter_mask(i1, i2) if df.filtered else None
                blocks = {e: df.evaluate_chunk(e, i1, i2, filter_mask) for e in expressions}
                for p in parts:
                    p.process(0, i1, i2, filter_mask, blocks)
            for p in parts:
                p.reduce([])
            self.combine_parts(parts)
            for t, p in zip(tasks, parts):
                t.fulfill(p.get_result())
        except Exception as e:
            for t in tasks:
                t.reject(e)
            raise


default_executor = ExecutorLocal()
