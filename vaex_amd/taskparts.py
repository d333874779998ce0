"""Task parts driving the HIP module (the role of ``packages/vaex-core/vaex/cpu.py``).

``TaskPartAggregation`` keeps ``cpu.py:449-639``'s structure -- build
``superagg.Grid([binner.copy()...])`` and one aggregator per (descriptor, selection),
``process`` hands each chunk's buffers to ``set_data``/``set_data_mask`` and calls
``grid.bin(all_aggregators, N)``, then ``reduce`` and ``get_result`` -- but the module it
drives is :mod:`vaex_amd.superagg`, whose grids live in HBM.  On the GPU one part is
enough (device atomics replace the per-thread private grids of ``ideal_splits``).
"""
import re

import numpy as np

from . import superagg
from .device import DeviceArray
from .utils import find_type_from_dtype

_ORDINAL_VALUES = re.compile(r"^_ordinal_values\((.+),\s*([A-Za-z_][A-Za-z0-9_]*)\)$")


def parse_ordinal_values(expression):
    """('key_expression', 'set_variable') of an ``_ordinal_values(key, set)`` binby expression."""
    m = _ORDINAL_VALUES.match(str(expression))
    return (m.group(1).strip(), m.group(2)) if m else None


def _rebase(view, host):
    """``view`` (a view into the 1-d host image ``host``, whatever it is based on) rebuilt as
    an array based on ``host`` alone; None when it does not lie inside ``host``."""
    if not np.may_share_memory(view, host) or view.size == 0 or any(s < 0 for s in view.strides):
        return None
    offset = view.__array_interface__["data"][0] - host.ctypes.data
    extent = sum((n - 1) * s for n, s in zip(view.shape, view.strides)) + view.itemsize
    if offset < 0 or offset + extent > host.nbytes:
        return None
    return np.ndarray(view.shape, view.dtype, buffer=host, offset=offset, strides=view.strides)


def create_binner(df, spec):
    """binner-cpu decode (cpu.py:40-51), plus the fused set-ordinal binner for groupby."""
    if spec.kind == "ordinal":
        parsed = parse_ordinal_values(spec.expression)
        if parsed is not None:
            key_expr, set_name = parsed
            ordered_set = df.variables[set_name]
            b = superagg.BinnerSetOrdinal(spec.expression, ordered_set, spec.count)
            b._data_expression = key_expr
            return b
        cls = find_type_from_dtype(superagg, "BinnerOrdinal_", spec.dtype)
        b = cls(spec.expression, spec.count, spec.minimum)
    else:
        cls = find_type_from_dtype(superagg, "BinnerScalar_", spec.dtype)
        b = cls(spec.expression, spec.minimum, spec.maximum, spec.count)
    b._data_expression = spec.expression
    return b


def _split_masked(block):
    if np.ma.isMaskedArray(block):
        return block.data, np.ma.getmaskarray(block)
    return block, None


def _prepare(block):
    """check_array (cpu.py:505-513): contiguous, datetime/timedelta passed as int64 bits."""
    if isinstance(block, DeviceArray):
        return block
    block = np.asarray(block)
    if not block.flags["C_CONTIGUOUS"]:
        block = block.copy()
    if block.dtype.kind in "mM":
        block = block.view("uint64" if block.dtype.byteorder in "<=|" else block.dtype.newbyteorder("=").str)
    return block


class DeviceResult:
    """An aggregation result left in HBM: the aggregator (its grid, Fortran order with edges).
    ``np.asarray`` reads the grid back like a plain result."""

    def __init__(self, agg):
        self.agg = agg

    def __array__(self, dtype=None, copy=None):
        a = np.asarray(self.agg)
        return a if dtype is None else a.astype(dtype)


class TaskPartAggregation:
    snake_name = "aggregations"

    def __init__(self, df, binners, aggregation_descriptions):
        self.df = df
        self.has_values = False
        self.aggregation_descriptions = aggregation_descriptions
        self._binners = [create_binner(df, b) for b in binners]
        # the expressions this part needs per chunk: binner data, then aggregator data
        self.expressions = [b._data_expression for b in self._binners]
        for desc in aggregation_descriptions:
            for e in desc.expressions:
                if e not in self.expressions:
                    self.expressions.append(e)
        self.grid = superagg.Grid([b.copy() for b in self._binners])
        self.nbytes = 0
        self.aggregations = []
        for desc in aggregation_descriptions:
            selection = desc.selection
            selection_waslist = isinstance(selection, (list, tuple))
            selections = list(selection) if selection_waslist else [selection]
            aggs = []
            for _ in selections:
                agg = desc._create_operation(self.grid)
                self.nbytes += agg.__sizeof__()
                aggs.append(agg)
            self.aggregations.append((desc, selections, aggs, selection_waslist))

    def ideal_splits(self, nthreads):
        return 1

    def process(self, thread_index, i1, i2, filter_mask, blocks):
        """cpu.py:501-583 with ``blocks`` a dict expression -> chunk buffer."""
        N = i2 - i1
        device_filter = isinstance(filter_mask, DeviceArray)  # HBM frame: chunk whole, filter as mask
        if filter_mask is not None and not device_filter:
            N = int(np.sum(filter_mask))
        references = []
        for binner in self.grid.binners:
            block, mask = _split_masked(blocks[binner._data_expression])
            block = _prepare(block)
            binner.set_data(block)
            if mask is not None:
                binner.set_data_mask(mask)
                references.append(mask)
            else:
                binner.clear_data_mask()
            references.append(block)
        all_aggregators = []
        # one mask per selection and chunk: every aggregator of a selection shares it (one
        # evaluation; the tile path runs a mask shared by all aggregators as a row mask)
        sel_masks = {}
        for desc, selections, aggs, _ in self.aggregations:
            for selection_index, selection in enumerate(selections):
                agg = aggs[selection_index]
                all_aggregators.append(agg)
                selection_mask = None
                if not (selection is None or selection is False):
                    skey = selection if isinstance(selection, (str, bool)) else None
                    if skey is not None and skey in sel_masks:
                        selection_mask = sel_masks[skey]
                    else:
                        selection_mask = self.df.evaluate_selection_mask(selection, i1=i1, i2=i2, filter_mask=filter_mask,
                                                                         cache=True)  # cpu.py:548
                        if not isinstance(selection_mask, DeviceArray):
                            selection_mask = np.asarray(selection_mask)
                        if skey is not None:
                            sel_masks[skey] = selection_mask
                elif device_filter:
                    selection_mask = filter_mask
                if selection_mask is not None and hasattr(agg, "set_selection_mask"):
                    # nunique tells rows outside the selection (or an HBM frame's filter)
                    # from missing values (cpu.py:551-554)
                    agg.set_selection_mask(selection_mask)
                for i, expression in enumerate(desc.expressions):
                    block, mask = _split_masked(blocks[expression])
                    block = _prepare(block)
                    if mask is not None:
                        if isinstance(selection_mask, DeviceArray):
                            raise NotImplementedError("masked host columns in a filtered / selected HBM frame")
                        selection_mask = ~mask if selection_mask is None else (selection_mask & ~mask)
                    agg.set_data(block, i)
                    references.append(block)
                if selection_mask is not None:
                    agg.set_data_mask(selection_mask)
                    references.append(selection_mask)
                else:
                    agg.clear_data_mask()
        self.grid.bin(all_aggregators, N)
        self.has_values = True

    def reduce(self, others):
        for agg_index, (desc, selections, aggs, _) in enumerate(self.aggregations):
            for selection_index in range(len(selections)):
                aggs[selection_index].reduce([o.aggregations[agg_index][2][selection_index] for o in others])

    def get_aggregators(self):
        return [agg for _, _, aggs, _ in self.aggregations for agg in aggs]

    def get_result(self):
        """cpu.py:592-605."""
        results = []
        for desc, selections, aggs, selection_waslist in self.aggregations:
            if getattr(desc, "keep_device", False) and len(aggs) == 1 and not selection_waslist:
                # the caller finishes on the device (a dense groupby in first-appearance order):
                # the aggregator itself is the result, its grid still in HBM (no read-back)
                if getattr(desc, "want_occupancy", False) and aggs[0].grid.dimensions == 1:
                    desc.occupancy = aggs[0].occupancy(2, aggs[0].grid.length1d - 1)
                results.append(DeviceResult(aggs[0]))
                continue
            grids = [desc.get_result(agg) for agg in aggs]
            result = np.asarray(grids) if selection_waslist else grids[0]
            dtype_out = np.dtype(desc.dtype_out)
            if dtype_out.kind in "mM" or result.dtype.itemsize == dtype_out.itemsize:
                result = result.view(dtype_out.newbyteorder("=") if dtype_out.byteorder not in "<=|" else dtype_out)
            host = getattr(aggs[0], "_host", None) if len(aggs) == 1 and not selection_waslist else None
            rebased = _rebase(result, host) if host is not None else None
            if rebased is not None:
                # the part is done with its aggregator: hand its (page-locked) host image over
                # (the result may be a strided view of it: the grid's central part) instead of
                # copying it (cpu.py:605 copies because its grids are reused; for an N-d grid
                # that copy is a transpose into C order, ~2 ms per 1e6 cells).  The view is
                # rebuilt over the image itself so it does not keep the aggregator (and the
                # columns it references) alive.
                aggs[0]._release_host()
                results.append(rebased)
            else:
                results.append(result.copy())
        return results


class TaskPartSetCreate:
    """cpu.py:117-237: one part shared by all chunks (see_all), GPU ordered set."""

    def __init__(self, df, expression, dtype, unique_limit=None, selection=None):
        from .superutils import ordered_set_type_from_dtype
        self.df = df
        self.expression = expression
        self.expressions = [expression]
        self.unique_limit = unique_limit
        self.selection = selection
        self.set = ordered_set_type_from_dtype(dtype)()

    def process(self, thread_index, i1, i2, filter_mask, blocks):
        ar = blocks[self.expression]
        if isinstance(ar, DeviceArray):
            # HBM frame: filter & selection as one device mask, the set skips the other rows
            keep = None
            if isinstance(filter_mask, DeviceArray) or self.selection:
                keep = self.df.device_keep_mask(i1, i2, self.selection or None)
            if len(ar):
                if keep is not None:
                    self.set.update(ar, select=keep)
                else:
                    self.set.update(ar)
            self._check_row_limit()
            return
        if self.selection:
            sel = self.df.evaluate_selection_mask(self.selection, i1=i1, i2=i2, filter_mask=filter_mask)
            ar = ar[np.asarray(sel)]
        if len(ar) == 0:
            return
        if isinstance(ar, DeviceArray):
            self.set.update(ar)
        else:
            ar = _prepare(ar) if not np.ma.isMaskedArray(ar) else ar
            self.set.update(ar)
        self._check_row_limit()

    def _check_row_limit(self):
        if self.unique_limit is not None and len(self.set) > self.unique_limit:
            from .dataframe import RowLimitException
            raise RowLimitException(f"Resulting set would have >= {self.unique_limit} unique combinations")

    def reduce(self, others):
        pass

    def get_result(self):
        return self.set


class TaskPartMinMax:
    """The limits pre-pass on the GPU: NaN-ignoring min/max (vaexfast.cpp:1043-1055,
    tasks.py:173-185 reduce with nanmin/nanmax)."""

    def __init__(self, df, expression, selection=None):
        self.df = df
        self.expression = expression
        self.expressions = [expression]
        self.selection = selection
        self.vmin = np.nan
        self.vmax = np.nan

    def process(self, thread_index, i1, i2, filter_mask, blocks):
        from . import _lib
        import ctypes
        block, mask = _split_masked(blocks[self.expression])
        block = _prepare(block)
        code, flip = _lib.dtype_code(block.dtype)
        lo, hi = ctypes.c_double(), ctypes.c_double()
        if isinstance(block, DeviceArray):
            # HBM frame: skip = ~(filter & selection), evaluated on the device
            skip = None
            if isinstance(filter_mask, DeviceArray) or self.selection not in (None, False):
                skip = self.df.device_keep_mask(i1, i2, self.selection if self.selection not in (None, False) else None,
                                                invert=True)
            _lib.call("vh_minmax", block.ptr, len(block), code, flip, None if skip is None else skip.ptr,
                      _lib.LOC_DEVICE, ctypes.byref(lo), ctypes.byref(hi))
        else:
            skip = None
            if mask is not None:
                skip = mask
            if self.selection not in (None, False):
                sel = np.asarray(self.df.evaluate_selection_mask(self.selection, i1=i1, i2=i2, filter_mask=filter_mask))
                skip = ~sel if skip is None else (skip | ~sel)
            skip_arr = None if skip is None else np.ascontiguousarray(skip, dtype=np.uint8)
            _lib.call("vh_minmax", block.ctypes.data, len(block), code, flip,
                      None if skip_arr is None else skip_arr.ctypes.data, _lib.LOC_HOST, ctypes.byref(lo), ctypes.byref(hi))
        self.vmin = np.nanmin([self.vmin, lo.value]) if not np.isnan(lo.value) else self.vmin
        self.vmax = np.nanmax([self.vmax, hi.value]) if not np.isnan(hi.value) else self.vmax

    def reduce(self, others):
        pass

    def get_result(self):
        return np.array([self.vmin, self.vmax])
