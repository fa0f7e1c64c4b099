"""Operator facades mirroring the reference's operator interfaces over the GPU engine.

DataStream  WindowOperator.processElement / processWatermark / close
            flink-streaming-java/.../runtime/operators/windowing/WindowOperator.java:278-481
Table       SlicingWindowProcessor.open/initializeWatermark/processElement/advanceProgress/
            prepareCheckpoint/fireWindow/clearWindow/close
            flink-table-runtime/.../window/slicing/SlicingWindowProcessor.java:33-126

Records are buffered columnar and handed to the engine in batches (the engine's unit of work);
every buffered record is pushed before a watermark is applied, so the observable results equal
per-record processing. Emission order among windows with the same end is
unspecified in the reference too (TimerHeapInternalTimer orders by timestamp only).
"""
import numpy as np

from . import _abi as A
from .assigners import WindowSpec, is_window_fired, to_utc_timestamp_mills


class _Batcher:
    def __init__(self, ncols, batch):
        self.ncols, self.batch = ncols, batch
        self.reset()

    def reset(self):
        self.keys, self.ts = [], []
        self.cols = [[] for _ in range(self.ncols)]

    def __len__(self):
        return len(self.keys)

    def add(self, key, ts, values):
        self.keys.append(key)
        self.ts.append(ts)
        for c, v in zip(self.cols, values):
            c.append(v)

    def arrays(self, dtypes):
        return (np.asarray(self.keys, np.int64), np.asarray(self.ts, np.int64),
                [np.asarray(c, dt) for c, dt in zip(self.cols, dtypes)])


def _col_dtypes(aggs, ncols):
    dts = ["i8"] * ncols
    for name, col in aggs:
        if A.AGG_INPUT_DTYPE[name]:
            dts[col] = A.AGG_INPUT_DTYPE[name]
    return dts


class _Base:
    def __init__(self, spec: WindowSpec, aggs, batch_size=1 << 20, engine_factory=None, track_late=False, **cfg_kw):
        if engine_factory is None:
            from .engine import WindowAggregator
            engine_factory = WindowAggregator
        self.aggs = list(aggs)
        self.ncols = max([c + 1 for n, c in self.aggs if A.AGG_INPUT_DTYPE[n]] + [0])
        self.dtypes = _col_dtypes(self.aggs, self.ncols)
        self.track_late = track_late
        self.cfg = A.make_config(aggs=self.aggs, late_indices=track_late, **spec.config_kwargs(), **cfg_kw)
        self.engine = engine_factory(self.cfg)
        self.buf = _Batcher(self.ncols, batch_size)
        self.num_late_records_dropped = 0
        self.late_records = []                 # (key, values, timestamp) of every record dropped as late
        self.current_watermark = A.LONG_MIN

    def _push(self):
        if len(self.buf):
            k, t, c = self.buf.arrays(self.dtypes)
            n = self.engine.push(k, t, c)
            if self.track_late:                # the batch's dropped records, by index (fwa_late_records)
                for i in self.engine.late_records().tolist():
                    self.late_records.append((self.buf.keys[i], tuple(col[i] for col in self.buf.cols), self.buf.ts[i]))
            self._count_late(n)
            self.buf.reset()

    def _count_late(self, n):
        self.num_late_records_dropped += n

    def _add(self, key, ts, values):
        self.buf.add(key, ts, values)
        if len(self.buf) >= self.buf.batch:
            self._push()

    def _rows(self, res):
        names = A.agg_names(self.cfg)
        out = []
        for i in range(len(res["key"])):
            out.append((int(res["key"][i]), int(res["win_start"][i]), int(res["win_end"][i]),
                        tuple(res["agg%d" % j][i].item() for j in range(len(names)))))
        return out

    def close(self):
        self.engine.close()


class WindowOperator(_Base):
    """DataStream window operator (event time, EventTimeTrigger, AggregateFunction/ReduceFunction
    restricted to the engine's built-in aggregates). Emits (key, window_start, window_end, aggs)
    with record timestamp window.maxTimestamp() = window_end - 1 (WindowOperator.java:552-557)."""

    def __init__(self, assigner: WindowSpec, aggs, allowed_lateness_ms=0, late_data_output=False, **kw):
        """late_data_output: a lateDataOutputTag is set -- late records go to `late_records` (the side output)
        instead of numLateRecordsDropped (WindowOperator.java:425-433)."""
        self.late_data_output = late_data_output
        super().__init__(assigner, aggs, allowed_lateness_ms=allowed_lateness_ms, track_late=late_data_output, **kw)

    def _count_late(self, n):
        if not self.late_data_output:
            self.num_late_records_dropped += n

    def process_element(self, key, value_columns, timestamp):
        self._add(key, timestamp, value_columns)

    def process_watermark(self, wm):
        self._push()
        if wm > self.current_watermark:
            self.current_watermark = wm
        return [(r, r[2] - 1) for r in self._rows(self.engine.advance_watermark(wm))]


_FIELD_DTYPE = {"I32": "i4", "I64": "i8", "F32": "f4", "F64": "f8"}
_REDUCE_PREFIX = {"sum": "SUM_", "min": "MIN_", "max": "MAX_", "min_by": "MINBY_", "max_by": "MAXBY_"}


def reduction_aggs(op, pos, field_types):
    """Aggregate list of WindowedStream.<op>(pos) over a tuple (key, f1, ..., fn) whose fields have the given types
    ("I32" Integer, "I64" Long, "F32" Float, "F64" Double; field i is value column i - 1): field pos is summed /
    folded (SumAggregator / ComparableAggregator, WindowedStream.java:680-890); every other field is the window's first
    element's (FIRST_*), or for min_by / max_by the selected element's (SEL_*)."""
    by = op in ("min_by", "max_by")
    aggs = []
    for f, t in enumerate(field_types, start=1):
        if f == pos:
            aggs.append((_REDUCE_PREFIX[op] + t, f - 1))
        else:
            aggs.append((("SEL_" if by else "FIRST_") + ("32" if t in ("I32", "F32") else "64"), f - 1))
    return aggs


class ReduceWindowOperator(WindowOperator):
    """DataStream window operator of the built-in reductions WindowedStream.sum / min / max / minBy / maxBy(pos)
    (WindowedStream.java:680-890: reduce() with SumAggregator / ComparableAggregator, ReducingState folded in arrival
    order) over tuples (key, f1, ..., fn). first=False is minBy / maxBy(pos, false): ties select the last element.
    Emits ((key, window_start, window_end, (f1, ..., fn)), window.maxTimestamp())."""

    def __init__(self, assigner: WindowSpec, op, pos, field_types, first=True, **kw):
        self.field_types = list(field_types)
        super().__init__(assigner, reduction_aggs(op, pos, self.field_types), reduce=True, by_last=not first, **kw)
        self.dtypes = [_FIELD_DTYPE[t] for t in self.field_types]

    def _rows(self, res):
        cols = []
        for j, t in enumerate(self.field_types):
            a = np.asarray(res["agg%d" % j])
            dt = np.dtype(_FIELD_DTYPE[t])
            cols.append(a.view(dt) if a.dtype.itemsize == dt.itemsize else a.astype(dt))   # FIRST_* / SEL_* bits
        return [(int(res["key"][i]), int(res["win_start"][i]), int(res["win_end"][i]),
                 tuple(c[i].item() for c in cols)) for i in range(len(res["key"]))]


class SlicingWindowProcessor(_Base):
    """Table window-TVF processor: one GPU processor replaces Slice{Shared,Unshared}WindowAggProcessor.
    Output rows are key ++ aggs ++ [window_start, window_end] (AbstractWindowAggProcessor.java:230-233)."""

    def open(self):
        return self

    def initialize_watermark(self, wm):
        self.current_watermark = wm

    def __init__(self, spec, aggs, **kw):
        kw.setdefault("track_late", True)
        self.spec = spec
        self.tz = kw.get("tz")
        super().__init__(spec, aggs, **kw)

    def process_element(self, key, row_values, rowtime):
        """True when the record is dropped as late, which SlicingWindowOperator turns into lateRecordsDroppedRate
        (SlicingWindowOperator.java:222-226): its slice fired and so did the last window containing that slice,
        under the current progress (AbstractWindowAggProcessor.processElement :142-182, TimeWindowUtil.isWindowFired
        :175-183, a shift time zone's local time and timer instants included). The record is buffered either way: the
        engine drops the same records when the batch is pushed (num_late_records_dropped, late_records)."""
        self._add(key, rowtime, row_values)
        if self.current_watermark == A.LONG_MIN:
            return False
        slice_end = self.spec.assign_slice_end(to_utc_timestamp_mills(rowtime, self.tz))
        return (is_window_fired(slice_end, self.current_watermark, self.tz) and
                is_window_fired(self.spec.last_window_end(slice_end), self.current_watermark, self.tz))

    def advance_progress(self, progress):
        self._push()
        if progress <= self.current_watermark:
            return []                                     # SlicingWindowOperator.java:231
        self.current_watermark = progress
        return [(k, *aggs, ws, we) for (k, ws, we, aggs) in self._rows(self.engine.advance_watermark(progress))]

    def prepare_checkpoint(self):
        self._push()
        self.engine.flush()

    def fire_window(self, window_end):
        """No-op: the GPU processor fires every due window inside advance_progress."""

    def clear_window(self, window_end):
        """No-op: slices are released by the engine when their last window fired."""
