"""CPU tests of the operator facades (flink_amd.operators / assigners) driven per record, with the
oracle standing in for the engine (engine_factory) -- checks the host-side batching/ordering logic."""
import pytest

from flink_amd import _abi as A
from flink_amd.assigners import (EventTimeSessionWindows, SliceAssigners, SlidingEventTimeWindows,
                                 TumblingEventTimeWindows)
from flink_amd.operators import SlicingWindowProcessor, WindowOperator
from helpers import load_kats
from oracle.oracle import Oracle

KATS = {c["name"].split(" ")[0]: c for c in load_kats()["operators"]}


def test_assigner_argument_checks():
    with pytest.raises(ValueError):
        TumblingEventTimeWindows.of(1000, 1000)
    with pytest.raises(ValueError):
        SlidingEventTimeWindows.of(1000, 100, 100)
    with pytest.raises(ValueError):
        SliceAssigners.hopping(1000, 300)
    with pytest.raises(ValueError):
        SliceAssigners.cumulative(1000, 300)
    with pytest.raises(ValueError):
        EventTimeSessionWindows.with_gap(0)
    assert SlidingEventTimeWindows.of(5000, 2000).slice_ms == 1000
    assert SliceAssigners.cumulative(3000, 1000).slice_ms == 1000


@pytest.mark.parametrize("batch", [1, 3, 1 << 20])
def test_window_operator_facade_tumbling_kat(batch):
    case = KATS["WindowOperatorTest.testTumblingEventTimeWindowsReduce"]
    op = WindowOperator(TumblingEventTimeWindows.of(3000), [("SUM_I64", 0)], batch_size=batch,
                        engine_factory=Oracle)
    for ev in case["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], [ev[2]], ev[3])
        else:
            got = sorted((r[0], r[1], r[2], r[3][0]) for r, ts in op.process_watermark(ev[1]))
            assert got == sorted(tuple(x) for x in ev[2])
    op.close()


TABLE_SPECS = {"SLIDE": lambda: SliceAssigners.hopping(3000, 1000), "CUMULATE": lambda: SliceAssigners.cumulative(3000, 1000),
               "TUMBLE": lambda: SliceAssigners.tumbling(3000)}


@pytest.mark.parametrize("kind", ["SLIDE", "CUMULATE", "TUMBLE"])
def test_slicing_processor_facade_kats(kind):
    """SlicingWindowAggOperatorTest sequences through the facade: rows per watermark, and processElement returns true
    exactly for the records the reference drops (SlicingWindowOperator.java:222-226 lateRecordsDroppedRate)."""
    name = {"SLIDE": "Hopping", "CUMULATE": "Cumulative", "TUMBLE": "Tumbling"}[kind]
    case = KATS["SlicingWindowAggOperatorTest.testEventTime%sWindows" % name]
    proc = SlicingWindowProcessor(TABLE_SPECS[kind](), [("SUM_I64", 0), ("COUNT", 0)], batch_size=2,
                                  engine_factory=Oracle).open()
    flagged = []
    for ev in case["events"]:
        if ev[0] == "e":
            if proc.process_element(ev[1], [ev[2]], ev[3]):
                flagged.append((ev[1], ev[3]))
        else:
            got = sorted(proc.advance_progress(ev[1]))
            exp = sorted((k, s, c, ws, we) for k, ws, we, s, c in ev[2])
            assert got == exp
    proc.prepare_checkpoint()
    assert proc.num_late_records_dropped == case["late_dropped"] == len(flagged)
    assert sorted(flagged) == sorted((k, ts) for k, _, ts in proc.late_records)
    proc.close()


def test_window_fired_and_slice_helpers():
    """TimeWindowUtil.isWindowFired / SliceAssigners geometry restated for the facade (UTC and a shift zone)."""
    from flink_amd.assigners import is_window_fired, to_epoch_mills_for_timer, window_start_with_offset
    assert window_start_with_offset(-1, 0, 1000) == -1000 and window_start_with_offset(1999, 300, 1000) == 1300
    hop = SliceAssigners.hopping(3000, 1000)
    assert hop.assign_slice_end(2999) == 3000 and hop.last_window_end(3000) == 5000
    cum = SliceAssigners.cumulative(3000, 1000)
    assert cum.assign_slice_end(4500) == 5000 and cum.last_window_end(5000) == 6000
    assert not is_window_fired(3000, 2998) and is_window_fired(3000, 2999) and not is_window_fired(A.LONG_MAX, A.LONG_MAX)
    shanghai = [(-2**63, 8 * 3600_000)]                # fixed +08:00
    assert to_epoch_mills_for_timer(10 * 3600_000, shanghai) == 2 * 3600_000


def test_window_operator_side_output_of_late_records():
    """lateDataOutputTag set: the late record goes to the side output, not to numLateRecordsDropped
    (WindowOperatorTest.testSideOutputDueToLatenessTumbling, WindowOperator.java:425-433)."""
    case = KATS["WindowOperatorTest.testSideOutputDueToLatenessTumbling"]
    op = WindowOperator(TumblingEventTimeWindows.of(case["size_ms"]), [("SUM_I64", 0)], batch_size=1,
                        engine_factory=Oracle, late_data_output=True)
    late = []
    for ev in case["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], [ev[2]], ev[3])
        else:
            op.process_watermark(ev[1])
    assert op.num_late_records_dropped == 0
    assert len(op.late_records) == case["late_dropped"] > 0
    op.close()


def test_slicing_processor_lists_dropped_records():
    case = KATS["SlicingWindowAggOperatorTest.testEventTimeHoppingWindows"]
    proc = SlicingWindowProcessor(SliceAssigners.hopping(3000, 1000), [("SUM_I64", 0), ("COUNT", 0)],
                                  batch_size=1, engine_factory=Oracle).open()
    for ev in case["events"]:
        if ev[0] == "e":
            proc.process_element(ev[1], [ev[2]], ev[3])
        else:
            proc.advance_progress(ev[1])
    assert [(k, ts) for k, _, ts in proc.late_records] == [(1, 2999)]   # "late for all assigned windows"
    proc.close()


def test_timer_and_local_time_against_reference_kats():
    """The facade's toEpochMillsForTimer / toUtcTimestampMills restatement against TimeWindowUtilTest's cases
    (Asia/Shanghai, America/Los_Angeles DST), and the slice assigners against the *SliceAssignerTest cases."""
    from flink_amd.assigners import to_epoch_mills_for_timer, to_utc_timestamp_mills
    from helpers import load_tz_kats
    tzk = load_tz_kats()
    n = 0
    for c in tzk["timer"]:
        tz = [tuple(p) for p in c["tz"]]
        for local, inst in c["timer"]:
            assert to_epoch_mills_for_timer(local, tz) == inst, (c["zone"], local)
            n += 1
        for inst, local in c.get("to_local", []):
            assert to_utc_timestamp_mills(inst, tz) == local, (c["zone"], inst)
    for c in tzk["slice_ends"]:
        tz = [tuple(p) for p in c["tz"]]
        spec = {"TUMBLE": lambda: SliceAssigners.tumbling(c["size"], c["offset"]),
                "SLIDE": lambda: SliceAssigners.hopping(c["size"], c["slide"], c["offset"]),
                "CUMULATE": lambda: SliceAssigners.cumulative(c["size"], c["slide"], c["offset"])}[c["kind"]]()
        for ts, end in c["cases"]:
            assert spec.assign_slice_end(to_utc_timestamp_mills(ts, tz)) == end, (c["src"], ts)
            n += 1
    assert n > 20


@pytest.mark.parametrize("kind", ["SLIDE", "CUMULATE", "TUMBLE"])
def test_slicing_processor_late_flags_shanghai(kind):
    """The Asia/Shanghai parameterisation of SlicingWindowAggOperatorTest through the facade (oracle engine): rows and
    the per-record late flag under a shift time zone."""
    from helpers import load_tz_kats
    case = [c for c in load_tz_kats()["operators"] if c["window_kind"] == kind and c["semantics"] == "TABLE"][0]
    tz = [tuple(p) for p in case["tz"]]
    proc = SlicingWindowProcessor(TABLE_SPECS[kind](), [("SUM_I64", 0), ("COUNT", 0)], batch_size=3,
                                  engine_factory=Oracle, tz=tz).open()
    flagged = 0
    for ev in case["events"]:
        if ev[0] == "e":
            flagged += bool(proc.process_element(ev[1], [ev[2]], ev[3]))
        else:
            got = sorted(proc.advance_progress(ev[1]))
            assert got == sorted((k, s, c, ws, we) for k, ws, we, s, c in ev[2])
    proc.prepare_checkpoint()
    assert flagged == proc.num_late_records_dropped == case["late_dropped"]
    proc.close()


@pytest.mark.parametrize("name", ["WindowOperatorTest.testTumblingEventTimeWindowsReduce",
                                  "WindowOperatorTest.testSlidingEventTimeWindowsReduce"])
def test_reduce_facade_on_sum_reducer_kats(name):
    """WindowOperatorTest's SumReducer sequences (Tuple2<String, Integer>, WindowedStream.sum(1) semantics) through the
    DataStream reduction facade (flink_amd.operators.ReduceWindowOperator) over the oracle."""
    from flink_amd.operators import ReduceWindowOperator
    case = KATS[name]
    spec = (TumblingEventTimeWindows.of(case["size_ms"], case["offset_ms"]) if case["window_kind"] == "TUMBLE" else
            SlidingEventTimeWindows.of(case["size_ms"], case["slide_ms"], case["offset_ms"]))
    op = ReduceWindowOperator(spec, "sum", 1, ["I32"], batch_size=3, engine_factory=Oracle)
    for ev in case["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], [ev[2]], ev[3])
        else:
            got = sorted((r[0], r[1], r[2], r[3][0]) for r, ts in op.process_watermark(ev[1]))
            assert got == sorted(tuple(x) for x in ev[2])
    op.close()


def test_reduction_aggs_of_windowed_stream_calls():
    from flink_amd.operators import reduction_aggs
    assert reduction_aggs("sum", 2, ["I64", "F64", "F32"]) == [("FIRST_64", 0), ("SUM_F64", 1), ("FIRST_32", 2)]
    assert reduction_aggs("min_by", 3, ["I64", "F64", "F32"]) == [("SEL_64", 0), ("SEL_64", 1), ("MINBY_F32", 2)]
