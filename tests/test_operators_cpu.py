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


def test_slicing_processor_facade_hopping_kat():
    case = KATS["SlicingWindowAggOperatorTest.testEventTimeHoppingWindows"]
    proc = SlicingWindowProcessor(SliceAssigners.hopping(3000, 1000), [("SUM_I64", 0), ("COUNT", 0)],
                                  batch_size=2, engine_factory=Oracle).open()
    for ev in case["events"]:
        if ev[0] == "e":
            assert proc.process_element(ev[1], [ev[2]], ev[3]) is False
        else:
            got = sorted(proc.advance_progress(ev[1]))
            exp = sorted((k, s, c, ws, we) for k, ws, we, s, c in ev[2])
            assert got == exp
    assert proc.num_late_records_dropped == case["late_dropped"]
    proc.prepare_checkpoint()
    proc.close()


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
