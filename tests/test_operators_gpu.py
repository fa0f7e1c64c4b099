"""GPU tests: the operator facades (flink_amd.operators, the host-side mirror of WindowOperator and
SlicingWindowProcessor) driven record by record over the HIP engine on the reference's operator KATs
(WindowOperatorTest, SlicingWindowAggOperatorTest in UTC and Asia/Shanghai). Rows per watermark, the drop metric,
the late side output and SlicingWindowProcessor.processElement's per-record late flag
(SlicingWindowOperator.java:222-226) must equal the reference's."""
import pytest

from flink_amd.assigners import SliceAssigners, WindowSpec
from flink_amd.operators import SlicingWindowProcessor, WindowOperator
from helpers import load_kats, load_tz_kats

pytestmark = pytest.mark.gpu

DS_KATS = [c for c in load_kats()["operators"] if c["semantics"] == "DATASTREAM" and "gap_col" not in c]
TABLE_KATS = ([c for c in load_kats()["operators"] if c["semantics"] == "TABLE" and c["window_kind"] != "SESSION"] +
              [c for c in load_tz_kats()["operators"] if c["semantics"] == "TABLE" and c["window_kind"] != "SESSION"])


def _spec(c):
    return WindowSpec(c["window_kind"], c["semantics"], size_ms=c["size_ms"], slide_ms=c["slide_ms"],
                      offset_ms=c["offset_ms"], gap_ms=c["gap_ms"])


@pytest.mark.parametrize("case", DS_KATS, ids=[c["name"].split(" ")[0].split(".")[1] for c in DS_KATS])
@pytest.mark.parametrize("batch", [1, 4, 1 << 20])
def test_window_operator_facade_on_gpu(case, batch):
    side = "side_output" in case
    op = WindowOperator(_spec(case), [tuple(a) for a in case["aggs"]], allowed_lateness_ms=case["allowed_lateness_ms"],
                        batch_size=batch, late_data_output=side, key_capacity=1 << 12)
    for ev in case["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], [ev[2]], ev[3])
        else:
            rows = op.process_watermark(ev[1])
            assert all(ts == r[2] - 1 for r, ts in rows)                # record timestamp = window.maxTimestamp()
            got = sorted((r[0], r[1], r[2], *r[3]) for r, _ in rows)
            assert got == sorted(tuple(x) for x in ev[2]), (case["name"], ev[1])
    if side:
        assert op.num_late_records_dropped == 0
        assert sorted((k, v[0], ts) for k, v, ts in op.late_records) == sorted(tuple(x) for x in case["side_output"])
    else:
        assert op.num_late_records_dropped == case["late_dropped"]
    op.close()


@pytest.mark.parametrize("case", TABLE_KATS, ids=[c["name"].split(" ")[0].split(".")[1] + ("_tz" if "tz" in c else "")
                                                  for c in TABLE_KATS])
@pytest.mark.parametrize("batch", [1, 3, 1 << 20])
def test_slicing_processor_facade_on_gpu(case, batch):
    tz = [tuple(p) for p in case["tz"]] if "tz" in case else None
    proc = SlicingWindowProcessor(_spec(case), [tuple(a) for a in case["aggs"]], batch_size=batch, tz=tz,
                                  key_capacity=1 << 12).open()
    flagged = []
    for ev in case["events"]:
        if ev[0] == "e":
            if proc.process_element(ev[1], [ev[2]], ev[3]):
                flagged.append((ev[1], ev[3]))
        else:
            got = sorted(proc.advance_progress(ev[1]))
            assert got == sorted((k, *aggs, ws, we) for k, ws, we, *aggs in ev[2]), (case["name"], ev[1])
    proc.prepare_checkpoint()
    assert proc.num_late_records_dropped == case["late_dropped"] == len(flagged)
    assert sorted(flagged) == sorted((k, ts) for k, _, ts in proc.late_records)
    proc.close()


def test_slicing_processor_late_flag_over_random_stream_on_gpu():
    """A HOP processor over a random stream with late records: the per-record flags equal the engine's per-push
    late indices (fwa_late_records) record for record."""
    import numpy as np
    rng = np.random.default_rng(12)
    proc = SlicingWindowProcessor(SliceAssigners.hopping(4000, 1000), [("COUNT", 0), ("SUM_I64", 0)], batch_size=500,
                                  key_capacity=1 << 12).open()
    n, flags = 20_000, []
    ts = np.sort(rng.integers(0, 100_000, n)) - rng.integers(0, 9000, n)
    keys = rng.integers(0, 300, n)
    wm = -2**63
    for i in range(n):
        flags.append(bool(proc.process_element(int(keys[i]), [int(i)], int(ts[i]))))
        if i % 1000 == 999:
            wm = max(wm, int(ts[i - 999:i + 1].max()) - 1500)
            proc.advance_progress(wm)
    proc.prepare_checkpoint()
    assert sum(flags) == proc.num_late_records_dropped > 0
    flagged = sorted(i for i, f in enumerate(flags) if f)
    assert flagged == sorted(v[0] for _, v, _ in proc.late_records)
    proc.close()


# WindowOperatorTest's reduce sequences (SumReducer over Tuple2<String, Integer>: WindowedStream.sum(1)'s semantics,
# WindowOperatorTest.java:224,406,668) through the DataStream reduction facade on the GPU: non-merging, lateness 0
REDUCE_KATS = [c for c in DS_KATS if c["window_kind"] in ("TUMBLE", "SLIDE") and c["allowed_lateness_ms"] == 0]


@pytest.mark.parametrize("case", REDUCE_KATS, ids=[c["name"].split(" ")[0].split(".")[1] for c in REDUCE_KATS])
@pytest.mark.parametrize("batch", [1, 1 << 20])
def test_reduce_facade_on_gpu(case, batch):
    from flink_amd.operators import ReduceWindowOperator
    side = "side_output" in case
    op = ReduceWindowOperator(_spec(case), "sum", 1, ["I32"], batch_size=batch, late_data_output=side,
                              key_capacity=1 << 12)
    for ev in case["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], [ev[2]], ev[3])
        else:
            got = sorted((r[0], r[1], r[2], r[3][0]) for r, ts in op.process_watermark(ev[1]))
            assert got == sorted(tuple(x) for x in ev[2]), case["name"]
    if not side:
        assert op.num_late_records_dropped == case["late_dropped"]
    op.close()
