"""Known-answer vectors transcribed from EventTimeSessionWindowsTest.java and TimeWindowTest.java (data only).

Paths relative to flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/.

* assigners: `EventTimeSessionWindowsTest.testWindowAssignment` :61-79 / `testTimeUnits` :177-197 (gap 5000:
  ts -> [ts, ts + gap)), `TimeWindowTest.testGetWindowStartWithOffset` :31-76 (window starts for size 7 with
  offsets 0, 3, -2 and a one-day window at GMT+08:00; expressed as tumbling windows [start, start + size)).
* operators: the mergeWindows cases of `EventTimeSessionWindowsTest` (:82-174) and `TimeWindowTest.testIntersect`
  (:84-97) as session operator sequences. A window [s, e) is the session window of a record with timestamp s and a
  per-record gap e - s (DynamicEventTimeSessionWindows, gap column 1); the windows of one key are pushed, the
  Long.MAX_VALUE watermark fires the merged sessions, and each row's SUM counts the windows merged into it (value
  1 per record). Zero-length windows ((0, 0) in testMergeSinglePointWindow, (1, 1) in testMergeCoveringWindow)
  have no record form (a dynamic gap must be > 0, DynamicEventTimeSessionWindows.java:62-66), so they are left
  out; the merges they take part in are unchanged ((1, 1) lies inside (0, 2)).
* invalid parameters: `testInvalidParameters` :199-214 (gap <= 0 rejected).

Run: python tests/golden/gen_session_kats.py  (writes tests/golden/session_kats.json)
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "session_kats.json")
SRC = "flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/"
LMAX = (1 << 63) - 1


def tumble_case(src, size, offset, pairs):
    return dict(src=src, kind="TUMBLE", size=size, offset=offset, cases=[[ts, [[st, st + size]]] for ts, st in pairs])


def merge_case(name, src, windows, merged):
    """windows: [(s, e)] pushed for key 1 in this order; merged: [(s, e, n_windows)] fired at Long.MAX_VALUE."""
    events = [["e", 1, 1, s, e - s] for s, e in windows]
    events.append(["w", LMAX, [[1, s, e, n] for s, e, n in merged]])
    return dict(name=name, src=src, semantics="DATASTREAM", window_kind="SESSION", size_ms=0, slide_ms=0,
                offset_ms=0, gap_ms=0, allowed_lateness_ms=0, aggs=[["SUM_I64", 0]], gap_col=1, events=events,
                late_dropped=0)


def main():
    assigners = [
        dict(src=SRC + "EventTimeSessionWindowsTest.java:61-79 (testWindowAssignment)", kind="SESSION", size=0,
             offset=0, gap=5000, cases=[[0, [[0, 5000]]], [4999, [[4999, 9999]]], [5000, [[5000, 10000]]]]),
        dict(src="EventTimeSessionWindowsTest.java:177-197 (testTimeUnits, Time.seconds(5))", kind="SESSION", size=0,
             offset=0, gap=5000, cases=[[0, [[0, 5000]]], [4999, [[4999, 9999]]], [5000, [[5000, 10000]]]]),
        tumble_case(SRC + "TimeWindowTest.java:32-41 (offset 0, size 7)", 7, 0,
                    [(-8, -14), (-7, -7), (-6, -7), (-1, -7), (1, 0), (6, 0), (7, 7), (8, 7)]),
        tumble_case("TimeWindowTest.java:43-54 (offset 3, size 7)", 7, 3,
                    [(-10, -11), (-9, -11), (-3, -4), (-2, -4), (-1, -4), (1, -4), (2, -4), (3, 3), (9, 3), (10, 10)]),
        tumble_case("TimeWindowTest.java:56-69 (offset -2, size 7)", 7, -2,
                    [(-12, -16), (-7, -9), (-4, -9), (-3, -9), (2, -2), (-1, -2), (1, -2), (-2, -2), (3, -2),
                     (4, -2), (7, 5), (12, 12)]),
        tumble_case("TimeWindowTest.java:71-75 (GMT+08:00 day windows)", 86400000, -8 * 3600000,
                    [(1470902048450, 1470844800000)]),
    ]
    operators = [
        merge_case("EventTimeSessionWindowsTest.testMergeSingleWindow", SRC + "EventTimeSessionWindowsTest.java:93-103",
                   [(0, 1)], [(0, 1, 1)]),
        merge_case("EventTimeSessionWindowsTest.testMergeConsecutiveWindows", "EventTimeSessionWindowsTest.java:105-140",
                   [(0, 1), (1, 2), (2, 3), (4, 5), (5, 6)], [(0, 3, 3), (4, 6, 2)]),
        merge_case("EventTimeSessionWindowsTest.testMergeCoveringWindow (zero-length (1, 1) left out)",
                   "EventTimeSessionWindowsTest.java:142-174", [(0, 2), (4, 7), (5, 6)], [(0, 2, 1), (4, 7, 2)]),
        merge_case("TimeWindowTest.testIntersect (adjacent windows merge)", SRC + "TimeWindowTest.java:84-97",
                   [(10, 20), (20, 30)], [(10, 30, 2)]),
        merge_case("TimeWindowTest.testIntersect (gap between windows)", "TimeWindowTest.java:92-93",
                   [(10, 20), (21, 30)], [(10, 20, 1), (21, 30, 1)]),
        merge_case("TimeWindowTest.testIntersect (overlap by one)", "TimeWindowTest.java:95-96",
                   [(10, 20), (19, 22)], [(10, 22, 2)]),
    ]
    invalid_gaps = dict(src=SRC + "EventTimeSessionWindowsTest.java:199-214 (testInvalidParameters)",
                        gaps=[-1000, 0])
    doc = ("Known-answer vectors transcribed from EventTimeSessionWindowsTest.java and TimeWindowTest.java "
           "(generated by tests/golden/gen_session_kats.py; see its docstring for the mapping).")
    with open(OUT, "w") as f:
        json.dump(dict(_doc=doc, assigners=assigners, operators=operators, invalid_gaps=invalid_gaps), f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
