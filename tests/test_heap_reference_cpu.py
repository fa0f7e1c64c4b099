"""Pin the heap keyed-state reader (tests/heap_reader.py) against checkpoints the reference itself wrote.

Fixtures: `tests/golden/flink_snapshots/win-op-migration-test-*-flink1.18-snapshot`, copied byte for byte from
`flink-streaming-java/src/test/resources/` (data files of the reference's own tests, written by
`WindowOperatorMigrationTest.java` through `OperatorSnapshotUtil.writeStateHandle` with the heap backend of the
`KeyedOneInputStreamOperatorTestHarness`). The same section reader parses the engine's `fwa_snapshot_heap` bytes in
tests/test_heap_snapshot_gpu.py, so these tests pin that check to the reference's real byte layout: the wrapper
(OperatorSnapshotUtil.java:48-123, MetadataV2V3SerializerBase.java:309-331,670-690), the state-id numbering (the
order of the proxy's meta infos: HashMap order of the state names, key/value states before timer queues,
HeapSnapshotResources.java:100-139), the per-key-group sections (HeapSnapshotStrategy.java:154-175), TimeWindow /
String / Tuple / List / VoidNamespace serializers and the timer entries (TimerSerializer.java:147-152).
"""
import os

import pytest

import heap_reader as H

D = os.path.join(os.path.dirname(__file__), "golden", "flink_snapshots")
WINDOW_OPERATOR_STATES = ["count", "window-contents", "merging-window-set",
                          "_timer_state/processing_window-timers", "_timer_state/event_window-timers"]
STR_INT = H.ser_tuple(H.ser_string, H.ser_int)


def load(name):
    b = open(os.path.join(D, name), "rb").read()
    hs = H.read_operator_snapshot(b)
    assert len(hs) == 1
    first, offs, data = hs[0]
    ids = H.state_ids(data[:offs[0]], WINDOW_OPERATOR_STATES)
    return first, offs, data, ids


def test_reduce_event_time_snapshot():
    """writeReducingEventTimeWindowsSnapshot (WindowOperatorMigrationTest.java:366-440): tumbling 3 s event-time
    windows, ReducingState "window-contents" of Tuple2<String, Integer> with a sum reducer, records :408-417,
    watermark 1999 (nothing fired). Restore expectations (:494-507): at 2999 key1 -> 3 and key2 -> 3, at 5999
    key2 -> 2 -- so the state holds [0,3000) key1 3, [0,3000) key2 3, [3000,6000) key2 2 and the event-time timers
    at window.maxTimestamp() (EventTimeTrigger.onElement; allowedLateness 0, so the cleanup timer is the same)."""
    first, offs, data, ids = load("win-op-migration-test-reduce-event-time-flink1.18-snapshot")
    assert ids == {"window-contents": 0, "_timer_state/processing_window-timers": 1,
                   "_timer_state/event_window-timers": 2}
    assert first == 0 and len(offs) == 1
    lay = {ids["window-contents"]: ("kv", H.ser_time_window, H.ser_string, STR_INT),
           ids["_timer_state/processing_window-timers"]: ("pq", H.ser_string, H.ser_time_window),
           ids["_timer_state/event_window-timers"]: ("pq", H.ser_string, H.ser_time_window)}
    kgs = H.read_key_groups(data, offs, first, lay)
    s = kgs[0]
    assert sorted(s) == [0, 1, 2]                                  # every registered state has a section
    assert sorted(s[0]) == [((0, 3000), "key1", ("key1", 3)), ((0, 3000), "key2", ("key2", 3)),
                            ((3000, 6000), "key2", ("key2", 2))]
    assert s[1] == []                                              # no processing-time timers
    assert sorted(s[2]) == [(2999, "key1", (0, 3000)), (2999, "key2", (0, 3000)), (5999, "key2", (3000, 6000))]


def test_session_with_stateful_trigger_snapshot():
    """writeSessionWindowsWithCountTriggerSnapshot (WindowOperatorMigrationTest.java:98-153): session gap 3 s,
    ListState "window-contents", PurgingTrigger.of(CountTrigger.of(4)) (trigger state "count"), records :135-141.
    key2's four records merge into [0, 6500) and fire-and-purge (count reached 4: contents and count cleared; the
    window stays in the merging-window-set until cleanup); key1's two records make [10, 4000) with count 2.
    MergingWindowSet.addWindow keeps the first window's state namespace for a merge ([0,3000) / [10,3010)).
    The cleanup timers are at maxTimestamp() + allowedLateness 0 (WindowOperator.registerCleanupTimer :608-620).
    Restore expectation (:201-217): one more key1 record at 4500 merges the sessions into [10, 10000)."""
    first, offs, data, ids = load("win-op-migration-test-session-with-stateful-trigger-flink1.18-snapshot")
    assert ids == {"count": 0, "window-contents": 1, "merging-window-set": 2,
                   "_timer_state/processing_window-timers": 3, "_timer_state/event_window-timers": 4}
    lay = {0: ("kv", H.ser_time_window, H.ser_string, H.ser_long),
           1: ("kv", H.ser_time_window, H.ser_string, H.ser_list(STR_INT)),
           2: ("kv", H.ser_void, H.ser_string, H.ser_list(H.ser_tuple(H.ser_time_window, H.ser_time_window))),
           3: ("pq", H.ser_string, H.ser_time_window),
           4: ("pq", H.ser_string, H.ser_time_window)}
    s = H.read_key_groups(data, offs, first, lay)[0]
    assert sorted(s) == [0, 1, 2, 3, 4]
    assert s[0] == [((10, 4000), "key1", 2)]                       # CountTrigger's count under the actual window
    assert s[1] == [((10, 3010), "key1", [("key1", 1), ("key1", 2)])]   # contents under the state window
    assert sorted(s[2]) == [(None, "key1", [((10, 4000), (10, 3010))]), (None, "key2", [((0, 6500), (0, 3000))])]
    assert s[3] == []
    assert sorted(s[4]) == [(3999, "key1", (10, 4000)), (6499, "key2", (0, 6500))]


def test_state_ids_follow_hashmap_order():
    """The id numbering the engine's heap writer uses for the states WindowOperator / SlicingWindowOperator
    register (include/flink_amd.h fwa_snapshot_heap): java.util.HashMap iteration order of the names (bucket =
    (h ^ h >>> 16) & 15 of String.hashCode, 16 buckets), key/value states first, then the timer queues."""
    def bucket(s):
        h = 0
        for ch in s:
            h = (31 * h + ord(ch)) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & 15
    kv = ["count", "window-contents", "merging-window-set"]
    assert sorted(kv, key=bucket) == kv                            # the order the session snapshot shows
    assert bucket("window-contents") < bucket("merging-window-set")
    pq = ["_timer_state/processing_window-timers", "_timer_state/event_window-timers"]
    assert sorted(pq, key=bucket) == pq


def test_truncated_snapshot_is_rejected():
    b = open(os.path.join(D, "win-op-migration-test-reduce-event-time-flink1.18-snapshot"), "rb").read()
    first, offs, data = H.read_operator_snapshot(b)[0]
    lay = {0: ("kv", H.ser_time_window, H.ser_string, STR_INT), 1: ("pq", H.ser_string, H.ser_time_window),
           2: ("pq", H.ser_string, H.ser_time_window)}
    with pytest.raises(Exception):
        H.read_key_groups(data[:-10], offs, first, lay)
