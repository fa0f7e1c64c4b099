"""CPU tests: the oracle restatement against the reference's own known-answer vectors."""
import ctypes as C

import numpy as np
import pytest

from flink_amd import _abi as A
from oracle import oracle as O
from helpers import load_kats, load_pyflink_kats, load_session_kats, load_sql_kats, load_tz_kats, replay_kat, replay_sql_kat

KATS = load_kats()
TZ_KATS = load_tz_kats()
PY_KATS = load_pyflink_kats()
SESSION_KATS = load_session_kats()


@pytest.mark.parametrize("case", KATS["assigners"] + SESSION_KATS["assigners"], ids=lambda c: c["src"].split("/")[-1])
def test_assigner_kats(case):
    cfg = A.make_config(window_kind=case["kind"], size_ms=case["size"], slide_ms=case.get("slide", 0),
                        offset_ms=case["offset"], gap_ms=case.get("gap", 0))
    for ts, exp in case["cases"]:
        starts = np.zeros(64, np.int64)
        ends = np.zeros(64, np.int64)
        n = O.lib().or_assign_windows(C.byref(cfg), ts, starts.ctypes.data, ends.ctypes.data, 64)
        got = sorted(zip(starts[:n].tolist(), ends[:n].tolist()))
        assert got == sorted(tuple(w) for w in exp), (ts, got, exp)


@pytest.mark.parametrize("case", KATS["slice_ends"], ids=lambda c: c["src"].split("/")[-1])
def test_slice_end_kats(case):
    cfg = A.make_config(window_kind=case["kind"], semantics="TABLE", size_ms=case["size"],
                        slide_ms=case["slide"], offset_ms=case["offset"])
    for ts, exp in case["cases"]:
        assert O.lib().or_assign_slice_end(C.byref(cfg), ts) == exp


@pytest.mark.parametrize("case", KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_operator_kats(case):
    replay_kat(case, O.Oracle)


@pytest.mark.parametrize("case", PY_KATS["operators"], ids=lambda c: c["name"].split(" ", 1)[1])
def test_pyflink_window_operator_sequences(case):
    """The oracle against the reference's own Python WindowOperator run over random streams
    (tests/golden/gen_pyflink_kats.py): every watermark's rows and the drop count."""
    replay_kat(case, O.Oracle)


@pytest.mark.parametrize("case", SESSION_KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_session_merge_kats(case):
    """EventTimeSessionWindowsTest mergeWindows / TimeWindowTest.testIntersect as session sequences."""
    replay_kat(case, O.Oracle)


@pytest.mark.parametrize("gap", SESSION_KATS["invalid_gaps"]["gaps"])
def test_session_invalid_gap(gap):
    """EventTimeSessionWindowsTest.testInvalidParameters: a gap <= 0 is rejected."""
    with pytest.raises(O.OracleError) as ei:
        O.Oracle(A.make_config(window_kind="SESSION", gap_ms=gap, size_ms=0))
    assert ei.value.code == -1


def test_murmur_properties():
    L = O.lib()
    # murmurHash is non-negative and INT_MIN folds to 0 (MathUtils.java:150-154)
    for code in [0, 1, -1, 42, 2**31 - 1, -2**31, 123456789, -987654321]:
        assert L.or_murmur_hash(code) >= 0
    # key groups within range and operator index formula
    for k in range(-1000, 1000, 7):
        kg = L.or_key_group(k, A.KEY_JAVA_LONG, 0, 128)
        assert 0 <= kg < 128
        assert L.or_operator_index(128, 8, kg) == kg * 8 // 128


def test_key_group_ranges_partition():
    L = O.lib()
    for maxp, par in [(128, 1), (128, 2), (128, 3), (128, 8), (32768, 7)]:
        covered = []
        for i in range(par):
            s, e = C.c_int32(), C.c_int32()
            L.or_key_group_range(maxp, par, i, C.byref(s), C.byref(e))
            covered.extend(range(s.value, e.value + 1))
            for kg in (s.value, e.value):
                assert L.or_operator_index(maxp, par, kg) == i
        assert covered == list(range(maxp))


def test_keygroup_violation_raises():
    cfg = A.make_config(kg_start=0, kg_end=0)
    o = O.Oracle(cfg)
    with pytest.raises(O.OracleError) as ei:
        o.push(np.arange(100), np.arange(100), [np.arange(100)])
    assert ei.value.code == -3


def test_ts_min_raises():
    o = O.Oracle(A.make_config())
    with pytest.raises(O.OracleError) as ei:
        o.push(np.array([1]), np.array([A.LONG_MIN]), [np.array([1])])
    assert ei.value.code == -2


@pytest.mark.parametrize("case", KATS["key_groups"], ids=lambda c: c["src"].split("/")[-1].split(" ")[0])
def test_key_group_literal_kats(case):
    """KeyGroupRangeAssignment integers asserted by the reference's own tests (String / Integer keys:
    key.hashCode() -> murmurHash -> % maxParallelism; operator index kg * P / maxP)."""
    from helpers import java_hash_code
    L = O.lib()
    maxp = case["max_parallelism"]
    for key, kg in case["cases"]:
        assert L.or_key_group(0, A.KEY_PREHASHED, java_hash_code(key, case["key_type"]), maxp) == kg, key
    for key, par, op in case["operator_index"]:
        kg = L.or_key_group(0, A.KEY_PREHASHED, java_hash_code(key, case["key_type"]), maxp)
        assert L.or_operator_index(maxp, par, kg) == op, (key, par)


@pytest.mark.parametrize("case", TZ_KATS["slice_ends"], ids=lambda c: c["src"].split("/")[-1])
def test_slice_end_kats_shift_time_zone(case):
    """TIMESTAMP_LTZ rowtimes: slice ends in local wall-clock millis (TimeWindowUtil.toUtcTimestampMills),
    incl. the America/Los_Angeles DST days of Tumbling/CumulativeSliceAssignerTest.testDstSaving."""
    cfg = A.make_config(window_kind=case["kind"], semantics="TABLE", size_ms=case["size"],
                        slide_ms=case["slide"], offset_ms=case["offset"], tz=case["tz"])
    for ts, exp in case["cases"]:
        assert O.lib().or_assign_slice_end(C.byref(cfg), ts) == exp, (ts, exp)


@pytest.mark.parametrize("case", TZ_KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_operator_kats_shift_time_zone(case):
    replay_kat(case, O.Oracle)


@pytest.mark.parametrize("case", TZ_KATS["timer"], ids=lambda c: c["zone"])
def test_time_zone_conversion_kats(case):
    """TimeWindowUtilTest integers: toEpochMillsForTimer (incl. the DST gap / overlap hours) and
    toUtcTimestampMills."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, tz=case["tz"])
    for local, exp in case["timer"]:
        assert O.lib().or_tz_timer(C.byref(cfg), local) == exp, (local, exp)
    for epoch, exp in case["to_local"]:
        assert O.lib().or_to_local(C.byref(cfg), epoch) == exp, (epoch, exp)


SQL_KATS = load_sql_kats()


@pytest.mark.parametrize("case", SQL_KATS["operators"], ids=lambda c: c["name"].split(".")[-1])
def test_sql_null_kats(case):
    """WindowAggregateITCase TUMBLE/HOP/CUMULATE over TestData.windowDataWithTimestamp: NULL values skipped by
    SUM/MAX/MIN, a NULL result where a window has no non-NULL value, a NULL grouping key."""
    replay_sql_kat(case, O.Oracle)
