"""Generates tests/golden/tz_kats.json: shift-time-zone KATs for the Table slicing path.

Data only. The expected values are the ones asserted by the reference's own tests (file:line in each
case's "src"); this script only (1) builds each zone's (utc_instant, offset) transition table with
Python's zoneinfo (the IANA rules java.time also uses) and (2) evaluates the tests' own input helpers,
localMills(str, zone) = LocalDateTime.parse(str).atZone(zone).toEpochMilli() and
utcMills(str) = LocalDateTime.parse(str).atZone(UTC).toEpochMilli()
(SliceAssignerTestBase.java:108-118), so the fixture holds plain epoch integers.

Run: python tests/golden/gen_tz_kats.py   (rewrites tz_kats.json next to this file)
"""
import datetime as dt
import json
import os
from zoneinfo import ZoneInfo

LONG_MIN = -(1 << 63)
UTC = dt.timezone.utc
SL = "flink-table/flink-table-runtime/src/test/java/org/apache/flink/table/runtime/operators/window/slicing/"
OP = "flink-table/flink-table-runtime/src/test/java/org/apache/flink/table/runtime/operators/aggregate/window/"


def ms(d):
    return int(d.timestamp() * 1000)


def offset_ms(z, instant_ms):
    return int(dt.datetime.fromtimestamp(instant_ms / 1000, tz=UTC).astimezone(z).utcoffset().total_seconds() * 1000)


def transitions(zone, y0=1969, y1=2023):
    """[(instant, offset)] with offset from instant on; the first pair covers everything before."""
    z = ZoneInfo(zone)
    t = ms(dt.datetime(y0, 1, 1, tzinfo=UTC))
    end = ms(dt.datetime(y1, 1, 1, tzinfo=UTC))
    out = [[LONG_MIN, offset_ms(z, t)]]
    step = 3600_000
    while t < end:
        a, b = offset_ms(z, t), offset_ms(z, t + step)
        if a != b:                                   # refine to the first instant with the new offset
            lo, hi = t, t + step
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if offset_ms(z, mid) == a:
                    lo = mid
                else:
                    hi = mid
            out.append([hi, b])
        t += step
    return out


def local_mills(s, zone):                             # LocalDateTime.parse(s).atZone(zone) (earlier offset)
    return ms(dt.datetime.fromisoformat(s).replace(tzinfo=ZoneInfo(zone), fold=0))


def utc_mills(s):
    return ms(dt.datetime.fromisoformat(s).replace(tzinfo=UTC))


def slice_cases(zone):
    out = []
    # TumblingSliceAssignerTest.java:44-54 (testSliceAssignment), 56-68 (withOffset), 70-104 (testDstSaving)
    out.append({"src": SL + "TumblingSliceAssignerTest.java:44-54 (%s)" % zone, "kind": "TUMBLE", "size": 5 * 3600_000,
                "slide": 0, "offset": 0, "cases": [
                    [local_mills("1970-01-01T00:00:00", zone), utc_mills("1970-01-01T05:00:00")],
                    [local_mills("1970-01-01T04:59:59.999", zone), utc_mills("1970-01-01T05:00:00")],
                    [local_mills("1970-01-01T05:00:00", zone), utc_mills("1970-01-01T10:00:00")]]})
    out.append({"src": SL + "TumblingSliceAssignerTest.java:56-68 (%s)" % zone, "kind": "TUMBLE", "size": 5 * 3600_000,
                "slide": 0, "offset": 100, "cases": [
                    [local_mills("1970-01-01T00:00:00.100", zone), utc_mills("1970-01-01T05:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.099", zone), utc_mills("1970-01-01T05:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.100", zone), utc_mills("1970-01-01T10:00:00.100")]]})
    # CumulativeSliceAssignerTest.java:45-57 (testSliceAssignment: max size 1 day, step 1 hour)
    out.append({"src": SL + "CumulativeSliceAssignerTest.java:45-57 (%s)" % zone, "kind": "CUMULATE",
                "size": 24 * 3600_000, "slide": 3600_000, "offset": 0, "cases": [
                    [local_mills("1970-01-01T00:00:00", zone), utc_mills("1970-01-01T01:00:00")],
                    [local_mills("1970-01-02T22:59:59.999", zone), utc_mills("1970-01-02T23:00:00")],
                    [local_mills("1970-01-02T23:00:00", zone), utc_mills("1970-01-03T00:00:00")]]})
    # CumulativeSliceAssignerTest.java:59-72 (withOffset: max size 5 h, step 1 h, offset 100 ms)
    out.append({"src": SL + "CumulativeSliceAssignerTest.java:59-72 (%s)" % zone, "kind": "CUMULATE",
                "size": 5 * 3600_000, "slide": 3600_000, "offset": 100, "cases": [
                    [local_mills("1970-01-01T00:00:00.100", zone), utc_mills("1970-01-01T01:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.099", zone), utc_mills("1970-01-01T05:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.100", zone), utc_mills("1970-01-01T06:00:00.100")]]})
    # HoppingSliceAssignerTest.java:45-70 (size 5 h, slide 1 h; withOffset 100 ms)
    out.append({"src": SL + "HoppingSliceAssignerTest.java:45-56 (%s)" % zone, "kind": "SLIDE",
                "size": 5 * 3600_000, "slide": 3600_000, "offset": 0, "cases": [
                    [local_mills("1970-01-01T00:00:00", zone), utc_mills("1970-01-01T01:00:00")],
                    [local_mills("1970-01-01T04:59:59.999", zone), utc_mills("1970-01-01T05:00:00")],
                    [local_mills("1970-01-01T05:00:00", zone), utc_mills("1970-01-01T06:00:00")]]})
    out.append({"src": SL + "HoppingSliceAssignerTest.java:58-70 (%s)" % zone, "kind": "SLIDE",
                "size": 5 * 3600_000, "slide": 3600_000, "offset": 100, "cases": [
                    [local_mills("1970-01-01T00:00:00.100", zone), utc_mills("1970-01-01T01:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.099", zone), utc_mills("1970-01-01T05:00:00.100")],
                    [local_mills("1970-01-01T05:00:00.100", zone), utc_mills("1970-01-01T06:00:00.100")]]})
    if zone == "America/Los_Angeles":                 # the DST cases run only where useDaylightTime()
        hdst = [(1615708800000, "2021-03-14T01:00"), (1615712400000, "2021-03-14T02:00"),
                (1615716000000, "2021-03-14T04:00"), (1615719600000, "2021-03-14T05:00"),
                (1636268400000, "2021-11-07T01:00"), (1636272000000, "2021-11-07T02:00"),
                (1636275600000, "2021-11-07T02:00"), (1636279200000, "2021-11-07T03:00"),
                (1636282800000, "2021-11-07T04:00"), (1636286400000, "2021-11-07T05:00")]
        out.append({"src": SL + "HoppingSliceAssignerTest.java:72-107 (testDstSaving: size 4 h, slide 1 h)",
                    "kind": "SLIDE", "size": 4 * 3600_000, "slide": 3600_000, "offset": 0,
                    "cases": [[e, utc_mills(s)] for e, s in hdst]})
        dst = [  # (epoch from the test, expected slice end "local as UTC")
            (1615708800000, "2021-03-14T04:00"), (1615712400000, "2021-03-14T04:00"),
            (1615716000000, "2021-03-14T04:00"), (1615719600000, "2021-03-14T08:00"),
            (1636268400000, "2021-11-07T04:00"), (1636272000000, "2021-11-07T04:00"),
            (1636275600000, "2021-11-07T04:00"), (1636279200000, "2021-11-07T04:00"),
            (1636282800000, "2021-11-07T04:00"), (1636286400000, "2021-11-07T08:00")]
        out.append({"src": SL + "TumblingSliceAssignerTest.java:70-104 (testDstSaving)", "kind": "TUMBLE",
                    "size": 4 * 3600_000, "slide": 0, "offset": 0,
                    "cases": [[e, utc_mills(s)] for e, s in dst]})
        cdst = [(1615708800000, "2021-03-14T01:00"), (1615712400000, "2021-03-14T02:00"),
                (1615716000000, "2021-03-14T04:00"), (1615719600000, "2021-03-14T05:00"),
                (1636268400000, "2021-11-07T01:00"), (1636272000000, "2021-11-07T02:00"),
                (1636275600000, "2021-11-07T02:00"), (1636279200000, "2021-11-07T03:00"),
                (1636282800000, "2021-11-07T04:00"), (1636286400000, "2021-11-07T05:00")]
        out.append({"src": SL + "CumulativeSliceAssignerTest.java:74-110 (testDstSaving: max size 4 h, step 1 h)",
                    "kind": "CUMULATE", "size": 4 * 3600_000, "slide": 3600_000, "offset": 0,
                    "cases": [[e, utc_mills(s)] for e, s in cdst]})
    tz = transitions(zone)
    for c in out:
        c["tz"] = tz
        c["zone"] = zone
    return out


def timer_cases():
    """TimeWindowUtilTest.java (flink-table-runtime/src/test/.../runtime/util): toEpochMillsForTimer and
    toUtcTimestampMills integers, Asia/Shanghai and the America/Los_Angeles DST days."""
    LONG_MAX = (1 << 63) - 1
    src = "flink-table/flink-table-runtime/src/test/java/org/apache/flink/table/runtime/util/TimeWindowUtilTest.java"
    sh = {"src": src + ":38-49 (testShiftedTimeZone), :131-137 (testMaxWatermark)", "zone": "Asia/Shanghai",
          "tz": transitions("Asia/Shanghai"),
          "timer": [[utc_mills("1970-01-01T00:00:01"), -28799000], [utc_mills("1970-01-01T07:59:59.999"), -1],
                    [utc_mills("1970-01-01T08:00:01"), 1000], [utc_mills("1970-01-01T08:00:00.001"), 1],
                    [LONG_MAX, LONG_MAX]],
          "to_local": [[LONG_MAX, LONG_MAX]]}
    la = {"src": src + ":51-129 (testDaylightSaving)", "zone": "America/Los_Angeles",
          "tz": transitions("America/Los_Angeles"),
          "timer": [[utc_mills("2021-03-14T00:00:00"), 1615708800000], [utc_mills("2021-03-14T01:00:00"), 1615712400000],
                    [utc_mills("2021-03-14T02:00:00"), 1615716000000], [utc_mills("2021-03-14T02:30:00"), 1615716000000],
                    [utc_mills("2021-03-14T02:59:59"), 1615716000000], [utc_mills("2021-03-14T03:00:00"), 1615716000000],
                    [utc_mills("2021-03-14T03:30:00"), 1615717800000], [utc_mills("2021-03-14T03:59:59"), 1615719599000],
                    [utc_mills("2021-11-07T00:00:00"), 1636268400000], [utc_mills("2021-11-07T01:00:00"), 1636275600000],
                    [utc_mills("2021-11-07T02:00:00"), 1636279200000], [utc_mills("2021-11-07T00:00:01"), 1636268401000],
                    [utc_mills("2021-11-07T01:59:59"), 1636279199000], [utc_mills("2021-11-07T02:00:01"), 1636279201000]],
          "to_local": [[1636272000000, utc_mills("2021-11-07T01:00:00")], [1636275600000, utc_mills("2021-11-07T01:00:00")],
                       [1636272001000, utc_mills("2021-11-07T01:00:01")], [1636275599000, utc_mills("2021-11-07T01:59:59")]]}
    return [sh, la]


def shanghai_operator_kats(utc_kats):
    """SlicingWindowAggOperatorTest and the Table WindowOperatorTest (legacy GROUP BY SESSION) are parameterised by
    shiftTimeZone (UTC, Asia/Shanghai): inputs are the same epoch rowtimes and watermarks; expected window bounds are
    localMills(x) = toUtcTimestampMills(x, zone) (SlicingWindowAggOperatorTest.java:116-222, 345-460, 596-692;
    table WindowOperatorTest.java:89-100 parameters, :1401-1514 testEventTimeSessionWindows, localMills :2066-2068)."""
    z = ZoneInfo("Asia/Shanghai")
    tz = transitions("Asia/Shanghai")
    out = []
    for c in utc_kats:
        if not (c["name"].startswith("SlicingWindowAggOperatorTest") or
                c["name"].startswith("TableWindowOperatorTest.testEventTimeSessionWindows")):
            continue
        d = json.loads(json.dumps(c))
        d["name"] = c["name"].replace("(UTC)", "(Asia/Shanghai)")
        d["src"] = c["src"].replace("(UTC)", "") + " (Asia/Shanghai parameterisation)"
        for ev in d["events"]:
            if ev[0] == "w":
                ev[2] = [[r[0], r[1] + offset_ms(z, r[1]), r[2] + offset_ms(z, r[2])] + r[3:] for r in ev[2]]
        d["tz"] = tz
        out.append(d)
    return out


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "reference_kats.json")) as f:
        kats = json.load(f)
    doc = {"_doc": __doc__.strip().splitlines()[0] + " Generated by gen_tz_kats.py; see its docstring.",
           "slice_ends": slice_cases("America/Los_Angeles") + slice_cases("Asia/Shanghai"),
           "timer": timer_cases(),
           "operators": shanghai_operator_kats(kats["operators"])}
    with open(os.path.join(here, "tz_kats.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
