"""Generates tests/golden/sql_kats.json: SQL NULL-semantics KATs for the Table window-TVF path.

Data only, transcribed by hand from the reference's own test:
  input  TestData.windowDataWithTimestamp
         flink-table/flink-table-planner/src/test/scala/org/apache/flink/table/planner/runtime/utils/TestData.scala:729-742
  output WindowAggregateITCase.testEventTimeTumbleWindow / testEventTimeHopWindow / testEventTimeCumulateWindow
         flink-table/flink-table-planner/src/test/scala/org/apache/flink/table/planner/runtime/stream/sql/WindowAggregateITCase.scala:174-207, 492-530, 696-741
The ITCase's columns this engine computes: COUNT(*), SUM(bigdec), MAX(double), MIN(float) (COUNT(DISTINCT) and
the UDAF are not on this path). Mapping: name "a" -> key 1, "b" -> 2, NULL -> 3 (a NULL grouping key is a key
like any other); bigdec DECIMAL(10, 2) -> its unscaled long, summed by SUM_DEC (scale 2: the DECIMAL(38, 2) result
as its unscaled value, x100);
rowtime TIMESTAMP(3) -> epoch millis of the local time read as UTC (the non-LTZ parameterisation). Watermark:
`rowtime - INTERVAL '1' SECOND` after every record (the ITCase's per-record watermark assigner), then MAX at
the end of input. The ITCase asserts the multiset of all emitted rows; so does the replay.

Run: python tests/golden/gen_sql_kats.py
"""
import json
import os
from decimal import Decimal

BASE = 1602288000000              # 2020-10-10T00:00:00 as UTC epoch millis
KEY = {"a": 1, "b": 2, None: 3}
SRC_IT = "flink-table/flink-table-planner/src/test/scala/org/apache/flink/table/planner/runtime/stream/sql/WindowAggregateITCase.scala"

# (second, int, double, float, bigdec, string, name) -- TestData.scala:729-742, in arrival order
ROWS = [
    (1, 1, 1.0, 1.0, "1.11", "Hi", "a"),
    (2, 2, 2.0, 2.0, "2.22", "Comment#1", "a"),
    (3, 2, 2.0, 2.0, "2.22", "Comment#1", "a"),
    (4, 5, 5.0, 5.0, "5.55", None, "a"),
    (7, 3, 3.0, 3.0, None, "Hello", "b"),
    (6, 6, 6.0, 6.0, "6.66", "Hi", "b"),
    (8, 3, None, 3.0, "3.33", "Comment#2", "a"),
    (4, 5, 5.0, None, "5.55", "Hi", "a"),
    (16, 4, 4.0, 4.0, "4.44", "Hi", "b"),
    (32, 7, 7.0, 7.0, "7.77", None, None),
    (34, 1, 3.0, 3.0, "3.33", "Comment#3", "b"),
]

TUMBLE = [
    "a,2020-10-10T00:00,2020-10-10T00:00:05,4,11.10,5.0,1.0",
    "a,2020-10-10T00:00:05,2020-10-10T00:00:10,1,3.33,null,3.0",
    "b,2020-10-10T00:00:05,2020-10-10T00:00:10,2,6.66,6.0,3.0",
    "b,2020-10-10T00:00:15,2020-10-10T00:00:20,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:30,2020-10-10T00:00:35,1,3.33,3.0,3.0",
    "null,2020-10-10T00:00:30,2020-10-10T00:00:35,1,7.77,7.0,7.0",
]
HOP = [
    "a,2020-10-09T23:59:55,2020-10-10T00:00:05,4,11.10,5.0,1.0",
    "a,2020-10-10T00:00,2020-10-10T00:00:10,6,19.98,5.0,1.0",
    "a,2020-10-10T00:00:05,2020-10-10T00:00:15,1,3.33,null,3.0",
    "b,2020-10-10T00:00,2020-10-10T00:00:10,2,6.66,6.0,3.0",
    "b,2020-10-10T00:00:05,2020-10-10T00:00:15,2,6.66,6.0,3.0",
    "b,2020-10-10T00:00:10,2020-10-10T00:00:20,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:15,2020-10-10T00:00:25,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:25,2020-10-10T00:00:35,1,3.33,3.0,3.0",
    "b,2020-10-10T00:00:30,2020-10-10T00:00:40,1,3.33,3.0,3.0",
    "null,2020-10-10T00:00:25,2020-10-10T00:00:35,1,7.77,7.0,7.0",
    "null,2020-10-10T00:00:30,2020-10-10T00:00:40,1,7.77,7.0,7.0",
]
CUMULATE = [
    "a,2020-10-10T00:00,2020-10-10T00:00:05,4,11.10,5.0,1.0",
    "a,2020-10-10T00:00,2020-10-10T00:00:10,6,19.98,5.0,1.0",
    "a,2020-10-10T00:00,2020-10-10T00:00:15,6,19.98,5.0,1.0",
    "b,2020-10-10T00:00,2020-10-10T00:00:10,2,6.66,6.0,3.0",
    "b,2020-10-10T00:00,2020-10-10T00:00:15,2,6.66,6.0,3.0",
    "b,2020-10-10T00:00:15,2020-10-10T00:00:20,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:15,2020-10-10T00:00:25,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:15,2020-10-10T00:00:30,1,4.44,4.0,4.0",
    "b,2020-10-10T00:00:30,2020-10-10T00:00:35,1,3.33,3.0,3.0",
    "b,2020-10-10T00:00:30,2020-10-10T00:00:40,1,3.33,3.0,3.0",
    "b,2020-10-10T00:00:30,2020-10-10T00:00:45,1,3.33,3.0,3.0",
    "null,2020-10-10T00:00:30,2020-10-10T00:00:35,1,7.77,7.0,7.0",
    "null,2020-10-10T00:00:30,2020-10-10T00:00:40,1,7.77,7.0,7.0",
    "null,2020-10-10T00:00:30,2020-10-10T00:00:45,1,7.77,7.0,7.0",
]


def ts_of(s):                     # "2020-10-09T23:59:55" / "2020-10-10T00:00" -> epoch millis (as UTC)
    date, t = s.split("T")
    parts = [int(x) for x in t.split(":")] + [0]
    sec = parts[0] * 3600 + parts[1] * 60 + parts[2]
    day = -86400 if date == "2020-10-09" else 0
    return BASE + (day + sec) * 1000


def parse(lines):
    out = []
    for ln in lines:
        name, ws, we, cnt, dec, dbl, flt = ln.split(",")
        nul = lambda v, f: None if v == "null" else f(v)
        out.append([KEY[None if name == "null" else name], ts_of(ws), ts_of(we), int(cnt),
                    nul(dec, lambda v: int(Decimal(v) * 100)), nul(dbl, float), nul(flt, float)])
    return out


def events():
    ev, mx = [], -(1 << 63)
    for sec, _i, dbl, flt, dec, _s, name in ROWS:
        ts = BASE + sec * 1000
        ev.append(["e", KEY[name], [None if dec is None else int(Decimal(dec) * 100), dbl, flt], ts])
        if ts - 1000 > mx:                       # WATERMARK rowtime - INTERVAL '1' SECOND, ascending only
            mx = ts - 1000
            ev.append(["w", mx])
    ev.append(["w", (1 << 63) - 1])
    return ev


def case(name, lines, lo, kind, size, slide):
    return {"name": "WindowAggregateITCase.%s" % name, "src": "%s:%s (input TestData.scala:729-742)" % (SRC_IT, lo),
            "window_kind": kind, "size_ms": size, "slide_ms": slide, "offset_ms": 0,
            "aggs": [["COUNT", 0], ["SUM_DEC", 0, 2], ["MAX_F64", 1], ["MIN_F32", 2]],
            "col_types": ["i8", "f8", "f4"], "nullable_cols": [0, 1, 2],
            "events": events(), "expected": parse(lines), "late_dropped": 1 if kind == "TUMBLE" else 0}


def main():
    doc = {"_doc": __doc__.strip().splitlines()[0] + " Generated by gen_sql_kats.py; see its docstring.",
           "operators": [case("testEventTimeTumbleWindow", TUMBLE, "174-207", "TUMBLE", 5000, 0),
                         case("testEventTimeHopWindow", HOP, "492-530", "SLIDE", 10000, 5000),
                         case("testEventTimeCumulateWindow", CUMULATE, "696-741", "CUMULATE", 15000, 5000)]}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sql_kats.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
