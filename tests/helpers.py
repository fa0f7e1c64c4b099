"""Shared test helpers: KAT replay and multiset comparison of fired rows."""
import json
import os

import numpy as np

from flink_amd import _abi as A

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def java_hash_code(key, key_type):
    """key.hashCode() per the Java SE spec: Integer -> the value; String -> s[0]*31^(n-1) + ... + s[n-1]
    over UTF-16 code units, int32 wrap-around (java.lang.String.hashCode)."""
    if key_type == "Integer":
        return int(np.int32(key))
    b = key.encode("utf-16-le")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + int.from_bytes(b[i:i + 2], "little")) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def load_kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


def load_pyflink_kats():
    """Operator sequences produced by the reference's own Python WindowOperator (tests/golden/gen_pyflink_kats.py)."""
    with open(os.path.join(GOLDEN, "pyflink_kats.json")) as f:
        return json.load(f)


def load_session_kats():
    """EventTimeSessionWindowsTest / TimeWindowTest vectors (tests/golden/gen_session_kats.py)."""
    with open(os.path.join(GOLDEN, "session_kats.json")) as f:
        return json.load(f)


def assigner_windows_by_rows(case, make_engine):
    """Window assignment seen through an engine: one record per timestamp (key = its index), fired at
    Long.MAX_VALUE; returns {ts: [(start, end)]}."""
    cfg = A.make_config(window_kind=case["kind"], size_ms=case["size"], slide_ms=case.get("slide", 0),
                        offset_ms=case["offset"], gap_ms=case.get("gap", 0), aggs=[("COUNT", 0)])
    eng = make_engine(cfg)
    ts = np.array([c[0] for c in case["cases"]], np.int64)
    eng.push(np.arange(len(ts), dtype=np.int64), ts, [])
    rows = eng.advance_watermark((1 << 63) - 1)
    eng.close()
    got = {}
    for i in range(len(rows["key"])):
        got.setdefault(int(ts[rows["key"][i]]), []).append((int(rows["win_start"][i]), int(rows["win_end"][i])))
    return {k: sorted(v) for k, v in got.items()}


def load_tz_kats():
    """Shift-time-zone KATs (tests/golden/gen_tz_kats.py)."""
    with open(os.path.join(GOLDEN, "tz_kats.json")) as f:
        return json.load(f)


def kat_config(case, **kw):
    return A.make_config(window_kind=case["window_kind"], semantics=case["semantics"],
                         size_ms=case["size_ms"], slide_ms=case["slide_ms"],
                         offset_ms=case["offset_ms"], gap_ms=case["gap_ms"],
                         allowed_lateness_ms=case["allowed_lateness_ms"],
                         aggs=[tuple(a) for a in case["aggs"]], gap_col=case.get("gap_col"),
                         tz=case.get("tz"), **kw)


def rows_to_tuples(rows, naggs):
    cols = [rows["key"], rows["win_start"], rows["win_end"]] + [rows["agg%d" % j] for j in range(naggs)]
    out = []
    for i in range(len(rows["key"])):
        out.append(tuple(c[i].item() for c in cols))
    return sorted(out)


def replay_kat(case, make_engine):
    """Feed a KAT event sequence through an engine; assert every watermark's fired multiset."""
    eng = make_engine(kat_config(case))
    naggs = len(case["aggs"])
    dropped = 0
    pend = []

    def flush():
        nonlocal dropped, pend
        if pend:
            k = np.array([p[0] for p in pend], np.int64)
            v = np.array([p[1] for p in pend], np.int64)
            t = np.array([p[2] for p in pend], np.int64)
            cols = [v]
            if case.get("gap_col") is not None:          # per-record session gap (5th event field)
                cols.append(np.array([p[3] for p in pend], np.int64))
            dropped += eng.push(k, t, cols)
            pend = []

    for ev in case["events"]:
        if ev[0] == "e":
            pend.append((ev[1], ev[2], ev[3], ev[4] if len(ev) > 4 else 0))
        else:
            flush()
            rows = eng.advance_watermark(ev[1])
            got = rows_to_tuples(rows, naggs)
            exp = sorted(tuple(r) for r in ev[2])
            assert got == exp, "%s: wm=%d expected %s got %s" % (case["name"], ev[1], exp, got)
    flush()
    assert dropped == case["late_dropped"], "%s: late dropped %d != %d" % (case["name"], dropped, case["late_dropped"])
    eng.close()


def load_sql_kats():
    """SQL NULL-semantics KATs (tests/golden/gen_sql_kats.py)."""
    with open(os.path.join(GOLDEN, "sql_kats.json")) as f:
        return json.load(f)


def replay_sql_kat(case, make_engine):
    """Feed a WindowAggregateITCase event sequence (multi-column, SQL NULLs) through an engine and compare
    the multiset of ALL emitted rows with the ITCase's expected rows; NULL results compare as None."""
    cfg = A.make_config(window_kind=case["window_kind"], semantics="TABLE", size_ms=case["size_ms"],
                        slide_ms=case["slide_ms"], offset_ms=case["offset_ms"],
                        aggs=[tuple(a) for a in case["aggs"]], nullable_cols=case["nullable_cols"])
    eng = make_engine(cfg)
    naggs, types = len(case["aggs"]), case["col_types"]
    dropped, got, pend = 0, [], []

    def flush():
        nonlocal dropped, pend
        if pend:
            k = np.array([p[0] for p in pend], np.int64)
            t = np.array([p[2] for p in pend], np.int64)
            cols = [np.array([0 if p[1][c] is None else p[1][c] for p in pend], types[c]) for c in range(len(types))]
            nulls = [np.array([p[1][c] is None for p in pend], np.uint8) for c in range(len(types))]
            dropped += eng.push(k, t, cols, nulls=nulls)
            pend = []

    for ev in case["events"]:
        if ev[0] == "e":
            pend.append((ev[1], ev[2], ev[3]))
            continue
        flush()
        rows = eng.advance_watermark(ev[1])
        for i in range(len(rows["key"])):
            r = [rows["key"][i].item(), rows["win_start"][i].item(), rows["win_end"][i].item()]
            for j in range(naggs):
                nul = rows.get("null%d" % j)
                v = rows["agg%d" % j][i]
                r.append(None if nul is not None and nul[i] else (v.item() if hasattr(v, "item") else v))
            got.append(r)
    flush()
    key = lambda r: tuple((x is None, x) for x in r)
    assert sorted(got, key=key) == sorted(case["expected"], key=key), "%s: got %s" % (case["name"], got)
    assert dropped == case["late_dropped"], "%s: late dropped %d != %d" % (case["name"], dropped, case["late_dropped"])
    eng.close()


def load_decimal_kats():
    """DECIMAL SUM / AVG KATs (tests/golden/gen_decimal_kats.py)."""
    with open(os.path.join(GOLDEN, "decimal_kats.json")) as f:
        return json.load(f)["cases"]


def dec_input(kind, values):
    """The engine's input column for unscaled DECIMAL values: int64 (SUM_DEC / AVG_DEC) or 16-byte (the *128 kinds)."""
    if kind.endswith("128"):
        return A.dec128_column(values)
    return np.array(values, np.int64)


def replay_decimal_kat(case, make_engine):
    """One key, one Table tumbling window holding the case's inputs; the fired value must be the expected one."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000,
                        aggs=[("COUNT", 0), (case["agg"], 0, case["scale"])])
    eng = make_engine(cfg)
    n = len(case["inputs"])
    eng.push(np.full(n, 7, np.int64), np.arange(n, dtype=np.int64), [dec_input(case["agg"], case["inputs"])])
    rows = eng.advance_watermark(A.LONG_MAX)
    assert len(rows["key"]) == 1 and int(rows["agg0"][0]) == n, case["name"]
    assert rows.get("null1") is None or not rows["null1"][0], case["name"]
    assert int(rows["agg1"][0]) == case["expected"], "%s: %s != %s" % (case["name"], rows["agg1"][0], case["expected"])
    eng.close()


def assert_rows_equal(a, b, names, rtol=None, ctx=""):
    """Multiset equality of two fired-row dicts. Integer columns bit-exact; float columns within rtol
    (relative, with the same absolute floor) when rtol is given, else exact."""
    n = len(a["key"])
    if n != len(b["key"]):                                 # name the (key, window) pairs only one side has
        ka = {(int(k), int(s), int(e)) for k, s, e in zip(a["key"], a["win_start"], a["win_end"])}
        kb = {(int(k), int(s), int(e)) for k, s, e in zip(b["key"], b["win_start"], b["win_end"])}
        raise AssertionError("%s row count %d != %d; only first: %s; only second: %s" %
                             (ctx, n, len(b["key"]), sorted(ka - kb)[:8], sorted(kb - ka)[:8]))
    if n == 0:
        return
    oa = np.lexsort((a["win_end"], a["win_start"], a["key"]))
    ob = np.lexsort((b["win_end"], b["win_start"], b["key"]))
    for f in ("key", "win_start", "win_end"):
        assert np.array_equal(a[f][oa], b[f][ob]), "%s column %s differs" % (ctx, f)
    for j, name in enumerate(names):
        x = a["agg%d" % j][oa]
        y = b["agg%d" % j][ob]
        na_, nb_ = a.get("null%d" % j), b.get("null%d" % j)
        if na_ is not None or nb_ is not None:           # SQL NULL results: same rows NULL, values compared elsewhere
            na_ = np.zeros(n, np.uint8) if na_ is None else na_[oa]
            nb_ = np.zeros(n, np.uint8) if nb_ is None else nb_[ob]
            assert np.array_equal(na_ != 0, nb_ != 0), "%s agg %s NULL flags differ" % (ctx, name)
            keep = nb_ == 0
            x, y = x[keep], y[keep]
        if x.dtype.kind == "f" and rtol is not None:
            tol = rtol(name) if callable(rtol) else rtol
            assert np.allclose(x, y, rtol=tol, atol=tol), "%s agg %s max rel err %g" % (
                ctx, name, np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-30)))
        else:
            bad = np.nonzero(x != y)[0]
            assert len(bad) == 0, "%s agg %s differs at %d rows, first %s vs %s" % (
                ctx, name, len(bad), x[bad[0]], y[bad[0]])


# ---- DataStream built-in reductions (WindowedStream.sum / min / max / minBy / maxBy over a Tuple4(key, Integer,
# Double, Long) -- tests/golden/gen_pyflink_reduce_kats.py): value columns f1 (int32), f2 (float64), f3 (int64)
REDUCE_FIELD_TYPES = ("I32", "F64", "I64")


def reduce_aggs(op, pos, types=REDUCE_FIELD_TYPES):
    """The engine aggregate list for <op>(pos) over fields 1..len(types) (column = field - 1)."""
    from flink_amd.operators import reduction_aggs
    return reduction_aggs(op, pos, types)


def load_reduce_kats():
    with open(os.path.join(GOLDEN, "pyflink_reduce_kats.json")) as f:
        return json.load(f)


def reduce_field_values(rows, names, types=REDUCE_FIELD_TYPES):
    """Fired rows -> list of (key, start, end, f1, f2, f3) with each field in its Python type (raw FIRST_/SEL_ bits
    viewed as the field's type)."""
    cols = []
    for j, t in enumerate(types):
        a = np.asarray(rows["agg%d" % j])
        dt = {"I32": np.int32, "I64": np.int64, "F64": np.float64, "F32": np.float32}[t]
        cols.append(a.view(dt) if a.dtype.itemsize == np.dtype(dt).itemsize else a.astype(dt))
    out = []
    for i in range(len(rows["key"])):
        out.append((int(rows["key"][i]), int(rows["win_start"][i]), int(rows["win_end"][i])) +
                   tuple(float(c[i]) if c.dtype.kind == "f" else int(c[i]) for c in cols))
    return sorted(out)


def replay_reduce_kat(case, make_engine):
    """Feed a reduce KAT through an engine built with the case's reduction; every watermark's rows must match."""
    import flink_amd._abi as A
    spec = case["spec"]
    kw = dict(window_kind=spec["window_kind"], size_ms=spec["size_ms"], offset_ms=spec["offset_ms"])
    if spec["window_kind"] == "SLIDE":
        kw["slide_ms"] = spec["slide_ms"]
    kw["allowed_lateness_ms"] = spec.get("allowed_lateness_ms", 0)
    cfg = A.make_config(aggs=reduce_aggs(case["op"], case["pos"]), reduce=True, **kw)
    names = A.agg_names(cfg)
    eng = make_engine(cfg)
    dropped, pend = 0, []

    def flush():
        nonlocal dropped, pend
        if pend:
            k = np.array([p[1] for p in pend], np.int64)
            cols = [np.array([p[2] for p in pend], np.int32), np.array([p[3] for p in pend], np.float64),
                    np.array([p[4] for p in pend], np.int64)]
            dropped += eng.push(k, np.array([p[5] for p in pend], np.int64), cols)
            pend = []

    for ev in case["events"]:
        if ev[0] == "e":
            pend.append(ev)
        else:
            flush()
            got = reduce_field_values(eng.advance_watermark(ev[1]), names)
            exp = sorted(tuple(r) for r in ev[2])
            assert got == exp, "%s: wm=%d expected %s got %s" % (case["name"], ev[1], exp, got)
    flush()
    assert dropped == case["late_dropped"], "%s: late dropped %d != %d" % (case["name"], dropped, case["late_dropped"])
    eng.close()
