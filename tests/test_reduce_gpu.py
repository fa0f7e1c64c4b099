"""DataStream built-in reductions on the GPU (FWA_CFG_REDUCE: WindowedStream.sum / min / max / minBy / maxBy,
WindowedStream.java:680-890): the reference's own Python WindowOperator sequences (tests/golden/
gen_pyflink_reduce_kats.py), random streams against the oracle's arrival-order fold (every field of the reduced tuple,
bit-exact except Double / Float sums, whose device order differs: relative 1e-9 / 2e-4 as SUM_F64 / SUM_F32 elsewhere),
ties in both directions, allowed lateness (late firings of the reduced element, in arrival order), and Java's
wrap-around and compareTo order."""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import load_reduce_kats, reduce_aggs, reduce_field_values, replay_reduce_kat

pytestmark = pytest.mark.gpu
KATS = load_reduce_kats()


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("case", KATS["cases"], ids=lambda c: c["name"].split(" ", 1)[1])
def test_reference_reduce_sequences_on_gpu(eng_mod, case):
    replay_reduce_kat(case, eng_mod.WindowAggregator)


def _stream(seed, n, nkeys, span, ties):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    keys[rng.random(n) < 0.002] = -2**63                  # the key-table sentinel is a legal key
    ts = np.sort(rng.integers(0, span, n)).astype(np.int64) - rng.integers(0, 800, n)
    late = rng.random(n) < 0.02
    ts[late] -= rng.integers(800, 3000, late.sum())
    f1 = (rng.integers(-4, 4, n) if ties else rng.integers(-2**31, 2**31 - 1, n)).astype(np.int32)
    f2 = (rng.integers(-4, 4, n) * 0.5 if ties else rng.standard_normal(n) * 1e3).astype(np.float64)
    f3 = (rng.integers(-4, 4, n) if ties else rng.integers(-2**62, 2**62, n)).astype(np.int64)
    return keys, ts, [f1, f2, f3]


def _close(a, b, names):
    assert len(a) == len(b), (len(a), len(b))
    for x, y in zip(a, b):
        assert x[:3] == y[:3]
        for j, (u, v) in enumerate(zip(x[3:], y[3:])):
            if names[j] in ("SUM_F64",):
                assert abs(u - v) <= 1e-9 * max(1.0, abs(v)), (x, y)
            elif names[j] in ("SUM_F32",):   # the reference adds in float, in order; the engine in double, rounded once
                assert abs(u - v) <= 1e-4 * max(1.0, abs(v)), (x, y)
            else:
                assert u == v or (u != u and v != v), (x, y)


@pytest.mark.parametrize("ties", [False, True], ids=["distinct", "ties"])
@pytest.mark.parametrize("by_last", [False, True], ids=["first", "last"])
@pytest.mark.parametrize("op,pos", [("sum", 1), ("sum", 2), ("sum", 3), ("min", 2), ("max", 3), ("min", 1),
                                    ("min_by", 2), ("max_by", 1), ("min_by", 3), ("max_by", 2)])
@pytest.mark.parametrize("win", [dict(window_kind="TUMBLE", size_ms=1000),
                                 dict(window_kind="SLIDE", size_ms=3000, slide_ms=1000, offset_ms=300),
                                 dict(window_kind="TUMBLE", size_ms=1000, allowed_lateness_ms=1500),
                                 dict(window_kind="SLIDE", size_ms=3000, slide_ms=1000, offset_ms=300,
                                      allowed_lateness_ms=2000)],
                         ids=["tumble", "slide", "tumble_late", "slide_late"])
def test_random_reductions_vs_oracle(eng_mod, win, op, pos, by_last, ties):
    from oracle.oracle import Oracle
    if by_last and not op.endswith("_by"):
        pytest.skip("the tie rule applies to minBy / maxBy")
    cfg = A.make_config(aggs=reduce_aggs(op, pos), reduce=True, by_last=by_last, key_capacity=4096, **win)
    names = A.agg_names(cfg)
    keys, ts, cols = _stream(7 + pos, 30_000, 500, 40_000, ties)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    nb, mx = 8, -2**63
    for b in range(nb + 1):
        sl = slice(b * len(keys) // nb, (b + 1) * len(keys) // nb) if b < nb else slice(0, 0)
        c = [x[sl] for x in cols]
        assert g.push(keys[sl], ts[sl], c) == o.push(keys[sl], ts[sl], c)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 801 if b < nb else A.LONG_MAX
        _close(reduce_field_values(g.advance_watermark(wm), names), reduce_field_values(o.advance_watermark(wm), names),
               names)
    g.close()
    o.close()


def test_java_semantics_on_gpu(eng_mod):
    """int / long wrap-around sums, Double.compareTo (-0.0 < 0.0, NaN greatest) and both tie rules, one window."""
    from oracle.oracle import Oracle
    d = np.array([0.0, -0.0, np.inf, np.nan, -0.0, np.nan, 2.0])
    cols = [np.array([2**31 - 1, 1, 5, 7, -3, 2, 9], np.int32), d, np.array([2**63 - 1, 1, 2, 3, 4, 5, 6], np.int64)]
    for aggs, last in (([("SUM_I32", 0), ("FIRST_64", 1), ("SUM_I64", 2)], False),
                       ([("SEL_32", 0), ("MINBY_F64", 1), ("SEL_64", 2)], False),
                       ([("SEL_32", 0), ("MINBY_F64", 1), ("SEL_64", 2)], True),
                       ([("SEL_32", 0), ("MAXBY_F64", 1), ("SEL_64", 2)], False),
                       ([("FIRST_32", 0), ("MIN_F64", 1), ("FIRST_64", 2)], False),
                       ([("FIRST_32", 0), ("MAX_F64", 1), ("FIRST_64", 2)], False)):
        cfg = A.make_config(window_kind="TUMBLE", size_ms=100, aggs=aggs, reduce=True, by_last=last)
        names = A.agg_names(cfg)
        k = np.full(7, 3, np.int64)
        t = np.arange(7, dtype=np.int64)
        rows = []
        for mk in (eng_mod.WindowAggregator, Oracle):
            h = mk(cfg)
            h.push(k[:3], t[:3], [c[:3] for c in cols])          # two pushes: selections survive across pushes
            h.push(k[3:], t[3:], [c[3:] for c in cols])
            r = h.advance_watermark(A.LONG_MAX)
            rows.append([tuple(np.asarray(r["agg%d" % j]).view(np.int64 if np.asarray(r["agg%d" % j]).itemsize == 8
                                                                else np.int32)[0] for j in range(3))])
            h.close()
        assert rows[0] == rows[1], (aggs, last, rows)


def test_reduce_handle_refusals(eng_mod):
    for kw in (dict(window_kind="SESSION", gap_ms=10, size_ms=0),):
        with pytest.raises(eng_mod.EngineError) as ei:
            eng_mod.WindowAggregator(A.make_config(aggs=[("SUM_I64", 0), ("FIRST_64", 1)], reduce=True, **kw))
        assert ei.value.code == -7
    g = eng_mod.WindowAggregator(A.make_config(aggs=[("SUM_I64", 0), ("FIRST_64", 1)], reduce=True))
    with pytest.raises(eng_mod.EngineError):
        g.drain_partials(0)                           # two-phase partials: the selection is not a partial aggregate
    with pytest.raises(eng_mod.EngineError):
        g.snapshot_heap()                             # heap layout: the shim writes the reduced tuple itself
    g.close()


@pytest.mark.parametrize("op,pos,by_last", [("sum", 2, False), ("min_by", 2, False), ("max_by", 1, True), ("min", 3, False)])
@pytest.mark.parametrize("win", [dict(window_kind="TUMBLE", size_ms=1000),
                                 dict(window_kind="SLIDE", size_ms=3000, slide_ms=1000),
                                 dict(window_kind="SLIDE", size_ms=3000, slide_ms=1000, allowed_lateness_ms=2000)],
                         ids=["tumble", "slide", "slide_late"])
def test_reduction_snapshot_restore_rescale(eng_mod, win, op, pos, by_last):
    """fwa_snapshot / fwa_restore of a reduction mid-stream, 1 subtask -> 2 subtasks (key-group halves) and back into
    one: every later watermark's rows equal an uninterrupted oracle run (the restored elements are pushed back in their
    original arrival order, so first-element and tie rules hold across the restore)."""
    from oracle.oracle import Oracle
    kw = dict(aggs=reduce_aggs(op, pos), reduce=True, by_last=by_last, key_capacity=4096, **win)
    cfg = A.make_config(**kw)
    names = A.agg_names(cfg)
    keys, ts, cols = _stream(31 + pos, 20_000, 300, 30_000, True)
    o = Oracle(cfg)
    g = eng_mod.WindowAggregator(cfg)
    nb, mx, cut = 8, -2**63, 4
    subs = None
    for b in range(nb + 1):
        sl = slice(b * len(keys) // nb, (b + 1) * len(keys) // nb) if b < nb else slice(0, 0)
        c = [x[sl] for x in cols]
        if b == cut:                                  # checkpoint, rescale to two subtasks
            blob = g.snapshot()
            g.close()
            subs = []
            for lo, hi in ((0, 63), (64, 127)):
                h = eng_mod.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **kw))
                h.restore([blob])
                subs.append((h, lo, hi))
        o.push(keys[sl], ts[sl], c)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 801 if b < nb else A.LONG_MAX
        exp = reduce_field_values(o.advance_watermark(wm), names)
        if subs is None:
            g.push(keys[sl], ts[sl], c)
            got = reduce_field_values(g.advance_watermark(wm), names)
        else:
            kg, _ = eng_mod.key_groups(keys[sl], 128, 1) if len(keys[sl]) else (np.zeros(0, np.int32), None)
            kg = np.asarray(kg)
            got = []
            for h, lo, hi in subs:
                m = (kg >= lo) & (kg <= hi)
                h.push(keys[sl][m], ts[sl][m], [x[m] for x in c])
                got += reduce_field_values(h.advance_watermark(wm), names)
            got = sorted(got)
        _close(got, exp, names)
    for h, _, _ in subs:
        h.close()
    o.close()


@pytest.mark.parametrize("lateness", [0, 1500], ids=["no_lateness", "lateness"])
@pytest.mark.parametrize("kind,col", [("SUM_I64", 2), ("SUM_I32", 0), ("SUM_F64", 1), ("SUM_F32", 3), ("MIN_I64", 2),
                                      ("MAX_I32", 0), ("MIN_F64", 1), ("MAX_F32", 3), ("MINBY_I64", 2),
                                      ("MAXBY_F64", 1), ("MAXBY_I32", 0), ("MINBY_F32", 3)])
def test_session_reductions_vs_oracle(eng_mod, kind, col, lateness):
    """Session windows over Tuple2<key, f1> reductions (sum / min / max / minBy / maxBy of the one value field): merging
    sessions cannot choose among other fields there, so the reference's result does not depend on its HashSet merge
    order. Ties and -0.0 / NaN-free values; late records take the arrival-order path."""
    from oracle.oracle import Oracle
    keys, ts, cols = _stream(101 + col, 30_000, 500, 40_000, True)
    cols = cols + [(cols[1] * 3).astype(np.float32)]
    cfg = A.make_config(window_kind="SESSION", gap_ms=500, size_ms=0, aggs=[(kind, col)], reduce=True,
                        allowed_lateness_ms=lateness, key_capacity=4096)
    names = A.agg_names(cfg)
    ty = [("I32", "F64", "I64", "F32")[col]]
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    nb, mx = 8, -2**63
    for b in range(nb + 1):
        sl = slice(b * len(keys) // nb, (b + 1) * len(keys) // nb) if b < nb else slice(0, 0)
        c = [x[sl] for x in cols]
        assert g.push(keys[sl], ts[sl], c) == o.push(keys[sl], ts[sl], c)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 801 if b < nb else A.LONG_MAX
        _close(reduce_field_values(g.advance_watermark(wm), names, ty), reduce_field_values(o.advance_watermark(wm), names, ty),
               names)
    g.close()
    o.close()


def test_session_reduction_scope(eng_mod):
    """A session reduction with more than the reduced field is refused (its other fields would follow the reference's
    HashSet merge order); Tuple2 reductions are accepted."""
    with pytest.raises(eng_mod.EngineError) as ei:
        eng_mod.WindowAggregator(A.make_config(window_kind="SESSION", gap_ms=10, size_ms=0, reduce=True,
                                               aggs=[("SUM_I64", 0), ("FIRST_64", 1)]))
    assert ei.value.code == -7
    eng_mod.WindowAggregator(A.make_config(window_kind="SESSION", gap_ms=10, size_ms=0, reduce=True,
                                           aggs=[("MAXBY_I64", 0)])).close()


@pytest.mark.parametrize("route", [0, 8], ids=["s5_hash_route", "s4_probe_route"])
@pytest.mark.parametrize("kind,col", [("SUM_I64", 2), ("MIN_I32", 0), ("MAXBY_F64", 1), ("SUM_F32", 3)])
def test_session_reduction_cell_preagg_vs_oracle(eng_mod, kind, col, route):
    """In-order session reductions take the cell pre-aggregation path (FWA_OPT_SESSION_PATH 2) on both of its routes;
    sessions stay in flight across pushes and merge with the next push's cells."""
    from oracle.oracle import Oracle
    rng = np.random.default_rng(300 + col)
    n, nb = 200_000, 12
    keys = rng.integers(0, 3000, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 600_000, n)).astype(np.int64) - rng.integers(0, 301, n)
    cols = [rng.integers(-50, 50, n).astype(np.int32), rng.standard_normal(n) * 10, rng.integers(-2**40, 2**40, n),
            (rng.standard_normal(n) * 10).astype(np.float32)]
    cfg = A.make_config(window_kind="SESSION", gap_ms=5000, size_ms=0, aggs=[(kind, col)], reduce=True,
                        key_capacity=8192)
    names, ty = A.agg_names(cfg), [("I32", "F64", "I64", "F32")[col]]
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    if route:
        g.set_option("ingest_variant", route)
    paths, mx = [], -2**63
    for b in range(nb + 1):
        sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
        c = [x[sl] for x in cols]
        assert g.push(keys[sl], ts[sl], c) == o.push(keys[sl], ts[sl], c)
        if b < nb:
            paths.append(g.get_option("session_path"))
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 301 if b < nb else A.LONG_MAX
        _close(reduce_field_values(g.advance_watermark(wm), names, ty), reduce_field_values(o.advance_watermark(wm), names, ty),
               names)
    assert paths == [2] * nb
    g.close()
    o.close()


@pytest.mark.parametrize("lateness", [0, 1500], ids=["no_lateness", "lateness"])
@pytest.mark.parametrize("kind,col", [("SUM_I64", 2), ("MIN_I32", 0), ("MAXBY_F64", 1), ("MINBY_F32", 3)])
def test_session_reduction_snapshot_restore_rescale(eng_mod, kind, col, lateness):
    """A session reduction checkpointed mid-stream (fwa_snapshot: its in-flight sessions) and restored into two subtasks
    (key-group halves): every later watermark's rows equal an uninterrupted oracle run."""
    from oracle.oracle import Oracle
    keys, ts, cols = _stream(61 + col, 20_000, 300, 30_000, False)
    cols = cols + [(cols[1] * 3).astype(np.float32)]
    kw = dict(window_kind="SESSION", gap_ms=500, size_ms=0, aggs=[(kind, col)], reduce=True,
              allowed_lateness_ms=lateness, key_capacity=4096)
    cfg = A.make_config(**kw)
    names, ty = A.agg_names(cfg), [("I32", "F64", "I64", "F32")[col]]
    o, g = Oracle(cfg), eng_mod.WindowAggregator(cfg)
    nb, mx, cut, subs = 8, -2**63, 4, None
    for b in range(nb + 1):
        sl = slice(b * len(keys) // nb, (b + 1) * len(keys) // nb) if b < nb else slice(0, 0)
        c = [x[sl] for x in cols]
        if b == cut:
            blob = g.snapshot()
            g.close()
            subs = []
            for lo, hi in ((0, 63), (64, 127)):
                h = eng_mod.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **kw))
                h.restore([blob])
                subs.append((h, lo, hi))
        o.push(keys[sl], ts[sl], c)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 801 if b < nb else A.LONG_MAX
        exp = reduce_field_values(o.advance_watermark(wm), names, ty)
        if subs is None:
            g.push(keys[sl], ts[sl], c)
            got = reduce_field_values(g.advance_watermark(wm), names, ty)
        else:
            kg, _ = eng_mod.key_groups(keys[sl], 128, 1) if len(keys[sl]) else (np.zeros(0, np.int32), None)
            kg = np.asarray(kg)
            got = []
            for h, lo, hi in subs:
                m = (kg >= lo) & (kg <= hi)
                h.push(keys[sl][m], ts[sl][m], [x[m] for x in c])
                got += reduce_field_values(h.advance_watermark(wm), names, ty)
            got = sorted(got)
        _close(got, exp, names)
    for h, _, _ in subs:
        h.close()
    o.close()
