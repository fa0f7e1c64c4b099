"""GPU tests: keyed window state in Flink's heap-backend byte layout (fwa_snapshot_heap / fwa_restore_heap).

The bytes are read back with tests/heap_reader.py -- the Python restatement of the reference's readers that
tests/test_heap_reference_cpu.py pins against checkpoints the reference itself wrote
(win-op-migration-test-*-flink1.18-snapshot): per key group (HeapSnapshotStrategy.java:154-175) int keyGroupId, then
one section per registered state (window contents, [merging-window-set], processing timers, event timers) with the
ids a heap backend gives them -- and compared with the engine's FWASNAP1 snapshot of the same handle; then a restore
from the heap bytes (with rescaling) must resume exactly like the oracle's uninterrupted run
(EventTimeWindowCheckpointingITCase.java:759-810).
"""
import struct

import numpy as np
import pytest

import heap_reader as H
from flink_amd import _abi as A
from flink_amd import snapshot as S
from helpers import assert_rows_equal, load_tz_kats
from test_gpu_parity import random_stream

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_F64", 2), ("AVG_F64", 2)]


def parse_heap(body, offs, ds, naggs, sess=False, nh=0, first_kg=0):
    """(key group -> [(key, start, end, acc fields[, null flags])], timers, merging sets) via the reader pinned by
    the reference's own snapshots (tests/heap_reader.py, tests/test_heap_reference_cpu.py)"""
    ents, timers, msets = H.parse_engine_heap(body, offs, ds, naggs + nh, sess, first_kg)
    return ({kg: [(k, st, en, acc) for k, st, en, acc, _ in v] for kg, v in ents.items()}, timers, msets,
            {kg: [nl for *_, nl in v] for kg, v in ents.items()})


def s64(x):
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= 1 << 63 else x


def to_engine_words(acc, kinds):
    """ACC fields back to the engine's words: ord keys for MIN / MAX"""
    enc = []
    for j, k in enumerate(kinds):
        x = acc[1 + j] & 0xFFFFFFFFFFFFFFFF
        if k in (4, 5):
            x ^= 1 << 63
        elif 6 <= k <= 9:
            x = (~x & 0xFFFFFFFFFFFFFFFF) if x >> 63 else x | (1 << 63)
        enc.append(s64(x))
    return enc


def merge_words(kind, x, y):
    if kind in (2, 3, 11, 12):
        return struct.unpack("<q", struct.pack("<d", struct.unpack("<d", struct.pack("<q", x))[0]
                                                + struct.unpack("<d", struct.pack("<q", y))[0]))[0]
    if kind in (4, 6, 8):
        return x if (x & 0xFFFFFFFFFFFFFFFF) <= (y & 0xFFFFFFFFFFFFFFFF) else y
    if kind in (5, 7, 9):
        return x if (x & 0xFFFFFFFFFFFFFFFF) >= (y & 0xFFFFFFFFFFFFFFFF) else y
    return s64(x + y)


TZ = {c["zone"]: c["tz"] for c in load_tz_kats()["timer"]}
NULL_AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("COUNT_COL", 2), ("MAX_F64", 2), ("AVG_F64", 2),
             ("SUM_F32", 1)]

CASES = {
    "ds_tumble": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=5000),
    "ds_tumble_late": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=5000, allowed_lateness_ms=3000),
    "ds_session": dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700),
    "ds_session_late": dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700, allowed_lateness_ms=1500),
    "table_tumble": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000),
    "table_hop": dict(window_kind="SLIDE", semantics="TABLE", size_ms=15000, slide_ms=5000),
    "table_cumulate": dict(window_kind="CUMULATE", semantics="TABLE", size_ms=20000, slide_ms=5000),
    # SQL NULLs: NULL bits in the accumulator row + one BIGINT per hidden non-NULL counter
    "table_tumble_null": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000, nullable_cols=(0, 1, 2)),
    "table_hop_null": dict(window_kind="SLIDE", semantics="TABLE", size_ms=15000, slide_ms=5000, nullable_cols=(0, 2)),
    # shift time zones: local slice ends, timers at toEpochMillsForTimer(end - 1)
    "table_tumble_tz": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000, tz=TZ["Asia/Shanghai"]),
    "table_cumulate_tz": dict(window_kind="CUMULATE", semantics="TABLE", size_ms=20000, slide_ms=5000,
                              tz=TZ["America/Los_Angeles"]),
    # DataStream sliding windows: per-window state (SlidingEventTimeWindows), from the engine's slices
    "ds_slide": dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=15000, slide_ms=5000),
    "ds_slide_late_odd": dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=5000, slide_ms=2000, offset_ms=300,
                              allowed_lateness_ms=2500),
    # legacy Table WindowOperator (GROUP BY SESSION): session-window-mapping + window-aggs
    "table_session": dict(window_kind="SESSION", semantics="TABLE", gap_ms=700),
    "table_session_null": dict(window_kind="SESSION", semantics="TABLE", gap_ms=700, nullable_cols=(0, 1, 2)),
    "table_session_tz": dict(window_kind="SESSION", semantics="TABLE", gap_ms=700, tz=TZ["Asia/Shanghai"]),
}


def aggs_of(case):
    return NULL_AGGS if "nullable_cols" in CASES[case] else AGGS


def nhid(case):
    cols = CASES[case].get("nullable_cols", ())
    return len({col for kind, col in aggs_of(case) if kind != "COUNT" and col in cols})


def make_cfg(case, **kw):
    c = dict(CASES[case])
    ds = c["semantics"] == "DATASTREAM"
    return A.make_config(aggs=aggs_of(case), key_capacity=4096, key_kind=A.KEY_JAVA_LONG if ds else A.KEY_BINROW_BIGINT,
                         **c, **kw)


def tz_timer(case, x):
    """toEpochMillsForTimer through the oracle's restatement (TimeWindowUtil.java:67-100); UTC: x"""
    if "tz" not in CASES[case]:
        return x
    from oracle import oracle as O
    cfg = make_cfg(case)
    return O.lib().or_tz_timer(cfg, x)


def stream_of(case, seed, n, nkeys, span, delay):
    keys, ts, vi, vf, vd = random_stream(seed, n, nkeys, span, delay)
    nulls = None
    if "nullable_cols" in CASES[case]:
        rng = np.random.default_rng(seed)
        nulls = [(rng.random(n) < 0.3).astype(np.uint8) for _ in range(3)]
        nulls[2] |= (keys % 7 == 0).astype(np.uint8)       # keys whose column 2 is always NULL: NULL results
    return keys, ts, [vi, vf, vd], nulls


def push(g, keys, ts, cols, nulls, m=slice(None)):
    if nulls is None:
        return g.push(keys[m], ts[m], [c[m] for c in cols])
    return g.push(keys[m], ts[m], [c[m] for c in cols], nulls=[z[m] for z in nulls])


def expected_state(case, snap, kg, wm):
    """(key, start, count, acc words..., hidden counters...) the heap bytes must hold for key group kg: the engine's
    entries, with a CUMULATE window's fired slices folded into its first slice (SliceSharedWindowAggProcessor.merge)"""
    c = CASES[case]
    sl = S.entries_of_key_group(snap, kg)
    rows = list(zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist(), snap["count"][sl].tolist(),
                    *[a[sl].tolist() for a in snap["acc"]], *[h[sl].tolist() for h in snap["hidden"]]))
    if c["semantics"] == "DATASTREAM" and c["window_kind"] == "SLIDE":
        # WindowOperator's per-window state: the merge of the slices inside each window that is not past cleanup
        size, slide, off, late = c["size_ms"], c["slide_ms"], c.get("offset_ms", 0), c.get("allowed_lateness_ms", 0)
        kinds = [A.AGG_KINDS[a] for a, _ in aggs_of(case)]
        win = {}
        for r in rows:
            st = r[1] - (r[1] - off) % slide
            while st > r[1] - size:
                if wm == A.LONG_MIN or st + size - 1 + late > wm:
                    w = win.get((r[0], st))
                    win[(r[0], st)] = list(r[2:]) if w is None else [w[0] + r[2]] + [
                        merge_words(k, w[1 + j], r[3 + j]) for j, k in enumerate(kinds)]
                st -= slide
        return sorted((k, st, *w) for (k, st), w in win.items() if w[0] > 0)
    if c["window_kind"] != "CUMULATE":
        return sorted(rows)
    step, size = c["slide_ms"], c["size_ms"]
    kinds = [A.AGG_KINDS[a] for a, _ in aggs_of(case)]
    nh = len(snap["hidden"])
    first, keep = {}, []
    for r in sorted(rows):
        if tz_timer(case, r[1] + step - 1) > wm:
            keep.append(r)
            continue
        ws = (r[1] // size) * size
        if (r[0], ws) not in first:
            first[(r[0], ws)] = (r[0], ws) + tuple(r[2:])
        else:
            f = first[(r[0], ws)]
            na = len(kinds)
            first[(r[0], ws)] = ((r[0], ws, f[2] + r[2]) + tuple(merge_words(k, f[3 + j], r[3 + j])
                                                                 for j, k in enumerate(kinds))
                                 + tuple(f[3 + na + h] + r[3 + na + h] for h in range(nh)))
    return sorted(list(first.values()) + keep)


IDENT = {4: -1, 6: -1, 8: -1}       # MIN kinds: an all-NULL aggregate's accumulator word (~0)


@pytest.mark.parametrize("case", list(CASES))
def test_heap_bytes_match_engine_state(case):
    from flink_amd import engine
    cfg = make_cfg(case)
    c = CASES[case]
    ds, sess = c["semantics"] == "DATASTREAM", c["window_kind"] == "SESSION"
    lateness = c.get("allowed_lateness_ms", 0)
    aggs = aggs_of(case)
    nh = nhid(case)
    g = engine.WindowAggregator(cfg)
    keys, ts, cols, nulls = stream_of(case, 77, 30_000, 300, 40_000, 1000)
    push(g, keys, ts, cols, nulls)
    wm = int(ts.max()) - 6000 - 2500                 # mid-window for HOP / CUMULATE (fired and unfired slices)
    g.advance_watermark(wm)
    snap = S.parse(g.snapshot())
    body, offs, hwm = g.snapshot_heap()
    assert hwm == snap["watermark"] == wm and len(offs) == 128 and offs[0] == 0
    assert len(snap["hidden"]) == nh
    ents, timers, msets, nulls_of = parse_heap(body, offs, ds, len(aggs), sess, nh)
    assert sorted(ents) == list(range(128))
    for kg in range(128):                                      # KeyGroupRangeOffsets point at each section
        assert struct.unpack_from(">i", body, int(offs[kg]))[0] == kg
    kinds = [A.AGG_KINDS[a] for a, _ in aggs]
    width = {"TUMBLE": c.get("size_ms"), "SLIDE": c.get("size_ms") if ds else 5000, "CUMULATE": 5000}.get(c["window_kind"])
    n = nulled = 0
    for kg in range(128):
        got = []
        for (key, start, end, acc), nl in zip(ents[kg], nulls_of[kg]):
            start = end - width if start is None else start
            if not sess:
                assert end - start == width
            words = to_engine_words(acc, kinds)
            for j, k in enumerate(kinds):                      # a NULL aggregate <=> its hidden counter is 0
                if nh and nl[1 + j]:
                    nulled += 1
                    assert acc[1 + j] == 0
                    words[j] = IDENT.get(k, 0)
            got.append((s64(key), start, s64(acc[0]), *words, *[s64(x) for x in acc[1 + len(kinds):]]))
        exp = expected_state(case, snap, kg, wm)
        if ds and c["window_kind"] == "SLIDE":
            # a window merges several slices: floating sums are added in another order than the test's (tolerance)
            fl = [3 + j for j, k in enumerate(kinds) if k in (2, 3, 11, 12)]
            as_f = lambda w: struct.unpack("<d", struct.pack("<q", w))[0]   # noqa: E731
            strip = lambda rows: [tuple(x for i, x in enumerate(r) if i not in fl) for r in rows]   # noqa: E731
            g_, e_ = sorted(got), sorted(exp)
            assert strip(g_) == strip(e_), kg
            assert all(np.isclose(as_f(a[i]), as_f(b[i]), rtol=1e-12, atol=1e-12) for a, b in zip(g_, e_) for i in fl), kg
        else:
            assert sorted(got) == exp, kg
        n += len(got)
        if sess:                                               # every in-flight session maps to itself
            sl = S.entries_of_key_group(snap, kg)
            want = {}
            for k, st, en in zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist(),
                                 snap["window_end"][sl].tolist()):
                want.setdefault(k, []).append((st, en, st, en))
            assert {s64(k): sorted(v) for k, v in msets[kg].items()} == {k: sorted(v) for k, v in want.items()}
            ends = {(s64(e[0]), e[1]): e[2] for e in ents[kg]}
            assert all(ends[(s64(k), st)] == en for k, v in msets[kg].items() for st, en, _, _ in v)
        if sess and not ds:
            # legacy Table WindowOperator: trigger and cleanup timer coincide at toEpochMillsForTimer(maxTimestamp)
            want_t = {(tz_timer(case, e[2] - 1), s64(e[0]), e[1], e[2]) for e in ents[kg]}
            assert sorted((t[0], s64(t[1]), t[2], t[3]) for t in timers[kg]) == sorted(want_t)
        elif ds:
            # window.maxTimestamp() while unfired (EventTimeTrigger) + the cleanup time, per (key, window)
            want_t = set()
            for e in ents[kg]:
                if e[2] - 1 > wm:
                    want_t.add((e[2] - 1, s64(e[0]), e[1], e[2]))
                want_t.add((e[2] - 1 + lateness, s64(e[0]), e[1], e[2]))
            assert sorted((t[0], s64(t[1]), t[2], t[3]) for t in timers[kg]) == sorted(want_t)
        else:
            # the first unfired window end of each live slice, at toEpochMillsForTimer(end - 1)
            # (AbstractWindowAggProcessor.processElement :160-164 / SliceSharedWindowAggProcessor.fireWindow :76-84)
            sl = S.entries_of_key_group(snap, kg)
            want_t = set()
            for k, st in zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist()):
                we = st + width
                if c["window_kind"] == "SLIDE":
                    we = -(-we // c["slide_ms"]) * c["slide_ms"]
                while tz_timer(case, we - 1) <= wm:
                    we += c["slide_ms"] if c["window_kind"] == "SLIDE" else width
                want_t.add((tz_timer(case, we - 1), k, we))
            assert sorted((t[0], s64(t[1]), t[2]) for t in timers[kg]) == sorted(want_t)
    assert n > 0
    if nh:
        assert nulled > 0                                      # the stream makes some aggregates NULL
    if CASES[case]["window_kind"] == "CUMULATE":
        assert n < snap["n"]                                   # some fired slices were folded
    elif not (ds and CASES[case]["window_kind"] == "SLIDE"):
        assert n == snap["n"]
    g.close()


def test_heap_timers_after_fire_before_cleanup():
    """DataStream with allowed lateness: a window that fired but is not past cleanup keeps its state and only its
    cleanup timer (EventTimeTrigger keeps no timer for a fired window; WindowOperator.registerCleanupTimer)."""
    from flink_amd import engine
    cfg = make_cfg("ds_tumble_late")
    g = engine.WindowAggregator(cfg)
    keys = np.array([1, 2, 1], np.int64)
    ts = np.array([100, 200, 5100], np.int64)
    g.push(keys, ts, [keys, keys.astype(np.float32), keys.astype(np.float64)])
    rows = g.advance_watermark(5500)                           # [0, 5000) fired, cleanup at 4999 + 3000 = 7999
    assert sorted(rows["key"].tolist()) == [1, 2]
    body, offs, wm = g.snapshot_heap()
    ents, timers, _, _ = parse_heap(body, offs, True, len(AGGS))
    allt = sorted((t[0], s64(t[1]), t[2], t[3]) for kg in timers for t in timers[kg])
    assert allt == [(4999 + 3000, 1, 0, 5000), (4999 + 3000, 2, 0, 5000), (9999, 1, 5000, 10000),
                    (9999 + 3000, 1, 5000, 10000)]
    g.close()


def write_session_body(ents, msets, timers, naggs):
    """Re-serialise a parsed session heap body (the writer side of parse_heap): ids 0 window-contents,
    1 merging-window-set, 2 processing timers, 3 event timers."""
    out = bytearray()
    for kg in sorted(ents):
        out += struct.pack(">ihi", kg, 0, len(ents[kg]))
        for key, start, end, acc in ents[kg]:
            out += struct.pack(">qqq", start, end, s64(key)) + b"".join(struct.pack(">Q", a) for a in acc)
        out += struct.pack(">hi", 1, len(msets[kg]))
        for key, pairs in msets[kg].items():
            out += struct.pack(">bqi", 0, s64(key), len(pairs))
            for p in pairs:
                out += struct.pack(">qqqq", *p)
        out += struct.pack(">hi", 2, 0)
        out += struct.pack(">hi", 3, len(timers[kg]))
        for t in timers[kg]:
            out += struct.pack(">Qqqq", (t[0] ^ (1 << 63)) & 0xFFFFFFFFFFFFFFFF, s64(t[1]), t[2], t[3])
    return bytes(out)


def offsets_of(body):
    """Section offsets of a re-serialised body (key groups in order, one section per state)."""
    offs, at = [], 0
    while at < len(body):
        offs.append(at)
        r = H.Reader(body, at)
        r.get(">i")
        for _ in range(4):
            sid, n = r.get(">h"), r.get(">i")
            for _ in range(n):
                if sid == 0:
                    r.get(">qqq"); [r.get(">Q") for _ in range(1 + len(AGGS))]
                elif sid == 1:
                    r.get(">bq")
                    for _ in range(r.get(">i")):
                        r.get(">qqqq")
                else:
                    r.get(">Qqqq")
        at = r.at
    return offs


@pytest.mark.parametrize("case", list(CASES))
def test_heap_restore_resumes_with_rescale(case):
    """Two subtasks (key groups [0,63], [64,127]) checkpoint in the heap layout; one subtask restores both
    (scale-in) and two subtasks restore one body each half (scale-out); rows equal the oracle's."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    cfg = make_cfg(case)
    kk = cfg.key_kind
    names = A.agg_names(cfg)
    keys, ts, cols, nulls = stream_of(case, 91, 40_000, 500, 60_000, 1000)
    cut = 20_000
    wm1 = int(ts[:cut].max()) - 1001 - 2500
    kgs, _ = engine.key_groups(keys, 128, 1, kk)
    o = Oracle(make_cfg(case))
    push(o, keys, ts, cols, nulls, slice(0, cut))
    first = o.advance_watermark(wm1)
    push(o, keys, ts, cols, nulls, slice(cut, None))
    final = o.advance_watermark(A.LONG_MAX)
    halves = [(0, 63), (64, 127)]
    bodies, wms, got1 = [], [], []
    rest = np.arange(cut, len(keys))
    head = np.arange(cut)
    for lo, hi in halves:
        m = head[(kgs[:cut] >= lo) & (kgs[:cut] <= hi)]
        g = engine.WindowAggregator(make_cfg(case, kg_start=lo, kg_end=hi))
        push(g, keys, ts, cols, nulls, m)
        got1.append(g.advance_watermark(wm1))
        b, offs, wm = g.snapshot_heap()
        assert len(offs) == hi - lo + 1
        bodies.append(b)
        wms.append(wm)
        g.close()
    tol = 1e-6 if "nullable_cols" in CASES[case] else 1e-9
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names, rtol=tol)
    if CASES[case]["window_kind"] == "SESSION" and CASES[case]["semantics"] == "DATASTREAM":
        # a run of the reference names an older window as a merged session's state namespace
        # (MergingWindowSet.addWindow :190-201): rename every state window and check the restore follows the mapping
        renamed = []
        for b, (lo, _) in zip(bodies, halves):
            ents, timers, msets, _ = parse_heap(b, offsets_of(b), True, len(AGGS), True, first_kg=lo)
            for kg in ents:
                ents[kg] = [(k, st - 7, st + 1, acc) for k, st, en, acc in ents[kg]]
                msets[kg] = {k: [(a, b_, a - 7, a + 1) for a, b_, _, _ in v] for k, v in msets[kg].items()}
            renamed.append(write_session_body(ents, msets, timers, len(AGGS)))
        variants = [bodies, renamed]
    else:
        variants = [bodies]
    for bl in variants:
        for layout in ([(0, 127)], [(0, 31), (32, 127)]):      # scale-in (1 subtask), then a new split (2)
            outs = []
            for lo, hi in layout:
                g = engine.WindowAggregator(make_cfg(case, kg_start=lo, kg_end=hi))
                g.restore_heap(bl, wms)
                m = rest[(kgs[cut:] >= lo) & (kgs[cut:] <= hi)]
                push(g, keys, ts, cols, nulls, m)
                outs.append(g.advance_watermark(A.LONG_MAX))
                g.close()
            assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, final, names, rtol=tol)


@pytest.mark.parametrize("kind", [dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000),
                                  dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=15000, slide_ms=5000)])
def test_heap_layout_unsupported_kinds(kind):
    """Host-computed key hashes (FWA_KEY_PREHASHED): the restore could not place a key in its key group."""
    from flink_amd import engine
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, key_capacity=64, key_kind=A.KEY_PREHASHED, **kind))
    with pytest.raises(engine.EngineError) as ei:
        g.snapshot_heap()
    assert A.STATUS[ei.value.code] == "E_UNSUPPORTED"
    g.close()


def test_restore_reference_reduce_snapshot():
    """Restore the window state of the reference's own checkpoint (win-op-migration-test-reduce-event-time-flink1.18
    -snapshot, WindowOperatorMigrationTest.java:366-440: tumbling 3 s, sum reducer over Tuple2<String, Integer>) into
    the engine and replay the reference's restore expectations (:494-507): watermark 2999 emits key1 -> 3 and
    key2 -> 3, 3999 and 4999 nothing, 5999 key2 -> 2. Adapter: String keys become Long ids (key1 -> 1, key2 -> 2; both
    land in key group 0 of the 1-key-group test harness, so maxParallelism 1 here), the reduced Integer field is
    a SUM(BIGINT) accumulator and COUNT(*) = 1 marks the window non-empty (the reduce state has no count)."""
    import os
    from flink_amd import engine
    f = os.path.join(os.path.dirname(__file__), "golden", "flink_snapshots",
                     "win-op-migration-test-reduce-event-time-flink1.18-snapshot")
    first, offs, data = H.read_operator_snapshot(open(f, "rb").read())[0]
    lay = {0: ("kv", H.ser_time_window, H.ser_string, H.ser_tuple(H.ser_string, H.ser_int)),
           1: ("pq", H.ser_string, H.ser_time_window), 2: ("pq", H.ser_string, H.ser_time_window)}
    sec = H.read_key_groups(data, offs, first, lay)[0]
    ids = {"key1": 1, "key2": 2}
    body = bytearray(struct.pack(">i", 0))
    body += struct.pack(">hi", 0, len(sec[0]))
    for (st, en), key, (_, v) in sec[0]:
        body += struct.pack(">qqqqqq", st, en, ids[key], 1, 1, v)   # ACC tuple: COUNT(*), COUNT, SUM
    body += struct.pack(">hi", 1, 0)
    body += struct.pack(">hi", 2, len(sec[2]))
    for ts_, key, (st, en) in sec[2]:
        body += struct.pack(">Qqqq", (ts_ ^ (1 << 63)) & 0xFFFFFFFFFFFFFFFF, ids[key], st, en)
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=3000, aggs=[("COUNT", 0), ("SUM_I64", 0)],
                        max_parallelism=1, key_capacity=64)
    g = engine.WindowAggregator(cfg)
    g.restore_heap([bytes(body)], [1999])                      # the harness's watermark at the snapshot
    out = {}
    for wm in (2999, 3999, 4999, 5999):
        r = g.advance_watermark(wm)
        out[wm] = sorted(zip(r["key"].tolist(), r["agg1"].tolist(), r["win_end"].tolist()))
    assert out == {2999: [(1, 3, 3000), (2, 3, 3000)], 3999: [], 4999: [], 5999: [(2, 2, 6000)]}
    g.close()
