"""GPU tests: keyed window state in Flink's heap-backend byte layout (fwa_snapshot_heap / fwa_restore_heap).

The bytes are read back by an independent Python restatement of the reference's readers -- per key group
(HeapSnapshotStrategy.java:154-175): int keyGroupId; short stateId, int n, n x (namespace, key, state)
(CopyOnWriteStateMapSnapshot.writeState :138-148); short stateId, int m, m x (flipSignBit(ts), key, namespace)
(TimerSerializer.serialize :147-152); TimeWindow.Serializer (long start, long end), LongSerializer, TupleSerializer
(big-endian), BinaryRowDataSerializer (int size + row, little-endian slots) -- and compared with the engine's
FWASNAP1 snapshot of the same handle; then a restore from the heap bytes (with rescaling) must resume exactly
like the oracle's uninterrupted run (EventTimeWindowCheckpointingITCase.java:759-810).
"""
import struct

import numpy as np
import pytest

from flink_amd import _abi as A
from flink_amd import snapshot as S
from helpers import assert_rows_equal
from test_gpu_parity import random_stream

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_F64", 2), ("AVG_F64", 2)]


class Reader:
    def __init__(self, b):
        self.b, self.at = b, 0

    def get(self, fmt):
        v = struct.unpack_from(fmt, self.b, self.at)
        self.at += struct.calcsize(fmt)
        return v[0] if len(v) == 1 else v

    def row(self, arity):
        size = self.get(">i")
        nb = ((arity + 63 + 8) // 64) * 8
        assert size == nb + 8 * arity
        hdr = self.b[self.at:self.at + nb]
        self.at += nb
        assert hdr[0] == 0 and not any(hdr[1:])               # RowKind INSERT, no NULLs
        return [self.get("<Q") for _ in range(arity)]


def parse_heap(body, ds, naggs, lateness=0, sess=False):
    """(key group -> [(key, start, end, acc fields)], timers, merging sets) -- sessions carry a third state, the
    merging-window-set (VoidNamespace byte, key, ListSerializer of (actual, state) TimeWindow pairs)"""
    r = Reader(body)
    out, timers, msets = {}, {}, {}
    while r.at < len(body):
        kg = r.get(">i")
        assert r.get(">h") == 0
        n = r.get(">i")
        ents = []
        for _ in range(n):
            if ds:
                start, end, key = r.get(">q"), r.get(">q"), r.get(">q")
                acc = [r.get(">Q") for _ in range(1 + naggs)]
            else:
                end = r.get(">q")
                key = r.row(1)[0]
                acc = r.row(1 + naggs)
                start = None
            ents.append((key, start, end, acc))
        if sess:
            assert r.get(">h") == 1
            ms = {}
            for _ in range(r.get(">i")):
                assert r.get(">b") == 0                               # VoidNamespaceSerializer
                key = r.get(">q")
                ms[key] = [tuple(r.get(">q") for _ in range(4)) for _ in range(r.get(">i"))]
            msets[kg] = ms
        assert r.get(">h") == (2 if sess else 1)
        m = r.get(">i")
        tl = []
        for _ in range(m):
            ts = r.get(">Q") ^ (1 << 63)
            ts = ts - (1 << 64) if ts >= 1 << 63 else ts
            if ds:
                tl.append((ts, r.get(">q"), r.get(">q"), r.get(">q")))
            else:
                tl.append((ts, r.row(1)[0], r.get(">q")))
        out[kg], timers[kg] = ents, tl
    return out, timers, msets


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


CASES = {
    "ds_tumble": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=5000),
    "ds_tumble_late": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=5000, allowed_lateness_ms=3000),
    "ds_session": dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700),
    "ds_session_late": dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700, allowed_lateness_ms=1500),
    "table_tumble": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000),
    "table_hop": dict(window_kind="SLIDE", semantics="TABLE", size_ms=15000, slide_ms=5000),
    "table_cumulate": dict(window_kind="CUMULATE", semantics="TABLE", size_ms=20000, slide_ms=5000),
}


def make_cfg(case, **kw):
    c = dict(CASES[case])
    ds = c["semantics"] == "DATASTREAM"
    return A.make_config(aggs=AGGS, key_capacity=4096, key_kind=A.KEY_JAVA_LONG if ds else A.KEY_BINROW_BIGINT,
                         **c, **kw)


def expected_state(case, snap, kg, wm):
    """(key, start, count, acc words...) the heap bytes must hold for key group kg: the engine's entries, with a
    CUMULATE window's fired slices folded into its first slice (SliceSharedWindowAggProcessor.merge)"""
    c = CASES[case]
    sl = S.entries_of_key_group(snap, kg)
    rows = list(zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist(), snap["count"][sl].tolist(),
                    *[a[sl].tolist() for a in snap["acc"]]))
    if c["window_kind"] != "CUMULATE":
        return sorted(rows)
    step, size = c["slide_ms"], c["size_ms"]
    kinds = [A.AGG_KINDS[a] for a, _ in AGGS]
    first, keep = {}, []
    for r in sorted(rows):
        if r[1] + step - 1 > wm:
            keep.append(r)
            continue
        ws = (r[1] // size) * size
        if (r[0], ws) not in first:
            first[(r[0], ws)] = (r[0], ws) + tuple(r[2:])
        else:
            f = first[(r[0], ws)]
            first[(r[0], ws)] = (r[0], ws, f[2] + r[2]) + tuple(merge_words(k, f[3 + j], r[3 + j])
                                                                 for j, k in enumerate(kinds))
    return sorted(list(first.values()) + keep)


@pytest.mark.parametrize("case", list(CASES))
def test_heap_bytes_match_engine_state(case):
    from flink_amd import engine
    cfg = make_cfg(case)
    c = CASES[case]
    ds, sess = c["semantics"] == "DATASTREAM", c["window_kind"] == "SESSION"
    lateness = c.get("allowed_lateness_ms", 0)
    g = engine.WindowAggregator(cfg)
    keys, ts, vi, vf, vd = random_stream(77, 30_000, 300, 40_000, 1000)
    g.push(keys, ts, [vi, vf, vd])
    wm = int(ts.max()) - 6000 - 2500                 # mid-window for HOP / CUMULATE (fired and unfired slices)
    g.advance_watermark(wm)
    snap = S.parse(g.snapshot())
    body, offs, hwm = g.snapshot_heap()
    assert hwm == snap["watermark"] == wm and len(offs) == 128 and offs[0] == 0
    ents, timers, msets = parse_heap(body, ds, len(AGGS), lateness, sess)
    assert sorted(ents) == list(range(128))
    for kg in range(128):                                      # KeyGroupRangeOffsets point at each section
        assert struct.unpack_from(">i", body, int(offs[kg]))[0] == kg
    kinds = [A.AGG_KINDS[a] for a, _ in AGGS]
    width = {"TUMBLE": c.get("size_ms"), "SLIDE": 5000, "CUMULATE": 5000}.get(c["window_kind"])
    n = 0
    for kg in range(128):
        got = []
        for key, start, end, acc in ents[kg]:
            start = end - width if start is None else start
            if not sess:
                assert end - start == width
            got.append((s64(key), start, s64(acc[0]), *to_engine_words(acc, kinds)))
        assert sorted(got) == expected_state(case, snap, kg, wm), kg
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
        if ds:
            # window.maxTimestamp() (+ the cleanup time with lateness), per (key, window)
            want_t = sorted({(e[2] - 1 + d, s64(e[0]), e[1], e[2]) for e in ents[kg]
                             for d in ([0, lateness] if lateness else [0])})
            assert sorted((t[0], s64(t[1]), t[2], t[3]) for t in timers[kg]) == want_t
        else:
            # the first unfired window end of each live slice, minus 1 (AbstractWindowAggProcessor.processElement
            # :160-164 / SliceSharedWindowAggProcessor.fireWindow :76-84), deduplicated per (key, window)
            sl = S.entries_of_key_group(snap, kg)
            want_t = set()
            for k, st in zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist()):
                we = st + width
                while we - 1 <= wm:
                    we += width
                want_t.add((we - 1, k, we))
            assert sorted((t[0], s64(t[1]), t[2]) for t in timers[kg]) == sorted(want_t)
    assert n > 0
    if CASES[case]["window_kind"] != "CUMULATE":
        assert n == snap["n"]
    else:
        assert n < snap["n"]                                   # some fired slices were folded
    g.close()


def write_session_body(ents, msets, timers, naggs):
    """Re-serialise a parsed session heap body (the writer side of parse_heap)."""
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
        out += struct.pack(">hi", 2, len(timers[kg]))
        for t in timers[kg]:
            out += struct.pack(">Qqqq", (t[0] ^ (1 << 63)) & 0xFFFFFFFFFFFFFFFF, s64(t[1]), t[2], t[3])
    return bytes(out)


@pytest.mark.parametrize("case", list(CASES))
def test_heap_restore_resumes_with_rescale(case):
    """Two subtasks (key groups [0,63], [64,127]) checkpoint in the heap layout; one subtask restores both
    (scale-in) and two subtasks restore one body each half (scale-out); rows equal the oracle's."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    cfg = make_cfg(case)
    kk = cfg.key_kind
    names = A.agg_names(cfg)
    keys, ts, vi, vf, vd = random_stream(91, 40_000, 500, 60_000, 1000)
    cut = 20_000
    wm1 = int(ts[:cut].max()) - 1001 - 2500
    kgs, _ = engine.key_groups(keys, 128, 1, kk)
    o = Oracle(make_cfg(case))
    o.push(keys[:cut], ts[:cut], [vi[:cut], vf[:cut], vd[:cut]])
    first = o.advance_watermark(wm1)
    o.push(keys[cut:], ts[cut:], [vi[cut:], vf[cut:], vd[cut:]])
    final = o.advance_watermark(A.LONG_MAX)
    halves = [(0, 63), (64, 127)]
    bodies, wms, got1 = [], [], []
    for lo, hi in halves:
        m = (kgs[:cut] >= lo) & (kgs[:cut] <= hi)
        g = engine.WindowAggregator(make_cfg(case, kg_start=lo, kg_end=hi))
        g.push(keys[:cut][m], ts[:cut][m], [vi[:cut][m], vf[:cut][m], vd[:cut][m]])
        got1.append(g.advance_watermark(wm1))
        b, offs, wm = g.snapshot_heap()
        assert len(offs) == hi - lo + 1
        bodies.append(b)
        wms.append(wm)
        g.close()
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names, rtol=1e-9)
    if CASES[case]["window_kind"] == "SESSION":
        # a run of the reference names an older window as a merged session's state namespace
        # (MergingWindowSet.addWindow :190-201): rename every state window and check the restore follows the mapping
        renamed = []
        for b in bodies:
            ents, timers, msets = parse_heap(b, True, len(AGGS), 0, True)
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
                m = (kgs[cut:] >= lo) & (kgs[cut:] <= hi)
                g.push(keys[cut:][m], ts[cut:][m], [vi[cut:][m], vf[cut:][m], vd[cut:][m]])
                outs.append(g.advance_watermark(A.LONG_MAX))
                g.close()
            assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, final, names, rtol=1e-9)


@pytest.mark.parametrize("kind", [dict(window_kind="SESSION", semantics="TABLE", gap_ms=700),
                                  dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=15000, slide_ms=5000)])
def test_heap_layout_unsupported_kinds(kind):
    from flink_amd import engine
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, key_capacity=64, **kind))
    with pytest.raises(engine.EngineError) as ei:
        g.snapshot_heap()
    assert A.STATUS[ei.value.code] == "E_UNSUPPORTED"
    g.close()
