"""Heap-layout keyed state of DECIMAL SUM / AVG handles (flink_amd/csrc/heap_snapshot.cpp over decimal.inc).

The accumulator row's DECIMAL field is the DECIMAL(38, s) running sum (LogicalTypeMerging.findSumAggType) written as
a non-compact DecimalData (AbstractBinaryWriter.writeDecimal :164-196: 16 bytes in the variable-length part, the
bytes of BigInteger.toByteArray); the engine rebuilds it from its 32-bit piece sums. Checks:
  1. every unfired TUMBLE slice's fields equal the exact sums of the records pushed into it (no record of an unfired
     slice can have been dropped as late), parsed by tests/heap_reader.py;
  2. two subtasks' heap bodies restore into one subtask and into a new split, and the rows equal the oracle's
     uninterrupted run (TUMBLE / HOP / CUMULATE / SESSION, NULL-free and nullable columns);
  3. hand-written bodies: a NULL DECIMAL sum restarts from the next value (the reference's DecimalSumAggFunction),
     38-digit sums round-trip through the 4-piece split, a sum past 2^95 of an int64-input column is refused.
"""
import struct

import numpy as np
import pytest

import heap_reader as H
from flink_amd import _abi as A
from helpers import assert_rows_equal
from test_decimal_gpu import random_batches

pytestmark = pytest.mark.gpu

AGG_SETS = {
    "both": ([("COUNT", 0), ("SUM_DEC", 0, 2), ("AVG_DEC", 0, 2), ("SUM_DEC128", 1, 20), ("AVG_DEC128", 1, 20),
              ("MAX_F64", 2)], False),
    "dec64_null": ([("COUNT", 0), ("SUM_DEC", 0, 2), ("AVG_DEC", 0, 2), ("MAX_F64", 2)], True),
    "dec128_null": ([("SUM_DEC128", 1, 20), ("AVG_DEC128", 1, 20), ("COUNT", 0)], True),
}
WINDOWS = {
    "tumble": dict(window_kind="TUMBLE", size_ms=1000),
    "hop": dict(window_kind="SLIDE", size_ms=4000, slide_ms=1000),
    "cumulate": dict(window_kind="CUMULATE", size_ms=3000, slide_ms=1000),
    "session": dict(window_kind="SESSION", gap_ms=900),
}


def make_cfg(aset, win, **kw):
    aggs, nullable = AGG_SETS[aset]
    return A.make_config(semantics="TABLE", aggs=aggs, key_capacity=4096, key_kind=A.KEY_BINROW_BIGINT,
                         nullable_cols=[0, 1, 2] if nullable else [], **WINDOWS[win], **kw)


def hidden_cols(aset):
    """the caller's hidden non-NULL counters: nullable columns in first-use order (heap_snapshot.cpp hidden_map)"""
    aggs, nullable = AGG_SETS[aset]
    out = []
    for a in aggs:
        if nullable and a[0] != "COUNT" and a[1] not in out:
            out.append(a[1])
    return out


def dec_of(col, i):
    c = col[i]
    if np.ndim(c) == 0:
        return int(c)
    return (int(c[0]) & ((1 << 64) - 1)) | (int(c[1]) << 64)


def push(g, batch, m=None):
    k, t, cols, nul, _ = batch
    if m is None:
        return g.push(k, t, cols, nulls=nul)
    return g.push(k[m], t[m], [c[m] for c in cols], nulls=None if nul is None else [z[m] for z in nul])


@pytest.mark.parametrize("aset", list(AGG_SETS))
def test_heap_decimal_fields_are_slice_sums(aset):
    from flink_amd import engine
    aggs, nullable = AGG_SETS[aset]
    cfg = make_cfg(aset, "tumble")
    g = engine.WindowAggregator(cfg)
    batches = random_batches(5, nullable=nullable)
    for b in batches[:5]:
        push(g, b)
        g.advance_watermark(b[4])
    last_wm = batches[4][4]
    body, offs, wm = g.snapshot_heap()
    g.close()
    assert wm == last_wm
    hcols = hidden_cols(aset)
    na = len(aggs)
    arity = 1 + na + len(hcols)
    dec = [1 + j for j, a in enumerate(aggs) if "DEC" in a[0]]
    lay = {0: ("kv", H.ser_long, H.ser_binrow(1), H.ser_binrow_dec(arity, dec)),
           1: ("pq", H.ser_binrow(1), H.ser_long), 2: ("pq", H.ser_binrow(1), H.ser_long)}
    secs = H.read_key_groups(body, offs, 0, lay)
    got = {}
    for kg, s in secs.items():
        for end, (_, _, kf), (rk, nl, f) in s[0]:
            assert rk == 0 and not nl[0]
            got[(H.s64(kf[0]), end)] = (nl, f)
    # the exact sums of the records of every unfired slice
    exp = {}
    for k, t, cols, nul, _ in batches[:5]:
        for i in range(len(k)):
            end = (int(t[i]) // 1000) * 1000 + 1000
            if end - 1 <= last_wm:
                continue
            e = exp.setdefault((int(k[i]), end), [0, [0, 0, 0], [0, 0, 0]])   # count, per-column sums, non-NULL counts
            e[0] += 1
            for c in (0, 1):
                if nul is None or not nul[c][i]:
                    e[1][c] += dec_of(cols[c], i)
                    e[2][c] += 1
            if nul is None or not nul[2][i]:
                e[2][2] += 1
    assert set(got) == set(exp)
    for key, (nl, f) in got.items():
        cnt, sums, nn = exp[key]
        assert f[0] == cnt, key
        for j, a in enumerate(aggs):
            if a[0] == "COUNT":
                assert f[1 + j] == cnt
            elif "DEC" in a[0]:
                empty = nullable and nn[a[1]] == 0
                assert nl[1 + j] == empty, (key, j)
                if not empty:
                    assert f[1 + j] == sums[a[1]], (key, j)
        for h, c in enumerate(hcols):
            assert f[1 + na + h] == nn[c], (key, h)


@pytest.mark.parametrize("win", list(WINDOWS))
@pytest.mark.parametrize("aset", list(AGG_SETS))
def test_heap_decimal_restore_resumes_with_rescale(aset, win):
    """Two subtasks (key groups [0,63], [64,127]) checkpoint in the heap layout; one subtask restores both (scale-in)
    and two restore a new split (scale-out); every fire equals the oracle's uninterrupted run."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    cfg = make_cfg(aset, win)
    names = A.agg_names(cfg)
    batches = random_batches(17, nullable=AGG_SETS[aset][1])
    cut = 5
    o = Oracle(make_cfg(aset, win))
    want = []
    for b in batches:
        push(o, b)
        want.append(o.advance_watermark(b[4]))
    o.close()
    kgs = [engine.key_groups(b[0], 128, 1, A.KEY_BINROW_BIGINT)[0] for b in batches]
    bodies, wms = [], []
    halves = [(0, 63), (64, 127)]
    subs = [engine.WindowAggregator(make_cfg(aset, win, kg_start=lo, kg_end=hi)) for lo, hi in halves]
    for i, b in enumerate(batches[:cut]):
        outs = []
        for g, (lo, hi) in zip(subs, halves):
            push(g, b, (kgs[i] >= lo) & (kgs[i] <= hi))
            outs.append(g.advance_watermark(b[4]))
        assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, want[i], names,
                          ctx="before the checkpoint, batch %d" % i)
    for g in subs:
        body, _, wm = g.snapshot_heap()
        bodies.append(body)
        wms.append(wm)
        g.close()
    for layout in ([(0, 127)], [(0, 31), (32, 127)]):
        subs = []
        for lo, hi in layout:
            g = engine.WindowAggregator(make_cfg(aset, win, kg_start=lo, kg_end=hi))
            g.restore_heap(bodies, wms)
            subs.append(g)
        for i in range(cut, len(batches)):
            b = batches[i]
            outs = []
            for g, (lo, hi) in zip(subs, layout):
                push(g, b, (kgs[i] >= lo) & (kgs[i] <= hi))
                outs.append(g.advance_watermark(b[4]))
            assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, want[i], names,
                              ctx="restored %s, batch %d" % (layout, i))
        for g in subs:
            g.close()


def key_row(key):
    return struct.pack(">i", 16) + bytes(8) + struct.pack("<q", key)


def acc_row(count, dec_value):
    """BinaryRowData of (COUNT(*), DECIMAL(38, 2)): a NULL DECIMAL is setNullAt, a value 16 reserved bytes"""
    hdr = bytearray(8)
    if dec_value is None:
        hdr[1] |= 1 << 1                                          # field 1: bit 9
        return struct.pack(">i", 24) + bytes(hdr) + struct.pack("<qQ", count, 0)
    b = dec_value.to_bytes(16, "big", signed=True)
    jbl = dec_value.bit_length() if dec_value >= 0 else (~dec_value).bit_length()
    b = b[16 - (jbl // 8 + 1):]
    return (struct.pack(">i", 40) + bytes(hdr) + struct.pack("<qQ", count, (24 << 32) | len(b)) + b
            + bytes(16 - len(b)))


def one_entry_body(kg, key, slice_end, count, dec_value):
    body = struct.pack(">i", kg) + struct.pack(">hi", 0, 1) + struct.pack(">q", slice_end) + key_row(key)
    body += acc_row(count, dec_value)
    return body + struct.pack(">hi", 1, 0) + struct.pack(">hi", 2, 0)   # timers: re-derived from the state


@pytest.mark.parametrize("kind,value,push_v,expect", [
    ("SUM_DEC", None, 7, 7),                                      # NULL sum + 7 -> 7 (restart)
    ("SUM_DEC128", None, -3, -3),
    ("SUM_DEC128", 10 ** 38 - 1, -1, 10 ** 38 - 2),               # 38 digits through the 4-piece split
    ("SUM_DEC128", -(10 ** 38 - 1), 0, -(10 ** 38 - 1)),
    ("SUM_DEC", -(2 ** 94), -5, -(2 ** 94) - 5),                  # 2 pieces: |T| < 2^95
    ("SUM_DEC", 2 ** 96, 1, "E_UNSUPPORTED"),
])
def test_heap_decimal_hand_written_bodies(kind, value, push_v, expect):
    from flink_amd import engine
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[(kind, 0, 2)], key_capacity=64,
                        key_kind=A.KEY_BINROW_BIGINT)
    key = 5
    kg = int(engine.key_groups(np.array([key], np.int64), 128, 1, A.KEY_BINROW_BIGINT)[0][0])
    g = engine.WindowAggregator(cfg)
    body = one_entry_body(kg, key, 1000, 3, value)
    if expect == "E_UNSUPPORTED":
        with pytest.raises(engine.EngineError) as ei:
            g.restore_heap([body], [500])
        assert A.STATUS[ei.value.code] == "E_UNSUPPORTED"
        g.close()
        return
    g.restore_heap([body], [500])
    col = A.dec128_column([push_v]) if kind == "SUM_DEC128" else np.array([push_v], np.int64)
    g.push(np.array([key], np.int64), np.array([100], np.int64), [col])
    r = g.advance_watermark(A.LONG_MAX)
    g.close()
    assert r["key"].tolist() == [key] and r["win_end"].tolist() == [1000]
    assert not (r.get("null0") is not None and r["null0"][0])
    assert int(r["agg0"][0]) == expect
