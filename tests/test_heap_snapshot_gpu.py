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


def parse_heap(body, ds, naggs, lateness):
    """(key group -> [(key, start, end, acc fields)], timers)"""
    r = Reader(body)
    out, timers = {}, {}
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
        assert r.get(">h") == 1
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
    return out, timers


@pytest.mark.parametrize("sem", ["DATASTREAM", "TABLE"])
@pytest.mark.parametrize("lateness", [0, 3000])
def test_heap_bytes_match_engine_state(sem, lateness):
    from flink_amd import engine
    if sem == "TABLE" and lateness:
        pytest.skip("allowed lateness is a DataStream setting")
    cfg = A.make_config(window_kind="TUMBLE", semantics=sem, size_ms=5000, aggs=AGGS, key_capacity=4096,
                        allowed_lateness_ms=lateness, key_kind=A.KEY_JAVA_LONG if sem == "DATASTREAM" else A.KEY_BINROW_BIGINT)
    g = engine.WindowAggregator(cfg)
    keys, ts, vi, vf, vd = random_stream(77, 30_000, 300, 40_000, 1000)
    g.push(keys, ts, [vi, vf, vd])
    g.advance_watermark(int(ts.max()) - 6000)
    snap = S.parse(g.snapshot())
    body, offs, wm = g.snapshot_heap()
    assert wm == snap["watermark"] and len(offs) == 128 and offs[0] == 0
    ds = sem == "DATASTREAM"
    ents, timers = parse_heap(body, ds, len(AGGS), lateness)
    assert sorted(ents) == list(range(128))
    for kg in range(128):                                      # KeyGroupRangeOffsets point at each section
        assert struct.unpack_from(">i", body, int(offs[kg]))[0] == kg
    n = 0
    for kg in range(128):
        sl = S.entries_of_key_group(snap, kg)
        exp = sorted(zip(snap["key"][sl].tolist(), snap["slice_start"][sl].tolist(), snap["count"][sl].tolist(),
                         *[a[sl].tolist() for a in snap["acc"]]))
        got = []
        for key, start, end, acc in ents[kg]:
            start = end - 5000 if start is None else start
            assert end - start == 5000
            f = list(acc)
            kinds = [A.AGG_KINDS[a] for a, _ in AGGS]
            enc = []
            for j, k in enumerate(kinds):          # back to the engine's words: ord keys for MIN/MAX
                x = f[1 + j] & 0xFFFFFFFFFFFFFFFF
                if k in (4, 5):
                    x ^= 1 << 63
                elif 6 <= k <= 9:
                    x = (~x & 0xFFFFFFFFFFFFFFFF) if x >> 63 else x | (1 << 63)
                enc.append(x - (1 << 64) if x >= 1 << 63 else x)
            cnt = f[0] - (1 << 64) if f[0] >= 1 << 63 else f[0]
            got.append((key if key < 1 << 63 else key - (1 << 64), start, cnt, *enc))
        assert sorted(got) == exp, kg
        n += len(got)
        # timers: window.maxTimestamp() (+ cleanup time with lateness), per (key, window)
        want_t = sorted((e[2] - 1 + d, e[0]) for e in ents[kg] for d in ([0, lateness] if ds and lateness else [0]))
        assert sorted((t[0], t[1]) for t in timers[kg]) == want_t
    assert n == snap["n"] > 0
    g.close()


@pytest.mark.parametrize("sem", ["DATASTREAM", "TABLE"])
def test_heap_restore_resumes_with_rescale(sem):
    """Two subtasks (key groups [0,63], [64,127]) checkpoint in the heap layout; one subtask restores both
    (scale-in) and two subtasks restore one body each half (scale-out); rows equal the oracle's."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    base = dict(window_kind="TUMBLE", semantics=sem, size_ms=5000, aggs=AGGS, key_capacity=4096,
                key_kind=A.KEY_JAVA_LONG if sem == "DATASTREAM" else A.KEY_BINROW_BIGINT)
    names = A.agg_names(A.make_config(**base))
    keys, ts, vi, vf, vd = random_stream(91, 40_000, 500, 60_000, 1000)
    cut = 20_000
    wm1 = int(ts[:cut].max()) - 1001
    kgs, _ = engine.key_groups(keys, 128, 1, base["key_kind"])
    o = Oracle(A.make_config(**base))
    o.push(keys[:cut], ts[:cut], [vi[:cut], vf[:cut], vd[:cut]])
    first = o.advance_watermark(wm1)
    o.push(keys[cut:], ts[cut:], [vi[cut:], vf[cut:], vd[cut:]])
    final = o.advance_watermark(A.LONG_MAX)
    halves = [(0, 63), (64, 127)]
    bodies, wms, got1 = [], [], []
    for lo, hi in halves:
        m = (kgs[:cut] >= lo) & (kgs[:cut] <= hi)
        g = engine.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **base))
        g.push(keys[:cut][m], ts[:cut][m], [vi[:cut][m], vf[:cut][m], vd[:cut][m]])
        got1.append(g.advance_watermark(wm1))
        b, offs, wm = g.snapshot_heap()
        assert len(offs) == hi - lo + 1
        bodies.append(b)
        wms.append(wm)
        g.close()
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names, rtol=1e-9)
    for layout in ([(0, 127)], [(0, 31), (32, 127)]):          # scale-in (1 subtask), then a new split (2)
        outs = []
        for lo, hi in layout:
            g = engine.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **base))
            g.restore_heap(bodies, wms)
            m = (kgs[cut:] >= lo) & (kgs[cut:] <= hi)
            g.push(keys[cut:][m], ts[cut:][m], [vi[cut:][m], vf[cut:][m], vd[cut:][m]])
            outs.append(g.advance_watermark(A.LONG_MAX))
            g.close()
        assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, final, names, rtol=1e-9)
