"""GPU tests: TUMBLE window state as record lists (FWA_CFG_RECORD_LISTS, flink_amd/csrc/sparse.inc) against the
CPU oracle -- the layout the engine selects for key spaces where keys barely repeat within a window (C4).

Same contract as the dense layout: rows equal the oracle's (WindowOperator / SlicingWindowOperator restatement) for
DataStream and Table TUMBLE with offsets, late drops and their indices, key-group ownership and Long.MIN_VALUE
errors, the Long.MIN_VALUE key, a push spanning many windows, partial accumulators and snapshot / restore with
rescaling; the fire's fine-bucket and split-pass paths are forced with small LDS tables (FWA_OPT_SP_TABLE /
FWA_OPT_SP_FMAX).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal
from test_gpu_parity import random_stream

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0), ("SUM_F64", 2), ("MAX_F32", 1),
        ("AVG_F64", 2), ("AVG_I64", 0)]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_both(cfg_kw, batches, wms, aggs=AGGS):
    from flink_amd import engine
    from oracle.oracle import Oracle
    g = engine.WindowAggregator(A.make_config(aggs=aggs, record_lists=True, **cfg_kw))
    assert g.record_lists
    o = Oracle(A.make_config(aggs=aggs, **cfg_kw))
    names = A.agg_names(A.make_config(aggs=aggs, **cfg_kw))
    for (k, t, cols), wm in zip(batches, wms):
        dg = g.push(k, t, cols)
        do = o.push(k, t, cols)
        assert dg == do
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9)
    st = g.stats()
    g.close()
    return st


@pytest.mark.parametrize("sem,offset", [("DATASTREAM", 0), ("DATASTREAM", 1300), ("TABLE", -700)])
def test_record_lists_vs_oracle(sem, offset):
    keys, ts, vi, vf, vd = random_stream(5, 200_000, 20_000, 60_000, 1500)
    cut = [0, 50_000, 120_000, 200_000]
    batches = [(keys[a:b], ts[a:b], [vi[a:b], vf[a:b], vd[a:b]]) for a, b in zip(cut, cut[1:])]
    wms = [int(ts[:b].max()) - 1501 for b in cut[1:-1]] + [A.LONG_MAX]
    st = run_both(dict(window_kind="TUMBLE", semantics=sem, size_ms=5000, offset_ms=offset), batches, wms)
    assert st.records_in == 200_000 and st.live_slices == 0


def test_record_lists_one_big_window_fine_buckets():
    """2M distinct-ish keys in one window: every (window, partition) takes the fine-bucket path."""
    rng = np.random.default_rng(11)
    n = 3_000_000
    keys = rng.integers(-2**62, 2**62, n).astype(np.int64)
    keys[::7] = keys[1::7][: len(keys[::7])]                    # some repeats
    keys[rng.random(n) < 1e-4] = -2**63                         # the table's empty marker is a legal key
    ts = rng.integers(0, 10_000, n).astype(np.int64)
    vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
    vf = rng.random(n).astype(np.float32)
    vd = rng.random(n) - 0.5
    run_both(dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000),
             [(keys, ts, [vi, vf, vd])], [A.LONG_MAX])


@pytest.mark.parametrize("opts", [{"sp_table": 128}, {"sp_table": 256, "sp_fmax": 1}])
def test_record_lists_split_passes(monkeypatch, opts):
    """Tables far smaller than a partition's distinct keys: overflowing passes are redone as half passes."""
    from flink_amd import engine
    for k, v in opts.items():
        monkeypatch.setitem(engine.DEFAULT_OPTIONS, k, v)
    test_record_lists_vs_oracle('TABLE', 0)
    test_record_lists_hot_keys()


def test_record_lists_hot_keys():
    rng = np.random.default_rng(3)
    n = 400_000
    keys = np.where(rng.random(n) < 0.5, 42, rng.integers(0, 50_000, n)).astype(np.int64)
    ts = np.sort(rng.integers(0, 40_000, n)).astype(np.int64)
    vi = rng.integers(-1000, 1000, n).astype(np.int64)
    vf = rng.random(n).astype(np.float32)
    vd = rng.random(n)
    half = n // 2
    run_both(dict(window_kind="TUMBLE", semantics="TABLE", size_ms=3000),
             [(keys[:half], ts[:half], [vi[:half], vf[:half], vd[:half]]),
              (keys[half:], ts[half:], [vi[half:], vf[half:], vd[half:]])],
             [int(ts[half - 1]) - 1, A.LONG_MAX])


def test_record_lists_wide_push_and_late_indices():
    """One push spanning ~40 windows (several push passes), then late records with their indices."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    kw = dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, late_indices=True)
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, record_lists=True, **kw))
    o = Oracle(A.make_config(aggs=AGGS, **kw))
    names = A.agg_names(A.make_config(aggs=AGGS, **kw))
    keys, ts, vi, vf, vd = random_stream(8, 100_000, 3000, 40_000, 500)
    assert g.push(keys, ts, [vi, vf, vd]) == o.push(keys, ts, [vi, vf, vd])
    assert_rows_equal(g.advance_watermark(20_000), o.advance_watermark(20_000), names, rtol=1e-9)
    k2, t2, vi2, vf2, vd2 = random_stream(9, 20_000, 3000, 40_000, 500)
    assert g.push(k2, t2, [vi2, vf2, vd2]) == o.push(k2, t2, [vi2, vf2, vd2]) > 0
    late = g.late_records()
    exp = np.nonzero(((t2 // 1000) * 1000 + 999) <= 20_000)[0]   # window maxTimestamp <= the watermark
    assert np.array_equal(np.sort(late), exp), (len(late), len(exp))
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), names, rtol=1e-9)
    g.close()


def test_record_lists_errors():
    from flink_amd import engine
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, record_lists=True, kg_start=0, kg_end=63))
    kgs, _ = engine.key_groups(np.arange(1000, dtype=np.int64), 128, 1, A.KEY_JAVA_LONG)
    bad = np.arange(1000, dtype=np.int64)[kgs > 63][:5]
    z = np.zeros(5, np.int64)
    with pytest.raises(engine.EngineError) as ei:
        g.push(bad, z, [z, z.astype(np.float32), z.astype(np.float64)])
    assert A.STATUS[ei.value.code] == "E_KEYGROUP"
    g.close()
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, record_lists=True))
    t = np.full(5, -2**63, np.int64)
    with pytest.raises(engine.EngineError) as ei:
        g.push(np.arange(5, dtype=np.int64), t, [z, z.astype(np.float32), z.astype(np.float64)])
    assert A.STATUS[ei.value.code] == "E_TS_MIN"
    g.close()
    with pytest.raises(engine.EngineError):                    # sliding windows keep the dense layout
        engine.WindowAggregator(A.make_config(window_kind="SLIDE", size_ms=3000, slide_ms=1000, record_lists=True))


def test_record_lists_auto_selected_for_huge_key_spaces():
    from flink_amd import engine
    g = engine.WindowAggregator(A.make_config(key_capacity=100_000_000))
    assert g.record_lists
    g.close()
    g = engine.WindowAggregator(A.make_config(key_capacity=1_000_000))
    assert not g.record_lists
    g.close()


def test_record_lists_partials_two_phase():
    """Local drain (raw accumulators, record lists) -> owner push_partials (record lists) == one operator."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    kw = dict(window_kind="TUMBLE", semantics="TABLE", size_ms=2000)
    aggs = [("COUNT", 0), ("SUM_I64", 0), ("MAX_F64", 2), ("AVG_F64", 2)]
    names = A.agg_names(A.make_config(aggs=aggs, **kw))
    local = engine.WindowAggregator(A.make_config(aggs=aggs, record_lists=True, **kw))
    owner = engine.WindowAggregator(A.make_config(aggs=aggs, record_lists=True, **kw))
    o = Oracle(A.make_config(aggs=aggs, **kw))
    keys, ts, vi, vf, vd = random_stream(21, 120_000, 5000, 30_000, 800)
    for a, b, wm in [(0, 60_000, int(ts[:60_000].max()) - 801), (60_000, 120_000, A.LONG_MAX)]:
        local.push(keys[a:b], ts[a:b], [vi[a:b], vf[a:b], vd[a:b]])
        o.push(keys[a:b], ts[a:b], [vi[a:b], vf[a:b], vd[a:b]])
        p = local.drain_partials(wm)
        owner.push_partials(p["key"], p["slice_start"], p["count"], [p["acc%d" % j] for j in range(len(aggs))])
        assert_rows_equal(owner.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9)
    local.close()
    owner.close()


def test_record_lists_snapshot_restore_rescale():
    from flink_amd import engine
    from oracle.oracle import Oracle
    base = dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=5000, aggs=AGGS)
    names = A.agg_names(A.make_config(**base))
    keys, ts, vi, vf, vd = random_stream(91, 60_000, 8000, 60_000, 1000)
    cut = 30_000
    wm1 = int(ts[:cut].max()) - 3001
    kgs, _ = engine.key_groups(keys, 128, 1, A.KEY_JAVA_LONG)
    o = Oracle(A.make_config(**base))
    o.push(keys[:cut], ts[:cut], [vi[:cut], vf[:cut], vd[:cut]])
    first = o.advance_watermark(wm1)
    o.push(keys[cut:], ts[cut:], [vi[cut:], vf[cut:], vd[cut:]])
    final = o.advance_watermark(A.LONG_MAX)
    blobs, got1 = [], []
    for lo, hi in [(0, 63), (64, 127)]:
        m = (kgs[:cut] >= lo) & (kgs[:cut] <= hi)
        g = engine.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, record_lists=True, **base))
        g.push(keys[:cut][m], ts[:cut][m], [vi[:cut][m], vf[:cut][m], vd[:cut][m]])
        got1.append(g.advance_watermark(wm1))
        blobs.append(g.snapshot())
        g.close()
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names, rtol=1e-9)
    for layout, dense in [([(0, 127)], False), ([(0, 31), (32, 127)], False), ([(0, 127)], True)]:
        outs = []
        for lo, hi in layout:   # record-list snapshots restore into either layout
            g = engine.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, record_lists=not dense, **base))
            g.restore(blobs)
            m = (kgs[cut:] >= lo) & (kgs[cut:] <= hi)
            g.push(keys[cut:][m], ts[cut:][m], [vi[cut:][m], vf[cut:][m], vd[cut:][m]])
            outs.append(g.advance_watermark(A.LONG_MAX))
            g.close()
        assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, final, names, rtol=1e-9)


def record_lists_compaction_check():
    """Few distinct keys, many records per window, a small FWA_OPT_SP_BUDGET (set by the caller): the growing windows'
    lists are folded into pre-aggregated runs, results still equal the oracle's, device memory stays bounded."""
    import torch
    rng = np.random.default_rng(29)
    batches, wms = [], []
    for b in range(30):
        n = 100_000
        keys = rng.integers(0, 500, n).astype(np.int64)
        ts = rng.integers(0, 1_900_000, n).astype(np.int64) + (100_000 if b >= 20 else 0)
        vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
        vf = rng.random(n).astype(np.float32)
        vd = rng.random(n) - 0.5
        batches.append((keys, ts, [vi, vf, vd]))
        wms.append(999_999 if b == 24 else (A.LONG_MAX if b == 29 else -1))
    from flink_amd import engine
    from oracle.oracle import Oracle
    kw = dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1_000_000)
    g = engine.WindowAggregator(A.make_config(aggs=AGGS, record_lists=True, **kw))
    o = Oracle(A.make_config(aggs=AGGS, **kw))
    names = A.agg_names(A.make_config(aggs=AGGS, **kw))
    free0 = None
    for b, ((k, t, cols), wm) in enumerate(zip(batches, wms)):
        assert g.push(k, t, cols) == o.push(k, t, cols)
        if b == 4:
            free0 = torch.cuda.mem_get_info()[0]
        if b == 19:   # 15 more batches (~100 MB of entries without compaction) in the same two windows
            grew = free0 - torch.cuda.mem_get_info()[0]
            assert grew < 48 << 20, "record lists grew by %d bytes" % grew
        if wm != -1:
            assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="batch %d" % b)
    st = g.stats()
    assert st.records_in == 30 * 100_000 and st.live_slices == 0
    g.close()


def test_record_lists_compaction_bounds_memory():
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from flink_amd import engine\n"
            "engine.DEFAULT_OPTIONS['sp_budget'] = 4 << 20\n"
            "from test_record_lists_gpu import record_lists_compaction_check\n"
            "record_lists_compaction_check()\n"
            "print('ok')\n") % (ROOT, os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_record_lists_owned_range_across_watermarks():
    """A subtask owning half the key groups (N = 2 keyBy owner) on the record lists: pushes after a watermark take the
    fused histogram pass (key-group check on the same loads); every push holds owned keys only."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    rng = np.random.default_rng(123)
    n = 1 << 20
    keys = rng.integers(0, 100_000_000, 4 * n).astype(np.int64)
    kgs, _ = engine.key_groups(keys, 128, 1, A.KEY_JAVA_LONG)
    keys = keys[kgs <= 63]
    m = len(keys)
    ts = np.sort(rng.integers(0, 40_000, m)).astype(np.int64) - rng.integers(0, 1000, m)
    vi = rng.integers(0, 1000, m).astype(np.int64)
    vf = rng.random(m).astype(np.float32)
    vd = rng.random(m)
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000, aggs=AGGS, record_lists=True,
                        kg_start=0, kg_end=63, key_capacity=1 << 26)
    names = A.agg_names(cfg)
    g, o = engine.WindowAggregator(cfg), Oracle(cfg)
    mx = -2**63
    for b in range(4):
        sl = slice(b * m // 4, (b + 1) * m // 4)
        cols = [vi[sl], vf[sl], vd[sl]]
        assert g.push(keys[sl], ts[sl], cols) == o.push(keys[sl], ts[sl], cols)
        mx = max(mx, int(ts[sl].max()))
        wm = mx - 1001 if b < 3 else A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-6, ctx="batch %d" % b)
    g.close()
    o.close()


@pytest.mark.parametrize("sem", ["DATASTREAM", "TABLE"])
def test_record_lists_narrow_entries(sem):
    """COUNT + SUM(BIGINT) with keys and values over the signed 32-bit range: the runs hold one-word entries (int32
    key | int32 value); a later push with keys and values past 32 bits is redone with 64-bit entries, which stay.
    Rows equal the oracle's throughout, and the one-word runs cost no extra replay."""
    rng = np.random.default_rng(17)
    n = 600_000
    keys = rng.integers(-2**31, 2**31, n).astype(np.int64)
    rep = rng.random(n) < 0.3                                 # some keys repeat within a window
    keys[rep] = keys[rng.integers(0, n, rep.sum())]
    ts = np.sort(rng.integers(0, 60_000, n)).astype(np.int64) - rng.integers(0, 1001, n)
    vi = rng.integers(-2**31, 2**31, n).astype(np.int64)
    late_wide = slice(400_000, 500_000)                       # the fifth push carries 64-bit keys and values
    keys[late_wide][::97] = 2**40 + 3
    vi[late_wide][::89] = -2**50
    cut = [0, 100_000, 200_000, 300_000, 400_000, 500_000, 600_000]
    batches = [(keys[a:b], ts[a:b], [vi[a:b]]) for a, b in zip(cut, cut[1:])]
    wms = [int(ts[:b].max()) - 1001 for b in cut[1:-1]] + [A.LONG_MAX]
    run_both(dict(window_kind="TUMBLE", semantics=sem, size_ms=5000, key_capacity=1 << 26), batches, wms,
             aggs=[("COUNT", 0), ("SUM_I64", 0)])
