"""GPU parity tests of the session-window path (DataStream EventTimeSessionWindows with allowed lateness,
DynamicEventTimeSessionWindows, Table GROUP BY SESSION) against the CPU oracle.

The engine splits a push into an order-free bulk path (sort by (key, start) + segmented gap-scan) and an
arrival-order walk for keys with records whose lone window already ended at the watermark;
these cases drive both paths, their mix inside one push, and the fallback when the start range is too wide
for one sort key. Integer aggregates, window bounds and late-drop counts are bit-exact; f64 sums within
1e-9 relative (reordered additions).
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0), ("SUM_F64", 2), ("AVG_F64", 2)]


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


def _run(eng_mod, cfg, batches):
    from oracle.oracle import Oracle
    names = A.agg_names(cfg)
    g = eng_mod.WindowAggregator(cfg)
    o = Oracle(cfg)
    dg = do = 0
    for k, t, cols, wm in batches:
        dg += g.push(k, t, cols)
        do += o.push(k, t, cols)
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="wm=%d" % wm)
    assert dg == do, (dg, do)
    st = g.stats()
    g.close()
    o.close()
    return dg, st


def _stream(seed, n, nkeys, span, delay, late_frac, t0=0):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    base = t0 + np.sort(rng.integers(0, span, n)).astype(np.int64)
    ts = base - rng.integers(0, delay + 1, n)
    late = rng.random(n) < late_frac
    ts[late] -= rng.integers(delay, 6 * delay + 1, late.sum())
    vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
    vd = rng.random(n) * 100.0
    return keys, ts, vi, vd


def _batches(keys, ts, cols, nb, delay):
    out, mx, n = [], -2**63, len(keys)
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        mx = max(mx, int(ts[sl].max()))
        out.append((keys[sl], ts[sl], [c[sl] for c in cols], mx - delay - 1))
    out.append((keys[:0], ts[:0], [c[:0] for c in cols], A.LONG_MAX))
    return out


@pytest.mark.parametrize("sem,lateness", [("DATASTREAM", 0), ("DATASTREAM", 800), ("DATASTREAM", 10_000), ("TABLE", 0)])
def test_sessions_random_vs_oracle(eng_mod, sem, lateness):
    keys, ts, vi, vd = _stream(7 + lateness, 60_000, 700, 80_000, 1200, 0.03)
    cfg = A.make_config(window_kind="SESSION", semantics=sem, gap_ms=600, allowed_lateness_ms=lateness,
                        aggs=AGGS, key_capacity=4096)
    dropped, _ = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 15, 1200))
    if lateness < 10_000:
        assert dropped > 0


def test_dynamic_gap_sessions_vs_oracle(eng_mod):
    keys, ts, vi, vd = _stream(11, 40_000, 300, 60_000, 900, 0.02)
    gaps = (np.random.default_rng(3).integers(1, 2000, len(keys))).astype(np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=0, gap_col=3, aggs=AGGS, key_capacity=1024)
    _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd, gaps], 10, 900))


def test_dynamic_gap_rejects_non_positive(eng_mod):
    cfg = A.make_config(window_kind="SESSION", gap_ms=0, gap_col=1, aggs=[("COUNT", 0)])
    g = eng_mod.WindowAggregator(cfg)
    with pytest.raises(eng_mod.EngineError) as ei:
        g.push(np.array([1, 2], np.int64), np.array([10, 20], np.int64),
               [np.zeros(2, np.int64), np.array([5, 0], np.int64)])
    assert ei.value.code == -1
    g.close()


def test_many_sessions_per_key(eng_mod):
    """One key holds hundreds of in-flight sessions (the r01 engine capped them at 16 per key)."""
    n = 3000
    ts = (np.arange(n, dtype=np.int64) * 1000)[::-1].copy()      # far apart, pushed newest first
    keys = np.full(n, 42, np.int64)
    keys[::3] = 7
    vi = np.arange(n, dtype=np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=100, aggs=AGGS, key_capacity=64)
    _, st = _run(eng_mod, cfg, [(keys, ts, [vi, vi, vi.astype(np.float64)], -1),
                                (keys[:0], ts[:0], [vi[:0], vi[:0], vi[:0].astype(np.float64)], A.LONG_MAX)])


def test_large_push_clusters_span_waves(eng_mod):
    """2^20 records over 20k keys: long sessions whose bulk-path clusters span many wavefronts."""
    keys, ts, vi, vd = _stream(5, 1 << 20, 20_000, 2_000_000, 3000, 0.001)
    cfg = A.make_config(window_kind="SESSION", gap_ms=5000, aggs=AGGS, key_capacity=1 << 15)
    _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 4, 3000))


def test_wide_start_range_falls_back_to_arrival_order(eng_mod):
    """Starts spanning ~2^61 ms do not fit next to the key bits in one 64-bit sort key: every key takes the
    arrival-order walk; results are unchanged."""
    rng = np.random.default_rng(9)
    n = 5000
    keys = rng.integers(0, 50, n).astype(np.int64)
    ts = np.sort(rng.integers(-2**60, 2**60, n)).astype(np.int64)
    ts[::50] = ts[::50] - 10                                    # a few touching / overlapping windows
    vi = rng.integers(0, 1000, n).astype(np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=1000, aggs=AGGS, key_capacity=256)
    _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vi.astype(np.float64)], 3, 0))


def test_session_late_firings_mixed_with_bulk(eng_mod):
    """Within one push the same key gets order-free records and records that merge into already fired
    sessions (allowed lateness): late-firing rows come back at the head of the next watermark."""
    cfg = A.make_config(window_kind="SESSION", gap_ms=1000, allowed_lateness_ms=5000, aggs=AGGS, key_capacity=64)
    k = lambda *x: np.array(x, np.int64)
    pushes = [
        (k(1, 1, 2, 2), k(0, 500, 100, 3000), 2500),
        (k(1, 2, 1, 1, 2), k(1200, 2600, 9000, 1800, 50), 4000),    # 1@1200, 1@1800 merge into fired [0,1500)
        (k(1, 1, 2), k(8000, 300, 4500), 7000),
        (k(2), k(20_000), A.LONG_MAX),
    ]
    batches = [(kk, tt, [tt * 3, tt * 3, (tt * 0.5).astype(np.float64)], wm) for kk, tt, wm in pushes]
    _run(eng_mod, cfg, batches)


# ---- cell path (sess3_*: fixed gap, every record of the push order-free) ---------------------------
# A stream without late records batched as _batches does is order-free in every push (each record's window ends after
# the previous watermark), so these pushes run on the cell path; FWA_OPT_SESSION_CELLS = 0 forces the general path on the same
# stream. replay_records counts the records of pushes the cell path had to hand back to the general path.
CELL_AGGS = {
    1: [("COUNT", 0)],
    2: [("COUNT", 0), ("SUM_I64", 0)],
    3: [("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)],
    4: [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_F64", 2)],
    5: AGGS,
}


@pytest.mark.parametrize("cell", ["1", "0"])
@pytest.mark.parametrize("nacc", [1, 2, 3, 4, 5])
def test_cell_path_order_free_vs_oracle(eng_mod, monkeypatch, nacc, cell):
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "session_cells", -1 if cell == "1" else 0)
    keys, ts, vi, vd = _stream(100 + nacc, 200_000, 3000, 400_000, 300, 0.0)
    cfg = A.make_config(window_kind="SESSION", gap_ms=700, aggs=CELL_AGGS[nacc], key_capacity=8192)
    dropped, st = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 12, 300))
    assert dropped == 0
    assert st.replay_records == 0


def test_cell_path_groups_span_many_chunks(eng_mod):
    """10 keys, ~1000 records per (key, cell): groups run over many 64-element chunks and wave ranges; holes in event
    time split sessions inside and across pushes."""
    rng = np.random.default_rng(21)
    n = 1 << 20
    keys = rng.integers(0, 10, n).astype(np.int64)
    base = np.sort(rng.integers(0, 500_000, n)).astype(np.int64)
    keep = (base % 97_000) > 8_000                               # 8 s holes: a new session after each
    keys, base = keys[keep], base[keep]
    ts = base - rng.integers(0, 200, len(base))
    vi = rng.integers(-2**40, 2**40, len(base)).astype(np.int64)
    vd = rng.random(len(base)) * 100.0
    cfg = A.make_config(window_kind="SESSION", gap_ms=5000, aggs=AGGS, key_capacity=64)
    _, st = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 5, 200))
    assert st.replay_records == 0


def test_cell_path_table_session_vs_oracle(eng_mod):
    keys, ts, vi, vd = _stream(23, 100_000, 1500, 300_000, 250, 0.0)
    cfg = A.make_config(window_kind="SESSION", semantics="TABLE", gap_ms=900, aggs=AGGS, key_capacity=4096)
    _, st = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 8, 250))
    assert st.replay_records == 0


def test_cell_range_overflow_is_redone(eng_mod):
    """A large key table leaves few bits for the cell (2^23 slots: 8 cell bits); a push spanning more than 256 gaps is
    handed back to the general path, with the same results."""
    keys, ts, vi, vd = _stream(29, 50_000, 500, 100_000, 5, 0.0)
    cfg = A.make_config(window_kind="SESSION", gap_ms=10, aggs=AGGS, key_capacity=1 << 22)
    _, st = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 3, 5))
    assert st.replay_records > 0


def test_cell_path_redo_on_order_sensitive_records(eng_mod):
    """Late records in a push hand it back to the general path (arrival-order walk for their keys); the pushes after
    the skip window take the cell path again."""
    keys, ts, vi, vd = _stream(31, 120_000, 800, 200_000, 400, 0.0)
    ts = ts.copy()
    ts[30_000:30_050] -= 20_000                                  # late records in the third push only
    cfg = A.make_config(window_kind="SESSION", gap_ms=1000, allowed_lateness_ms=500, aggs=AGGS, key_capacity=2048)
    dropped, st = _run(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 24, 400))
    assert dropped > 0
    assert 0 < st.replay_records < len(keys)


# ---- cell pre-aggregation (sessions4.inc: <= 16 cells per push, <= 8 in-flight sessions per key) ------------------
def _run_paths(eng_mod, cfg, batches, variant=0):
    """_run, recording the path each push took (FWA_OPT_SESSION_PATH: 0 general, 1 sort-based cells, 2 pre-agg).
    variant 8: the pre-aggregation path's s4 probe route instead of the s5 hash route (FWA_OPT_INGEST_VARIANT)."""
    from oracle.oracle import Oracle
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    if variant:
        g.set_option("ingest_variant", variant)
    paths, dg, do = [], 0, 0
    for k, t, cols, wm in batches:
        dg += g.push(k, t, cols)
        do += o.push(k, t, cols)
        if len(k):
            paths.append(g.get_option("session_path"))
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="wm=%d" % wm)
    assert dg == do
    st = g.stats()
    g.close()
    o.close()
    return paths, st


@pytest.mark.parametrize("route", [0, 8], ids=["s5_hash_route", "s4_probe_route"])
@pytest.mark.parametrize("sem", ["DATASTREAM", "TABLE"])
@pytest.mark.parametrize("nacc", [1, 2, 3, 4, 5])
def test_cell_preagg_vs_oracle(eng_mod, nacc, sem, route):
    """Pushes of 50 s of event time with a 5 s gap (about 11 cells): every push on the pre-aggregation path, sessions
    kept in flight across pushes, closed and fired between them; both routes of the path."""
    keys, ts, vi, vd = _stream(200 + nacc, 200_000, 3000, 600_000, 300, 0.0)
    cfg = A.make_config(window_kind="SESSION", semantics=sem, gap_ms=5000, aggs=CELL_AGGS[nacc], key_capacity=8192)
    paths, st = _run_paths(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 12, 300), variant=route)
    assert paths == [2] * 12
    assert st.replay_records == 0


@pytest.mark.parametrize("route", [0, 8], ids=["s5_hash_route", "s4_probe_route"])
def test_cell_preagg_many_partitions_vs_oracle(eng_mod, route):
    """A key table of 2^18 slots (32 partitions of 8192 keys; the s5 route resolves each in its own workgroup), 60K keys
    with the sentinel key among them, 8 pushes; the key table the route built serves the later pushes' probes."""
    keys, ts, vi, vd = _stream(77, 400_000, 60_000, 400_000, 300, 0.0)
    keys[::997] = -2**63
    cfg = A.make_config(window_kind="SESSION", gap_ms=5000, aggs=AGGS, key_capacity=1 << 17)
    paths, st = _run_paths(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 8, 300), variant=route)
    assert paths == [2] * 8
    assert st.replay_records == 0


def test_cell_preagg_touching_and_bucket_edges(eng_mod):
    """Windows exactly `gap` apart touch and merge (TimeWindow.intersects), inside one push and against an in-flight
    session; keys on both sides of a 128-kid bucket edge, the sentinel key (side slot) and a NULL-free wide value."""
    gap = 1000
    k = lambda *x: np.array(x, np.int64)
    keys1 = np.concatenate([k(1, 1, 1, 2, 2), np.arange(100, 400, dtype=np.int64), k(-2**63, -2**63)])
    ts1 = np.concatenate([k(0, 1000, 2000, 0, 2001), np.full(300, 1500, np.int64), k(10, 1010)])
    keys2 = k(1, 2, 2, 7, -2**63)
    ts2 = k(3000, 3001, 5003, 4000, 2010)                        # 1@3000 touches [0, 3000); 2@3001 touches [2001, 3001)
    batches = []
    for kk, tt, wm in [(keys1, ts1, 1500), (keys2, ts2, 2500), (keys2[:0], ts2[:0], A.LONG_MAX)]:
        vi = (tt * 7 + kk % 13).astype(np.int64)
        batches.append((kk, tt, [vi, vi, (tt * 0.25).astype(np.float64)], wm))
    cfg = A.make_config(window_kind="SESSION", gap_ms=gap, aggs=AGGS, key_capacity=512)
    paths, _ = _run_paths(eng_mod, cfg, batches)
    assert paths == [2, 2]


def test_cell_preagg_many_sessions_per_key_falls_back(eng_mod):
    """A key holding more than 8 in-flight sessions (allowed lateness keeps them) hands a narrow push to the sort-based
    cell path; the results are unchanged."""
    n = 200
    ts = np.arange(n, dtype=np.int64) * 300                        # gap 100: every record its own session
    keys = np.full(n, 5, np.int64)
    keys[::2] = 9
    vi = np.arange(n, dtype=np.int64)
    k2, t2 = np.array([5, 5, 9], np.int64), np.array([60_000, 60_050, 60_020], np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=100, allowed_lateness_ms=1_000_000, aggs=AGGS, key_capacity=64)
    batches = [(keys, ts, [vi, vi, vi * 0.5], 100), (k2, t2, [k2, k2, k2 * 0.5], 70_000),
               (keys[:0], ts[:0], [vi[:0], vi[:0], vi[:0] * 0.5], A.LONG_MAX)]
    paths, _ = _run_paths(eng_mod, cfg, batches)
    assert paths == [1, 1]


def test_cell_preagg_wide_push_uses_sorted_cells(eng_mod):
    """A push spanning more than 16 cells takes the sort-based cell path; a narrow one the pre-aggregation path."""
    keys, ts, vi, vd = _stream(41, 60_000, 500, 100_000, 100, 0.0)
    cfg = A.make_config(window_kind="SESSION", gap_ms=1000, aggs=AGGS, key_capacity=1024)
    paths, st = _run_paths(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 2, 100))
    assert paths == [1, 1]
    paths, st = _run_paths(eng_mod, cfg, _batches(keys, ts, [vi, vi, vd], 20, 100))
    assert paths == [2] * 20
    assert st.replay_records == 0
