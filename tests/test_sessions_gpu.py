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
