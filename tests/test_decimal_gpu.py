"""DECIMAL SUM / AVG on the GPU (flink_amd/csrc/decimal.inc) against the oracle and the reference's KATs.

The engine sums 32-bit pieces of the unscaled values in ordinary SUM(BIGINT) accumulators and rebuilds the exact
total at the fire; overflow is decided on that total (include/flink_amd.h). The oracle follows the reference's
arrival-order running sums, so the random streams keep every running sum within 38 digits (where the two agree by
construction); overflow is tested on windows whose last record crosses the bound, and the documented difference
(a running sum that overflows before the window's last record) is asserted as such.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal, dec_input, load_decimal_kats, replay_decimal_kat

pytestmark = pytest.mark.gpu

DEC_KATS = load_decimal_kats()


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


def one_window(eng_mod, kind, scale, values, device=False):
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[("COUNT", 0), (kind, 0, scale)])
    g = eng_mod.WindowAggregator(cfg)
    n = len(values)
    k, t, v = np.full(n, 3, np.int64), np.arange(n, dtype=np.int64) % 1000, dec_input(kind, values)
    if device:
        import torch
        k, t, v = (torch.from_numpy(x).cuda() for x in (k, t, v))
    g.push(k, t, [v])
    r = g.advance_watermark(A.LONG_MAX)
    g.close()
    assert len(r["key"]) == 1 and int(r["agg0"][0]) == n
    return None if r.get("null1") is not None and r["null1"][0] else int(r["agg1"][0])


@pytest.mark.parametrize("case", DEC_KATS, ids=lambda c: c["name"].split(" ", 1)[1])
def test_decimal_kats_on_gpu(eng_mod, case):
    replay_decimal_kat(case, eng_mod.WindowAggregator)


def test_avg_double_rounding_on_gpu(eng_mod):
    i0 = 9 * 10 ** 34 + 12345
    vals = [i0] * 1000 + [i0 + 500]
    assert one_window(eng_mod, "AVG_DEC128", 6, vals) == i0 + 1
    assert one_window(eng_mod, "AVG_DEC128", 6, vals, device=True) == i0 + 1


def test_overflow_and_result_type_bounds_on_gpu(eng_mod):
    big = 6 * 10 ** 37
    assert one_window(eng_mod, "SUM_DEC128", 2, [big, big]) is None          # the last record crosses 10^38
    assert one_window(eng_mod, "AVG_DEC128", 2, [big, big]) is None
    assert one_window(eng_mod, "SUM_DEC128", 2, [big, -big, big]) == big
    assert one_window(eng_mod, "SUM_DEC128", 0, [10 ** 38 - 1]) == 10 ** 38 - 1
    assert one_window(eng_mod, "SUM_DEC128", 0, [10 ** 38 - 1, 1]) is None
    assert one_window(eng_mod, "AVG_DEC128", 0, [10 ** 37]) is None         # 38 integer digits > DECIMAL(38, 6)
    assert one_window(eng_mod, "AVG_DEC128", 0, [10 ** 31]) == 10 ** 37
    assert one_window(eng_mod, "SUM_DEC", 0, [2 ** 63 - 1] * 3) == 3 * (2 ** 63 - 1)
    assert one_window(eng_mod, "AVG_DEC", 3, [-7, -8]) == -7500              # -0.0075 at scale 6
    assert one_window(eng_mod, "AVG_DEC", 0, [-1, -2]) == -1500000


def test_documented_overflow_difference(eng_mod):
    """The reference restarts SUM from the value after an overflowed running sum (arrival order); the engine decides
    on the window's exact total (include/flink_amd.h)."""
    from oracle.oracle import Oracle
    big = 6 * 10 ** 37
    vals = [big, big, 5]
    assert one_window(eng_mod, "SUM_DEC128", 2, vals) is None
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[("SUM_DEC128", 0, 2)])
    o = Oracle(cfg)
    o.push(np.full(3, 1, np.int64), np.arange(3, dtype=np.int64), [dec_input("SUM_DEC128", vals)])
    assert int(o.advance_watermark(A.LONG_MAX)["agg0"][0]) == 5
    o.close()
    # AVG has no restart (AvgAggFunction.java:79): the reference's AVG stays NULL once a running sum passed 38 digits,
    # the engine's is the exact total (6 * 10^37) over the count when that is back in range
    vals = [big, big, -big]
    assert one_window(eng_mod, "AVG_DEC128", 20, vals) == 2 * 10 ** 37
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[("AVG_DEC128", 0, 20)])
    o = Oracle(cfg)
    o.push(np.full(3, 1, np.int64), np.arange(3, dtype=np.int64), [dec_input("AVG_DEC128", vals)])
    r = o.advance_watermark(A.LONG_MAX)
    assert r["null0"][0]
    o.close()


CONFIGS = [
    dict(window_kind="TUMBLE", size_ms=1000),
    dict(window_kind="TUMBLE", size_ms=700, offset_ms=100),
    dict(window_kind="SLIDE", size_ms=4000, slide_ms=1000),
    dict(window_kind="CUMULATE", size_ms=3000, slide_ms=1000),
    dict(window_kind="SESSION", gap_ms=900),
]


def random_batches(seed, n=30_000, nkeys=500, nb=10, delay=1500, nullable=False, wide=True):
    rng = np.random.default_rng(seed)
    keys = rng.zipf(1.3, n).astype(np.int64) % nkeys
    ts = np.sort(rng.integers(0, 50_000, n)).astype(np.int64) - rng.integers(0, delay + 1, n)
    late = rng.random(n) < 0.02
    ts[late] -= rng.integers(delay, 3 * delay, late.sum())
    v64 = rng.integers(-10 ** 15, 10 ** 15, n).astype(np.int64)
    v64[rng.random(n) < 0.01] = 2 ** 62 + 7                                   # past 2^32 pieces, within the long
    big = [int(x) * 10 ** 18 + int(y) for x, y in zip(rng.integers(-10 ** 14, 10 ** 14, n), rng.integers(0, 10 ** 18, n))]
    v128 = A.dec128_column(big) if wide else None
    vd = rng.random(n) * 100.0
    nul = [(rng.random(n) < 0.1).astype(np.uint8) for _ in range(3)] if nullable else None
    out, mx = [], -2 ** 63
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        mx = max(mx, int(ts[sl].max()))
        cols = [v64[sl], v128[sl] if wide else v64[sl], vd[sl]]
        out.append((keys[sl], ts[sl], cols, None if nul is None else [x[sl] for x in nul], mx - delay - 1))
    out.append((keys[:0], ts[:0], [v64[:0], (v128 if wide else v64)[:0], vd[:0]],
                None if nul is None else [x[:0] for x in nul], A.LONG_MAX))
    return out


# DECIMAL aggregate lists: each DECIMAL source column takes 2 (int64 input) or 4 (16-byte) internal piece sums plus a
# count, within the handle's 8 aggregates (include/flink_amd.h)
AGG_SETS = {
    "both": [("COUNT", 0), ("SUM_DEC", 0, 2), ("AVG_DEC", 0, 2), ("SUM_DEC128", 1, 20), ("AVG_DEC128", 1, 20),
             ("MAX_F64", 2)],
    "dec64": [("COUNT", 0), ("SUM_DEC", 0, 2), ("AVG_DEC", 0, 2), ("MAX_F64", 2)],
    "dec128": [("SUM_DEC128", 1, 20), ("AVG_DEC128", 1, 20), ("COUNT", 0)],
}


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
@pytest.mark.parametrize("aset,nullable", [("both", False), ("dec64", True), ("dec128", True)],
                         ids=["both-notnull", "dec64-nullable", "dec128-nullable"])
def test_random_streams_decimal_vs_oracle(eng_mod, ci, aset, nullable):
    from oracle.oracle import Oracle
    aggs = AGG_SETS[aset]
    cfg = A.make_config(semantics="TABLE", aggs=aggs, key_capacity=2048, nullable_cols=[0, 1, 2] if nullable else [],
                        **CONFIGS[ci])
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    for k, t, cols, nul, wm in random_batches(40 + ci, nullable=nullable):
        assert g.push(k, t, cols, nulls=nul) == o.push(k, t, cols, nulls=nul)
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, ctx="config %d wm=%d" % (ci, wm))
    g.close()
    o.close()


def test_decimal_device_push_and_snapshot_roundtrip(eng_mod):
    """Device-pointer pushes split on the GPU; a snapshot of a DECIMAL handle restores into a fresh one."""
    import torch
    from oracle.oracle import Oracle
    aggs = [("COUNT", 0), ("SUM_DEC", 0, 4), ("AVG_DEC128", 1, 10)]
    cfg = A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=3000, slide_ms=1000, aggs=aggs,
                        key_capacity=4096)
    names = A.agg_names(cfg)
    batches = random_batches(77, n=20_000, nkeys=300, nb=6)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    for i, (k, t, cols, _, wm) in enumerate(batches[:-1]):
        dk, dt = torch.from_numpy(k).cuda(), torch.from_numpy(t).cuda()
        dc = [torch.from_numpy(np.ascontiguousarray(c)).cuda() for c in cols[:2]]
        assert g.push(dk, dt, dc) == o.push(k, t, cols[:2])
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, ctx="batch %d" % i)
        if i == 2:                                         # checkpoint, then continue on a restored handle
            blobs = g.snapshot()
            g.close()
            g = eng_mod.WindowAggregator(cfg)
            g.restore(blobs)
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), names, ctx="final")
    g.close()
    o.close()


def test_decimal_aggregate_budget(eng_mod):
    """Two nullable DECIMAL sources (one 16-byte) plus two more aggregates need 10 internal aggregates: refused."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, nullable_cols=[0, 1, 2],
                        aggs=AGG_SETS["both"])
    with pytest.raises(eng_mod.EngineError) as ei:
        eng_mod.WindowAggregator(cfg)
    assert "UNSUPPORTED" in str(ei.value)
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, aggs=[("SUM_DEC", 0, 2)])
    with pytest.raises(eng_mod.EngineError):                 # SQL aggregates: Table semantics only
        eng_mod.WindowAggregator(cfg)


def test_decimal_partials_unsupported(eng_mod):
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[("SUM_DEC", 0, 2)])
    g = eng_mod.WindowAggregator(cfg)
    with pytest.raises(eng_mod.EngineError) as ei:
        g.drain_partials(1000)
    assert "UNSUPPORTED" in str(ei.value)
    g.close()


@pytest.mark.parametrize("wrap_null", [1, 0])
def test_window_past_2_32_records_gives_null_decimal_rows(eng_mod, wrap_null):
    """The piece sums are exact below 2^32 records per (key, window); a window with more (forced here through a
    restored snapshot whose COUNT(*) says 2^32 + 5) fails the watermark step by default (FWA_E_UNSUPPORTED: the
    reference's total would be exact), and with FWA_OPT_DEC_WRAP_NULL fires its DECIMAL results as NULL, counted in
    fwa_stats.dec_inexact, every other row of the watermark emitted as usual."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, key_capacity=64,
                        aggs=[("COUNT", 0), ("SUM_DEC", 0, 2), ("AVG_DEC", 0, 2)])
    g = eng_mod.WindowAggregator(cfg)
    g.push(np.array([1, 2], np.int64), np.array([10, 20], np.int64), [np.array([5, 7], np.int64)])
    w = np.frombuffer(g.snapshot(), np.int64).copy()
    g.close()
    maxp, n = int(w[9]), int(w[21])
    body = 32 + maxp + 1
    keys = w[body:body + n]
    i = int(np.nonzero(keys == 1)[0][0])
    big = (1 << 32) + 5
    w[body + 2 * n + i] = big                    # COUNT(*) of key 1's slice
    naggs = int(w[11])
    kinds = w[12:12 + naggs]
    for j in range(naggs):
        if kinds[j] == A.AGG_KINDS["COUNT"]:
            w[body + (3 + j) * n + i] = big      # ... and the COUNT aggregate's word
    g = eng_mod.WindowAggregator(cfg, options={"dec_wrap_null": wrap_null})
    g.restore(w.tobytes())
    if not wrap_null:
        with pytest.raises(eng_mod.EngineError) as ei:
            g.advance_watermark(A.LONG_MAX)
        assert ei.value.code == -7 and g.stats().dec_inexact == 2
        g.close()
        return
    r = g.advance_watermark(A.LONG_MAX)
    st = g.stats()
    g.close()
    rows = {int(k): j for j, k in enumerate(r["key"])}
    assert set(rows) == {1, 2}
    a, b = rows[1], rows[2]
    assert int(r["agg0"][a]) == big and r["null1"][a] and r["null2"][a]
    assert int(r["agg0"][b]) == 1 and not r["null1"][b] and int(r["agg1"][b]) == 7
    assert st.dec_inexact == 2                   # SUM and AVG of key 1
