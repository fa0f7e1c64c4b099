"""GPU parity of SQL NULL semantics (Table window TVF aggregates over nullable columns) against the oracle and
the WindowAggregateITCase KATs.

SUM / MIN / MAX / AVG skip NULL inputs and are NULL for a window with no non-NULL input; COUNT(col) counts
the non-NULL values; COUNT(*) counts rows (the reference's SumAggFunction / MinAggFunction / AvgAggFunction /
CountAggFunction, DESIGN.md §2 "SQL NULLs"). NULL flags must agree row for row; values of non-NULL results
are bit-exact for integers and within the parity tolerances of test_gpu_parity.py for floats.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal, load_sql_kats, replay_sql_kat

pytestmark = pytest.mark.gpu

SQL_KATS = load_sql_kats()
TOL = {"SUM_F32": 2e-4, "AVG_F32": 1e-6, "SUM_F64": 1e-9, "AVG_F64": 1e-9}

AGGS = [("COUNT", 0), ("COUNT_COL", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0), ("AVG_I64", 0),
        ("COUNT_COL", 2), ("MAX_F64", 2)]
AGGS_F = [("SUM_F64", 2), ("AVG_F64", 2), ("MIN_F32", 1), ("SUM_F32", 1), ("MAX_F32", 1), ("AVG_F32", 1),
          ("COUNT_COL", 1), ("MIN_F64", 2)]

CONFIGS = [
    dict(window_kind="TUMBLE", size_ms=1000),
    dict(window_kind="TUMBLE", size_ms=700, offset_ms=100),
    dict(window_kind="SLIDE", size_ms=4000, slide_ms=1000),
    dict(window_kind="CUMULATE", size_ms=3000, slide_ms=1000),
    dict(window_kind="SESSION", gap_ms=900),
]


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("case", SQL_KATS["operators"], ids=lambda c: c["name"].split(".")[-1])
def test_sql_null_kats_on_gpu(eng_mod, case):
    replay_sql_kat(case, eng_mod.WindowAggregator)


def _stream(seed, n, nkeys, span, delay, null_frac, late_frac=0.02):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    ts = np.sort(rng.integers(0, span, n)).astype(np.int64) - rng.integers(0, delay + 1, n)
    late = rng.random(n) < late_frac
    ts[late] -= rng.integers(delay, 4 * delay + 1, late.sum())
    vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
    vf = (rng.random(n) * 100).astype(np.float32)
    vd = rng.random(n) * 1000.0 - 500.0
    nulls = [rng.random(n) < null_frac for _ in range(3)]
    quiet = keys % 11 == 0                        # keys whose column 0 is always NULL: NULL results
    nulls[0] |= quiet
    return keys, ts, [vi, vf, vd], [x.astype(np.uint8) for x in nulls]


def _run(eng_mod, cfg, stream, nb, delay, device=False):
    from oracle.oracle import Oracle
    import torch
    keys, ts, cols, nulls = stream
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    n, mx, dg, do = len(keys), -2**63, 0, 0
    for b in range(nb + 1):
        sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
        k, t, c, z = keys[sl], ts[sl], [x[sl] for x in cols], [x[sl] for x in nulls]
        wm = A.LONG_MAX if b == nb else None
        if b < nb:
            mx = max(mx, int(t.max()))
            wm = mx - delay - 1
        if device:
            dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
            dg += g.push(dev(k), dev(t), [dev(x) for x in c], nulls=[dev(x) for x in z])
        else:
            dg += g.push(k, t, c, nulls=z)
        do += o.push(k, t, c, nulls=z)
        rg, ro = g.advance_watermark(wm), o.advance_watermark(wm)
        assert_rows_equal(rg, ro, names, rtol=lambda nm: TOL.get(nm, 0.0), ctx="wm=%d" % wm)
        for j, nm in enumerate(names):                 # COUNT / COUNT(col) are never NULL
            if nm.startswith("COUNT"):
                assert not rg.get("null%d" % j, np.zeros(1, np.uint8)).any()
    assert dg == do, (dg, do)
    g.close()
    o.close()
    return dg


@pytest.mark.parametrize("ci", range(len(CONFIGS)), ids=[c["window_kind"] + str(i) for i, c in enumerate(CONFIGS)])
@pytest.mark.parametrize("aggs", [AGGS, AGGS_F], ids=["int", "float"])
def test_nullable_random_streams_vs_oracle(eng_mod, ci, aggs):
    cfg = A.make_config(semantics="TABLE", aggs=aggs, key_capacity=2048, nullable_cols=(0, 1, 2), **CONFIGS[ci])
    stream = _stream(300 + ci, 40_000, 500, 60_000, 1500, 0.2)
    assert _run(eng_mod, cfg, stream, 10, 1500) > 0


def test_nullable_large_pushes_mostly_non_null(eng_mod):
    """2^20-record pushes with rare NULLs: the NULL-free rows take the two-phase partition/combine path, rows
    with a NULL the slow path, both into the same windows."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=AGGS, key_capacity=1 << 15,
                        nullable_cols=(0, 1, 2))
    stream = _stream(77, 1 << 21, 20_000, 4_000_000, 2000, 0.002, late_frac=0.001)
    _run(eng_mod, cfg, stream, 2, 2000)


def test_nullable_device_inputs(eng_mod):
    cfg = A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=3000, slide_ms=1000, aggs=AGGS_F,
                        key_capacity=1024, nullable_cols=(0, 1, 2))
    _run(eng_mod, cfg, _stream(5, 20_000, 300, 30_000, 800, 0.3), 5, 800, device=True)


def test_partially_nullable_columns(eng_mod):
    """Only column 2 nullable: COUNT(col0) equals COUNT(*), aggregates over column 0/1 are never NULL."""
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=AGGS, key_capacity=1024,
                        nullable_cols=(2,))
    keys, ts, cols, nulls = _stream(9, 20_000, 300, 30_000, 800, 0.3)
    _run(eng_mod, cfg, (keys, ts, cols, [np.zeros_like(nulls[0]), np.zeros_like(nulls[1]), nulls[2]]), 5, 800)


def test_nullable_requires_table_semantics(eng_mod):
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, aggs=AGGS, nullable_cols=(0,))
    with pytest.raises(eng_mod.EngineError):
        eng_mod.WindowAggregator(cfg)


def _batches(stream, nb, delay):
    keys, ts, cols, nulls = stream
    n, mx = len(keys), -2**63
    for b in range(nb + 1):
        sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        yield keys[sl], ts[sl], [x[sl] for x in cols], [x[sl] for x in nulls], (mx - delay - 1 if b < nb else A.LONG_MAX)


@pytest.mark.parametrize("ci", [0, 2, 3], ids=["TUMBLE", "SLIDE", "CUMULATE"])
@pytest.mark.parametrize("aggs", [AGGS, AGGS_F], ids=["int", "float"])
def test_nullable_two_phase_partials_vs_oracle(eng_mod, ci, aggs):
    """Two-phase plan over nullable columns (LocalSlicingWindowAggOperator -> GlobalAggCombiner, whose nullable
    buffers merge with their NULL flags, GlobalAggCombiner.java:77-110): two local handles drain (key, slice)
    partials with the hidden non-NULL counters (fwa_partials.hidden), the owner merges them and fires. Rows, NULL
    flags and late drops equal one operator over the union of the streams."""
    from oracle.oracle import Oracle
    cfg = A.make_config(semantics="TABLE", aggs=aggs, key_capacity=2048, nullable_cols=(0, 1, 2), **CONFIGS[ci])
    names = A.agg_names(cfg)
    loc = [eng_mod.WindowAggregator(cfg) for _ in range(2)]
    glob, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    dg = do = 0
    for k, t, c, z, wm in _batches(_stream(400 + ci, 30_000, 400, 50_000, 1200, 0.25), 8, 1200):
        do += o.push(k, t, c, nulls=z)
        for s in range(2):
            sl = slice(s, None, 2)
            dg += loc[s].push(k[sl], t[sl], [x[sl] for x in c], nulls=[x[sl] for x in z])
        for s in range(2):
            p = loc[s].drain_partials(wm)
            nh = sum(1 for f in p if f.startswith("hidden"))
            assert nh == len({col for kind, col in aggs if kind != "COUNT"})
            dg += glob.push_partials(p["key"], p["slice_start"], p["count"], [p["acc%d" % j] for j in range(len(names))],
                                     hidden=[p["hidden%d" % h] for h in range(nh)])
        assert_rows_equal(glob.advance_watermark(wm), o.advance_watermark(wm), names,
                          rtol=lambda nm: TOL.get(nm, 0.0), ctx="wm=%d" % wm)
    assert dg == do and do > 0
    for x in loc + [glob]:
        x.close()
    o.close()


@pytest.mark.parametrize("ci", range(len(CONFIGS)), ids=[c["window_kind"] + str(i) for i, c in enumerate(CONFIGS)])
def test_nullable_snapshot_restore_with_rescale(eng_mod, ci):
    """Checkpoint / restore of nullable handles (FWASNAP1 carries the hidden non-NULL counters after the
    accumulator columns): two subtasks checkpoint mid-stream, one subtask (scale-in) and then two with a new split
    restore, and the resumed rows -- NULL flags included -- equal the oracle's uninterrupted run."""
    from flink_amd import snapshot as S
    from oracle.oracle import Oracle
    cfg_kw = dict(semantics="TABLE", aggs=AGGS_F if ci % 2 else AGGS, key_capacity=2048, nullable_cols=(0, 1, 2),
                  **CONFIGS[ci])
    cfg = A.make_config(**cfg_kw)
    names = A.agg_names(cfg)
    keys, ts, cols, nulls = _stream(500 + ci, 30_000, 400, 50_000, 1000, 0.25)
    kgs, _ = eng_mod.key_groups(keys, 128, 1, cfg.key_kind)
    cut = 15_000
    wm1 = int(ts[:cut].max()) - 1001
    o = Oracle(cfg)
    o.push(keys[:cut], ts[:cut], [c[:cut] for c in cols], nulls=[z[:cut] for z in nulls])
    first = o.advance_watermark(wm1)
    o.push(keys[cut:], ts[cut:], [c[cut:] for c in cols], nulls=[z[cut:] for z in nulls])
    final = o.advance_watermark(A.LONG_MAX)
    blobs, got1 = [], []
    for lo, hi in ((0, 63), (64, 127)):
        m = (kgs[:cut] >= lo) & (kgs[:cut] <= hi)
        g = eng_mod.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **cfg_kw))
        g.push(keys[:cut][m], ts[:cut][m], [c[:cut][m] for c in cols], nulls=[z[:cut][m] for z in nulls])
        got1.append(g.advance_watermark(wm1))
        b = g.snapshot()
        assert S.parse(b)["watermark"] == wm1
        blobs.append(b)
        g.close()
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names,
                      rtol=lambda nm: TOL.get(nm, 0.0))
    for layout in ([(0, 127)], [(0, 31), (32, 127)]):
        outs = []
        for lo, hi in layout:
            g = eng_mod.WindowAggregator(A.make_config(kg_start=lo, kg_end=hi, **cfg_kw))
            g.restore(blobs)
            m = (kgs[cut:] >= lo) & (kgs[cut:] <= hi)
            g.push(keys[cut:][m], ts[cut:][m], [c[cut:][m] for c in cols], nulls=[z[cut:][m] for z in nulls])
            outs.append(g.advance_watermark(A.LONG_MAX))
            g.close()
        assert_rows_equal({f: np.concatenate([r[f] for r in outs]) for f in outs[0]}, final, names,
                          rtol=lambda nm: TOL.get(nm, 0.0))
    o.close()
