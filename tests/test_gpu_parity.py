"""GPU parity tests: the HIP engine (through the C-ABI) against the CPU oracle and the reference KATs.

Integer aggregates, window bounds, keys and late-drop counts must be bit-exact; floating-point
aggregates are compared within the tolerances stated per aggregate below (GPU accumulates float
inputs in f64 with atomics, the reference in f32/f64 sequential order).
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal, assigner_windows_by_rows, load_kats, load_pyflink_kats, load_session_kats, load_tz_kats, replay_kat

pytestmark = pytest.mark.gpu

KATS = load_kats()
TZ_KATS = load_tz_kats()
PY_KATS = load_pyflink_kats()
SESSION_KATS = load_session_kats()

# Relative tolerances per aggregate (absolute floor equal to the same number, values are O(1..1e3)).
#  SUM_F32: reference accumulates in float32 sequentially: |err| <= n * 2^-24 * sum|x|; n <= ~2e3 here.
#  AVG_F32: both sides sum in double, result cast to float: one float rounding apart.
#  *_F64 sums/avgs: reordering of <= 1e4 additions of [0,1) values.
TOL = {"SUM_F32": 2e-4, "AVG_F32": 1e-6, "SUM_F64": 1e-9, "AVG_F64": 1e-9}


def tol(name):
    return TOL.get(name, 0.0)


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("case", KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_reference_kats_on_gpu(eng_mod, case):
    replay_kat(case, eng_mod.WindowAggregator)


@pytest.mark.parametrize("case", PY_KATS["operators"], ids=lambda c: c["name"].split(" ", 1)[1])
def test_pyflink_window_operator_sequences_on_gpu(eng_mod, case):
    """Random tumbling / sliding / session / dynamic-gap streams with lateness and late records, expected rows
    and drop counts produced by the reference's own Python WindowOperator (tests/golden/gen_pyflink_kats.py)."""
    replay_kat(case, eng_mod.WindowAggregator)


@pytest.mark.parametrize("case", SESSION_KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_session_merge_kats_on_gpu(eng_mod, case):
    """EventTimeSessionWindowsTest mergeWindows / TimeWindowTest.testIntersect as session sequences."""
    replay_kat(case, eng_mod.WindowAggregator)


@pytest.mark.parametrize("case", KATS["assigners"] + SESSION_KATS["assigners"], ids=lambda c: c["src"].split("/")[-1])
def test_assigner_kats_on_gpu(eng_mod, case):
    """Assigner / TimeWindowTest window starts as the windows the engine fires."""
    got = assigner_windows_by_rows(case, eng_mod.WindowAggregator)
    for ts, exp in case["cases"]:
        assert got[ts] == sorted(tuple(w) for w in exp), (ts, got[ts], exp)


@pytest.mark.parametrize("gap", SESSION_KATS["invalid_gaps"]["gaps"])
def test_session_invalid_gap_on_gpu(eng_mod, gap):
    """EventTimeSessionWindowsTest.testInvalidParameters: a gap <= 0 is rejected at create."""
    with pytest.raises(eng_mod.EngineError) as ei:
        eng_mod.WindowAggregator(A.make_config(window_kind="SESSION", gap_ms=gap, size_ms=0))
    assert ei.value.code == -1


@pytest.mark.parametrize("case", TZ_KATS["operators"], ids=lambda c: c["name"].split(" ")[0])
def test_reference_kats_shift_time_zone_on_gpu(eng_mod, case):
    """SlicingWindowAggOperatorTest's Asia/Shanghai parameterisation through the engine."""
    replay_kat(case, eng_mod.WindowAggregator)


I64_AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0), ("AVG_I64", 0)]
F64_AGGS = [("SUM_F64", 2), ("AVG_F64", 2), ("MIN_F64", 2), ("MAX_F64", 2), ("COUNT", 0)]
F32_AGGS = [("COUNT", 0), ("SUM_F32", 1), ("MIN_F32", 1), ("MAX_F32", 1), ("AVG_F32", 1)]

CONFIGS = [
    dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000),
    dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, offset_ms=-300),
    dict(window_kind="TUMBLE", semantics="TABLE", size_ms=700, offset_ms=100),
    dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=3000, slide_ms=1000),
    dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=5000, slide_ms=2000, offset_ms=300),
    dict(window_kind="SLIDE", semantics="TABLE", size_ms=4000, slide_ms=1000),
    dict(window_kind="CUMULATE", semantics="TABLE", size_ms=3000, slide_ms=1000),
    dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700),
    dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=2500),
    dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=700, allowed_lateness_ms=1200),
    dict(window_kind="SESSION", semantics="TABLE", gap_ms=900),
]


def random_stream(seed, n, nkeys, span, delay, late_frac=0.02):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-nkeys // 2, nkeys // 2, n).astype(np.int64)
    keys[rng.random(n) < 0.001] = -2**63          # the key-table sentinel value is a legal key
    base = np.sort(rng.integers(0, span, n)).astype(np.int64)
    ts = base - rng.integers(0, delay + 1, n)
    late = rng.random(n) < late_frac
    ts[late] -= rng.integers(delay, 4 * delay + 1, late.sum())
    vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
    vi[rng.random(n) < 0.01] = 2**62 + 12345     # exercise i64 wrap-around in SUM
    vf = rng.random(n).astype(np.float32) * 100
    vd = rng.random(n) * 1000.0 - 500.0
    return keys, ts, vi, vf, vd


def run_pair(cfg, batches, mk_gpu, mk_cpu, names):
    g = mk_gpu(cfg)
    o = mk_cpu(cfg)
    total_g = total_o = 0
    for (k, t, cols, wm) in batches:
        total_g += g.push(k, t, cols)
        total_o += o.push(k, t, cols)
        rg = g.advance_watermark(wm)
        ro = o.advance_watermark(wm)
        assert_rows_equal(rg, ro, names, rtol=tol, ctx="wm=%d" % wm)
    assert total_g == total_o
    g.close()
    o.close()
    return total_g


def batches_of(stream, nb, delay, final=True):
    keys, ts, vi, vf, vd = stream
    n = len(keys)
    out = []
    max_ts = -2**63
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        max_ts = max(max_ts, int(ts[sl].max()))
        out.append((keys[sl], ts[sl], [vi[sl], vf[sl], vd[sl]], max_ts - delay - 1))
    if final:
        out.append((keys[:0], ts[:0], [vi[:0], vf[:0], vd[:0]], A.LONG_MAX))
    return out


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
@pytest.mark.parametrize("aggs", [I64_AGGS, F64_AGGS, F32_AGGS], ids=["i64", "f64", "f32"])
def test_random_streams_vs_oracle(eng_mod, ci, aggs):
    from oracle.oracle import Oracle
    cfg_kw = CONFIGS[ci]
    cfg = A.make_config(aggs=aggs, key_capacity=4096, **cfg_kw)
    names = A.agg_names(cfg)
    stream = random_stream(100 + ci, 40_000, 600, 60_000, 1500)
    dropped = run_pair(cfg, batches_of(stream, 12, 1500), eng_mod.WindowAggregator, Oracle, names)
    assert dropped > 0  # the stream has late records


@pytest.mark.parametrize("ci", range(7))
@pytest.mark.parametrize("aggs", [I64_AGGS, F64_AGGS], ids=["i64", "f64"])
def test_random_streams_window_passes_vs_oracle(eng_mod, ci, aggs):
    """The combiner's window passes (FWA_OPT_WINDOW_PASSES) from the first push, over every non-session config. These
    streams leave most lanes of a chunk as padding (rel = -1), which is what the r04 spilling build corrupted: its
    padding lanes came back as slice 0 with key 0 (extra rows, DESIGN.md section 4 "Skewed keys")."""
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=aggs, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(cfg)
    stream = random_stream(100 + ci, 40_000, 600, 60_000, 1500)
    run_pair(cfg, batches_of(stream, 12, 1500), lambda c: eng_mod.WindowAggregator(c, options={"window_passes": 1}),
             Oracle, names)


def test_binrow_and_prehashed_keys(eng_mod):
    from oracle.oracle import Oracle
    for kind in (A.KEY_BINROW_BIGINT, A.KEY_PREHASHED):
        cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, key_kind=kind,
                            aggs=[("COUNT", 0), ("SUM_I64", 0)], max_parallelism=128, kg_start=0, kg_end=127)
        rng = np.random.default_rng(5)
        k = rng.integers(0, 1000, 5000).astype(np.int64)
        t = np.sort(rng.integers(0, 20_000, 5000)).astype(np.int64)
        v = rng.integers(0, 100, 5000).astype(np.int64)
        kh = (k * 31 + 7).astype(np.int32) if kind == A.KEY_PREHASHED else None
        g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
        g.push(k, t, [v], key_hash=kh)
        o.push(k, t, [v], key_hash=kh)
        assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), A.agg_names(cfg))


def test_key_groups_vs_oracle(eng_mod):
    from oracle import oracle as O
    L = O.lib()
    rng = np.random.default_rng(7)
    keys = np.concatenate([rng.integers(-2**63, 2**63 - 1, 100_000, dtype=np.int64),
                           np.array([0, 1, -1, -2**63, 2**63 - 1], np.int64)])
    for kind in (A.KEY_JAVA_LONG, A.KEY_BINROW_BIGINT):
        for maxp, par in ((128, 8), (128, 3), (32768, 7)):
            kg, op = eng_mod.key_groups(keys, maxp, par, key_kind=kind)
            exp = np.array([L.or_key_group(int(x), kind, 0, maxp) for x in keys[:3000]], np.int32)
            assert np.array_equal(kg[:3000], exp)
            assert np.array_equal(op, (kg.astype(np.int64) * par // maxp).astype(np.int32))


def test_keygroup_violation_and_ts_min(eng_mod):
    cfg = A.make_config(kg_start=0, kg_end=0)
    g = eng_mod.WindowAggregator(cfg)
    with pytest.raises(eng_mod.EngineError) as ei:
        g.push(np.arange(1000), np.arange(1000), [np.arange(1000)])
    assert ei.value.code == -3
    g2 = eng_mod.WindowAggregator(A.make_config())
    with pytest.raises(eng_mod.EngineError) as ei:
        g2.push(np.array([5]), np.array([A.LONG_MIN]), [np.array([1])])
    assert ei.value.code == -2


def test_invalid_configs(eng_mod):
    with pytest.raises(eng_mod.EngineError) as ei:
        eng_mod.WindowAggregator(A.make_config(window_kind="TUMBLE", size_ms=1000, offset_ms=1000))
    assert ei.value.code == -1
    with pytest.raises(eng_mod.EngineError) as ei:
        eng_mod.WindowAggregator(A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=1000, slide_ms=300))
    assert ei.value.code == -1


def test_device_generator_bit_exact(eng_mod):
    import torch
    from oracle import oracle as O
    n = 1 << 16
    for dist in (0, 1):
        p = A.GenParams(seed_k=11, seed_t=22, seed_v=33, first_index=12345, total_records=1 << 24,
                        num_keys=50_000, t0_ms=1_700_000_000_000, span_ms=1_000_000, max_delay_ms=1000,
                        key_dist=dist, val_kind=1)
        cdf = None
        dcdf = None
        if dist == 1:
            w = 1.0 / np.arange(1, 50_001, dtype=np.float64) ** 1.1
            cdf = np.cumsum(w) / w.sum()
            dcdf = torch.from_numpy(cdf).cuda()
            p.zipf_cdf = dcdf.data_ptr()
        dev = [torch.empty(n, dtype=dt, device="cuda") for dt in (torch.int64, torch.int64, torch.int64, torch.float32, torch.float64)]
        eng_mod.generate(p, n, *dev)
        torch.cuda.synchronize()
        host = O.generate(p, n, want_floats=True, cdf=cdf)
        for d, h in zip(dev, host):
            assert np.array_equal(d.cpu().numpy(), h)


def test_device_pointer_push_and_output(eng_mod):
    """Zero-copy path used by bench.py: device inputs, device-resident outputs."""
    import torch
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)],
                        key_capacity=1 << 14, output_on_device=1)
    n = 1 << 18
    p = A.GenParams(seed_k=1, seed_t=2, seed_v=3, first_index=0, total_records=n, num_keys=10_000, t0_ms=0,
                    span_ms=100_000, max_delay_ms=1000, key_dist=0, val_kind=0)
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty_like(k)
    v = torch.empty_like(k)
    eng_mod.generate(p, n, k, t, v)
    torch.cuda.synchronize()
    g = eng_mod.WindowAggregator(cfg)
    g.push(k, t, [v])
    rows = g.advance_watermark(A.LONG_MAX)
    cfg2 = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)])
    o = Oracle(cfg2)
    o.push(k.cpu().numpy(), t.cpu().numpy(), [v.cpu().numpy()])
    assert_rows_equal(rows, o.advance_watermark(A.LONG_MAX), ["COUNT", "SUM_I64"])


def test_c2_scaled_properties(eng_mod):
    """C2 shape at 2^24 records: exact equality with the oracle plus conservation of COUNT/SUM."""
    import torch
    from oracle.oracle import Oracle
    n = 1 << 24
    nk = 1 << 20
    p = A.GenParams(seed_k=0x1234, seed_t=0x5678, seed_v=0x9abc, first_index=0, total_records=n, num_keys=nk,
                    t0_ms=0, span_ms=1_000_000 * n // 1_000_000_000, max_delay_ms=1000, key_dist=0, val_kind=0)
    aggs = [("COUNT", 0), ("SUM_I64", 0)]
    cfg = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=aggs, key_capacity=nk)
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty_like(k)
    v = torch.empty_like(k)
    eng_mod.generate(p, n, k, t, v)
    g = eng_mod.WindowAggregator(cfg)
    o = Oracle(cfg)
    kh, th, vh = k.cpu().numpy(), t.cpu().numpy(), v.cpu().numpy()
    nb = 4
    tot_cnt = 0
    tot_sum = 0
    dropped = 0
    max_ts = -2**63
    for b in range(nb + 1):
        if b < nb:
            sl = slice(b * n // nb, (b + 1) * n // nb)
            dropped += g.push(k[sl], t[sl], [v[sl]])
            o.push(kh[sl], th[sl], [vh[sl]])
            max_ts = max(max_ts, int(th[sl].max()))
            wm = max_ts - 1000 - 1
        else:
            wm = A.LONG_MAX
        rg = g.advance_watermark(wm)
        ro = o.advance_watermark(wm)
        assert_rows_equal(rg, ro, ["COUNT", "SUM_I64"], ctx="batch %d" % b)
        tot_cnt += int(rg["agg0"].sum())
        tot_sum += int(rg["agg1"].astype(object).sum())
    assert tot_cnt + dropped == n
    assert dropped == 0  # bounded out-of-orderness D: nothing is late
    assert tot_sum == int(vh.astype(object).sum())


def test_session_edge_cases(eng_mod):
    """Touching windows merge (TimeWindow.intersects is inclusive), a late record survives only when it
    touches an in-flight session, a fired session is retired (a later touching record opens a new one),
    the INT64_MIN key and window-end overflow (ts + gap wraps) behave as in the reference."""
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="SESSION", gap_ms=1000, aggs=[("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)],
                        key_capacity=1024)
    L = A.LONG_MAX
    steps = [
        ([(1, 0), (1, 1000), (1, 2000), (2, 5), (-2**63, 7)], 500),      # 1: [0,3000) via touching merges
        ([(1, 100), (2, 6000), (1, 2999)], 1500),                          # late 100 merges into in-flight session
        ([(2, 100), (1, 5000), (2, 4000), (5, 2500)], 2998),               # key 2 @100: late, alone -> dropped
        ([(1, 2500), (1, 3000), (3, L - 10), (5, 1600), (6, 1600)], 4000), # late 5@1600 touches in-flight -> kept
        ([(1, 4100), (1, 3999), (3, L - 5)], L),                           # 1@3999: fired session retired -> new
    ]
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    for recs, wm in steps:
        k = np.array([r[0] for r in recs], np.int64)
        t = np.array([r[1] for r in recs], np.int64)
        v = np.arange(len(recs), dtype=np.int64) * 7 + 3
        assert g.push(k, t, [v]) == o.push(k, t, [v])
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), A.agg_names(cfg), ctx="wm=%d" % wm)
    assert g.stats().late_dropped == o.stats().late_dropped


def test_session_hot_key_many_records(eng_mod):
    """One key with thousands of records in a batch (a long sequential run) plus many short keys."""
    from oracle.oracle import Oracle
    rng = np.random.default_rng(3)
    n = 20_000
    k = np.where(rng.random(n) < 0.3, 42, rng.integers(0, 3000, n)).astype(np.int64)
    t = np.sort(rng.integers(0, 200_000, n)).astype(np.int64) - rng.integers(0, 3000, n)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=300, aggs=[("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0)],
                        key_capacity=4096)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    for b in range(4):
        sl = slice(b * n // 4, (b + 1) * n // 4)
        assert g.push(k[sl], t[sl], [v[sl]]) == o.push(k[sl], t[sl], [v[sl]])
        wm = int(t[: (b + 1) * n // 4].max()) - 3001 if b < 3 else A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), A.agg_names(cfg), ctx="b=%d" % b)


C2_AGGS = [("COUNT", 0), ("SUM_I64", 0)]


@pytest.mark.parametrize("ci", [i for i, c in enumerate(CONFIGS) if c["window_kind"] != "SESSION"])
@pytest.mark.parametrize("aggs", [I64_AGGS, F64_AGGS, C2_AGGS, [("COUNT", 0)]], ids=["i64", "f64", "c2", "count"])
def test_two_phase_partials_vs_oracle(eng_mod, ci, aggs):
    """Flink's two-phase plan (TwoStageOptimizedWindowAggregateRule.java:88-103): two local
    pre-aggregators (LocalSlicingWindowAggOperator) drain (key, slice) partials at every watermark, the
    owner merges them (GlobalAggCombiner.java:77-110) and fires. Rows and late-drop totals must equal
    one operator over the union of the streams."""
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=aggs, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(cfg)
    stream = random_stream(300 + ci, 30_000, 500, 50_000, 1200)
    loc = [eng_mod.WindowAggregator(cfg) for _ in range(2)]
    glob, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    dropped_g = dropped_o = 0
    for (k, t, cols, wm) in batches_of(stream, 9, 1200):
        dropped_o += o.push(k, t, cols)
        for s in range(2):
            sl = slice(s, None, 2)
            dropped_g += loc[s].push(k[sl], t[sl], [c[sl] for c in cols])
        for s in range(2):
            p = loc[s].drain_partials(wm)
            dropped_g += glob.push_partials(p["key"], p["slice_start"], p["count"],
                                            [p["acc%d" % j] for j in range(len(names))])
        assert_rows_equal(glob.advance_watermark(wm), o.advance_watermark(wm), names, rtol=tol, ctx="wm=%d" % wm)
    assert dropped_g == dropped_o and dropped_o > 0
    assert all(l.stats().rows_out == 0 for l in loc)   # pre-aggregators never fire windows themselves


@pytest.mark.parametrize("ci", [0, 3, 6])
def test_async_push_vs_oracle(eng_mod, ci):
    """FWA_PUSH_ASYNC: batches are enqueued without a host sync and settled by the next call (a
    following push or the watermark). Two pushes per watermark, late records and slice misses
    (replays) included; rows and the late-drop total must equal the oracle's."""
    import torch
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=I64_AGGS, key_capacity=4096, output_on_device=0, **CONFIGS[ci])
    names = A.agg_names(cfg)
    keys, ts, vi, vf, vd = random_stream(300 + ci, 48_000, 600, 60_000, 1500)
    g = eng_mod.WindowAggregator(cfg)
    o = Oracle(cfg)
    n = len(keys)
    dk, dt, dv = (torch.from_numpy(x).cuda() for x in (keys, ts, vi))
    nb = 12
    max_ts = -2**63
    dropped_o = 0
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        max_ts = max(max_ts, int(ts[sl].max()))
        assert g.push(dk[sl], dt[sl], [dv[sl]], sync=False) == 0
        dropped_o += o.push(keys[sl], ts[sl], [vi[sl]])
        if b % 2 == 1:
            wm = max_ts - 1500 - 1
            assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=tol, ctx="wm=%d" % wm)
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), names, rtol=tol)
    st = g.stats()
    assert dropped_o > 0 and st.late_dropped == dropped_o and st.records_in == n
    g.close()
    o.close()


SLIDE_SUM_AGGS = [("COUNT", 0), ("SUM_I64", 0), ("AVG_I64", 0)]


@pytest.mark.parametrize("ci", [3, 4, 5])
def test_slide_running_fire_vs_oracle(eng_mod, ci):
    """Hop windows with invertible accumulators fire through fire_slide_kernel (running sums over a
    run of consecutive windows): bit-exact against the oracle, including i64 wrap-around."""
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=SLIDE_SUM_AGGS, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(cfg)
    stream = random_stream(500 + ci, 40_000, 600, 60_000, 1500)
    dropped = run_pair(cfg, batches_of(stream, 8, 1500), eng_mod.WindowAggregator, Oracle, names)
    assert dropped > 0


def test_c3_shape_zipf_hop_vs_oracle(eng_mod):
    """C3 shape at 2^19 records: Table HOP 60 s / 1 s, Zipf(1.1) keys (one key carries ~11 % of the
    records: bucket overflow and replay), COUNT + SUM(long), device generator, exact equality."""
    import torch
    from oracle import oracle as O
    n, nkeys = 1 << 19, 100_000
    w = 1.0 / np.arange(1, nkeys + 1, dtype=np.float64) ** 1.1
    cdf = np.cumsum(w) / w.sum()
    dcdf = torch.from_numpy(cdf).cuda()
    p = A.GenParams(seed_k=5, seed_t=6, seed_v=7, first_index=0, total_records=n, num_keys=nkeys, t0_ms=0,
                    span_ms=200_000, max_delay_ms=1000, key_dist=1, val_kind=0)
    p.zipf_cdf = dcdf.data_ptr()
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty_like(k)
    v = torch.empty_like(k)
    eng_mod.generate(p, n, k, t, v)
    torch.cuda.synchronize()
    kh, th, vh = k.cpu().numpy(), t.cpu().numpy(), v.cpu().numpy()
    assert np.array_equal((kh, th, vh)[0], O.generate(p, n, cdf=cdf)[0])
    cfg = A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=60_000, slide_ms=1_000,
                        aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=nkeys)
    g = eng_mod.WindowAggregator(cfg)
    o = O.Oracle(cfg)
    nb = 4
    for b in range(nb + 1):
        if b < nb:
            sl = slice(b * n // nb, (b + 1) * n // nb)
            g.push(k[sl], t[sl], [v[sl]])
            o.push(kh[sl], th[sl], [vh[sl]])
            wm = int(th[: (b + 1) * n // nb].max()) - 1001
        else:
            wm = A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), ["COUNT", "SUM_I64"], ctx="wm=%d" % wm)
    g.close()
    o.close()


@pytest.mark.parametrize("case", KATS["key_groups"], ids=lambda c: c["src"].split("/")[-1].split(" ")[0])
def test_key_group_literal_kats_on_gpu(eng_mod, case):
    """fwa_key_groups (PREHASHED: the caller passes key.hashCode()) reproduces the key groups and
    operator indices the reference's tests assert (RocksIncrementalCheckpointRescalingTest, CEPRescalingTest)."""
    from helpers import java_hash_code
    maxp = case["max_parallelism"]
    keys = np.array([i for i, _ in enumerate(case["cases"])], np.int64)
    kh = np.array([java_hash_code(k, case["key_type"]) for k, _ in case["cases"]], np.int32)
    kg, _ = eng_mod.key_groups(keys, maxp, 1, key_kind=A.KEY_PREHASHED, key_hash=kh)
    assert kg.tolist() == [g for _, g in case["cases"]]
    for key, par, op in case["operator_index"]:
        _, o = eng_mod.key_groups(np.array([0], np.int64), maxp, par, key_kind=A.KEY_PREHASHED,
                                  key_hash=np.array([java_hash_code(key, case["key_type"])], np.int32))
        assert int(o[0]) == op, (key, par)


def test_late_firing_rows_survive_snapshot(eng_mod):
    """a snapshot (non-destructive raw fire) taken after a push with late firings must not
    discard the pending late-firing rows; the next watermark returns them, as without the snapshot."""
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, allowed_lateness_ms=5000,
                        aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1024)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    k = np.array([1, 2, 1, 3], np.int64)
    t = np.array([100, 200, 1500, 2500], np.int64)
    v = np.array([1, 2, 3, 4], np.int64)
    for x in (g, o):
        x.push(k, t, [v])
    assert_rows_equal(g.advance_watermark(3000), o.advance_watermark(3000), ["COUNT", "SUM_I64"])
    k2 = np.array([1, 1, 2], np.int64)           # windows [0,1000) fired at 3000, not past cleanup (5999)
    t2 = np.array([300, 400, 999], np.int64)
    v2 = np.array([10, 20, 30], np.int64)
    for x in (g, o):
        x.push(k2, t2, [v2])
    blob = g.snapshot()
    assert len(blob) > 0
    rg, ro = g.advance_watermark(3000), o.advance_watermark(3000)   # non-advancing: only the late rows
    assert len(ro["key"]) == 3
    assert_rows_equal(rg, ro, ["COUNT", "SUM_I64"])
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), ["COUNT", "SUM_I64"])


@pytest.mark.parametrize("zone", ["America/Los_Angeles", "Asia/Shanghai"])
@pytest.mark.parametrize("kind,size,slide", [("TUMBLE", 3_600_000, 0), ("SLIDE", 4 * 3_600_000, 3_600_000),
                                             ("CUMULATE", 4 * 3_600_000, 3_600_000)])
def test_shift_time_zone_streams_vs_oracle(eng_mod, zone, kind, size, slide):
    """TIMESTAMP_LTZ rowtime: slices in local wall-clock time, windows fire at toEpochMillsForTimer(end - 1);
    streams span the 2021 America/Los_Angeles DST days (a 23 h and a 25 h day)."""
    from oracle.oracle import Oracle
    tzk = {c["zone"]: c["tz"] for c in TZ_KATS["timer"]}
    cfg = A.make_config(window_kind=kind, semantics="TABLE", size_ms=size, slide_ms=slide, tz=tzk[zone],
                        aggs=[("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)], key_capacity=2048)
    names = A.agg_names(cfg)
    rng = np.random.default_rng(17)
    batches = []
    for t0 in (1615593600000, 1636156800000):         # 2021-03-13 and 2021-11-06, 00:00 UTC
        n = 30_000
        base = t0 + np.sort(rng.integers(0, 3 * 86_400_000, n)).astype(np.int64)
        ts = base - rng.integers(0, 600_000, n)
        keys = rng.integers(0, 300, n).astype(np.int64)
        vi = rng.integers(-1000, 1000, n).astype(np.int64)
        for b in range(12):
            sl = slice(b * n // 12, (b + 1) * n // 12)
            batches.append((keys[sl], ts[sl], [vi[sl]], int(ts[sl].max()) - 600_001))
    batches.append((batches[0][0][:0], batches[0][1][:0], [batches[0][2][0][:0]], A.LONG_MAX))
    run_pair(cfg, batches, eng_mod.WindowAggregator, Oracle, names)


@pytest.mark.parametrize("zone", ["America/Los_Angeles", "Asia/Shanghai"])
@pytest.mark.parametrize("gap", [300_000, 1_800_000])
def test_shift_time_zone_sessions_vs_oracle(eng_mod, zone, gap):
    """Table GROUP BY SESSION over a TIMESTAMP_LTZ rowtime (TR WindowOperator.processElement :340): sessions are
    formed on local wall-clock time and every watermark comparison / timer is toEpochMillsForTimer of the local
    instant (InternalWindowProcessFunction.isWindowLate :119-123, MergingWindowProcessFunction :137-141). Streams
    cross the 2021 America/Los_Angeles DST changes (a 23 h and a 25 h day), with late records."""
    from oracle.oracle import Oracle
    tzk = {c["zone"]: c["tz"] for c in TZ_KATS["timer"]}
    cfg = A.make_config(window_kind="SESSION", semantics="TABLE", gap_ms=gap, tz=tzk[zone],
                        aggs=[("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)], key_capacity=2048)
    names = A.agg_names(cfg)
    rng = np.random.default_rng(29 + gap)
    batches = []
    for t0 in (1615593600000, 1636156800000):         # 2021-03-13 and 2021-11-06, 00:00 UTC
        n = 20_000
        base = t0 + np.sort(rng.integers(0, 2 * 86_400_000, n)).astype(np.int64)
        ts = base - rng.integers(0, 900_000, n)
        keys = rng.integers(0, 200, n).astype(np.int64)
        vi = rng.integers(-1000, 1000, n).astype(np.int64)
        for b in range(10):
            sl = slice(b * n // 10, (b + 1) * n // 10)
            batches.append((keys[sl], ts[sl], [vi[sl]], int(ts[sl].max()) - 600_001))
    batches.append((batches[0][0][:0], batches[0][1][:0], [batches[0][2][0][:0]], A.LONG_MAX))
    run_pair(cfg, batches, eng_mod.WindowAggregator, Oracle, names)


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_late_record_indices_vs_oracle(eng_mod, ci):
    """FWA_CFG_LATE_INDICES: per push, exactly the records the reference drops as late (the ones WindowOperator
    sends to lateDataOutputTag, and SlicingWindowProcessor.processElement returns true for)."""
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=I64_AGGS, key_capacity=4096, late_indices=True, **CONFIGS[ci])
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    total = 0
    for k, t, cols, wm in batches_of(random_stream(900 + ci, 30_000, 500, 50_000, 1500, late_frac=0.05), 10, 1500):
        dg, do = g.push(k, t, cols), o.push(k, t, cols)
        lg, lo = g.late_records(), o.late_records()
        assert dg == do == len(lg) == len(lo)
        assert np.array_equal(lg, lo)
        total += dg
        g.advance_watermark(wm)
        o.advance_watermark(wm)
    assert total > 0
    g.close()
    o.close()


@pytest.mark.parametrize("ci", [0, 3])
def test_partials_large_counts_and_late(eng_mod, ci):
    """Partial rows through the owner's two-phase path (COUNT + SUM(BIGINT): PRE buckets carry each row's record
    count) against the per-row v1 path (FWA_OPT_PARTIALS_ONE_PASS) on the same rows: counts above a bucket's u16 take the v1
    path, late partials add their counts to the drops, rows are identical."""
    cfg = A.make_config(aggs=C2_AGGS, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(cfg)
    rng = np.random.default_rng(17)
    n = 40_000
    keys = rng.integers(0, 3000, n).astype(np.int64)
    sts = np.sort(rng.integers(0, 60_000, n)).astype(np.int64)
    sts[rng.random(n) < 0.05] -= 25_000                             # late once the first watermark fired
    cnt = rng.integers(1, 50, n).astype(np.int64)
    big = rng.random(n) < 0.01
    cnt[big] = rng.integers(65_536, 1 << 40, int(big.sum()))
    acc = rng.integers(-2**40, 2**40, n).astype(np.int64)
    handles = {}
    for mode in ("v2", "v1"):
        g = eng_mod.WindowAggregator(cfg, options={"partials_one_pass": 1} if mode == "v1" else None)
        out, drops = [], 0
        for sl, wm in ((slice(0, n // 2), 30_000), (slice(n // 2, n), A.LONG_MAX)):
            drops += g.push_partials(keys[sl], sts[sl], cnt[sl], [cnt[sl], acc[sl]])
            out.append(g.advance_watermark(wm))
        handles[mode] = (out, drops, g.stats().ingest_launches)
        g.close()
    (o2, d2, _), (o1, d1, _) = handles["v2"], handles["v1"]
    assert d2 == d1 and d1 > 0
    for a_, b_ in zip(o2, o1):
        assert_rows_equal(a_, b_, names, ctx="partials v2 vs v1")
