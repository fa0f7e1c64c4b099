"""GPU tests: fwa_fire_partials, the owner's merge + fire over the exchange's packed partial rows (include/flink_amd.h).

Its contract is fwa_push_partials of the rows' cells followed by fwa_advance_watermark (GlobalAggCombiner.combine,
GlobalAggCombiner.java:77-110, then WindowOperator.onEventTime). Checked three ways:
  * the two-phase plan -- four local handles drain (key, slice) partials, the owner fires their concatenated rows --
    against one oracle operator over the union of the streams (the reference's WindowOperator /
    SlicingWindowOperator restatement), with the on-chip path asserted to have run;
  * the on-chip path against a handle with it switched off (the two defining calls) on row sets with late partials,
    windows not yet due at the owner's watermark (the call is redone), one key spanning thousands of windows (a
    bucket past its region: redone) and the INT64_MIN key;
  * key-group ownership errors like fwa_push_partials."""
import numpy as np
import pytest
import torch

from flink_amd import _abi as A
from helpers import assert_rows_equal
from test_gpu_parity import random_stream

pytestmark = pytest.mark.gpu

# float sums merge in another order than the single operator's arrival order (SUM(FLOAT) accumulates in f64 and
# rounds once)
TOL = {"SUM_F32": 2e-4, "AVG_F32": 1e-6, "SUM_F64": 1e-9, "AVG_F64": 1e-9}
AGGS_I = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0), ("AVG_I64", 0)]
AGGS_F = [("COUNT", 0), ("SUM_F64", 2), ("AVG_F64", 2), ("MAX_F32", 1), ("MIN_F64", 2), ("SUM_F32", 1)]
AGGS_N = [("COUNT", 0), ("COUNT_COL", 0), ("SUM_I64", 0), ("AVG_F64", 2), ("MIN_F32", 1), ("MAX_I64", 0)]
CASES = {
    "ds_tumble_int": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=2000, aggs=AGGS_I),
    "ds_tumble_offset": dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000, offset_ms=-250, aggs=AGGS_I),
    "table_tumble_float": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=1500, offset_ms=300, aggs=AGGS_F),
    "table_tumble_nullable": dict(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=AGGS_N,
                                  nullable_cols=(0, 1, 2)),
}
NSRC = 4


def rtol(name):
    return TOL.get(name, 0.0)


def pack(parts, names):
    """drain_partials dicts (device views) -> packed int64 rows [n, m] and the accumulator cells, in the layout the
    two-phase pipeline ships (distributed.TwoPhaseKeyedWindowPipeline)."""
    ship = [j for j, nm in enumerate(names) if nm != "COUNT"]
    nh = sum(1 for f in parts[0] if f.startswith("hidden"))
    blocks = []
    for p in parts:
        cols = [p["key"], p["slice_start"], p["count"]] + [p["acc%d" % j] for j in ship] + \
            [p["hidden%d" % h] for h in range(nh)]
        blocks.append(torch.stack([c.view(torch.int64) for c in cols], dim=1))
    cells = [2 if nm == "COUNT" else 3 + ship.index(j) for j, nm in enumerate(names)] + \
        [3 + len(ship) + h for h in range(nh)]
    return torch.cat(blocks), cells


def stream(case, seed, n=160_000, nb=10, delay=800):
    keys, ts, vi, vf, vd = random_stream(seed, n, 3000, 60_000, delay, 0.02)
    rng = np.random.default_rng(seed + 1)
    nulls = [(rng.random(n) < 0.2).astype(np.uint8) for _ in range(3)] if "nullable_cols" in CASES[case] else None
    mx = -2**63
    for b in range(nb + 1):
        if b < nb:
            sl = slice(b * n // nb, (b + 1) * n // nb)
            mx = max(mx, int(ts[sl].max()))
            yield sl, keys, ts, [vi, vf, vd], nulls, mx - delay - 1
        else:
            yield slice(0, 0), keys, ts, [vi, vf, vd], nulls, A.LONG_MAX


def local_push(loc, s, sl, keys, ts, cols, nulls):
    idx = np.arange(sl.start, sl.stop)[s::NSRC]
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x[idx])).cuda()  # noqa: E731
    return loc.push(dev(keys), dev(ts), [dev(c) for c in cols], nulls=None if nulls is None else [dev(x) for x in nulls])


@pytest.mark.parametrize("case", list(CASES))
def test_two_phase_fire_partials_vs_oracle(case):
    from flink_amd import engine
    from oracle.oracle import Oracle
    kw = dict(key_capacity=4096, **CASES[case])
    cfg = A.make_config(output_on_device=1, **kw)
    names = A.agg_names(cfg)
    locs = [engine.WindowAggregator(cfg) for _ in range(NSRC)]
    owner = engine.WindowAggregator(A.make_config(**kw))
    o = Oracle(A.make_config(**kw))
    late_o = late_l = 0
    for b, (sl, keys, ts, cols, nulls, wm) in enumerate(stream(case, 21)):
        if sl.stop > sl.start:
            late_o += o.push(keys[sl], ts[sl], [c[sl] for c in cols], nulls=None if nulls is None else [x[sl] for x in nulls])
            for s in range(NSRC):
                late_l += local_push(locs[s], s, sl, keys, ts, cols, nulls)
        rows, cells = pack([loc.drain_partials(wm) for loc in locs], names)
        assert_rows_equal(owner.fire_partials(rows, cells, wm), o.advance_watermark(wm), names, rtol=rtol,
                          ctx="%s wm=%d" % (case, wm))
    assert owner.get_option("fire_partials") >= 10          # every step merged and fired on chip
    assert late_l + owner.stats().late_dropped == late_o and late_o > 0
    for x in locs + [owner]:
        x.close()
    o.close()


def pair(kw):
    from flink_amd import engine
    fast = engine.WindowAggregator(A.make_config(**kw))
    slow = engine.WindowAggregator(A.make_config(**kw))
    slow.set_option("fire_partials", 0)
    return fast, slow


@pytest.mark.parametrize("case", list(CASES))
def test_fire_partials_equals_push_partials_then_fire(case):
    """Each call re-sends the previous step's rows (late at the owner by then: dropped, counted) and every third
    call lags the owner's watermark one step behind the drains (windows not yet due: the call is redone through the
    defining calls, and the owner then holds their state until a later watermark fires them)."""
    from flink_amd import engine
    kw = dict(key_capacity=4096, **CASES[case])
    cfg = A.make_config(output_on_device=1, **kw)
    names = A.agg_names(cfg)
    locs = [engine.WindowAggregator(cfg) for _ in range(NSRC)]
    fast, slow = pair(kw)
    prev, prev_wm = None, A.LONG_MIN
    for b, (sl, keys, ts, cols, nulls, wm) in enumerate(stream(case, 33, nb=12)):
        if sl.stop > sl.start:
            for s in range(NSRC):
                local_push(locs[s], s, sl, keys, ts, cols, nulls)
        rows, cells = pack([loc.drain_partials(wm) for loc in locs], names)
        send = rows if prev is None else torch.cat([prev, rows])
        owm = prev_wm if (b % 3 == 1 and prev_wm > A.LONG_MIN and wm != A.LONG_MAX) else wm
        assert_rows_equal(fast.fire_partials(send, cells, owm), slow.fire_partials(send, cells, owm), names,
                          rtol=rtol, ctx="%s step %d" % (case, b))
        assert fast.stats().late_dropped == slow.stats().late_dropped
        prev, prev_wm = rows, wm
    assert fast.stats().late_dropped > 0
    assert fast.get_option("fire_partials") >= 4 and slow.get_option("fire_partials") == 0
    for x in locs + [fast, slow]:
        x.close()


def test_one_key_across_thousands_of_windows_is_redone():
    """Every slice of a key hashes to one bucket: 6000 windows of one key overflow its region, the call is redone
    through the defining calls; a later call with ordinary rows takes the on-chip path again."""
    from flink_amd import engine
    kw = dict(window_kind="TUMBLE", size_ms=10, aggs=AGGS_I, key_capacity=8192)
    cfg = A.make_config(output_on_device=1, **kw)
    names = A.agg_names(cfg)
    loc = engine.WindowAggregator(cfg)
    n = 6000
    k = torch.full((n,), -2**63, dtype=torch.int64, device="cuda")     # the key-table sentinel value as the key
    t = torch.arange(n, dtype=torch.int64, device="cuda") * 10 + 3
    v = torch.arange(n, dtype=torch.int64, device="cuda") - 77
    loc.push(k, t, [v])
    rows, cells = pack([loc.drain_partials(n * 10)], names)
    fast, slow = pair(kw)
    r = fast.fire_partials(rows, cells, n * 10)
    assert len(r["key"]) == n and fast.get_option("fire_partials") == 0
    assert_rows_equal(r, slow.fire_partials(rows, cells, n * 10), names)
    k2 = torch.arange(5000, dtype=torch.int64, device="cuda")
    loc.push(k2, torch.full_like(k2, n * 10 + 5), [k2 * 3])
    rows, cells = pack([loc.drain_partials(A.LONG_MAX)], names)
    assert_rows_equal(fast.fire_partials(rows, cells, A.LONG_MAX), slow.fire_partials(rows, cells, A.LONG_MAX), names)
    assert fast.get_option("fire_partials") == 1
    for x in (loc, fast, slow):
        x.close()


def test_fire_partials_key_group_error():
    from flink_amd import engine
    kw = dict(window_kind="TUMBLE", size_ms=1000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1024)
    names = A.agg_names(A.make_config(**kw))
    keys = np.arange(2000, dtype=np.int64)
    kgs, _ = engine.key_groups(keys, 128, 1)
    loc = engine.WindowAggregator(A.make_config(output_on_device=1, **kw))
    dk = torch.from_numpy(keys).cuda()
    loc.push(dk, torch.full_like(dk, 10), [dk])
    rows, cells = pack([loc.drain_partials(A.LONG_MAX)], names)
    assert (kgs > 63).any()
    for off in (1, 0):
        own = engine.WindowAggregator(A.make_config(kg_start=0, kg_end=63, **kw))
        own.set_option("fire_partials", off)
        with pytest.raises(engine.EngineError) as ei:
            own.fire_partials(rows, cells, A.LONG_MAX)
        assert ei.value.code == -3          # FWA_E_KEYGROUP
        own.close()
    loc.close()


@pytest.mark.parametrize("par", [1, 3, 8])
@pytest.mark.parametrize("case", ["ds_tumble_int", "table_tumble_nullable"])
def test_drain_route_equals_drain_then_route(case, par):
    """fwa_drain_route: the rows of fwa_drain_partials, packed in the exchange's layout and grouped by owning subtask
    exactly as fwa_route_rows groups them (row order inside a destination aside)."""
    from flink_amd import engine
    cfg = A.make_config(output_on_device=1, key_capacity=4096, **CASES[case])
    names = A.agg_names(cfg)
    a, b = engine.WindowAggregator(cfg), engine.WindowAggregator(cfg)
    srt = lambda x: x[np.lexsort((x[:, 1], x[:, 0]))] if len(x) else x  # noqa: E731   (key, slice): unique
    total = 0
    for sl, keys, ts, cols, nulls, wm in stream(case, 45, nb=6):
        if sl.stop > sl.start:
            for x in (a, b):
                local_push(x, 0, sl, keys, ts, cols, nulls)
        parts, counts, m = a.drain_route(wm, par)
        rows, _ = pack([b.drain_partials(wm)], names)
        packed, cnt = engine.route_rows(rows[:, 0].contiguous(), [rows[:, j].contiguous() for j in range(rows.shape[1])],
                                        128, par)
        assert m == rows.shape[1] and counts == cnt.tolist()
        # float sums accumulate with LDS atomics in either handle: their bits may differ in the last place
        ship = [j for j, nm in enumerate(names) if nm != "COUNT"]
        fcell = [3 + i for i, j in enumerate(ship) if names[j] in ("SUM_F64", "AVG_F64", "SUM_F32", "AVG_F32")]
        icell = [c for c in range(m) if c not in fcell]
        off = 0
        for d in range(par):
            got = srt(parts[d].cpu().numpy())
            exp = srt(packed[off:off + counts[d]].cpu().numpy())
            off += counts[d]
            assert np.array_equal(got[:, icell], exp[:, icell]), (case, par, d)
            assert np.allclose(got[:, fcell].view(np.float64), exp[:, fcell].view(np.float64), rtol=1e-12, atol=1e-9)
        total += sum(counts)
    assert total > 1000
    a.close()
    b.close()


def test_table_full_after_a_duplicated_call_is_redone():
    """Buckets are sized from the groups per row the last call saw: after a call whose rows repeat each group 8 times,
    a call of distinct groups overfills the LDS tables, the call is redone through the defining calls (same rows) and
    the next call is sized for one group per row again and merges on chip."""
    from flink_amd import engine
    kw = dict(window_kind="TUMBLE", size_ms=1000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1 << 18)
    names = A.agg_names(A.make_config(**kw))
    fast, slow = pair(kw)
    cells = [2, 3]

    def rows_of(keys, start, copies):
        k = torch.as_tensor(np.repeat(keys, copies), device="cuda")
        return torch.stack([k, torch.full_like(k, start), torch.ones_like(k), k * 7], dim=1)

    steps = [(rows_of(np.arange(12_500), 0, 8), 999),            # 8 copies per group: ~1/8 group per row
             (rows_of(np.arange(100_000), 1000, 1), 1999),       # distinct groups: the tables overfill -> redone
             (rows_of(np.arange(100_000), 2000, 1), 2999)]       # sized for one group per row again: on chip
    used = []
    for rows, wm in steps:
        assert_rows_equal(fast.fire_partials(rows, cells, wm), slow.fire_partials(rows, cells, wm), names)
        used.append(fast.get_option("fire_partials"))
    assert used == [1, 1, 2]
    fast.close()
    slow.close()
