"""GPU tests: fwa_advance_watermark_async / fwa_fired_output (include/flink_amd.h) give the rows fwa_advance_watermark
gives at the same point, with the next batch pushed while the fire runs (the bench's pipelined loop), against the
oracle (the reference's WindowOperator / SlicingWindowOperator restatement). Pushes that need a replay (slice misses
of a fresh handle, records that take the one-pass path) fall back to the synchronous step and stay exact."""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu


def _device_batches(seed, n, nkeys, span, delay, nb, late_frac=0.0):
    import torch
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    ts = np.sort(rng.integers(0, span, n)).astype(np.int64) - rng.integers(0, delay + 1, n)
    late = rng.random(n) < late_frac
    ts[late] -= rng.integers(delay, 4 * delay + 1, late.sum())
    vals = rng.integers(-2**31, 2**31, n).astype(np.int64)
    out, mx = [], -2**63
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        mx = max(mx, int(ts[sl].max()))
        out.append((keys[sl], ts[sl], vals[sl], mx - delay - 1))
    dev = [(torch.from_numpy(k).cuda(), torch.from_numpy(t).cuda(), torch.from_numpy(v).cuda(), wm) for k, t, v, wm in out]
    return out, dev


@pytest.mark.parametrize("sem,aggs,lateness", [("DATASTREAM", [("COUNT", 0), ("SUM_I64", 0)], 0),
                                               ("TABLE", [("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)], 0),
                                               ("DATASTREAM", [("SUM_I64", 0), ("AVG_I64", 0)], 0),
                                               ("DATASTREAM", [("COUNT", 0), ("SUM_I64", 0)], 1500)])
@pytest.mark.parametrize("late", [0.0, 0.01])
def test_async_watermark_pipeline_vs_oracle(sem, aggs, lateness, late):
    """Without allowed lateness the fire runs on the fire stream beside the next push (its windows retire at once);
    with it (fired windows still take late records) on the push's stream."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    host, dev = _device_batches(31, 1 << 20, 20_000, 200_000, 500, 10, late)
    kw = dict(window_kind="TUMBLE", semantics=sem, size_ms=7_000, aggs=aggs, key_capacity=1 << 16,
              allowed_lateness_ms=lateness)
    cfg = A.make_config(output_on_device=1, **kw)
    names = A.agg_names(cfg)
    g, o = engine.WindowAggregator(cfg), Oracle(A.make_config(**kw))
    expected = []
    for k, t, v, wm in host:
        o.push(k, t, [v])
        expected.append(o.advance_watermark(wm))
    expected.append(o.advance_watermark(A.LONG_MAX))
    got = []
    for b, (k, t, v, wm) in enumerate(dev):
        g.push(k, t, [v], sync=False)
        if b > 0:
            got.append(g.fired_output())
        g.advance_watermark_async(wm)
    got.append(g.fired_output())
    g.advance_watermark_async(A.LONG_MAX)          # no pending push: the synchronous path
    got.append(g.fired_output())
    assert len(got) == len(expected)
    for b, (rg, ro) in enumerate(zip(got, expected)):
        assert_rows_equal(rg, ro, names, ctx="watermark %d" % b)
    st = g.stats()
    assert st.records_in == sum(len(k) for k, _, _, _ in host)
    assert st.late_dropped == o.stats().late_dropped
    g.close()
    o.close()


def test_async_output_is_taken_once_and_other_calls_complete_the_fire():
    from flink_amd import engine
    host, dev = _device_batches(7, 1 << 18, 5_000, 60_000, 300, 3)
    cfg = A.make_config(window_kind="TUMBLE", size_ms=5_000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1 << 14,
                        output_on_device=1)
    g = engine.WindowAggregator(cfg)
    with pytest.raises(engine.EngineError):
        g.fired_output_raw()                        # nothing pending
    k, t, v, wm = dev[0]
    g.push(k, t, [v], sync=False)
    g.advance_watermark_async(wm)
    n0 = g.stats().rows_out                         # completes the fire
    k, t, v, wm = dev[1]
    g.push(k, t, [v], sync=False)
    g.advance_watermark_async(wm)
    out = g.fired_output_raw()
    assert out.n_rows == g.stats().rows_out - n0
    with pytest.raises(engine.EngineError):
        g.fired_output_raw()                        # taken
    g.close()
