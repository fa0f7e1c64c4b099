"""GPU parity: late firings within allowed lateness (DataStream WindowOperator + EventTimeTrigger).

WindowOperator.processElement (:391-420) adds a late element to every window that is not past cleanup
(isWindowLate :586-589) and EventTimeTrigger.onElement (:37-45) FIREs at once when the window's
maxTimestamp <= watermark, emitting the window's whole contents (FIRE, not PURGE). Each such element
emits one row per fired window, showing the state after that element, so a (key, window) with m late
elements in a batch emits m rows. The engine returns these push-time rows with the next
fwa_advance_watermark; the oracle does the same. Rows and late-drop totals must match per watermark.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal
from test_gpu_parity import F64_AGGS, I64_AGGS, random_stream, tol

pytestmark = pytest.mark.gpu

LATE_CONFIGS = [
    dict(window_kind="TUMBLE", size_ms=1000, allowed_lateness_ms=2000),
    dict(window_kind="TUMBLE", size_ms=700, offset_ms=100, allowed_lateness_ms=900),
    dict(window_kind="SLIDE", size_ms=3000, slide_ms=1000, allowed_lateness_ms=1500),
    dict(window_kind="SLIDE", size_ms=5000, slide_ms=2000, offset_ms=300, allowed_lateness_ms=2500),
]


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("ci", range(len(LATE_CONFIGS)))
@pytest.mark.parametrize("aggs", [I64_AGGS, F64_AGGS], ids=["i64", "f64"])
def test_late_firings_vs_oracle(eng_mod, ci, aggs):
    from oracle.oracle import Oracle
    cfg = A.make_config(semantics="DATASTREAM", aggs=aggs, key_capacity=4096, **LATE_CONFIGS[ci])
    names = A.agg_names(cfg)
    keys, ts, vi, vf, vd = random_stream(900 + ci, 30_000, 300, 50_000, 1000, late_frac=0.05)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    n, nb = len(keys), 12
    max_ts = -2**63
    dg = do = 0
    late_rows = 0
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        cols = [vi[sl], vf[sl], vd[sl]]
        dg += g.push(keys[sl], ts[sl], cols)
        do += o.push(keys[sl], ts[sl], cols)
        max_ts = max(max_ts, int(ts[sl].max()))
        wm = max_ts - 1000 - 1 if b < nb - 1 else A.LONG_MAX
        if b % 4 == 2:     # a non-advancing watermark still returns the push-time late firings
            wm_same = g.stats().current_watermark
            rg, ro = g.advance_watermark(wm_same), o.advance_watermark(wm_same)
            late_rows += len(ro["key"])
            assert_rows_equal(rg, ro, names, rtol=tol, ctx="b=%d same wm" % b)
        rg, ro = g.advance_watermark(wm), o.advance_watermark(wm)
        assert_rows_equal(rg, ro, names, rtol=tol, ctx="b=%d wm=%d" % (b, wm))
    assert dg == do
    st = o.stats()
    assert st.rows_out > 0 and late_rows > 0   # push-time late firings did occur (oracle: 77..149)


def test_repeated_late_elements_same_window(eng_mod):
    """Three late elements for one (key, window) in one batch: three rows with counts 2, 3, 4 (after one
    on-time element); one more within lateness in the next batch; then one past cleanup is dropped."""
    from oracle.oracle import Oracle
    cfg = A.make_config(semantics="DATASTREAM", window_kind="TUMBLE", size_ms=1000, allowed_lateness_ms=500,
                        aggs=[("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)], key_capacity=1024)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    names = A.agg_names(cfg)
    steps = [([(7, 100, 1)], 1200), ([(7, 200, 5), (8, 300, 2), (7, 999, 3), (7, 500, 9)], 1300),
             ([(7, 10, 4), (9, 2500, 1)], 1600), ([(7, 20, 1)], A.LONG_MAX)]
    for recs, wm in steps:
        if recs:
            k = np.array([r[0] for r in recs], np.int64)
            t = np.array([r[1] for r in recs], np.int64)
            v = np.array([r[2] for r in recs], np.int64)
            assert g.push(k, t, [v]) == o.push(k, t, [v])
        rg, ro = g.advance_watermark(wm), o.advance_watermark(wm)
        assert_rows_equal(rg, ro, names, ctx="wm=%d" % wm)
    assert g.stats().late_dropped == o.stats().late_dropped == 1


@pytest.mark.parametrize("ci", [0, 2])
def test_fire_output_regrow_relaunch(eng_mod, ci):
    """Output capacity smaller than one watermark's rows (FWA_OPT_OUT_MIN_ROWS forces a 16-row first sizing):
    the fire counts past the capacity, the host grows the output and relaunches, late-firing rows at the
    head included. Rows must still equal the oracle's."""
    eng_mod.DEFAULT_OPTIONS["out_min_rows"] = 16
    try:
        test_late_firings_vs_oracle(eng_mod, ci, I64_AGGS)
    finally:
        del eng_mod.DEFAULT_OPTIONS["out_min_rows"]
