"""GPU tests: the sliding fire's carried window sums (flink_amd/csrc/engine.hip fire_slide, FWA_OPT_SLIDE_CARRIED).

A run of hop windows starts from the sums the previous run stored for the slices its successor window shares with
the last fired window (all but the last few, which later records may still reach); a push that touches a carried
slice after that fire invalidates them. Every watermark's rows must equal the oracle's (the reference's
SlicingWindowOperator / WindowOperator restatement), whether the sums are reused, invalidated by late-arriving
records, or switched off -- and the reuse path must actually run on in-order streams."""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal
from test_gpu_parity import random_stream

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0), ("AVG_I64", 0)]
CASES = {
    "table_hop_10s_1s": dict(window_kind="SLIDE", semantics="TABLE", size_ms=10_000, slide_ms=1_000),
    "table_hop_12s_4s": dict(window_kind="SLIDE", semantics="TABLE", size_ms=12_000, slide_ms=4_000),
    "ds_slide_10s_4s_g2s": dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=10_000, slide_ms=4_000),
    "table_hop_offset": dict(window_kind="SLIDE", semantics="TABLE", size_ms=6_000, slide_ms=1_500, offset_ms=700),
    "ds_slide_8s_1s": dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=8_000, slide_ms=1_000),
}


def batches_of(seed, n, nb, delay, late_frac, span=120_000, nkeys=3000):
    keys, ts, vi, _, _ = random_stream(seed, n, nkeys, span, delay, late_frac)
    out, mx = [], -2 ** 63
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        mx = max(mx, int(ts[sl].max()))
        out.append((keys[sl], ts[sl], [vi[sl]], mx - delay - 1))
    out.append((keys[:0], ts[:0], [vi[:0]], A.LONG_MAX))
    return out


def run(case, batches, carried):
    from flink_amd import engine
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=AGGS, key_capacity=8192, **CASES[case])
    names = A.agg_names(cfg)
    g, o = engine.WindowAggregator(cfg), Oracle(cfg)
    g.set_option("slide_carried", 1 if carried else 0)
    for i, (k, t, cols, wm) in enumerate(batches):
        assert g.push(k, t, cols) == o.push(k, t, cols)
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, ctx="%s batch %d" % (case, i))
    used = g.get_option("slide_carried")
    g.close()
    o.close()
    return used


@pytest.mark.parametrize("case", list(CASES))
def test_carried_sums_in_order_stream(case):
    """Small out-of-orderness: the carried sums are reused at most fires (every batch spans >= 2 slides, so each
    watermark fires a run of windows through fire_slide)."""
    used = run(case, batches_of(3, 300_000, 12, delay=200, late_frac=0.0), True)
    assert used >= 5


@pytest.mark.parametrize("case", list(CASES))
def test_carried_sums_with_late_records_into_carried_slices(case):
    """Out-of-orderness of several slices plus late records: pushes hit carried slices (the sums are dropped and
    the left-out tail grows); rows stay exact."""
    run(case, batches_of(5, 300_000, 12, delay=4_000, late_frac=0.05), True)


def test_carried_sums_off_gives_the_same_rows():
    b = batches_of(7, 200_000, 12, delay=800, late_frac=0.02)
    assert run("table_hop_10s_1s", b, False) == 0
    assert run("table_hop_10s_1s", b, True) > 0
