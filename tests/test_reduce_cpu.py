"""The oracle's DataStream built-in reductions (FWA_CFG_REDUCE: WindowedStream.sum / min / max / minBy / maxBy,
WindowedStream.java:680-890), pinned by sequences the reference's own Python WindowOperator produced with the
reference's AccumulateReduceFunction (tests/golden/gen_pyflink_reduce_kats.py), plus the Java-only semantics the Python
restatement does not have: int / long wrap-around (SumFunction), Double.compareTo order (-0.0 < 0.0, NaN greatest) and
minBy(pos, first = false) (ComparableAggregator.java:83-107)."""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import load_reduce_kats, reduce_aggs, reduce_field_values, replay_reduce_kat

KATS = load_reduce_kats()


@pytest.mark.parametrize("case", KATS["cases"], ids=lambda c: c["name"].split(" ", 1)[1])
def test_oracle_reduce_kats(case):
    from oracle.oracle import Oracle
    replay_reduce_kat(case, Oracle)


def _one_window(aggs, cols, flags=()):
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", size_ms=100, aggs=aggs, reduce=True, **dict.fromkeys(flags, True))
    o = Oracle(cfg)
    n = len(cols[0])
    o.push(np.full(n, 7, np.int64), np.arange(n, dtype=np.int64), cols)
    r = o.advance_watermark(A.LONG_MAX)
    o.close()
    return r


def test_java_wraparound_sums():
    """SumFunction.IntSum / LongSum: Java int and long addition wrap (Tuple2<Long, Integer>.sum(1))."""
    i32 = np.array([2**31 - 1, 1, 5], np.int32)
    i64 = np.array([2**63 - 1, 1, 2], np.int64)
    r = _one_window([("SUM_I32", 0), ("SUM_I64", 1)], [i32, i64])
    assert int(r["agg0"][0]) == -2**31 + 5 and int(r["agg1"][0]) == -2**63 + 2


def test_double_compare_order_and_tie_rule():
    """Double.compareTo: -0.0 < 0.0 and NaN above +Inf; minBy/maxBy ties to the first element unless first=false."""
    d = np.array([0.0, -0.0, np.inf, np.nan, -0.0, np.nan])
    tag = np.arange(10, 16, dtype=np.int64)
    cols = [d, tag]
    r = _one_window([("MINBY_F64", 0), ("SEL_64", 1)], cols)
    assert np.signbit(r["agg0"][0]) and int(r["agg1"][0]) == 11           # the first -0.0
    r = _one_window([("MINBY_F64", 0), ("SEL_64", 1)], cols, flags=("by_last",))
    assert int(r["agg1"][0]) == 14                                         # the last -0.0
    r = _one_window([("MAXBY_F64", 0), ("SEL_64", 1)], cols)
    assert np.isnan(r["agg0"][0]) and int(r["agg1"][0]) == 13              # NaN is the largest
    r = _one_window([("MIN_F64", 0), ("FIRST_64", 1)], cols)
    assert np.signbit(r["agg0"][0]) and r["agg0"][0] == 0 and int(r["agg1"][0]) == 10
    r = _one_window([("MAX_F64", 0), ("FIRST_64", 1)], cols)
    assert np.isnan(r["agg0"][0]) and int(r["agg1"][0]) == 10


def test_reduce_handles_refuse_merging_windows():
    from oracle.oracle import Oracle, OracleError
    for kw in (dict(window_kind="SESSION", gap_ms=10, size_ms=0), dict(window_kind="TUMBLE", semantics="TABLE")):
        with pytest.raises(OracleError):
            Oracle(A.make_config(aggs=[("SUM_I64", 0), ("FIRST_64", 1)], reduce=True, **kw))
    with pytest.raises(OracleError):                        # FIRST_* needs FWA_CFG_REDUCE
        Oracle(A.make_config(aggs=[("SUM_I64", 0), ("FIRST_64", 1)]))


def test_reduce_aggs_mapping():
    assert reduce_aggs("sum", 2) == [("FIRST_32", 0), ("SUM_F64", 1), ("FIRST_64", 2)]
    assert reduce_aggs("max_by", 1) == [("MAXBY_I32", 0), ("SEL_64", 1), ("SEL_64", 2)]
    assert reduce_field_values({"key": [1], "win_start": [0], "win_end": [5], "agg0": np.array([3], np.int32),
                                "agg1": np.array([1.5]).view(np.int64), "agg2": np.array([9])}, None) == \
        [(1, 0, 5, 3, 1.5, 9)]


@pytest.mark.parametrize("kind", ["SUM_I64", "MIN_I64", "MAX_I64", "MINBY_I64", "MAXBY_I64"])
def test_oracle_session_reduction_matches_model(kind):
    """The oracle's session reduction (red_merge restating reduce(a, b) for MergingWindowSet merges) against a direct
    model: sessions of gap 50 per key from the sorted timestamps, the field reduced over each; records arrive shuffled
    within a push so that sessions merge."""
    from oracle.oracle import Oracle
    rng = np.random.default_rng(5)
    n = 3000
    keys = rng.integers(0, 20, n).astype(np.int64)
    ts = rng.integers(0, 20_000, n).astype(np.int64)
    v = rng.integers(-2**62, 2**62, n).astype(np.int64)
    cfg = A.make_config(window_kind="SESSION", gap_ms=50, size_ms=0, aggs=[(kind, 0)], reduce=True)
    o = Oracle(cfg)
    o.push(keys, ts, [v])
    got = reduce_field_values(o.advance_watermark(A.LONG_MAX), A.agg_names(cfg), ["I64"])
    o.close()
    f = {"SUM": lambda x: int(np.sum(x.astype(np.uint64)).astype(np.int64)), "MIN": min, "MAX": max}[kind[:3]]
    want = []
    for k in np.unique(keys):
        sel = np.argsort(ts[keys == k], kind="stable")
        t, x = ts[keys == k][sel], v[keys == k][sel]
        cut = np.flatnonzero(np.diff(t) > 50) + 1          # TimeWindow.intersects: touching windows merge
        for tt, xx in zip(np.split(t, cut), np.split(x, cut)):
            want.append((int(k), int(tt[0]), int(tt[-1]) + 50, int(f(xx))))
    assert got == sorted(want)
