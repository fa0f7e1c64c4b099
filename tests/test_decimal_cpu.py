"""DECIMAL SUM / AVG on the CPU oracle: the reference's KATs and its division semantics.

The oracle's decimal aggregates restate DecimalSumAggFunction / DecimalAvgAggFunction in arrival order
(oracle/fwa_oracle.c dec_divide, acc_add / acc_merge). Pinned here by
  * AggregateITCase's DECIMAL precision KATs (tests/golden/decimal_kats.json) and WindowAggregateITCase's SUM(bigdec)
    (tests/golden/sql_kats.json, test_oracle.py);
  * an independent model of the division: Python's decimal module (General Decimal Arithmetic, whose context division
    with precision 38 and ROUND_HALF_UP is BigDecimal.divide(divisor, new MathContext(38, HALF_UP)), and quantize is
    setScale(t, HALF_UP)), then DecimalData.fromBigDecimal's 38-digit check.
"""
from decimal import ROUND_HALF_UP, Context, Decimal

import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import dec_input, load_decimal_kats, replay_decimal_kat

DEC_KATS = load_decimal_kats()


def ref_avg(total, cnt, s):
    """DecimalAvgAggFunction's value: DecimalDataUtils.divide(sum, count) at DECIMAL(38, max(6, s)), or None (NULL)."""
    if cnt == 0 or abs(total) >= 10 ** 38:
        return None
    t = max(6, s)
    wide = Context(prec=400)
    q = Context(prec=38, rounding=ROUND_HALF_UP).divide(Decimal(total).scaleb(-s, context=wide), Decimal(cnt))
    r = q.quantize(Decimal(1).scaleb(-t), rounding=ROUND_HALF_UP, context=wide)
    u = int(r.scaleb(t, context=wide))
    return None if len(str(abs(u))) > 38 else u


def oracle_window(kind, scale, values, nulls=None):
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=[("COUNT", 0), (kind, 0, scale)],
                        nullable_cols=[0] if nulls is not None else [])
    o = Oracle(cfg)
    n = len(values)
    o.push(np.full(n, 3, np.int64), np.arange(n, dtype=np.int64) % 1000, [dec_input(kind, values)],
           nulls=None if nulls is None else [np.array(nulls, np.uint8)])
    r = o.advance_watermark(A.LONG_MAX)
    o.close()
    assert len(r["key"]) == 1
    return None if r.get("null1") is not None and r["null1"][0] else int(r["agg1"][0])


@pytest.mark.parametrize("case", DEC_KATS, ids=lambda c: c["name"].split(" ", 1)[1])
def test_decimal_kats_on_oracle(case):
    from oracle.oracle import Oracle
    replay_decimal_kat(case, Oracle)


def test_avg_matches_python_decimal_model():
    rng = np.random.default_rng(11)
    for trial in range(400):
        s = int(rng.choice([0, 1, 2, 6, 7, 8, 12, 20, 30, 37, 38]))
        n = int(rng.integers(1, 7))
        mag = int(rng.choice([3, 9, 18, 25, 33, 36]))
        vals = [int(rng.integers(-10 ** min(mag, 18), 10 ** min(mag, 18))) * 10 ** max(0, mag - 18) +
                int(rng.integers(0, 1000)) for _ in range(n)]
        if abs(sum(vals)) >= 10 ** 38:
            continue
        got = oracle_window("AVG_DEC128", s, vals)
        assert got == ref_avg(sum(vals), n, s), (trial, s, vals)


def test_avg_double_rounding_kat():
    """Both HALF_UP roundings of DecimalDataUtils.divide: 1001 records summing to 1001 * I + 500 (I of 35 digits) at
    scale 6 average to I + 0.4995..., which rounds to I.500 at 38 significant digits and then up to I + 1 at the
    result scale (a single rounding would give I)."""
    i0 = 9 * 10 ** 34 + 12345
    vals = [i0] * 1000 + [i0 + 500]
    assert ref_avg(sum(vals), len(vals), 6) == i0 + 1
    assert oracle_window("AVG_DEC128", 6, vals) == i0 + 1


def test_avg_integer_digits_past_the_result_type_is_null():
    """AVG(DECIMAL(38, 0)) of 10^37: the quotient needs 38 integer digits, DECIMAL(38, 6) holds 32 -> NULL."""
    assert ref_avg(10 ** 37, 1, 0) is None
    assert oracle_window("AVG_DEC128", 0, [10 ** 37]) is None
    assert oracle_window("AVG_DEC128", 0, [10 ** 31]) == 10 ** 37      # 32 integer digits still fit


def test_sum_overflow_follows_arrival_order():
    """DecimalSumAggFunction: a running sum past 38 digits is NULL, and the next value restarts it
    (ifThenElse(isNull(sum), operand, ...)); AVG's NULL sum stays NULL."""
    big = 6 * 10 ** 37
    assert oracle_window("SUM_DEC128", 2, [big, big]) is None
    assert oracle_window("SUM_DEC128", 2, [big, big, 5]) == 5
    assert oracle_window("AVG_DEC128", 2, [big, big, 5]) is None
    assert oracle_window("SUM_DEC128", 2, [big, -big, big]) == big
    # AVG: no restart (AvgAggFunction.java:79) -- NULL even though the total 6e37 is back within 38 digits
    assert oracle_window("AVG_DEC128", 20, [big, big, -big]) is None
    assert oracle_window("AVG_DEC128", 20, [big, -big, big]) == 2 * 10 ** 37


def test_sum_nulls_and_int64_input():
    assert oracle_window("SUM_DEC", 2, [111, 0, 222], nulls=[0, 1, 0]) == 333
    assert oracle_window("SUM_DEC", 2, [111, 222], nulls=[1, 1]) is None
    assert oracle_window("AVG_DEC", 2, [100, 0, 201], nulls=[0, 1, 0]) == 1505000   # 1.505 at scale 6
    assert oracle_window("SUM_DEC", 0, [2 ** 63 - 1, 2 ** 63 - 1]) == 2 ** 64 - 2   # past the long range, exact


def test_dec128_column_roundtrip():
    vals = [0, 1, -1, 10 ** 38 - 1, -(10 ** 38 - 1), 2 ** 64, -(2 ** 64) - 5]
    assert list(A.dec128_values(A.dec128_column(vals).tobytes())) == vals
