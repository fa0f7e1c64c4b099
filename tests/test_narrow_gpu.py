"""Narrow bucket entries of the two-phase ingest (partition3 / combine3 NW): COUNT + SUM(BIGINT) handles
keep each bucket entry as sign-extended 32-bit key and value halves of one u64. Records whose key or value needs 64
bits take the v1 replay; a push where more than 1/64 of the records do switches the handle to 64-bit entries. Parity
with the oracle is bit-exact in every case."""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu

AGGS = [("COUNT", 0), ("SUM_I64", 0)]


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


def _run(eng_mod, keys, ts, vals, nb, delay, size_ms=1000):
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", size_ms=size_ms, aggs=AGGS, key_capacity=1 << 16)
    names = A.agg_names(cfg)
    g = eng_mod.WindowAggregator(cfg)
    o = Oracle(cfg)
    n = len(keys)
    mx = -2**63
    for b in range(nb + 1):
        sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - delay - 1 if b < nb else A.LONG_MAX
        assert g.push(keys[sl], ts[sl], [vals[sl]]) == o.push(keys[sl], ts[sl], [vals[sl]])
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, ctx="batch %d" % b)
    st = g.stats()
    g.close()
    o.close()
    return st


def _stream(seed, n, nkeys, span, delay):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-nkeys // 2, nkeys // 2, n).astype(np.int64)
    ts = np.sort(rng.integers(0, span, n)).astype(np.int64) - rng.integers(0, delay + 1, n)
    vals = rng.integers(-2**31, 2**31, n).astype(np.int64)             # the full signed 32-bit range
    return keys, ts, vals


def test_narrow_entries_vs_oracle(eng_mod, monkeypatch):
    """Keys and values over the whole signed 32-bit range: no replay beyond the 64-bit entries' own (slice misses)."""
    keys, ts, vals = _stream(1, 1 << 20, 50_000, 40_000, 300)
    monkeypatch.setenv("FWA_NARROW", "0")
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.setenv("FWA_NARROW", "1")
    assert _run(eng_mod, keys, ts, vals, 8, 300).replay_records == wide


def test_narrow_entries_with_a_few_wide_records(eng_mod, monkeypatch):
    """Keys and values at and past the 32-bit edges, under 1/64 of the records: replayed, handle stays narrow."""
    keys, ts, vals = _stream(2, 1 << 20, 50_000, 40_000, 300)
    rng = np.random.default_rng(3)
    k = rng.random(len(keys)) < 0.004
    keys[k] = rng.choice(np.array([2**31, -2**31 - 1, 2**40 + 7, -2**62, 2**31 - 1, -2**31], np.int64), k.sum())
    v = rng.random(len(keys)) < 0.004
    vals[v] = rng.choice(np.array([2**31, -2**31 - 1, 2**62 + 5, -2**63, 2**31 - 1, -2**31], np.int64), v.sum())
    monkeypatch.setenv("FWA_NARROW", "0")
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.delenv("FWA_NARROW")
    assert _run(eng_mod, keys, ts, vals, 8, 300).replay_records > wide


def test_wide_values_switch_the_handle_to_64bit_entries(eng_mod, monkeypatch):
    keys, ts, vals = _stream(4, 1 << 19, 20_000, 30_000, 300)
    vals = vals * 4096                                                  # most values need 64 bits
    monkeypatch.setenv("FWA_NARROW", "0")
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.delenv("FWA_NARROW")
    extra = _run(eng_mod, keys, ts, vals, 8, 300).replay_records - wide
    assert 0 < extra <= (1 << 19) // 8                                  # only the first push is replayed


C5_AGGS = [("COUNT", 0), ("SUM_F64", 1), ("AVG_F64", 1), ("MAX_F32", 0), ("MAX_F64", 1)]


@pytest.mark.parametrize("wide_keys", [False, True], ids=["keys32", "keys64"])
def test_narrow_float_column_entries_vs_oracle(eng_mod, monkeypatch, wide_keys):
    """C5's shape: FLOAT + DOUBLE columns; the FLOAT's raw bits share the u64 with the 32-bit key (NW 3). With 64-bit
    keys (some, then most) the records are replayed and the handle switches back; rows equal the oracle's within the
    float-sum tolerance."""
    from oracle.oracle import Oracle
    monkeypatch.setenv("FWA_NARROW3", "1")
    rng = np.random.default_rng(11)
    n = 1 << 20
    keys = rng.integers(-30_000, 30_000, n).astype(np.int64)
    if wide_keys:
        keys[rng.random(n) < 0.3] += 2**40
    ts = np.sort(rng.integers(0, 40_000, n)).astype(np.int64) - rng.integers(0, 301, n)
    f = (rng.random(n) * 200 - 100).astype(np.float32)
    d = rng.random(n) * 1000.0 - 500.0
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=1000, aggs=C5_AGGS, key_capacity=1 << 17)
    names = A.agg_names(cfg)
    g = eng_mod.WindowAggregator(cfg)
    o = Oracle(cfg)
    mx = -2**63
    for b in range(9):
        sl = slice(b * n // 8, (b + 1) * n // 8) if b < 8 else slice(0, 0)
        if b < 8:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - 301 if b < 8 else A.LONG_MAX
        assert g.push(keys[sl], ts[sl], [f[sl], d[sl]]) == o.push(keys[sl], ts[sl], [f[sl], d[sl]])
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="batch %d" % b)
    g.close()
    o.close()
