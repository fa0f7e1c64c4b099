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
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 0)
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 1)
    assert _run(eng_mod, keys, ts, vals, 8, 300).replay_records == wide


def test_narrow_entries_with_a_few_wide_records(eng_mod, monkeypatch):
    """Keys and values at and past the 32-bit edges, under 1/64 of the records: replayed, handle stays narrow."""
    keys, ts, vals = _stream(2, 1 << 20, 50_000, 40_000, 300)
    rng = np.random.default_rng(3)
    k = rng.random(len(keys)) < 0.004
    keys[k] = rng.choice(np.array([2**31, -2**31 - 1, 2**40 + 7, -2**62, 2**31 - 1, -2**31, -2**31 + 1], np.int64), k.sum())
    v = rng.random(len(keys)) < 0.004
    vals[v] = rng.choice(np.array([2**31, -2**31 - 1, 2**62 + 5, -2**63, 2**31 - 1, -2**31], np.int64), v.sum())
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 0)
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.delitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries")
    assert _run(eng_mod, keys, ts, vals, 8, 300).replay_records > wide


def test_wide_values_switch_the_handle_to_64bit_entries(eng_mod, monkeypatch):
    keys, ts, vals = _stream(4, 1 << 19, 20_000, 30_000, 300)
    vals = vals * 4096                                                  # most values need 64 bits
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 0)
    wide = _run(eng_mod, keys, ts, vals, 8, 300).replay_records
    monkeypatch.delitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries")
    extra = _run(eng_mod, keys, ts, vals, 8, 300).replay_records - wide
    assert 0 < extra <= (1 << 19) // 8                                  # only the first push is replayed


@pytest.mark.parametrize("hot", [32_767, 32_768, 65_536 + 3, 300_000])
def test_narrow_combiner_hot_keys(eng_mod, monkeypatch, hot):
    """Hot keys through the narrow combiner's LDS accumulators: tens of thousands of records of one (key, slice) in one
    push (the counts around 2^15 / 2^16 a packed 16-bit count field would wrap at -- r06 measured such a layout and
    kept the separate COUNT / SUM words), values at both ends of the signed 32-bit range, one combiner block (a small
    key capacity: one partition) and tile pre-aggregation off; rows equal the oracle's."""
    from oracle.oracle import Oracle
    rng = np.random.default_rng(hot)
    n = hot * 2 + 50_000
    keys = rng.integers(-500, 500, n).astype(np.int64)
    keys[rng.permutation(n)[:hot]] = 7                                  # one key with `hot` records of each slice...
    keys[rng.permutation(n)[:hot]] = -3                                 # (two, overlapping draws)
    ts = rng.integers(0, 1000, n).astype(np.int64)                      # ...all in one slice
    ts[: n // 4] += 1000                                                # and a second slice for a quarter of them
    vals = rng.choice(np.array([2**31 - 1, -2**31, -2**31 + 1, 0, -1, 1, 2**31 - 2], np.int64), n)
    r = rng.random(n) < 0.5
    vals[r] = rng.integers(-2**31, 2**31, r.sum())
    cfg = A.make_config(window_kind="TUMBLE", size_ms=1000, aggs=AGGS, key_capacity=1024)
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg, options={"skew_merge": 0, "narrow_entries": 1}), Oracle(cfg)
    for sl in (slice(0, 2), slice(2, n)):   # the first push allocates the slices (its records are replayed)
        k2, t2, v2 = keys[sl], ts[sl], vals[sl]
        if sl.start == 0:
            t2 = np.array([5, 1005], np.int64)
        assert g.push(k2, t2, [v2]) == o.push(k2, t2, [v2])
    assert g.get_option("narrow_entries") == 1
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), o.advance_watermark(A.LONG_MAX), names)
    assert g.stats().replay_records < n // 8   # the first push; sub-buckets of the few tiles that overflow
    g.close()
    o.close()


# NW = 2: a DOUBLE column beside a FLOAT one (C5's aggregate list): the key's 32 bits and the FLOAT's bits share one
# word, the DOUBLE keeps its own; keys needing 64 bits take the v1 replay (the FLOAT always fits)
AGGS_F = [("COUNT", 0), ("SUM_F64", 1), ("AVG_F64", 1), ("MAX_F32", 0), ("MAX_F64", 1), ("MIN_F32", 0)]


def _run_f(eng_mod, keys, ts, f, d, nb, delay, window="TUMBLE"):
    from oracle.oracle import Oracle
    kw = dict(window_kind=window, semantics="TABLE", aggs=AGGS_F, key_capacity=1 << 16, size_ms=2000)
    if window == "SLIDE":
        kw.update(size_ms=4000, slide_ms=1000)
    cfg = A.make_config(**kw)
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    n, mx = len(keys), -2**63
    for b in range(nb + 1):
        sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
        if b < nb:
            mx = max(mx, int(ts[sl].max()))
        wm = mx - delay - 1 if b < nb else A.LONG_MAX
        cols = [f[sl], d[sl]]
        assert g.push(keys[sl], ts[sl], cols) == o.push(keys[sl], ts[sl], cols)
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="batch %d" % b)
    st = g.stats()
    g.close()
    o.close()
    return st


@pytest.mark.parametrize("window", ["TUMBLE", "SLIDE"])
def test_narrow_entries_double_beside_float(eng_mod, monkeypatch, window):
    keys, ts, _ = _stream(5, 1 << 20, 50_000, 40_000, 300)
    rng = np.random.default_rng(6)
    f = (rng.random(len(keys)).astype(np.float32) - 0.5) * 1e4
    f[rng.random(len(keys)) < 0.01] = np.float32(-0.0)
    f[rng.random(len(keys)) < 0.001] = np.float32(np.inf)
    d = rng.random(len(keys)) * 1e6 - 5e5
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 0)
    wide = _run_f(eng_mod, keys, ts, f, d, 8, 300, window).replay_records
    monkeypatch.setitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries", 1)
    assert _run_f(eng_mod, keys, ts, f, d, 8, 300, window).replay_records == wide
    k = rng.random(len(keys)) < 0.004                                  # a few keys past 32 bits / at the markers
    keys[k] = rng.choice(np.array([2**31, -2**31 - 1, 2**40 + 7, -2**31, -2**31 + 1], np.int64), k.sum())
    monkeypatch.delitem(eng_mod.DEFAULT_OPTIONS, "narrow_entries")
    assert _run_f(eng_mod, keys, ts, f, d, 8, 300, window).replay_records > wide
