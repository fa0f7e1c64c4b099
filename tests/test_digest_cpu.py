"""The full-size parity check's tools on the CPU: the torch row digest (tests/digest.py) equals the oracle's
or_row_digest, and the threaded generating pipeline (or_pipeline_digests, several operator instances over key-group
ranges) yields per watermark the rows of one sequential oracle over the whole stream (WindowOperator.onEventTime,
WindowOperator.java:437-481; the keyBy split must not change the fired multiset)."""
import numpy as np
import torch

from digest import bucket_sums, f32_word, f64_word, rows_digest
from flink_amd import _abi as A
from oracle import oracle as O


def test_torch_digest_matches_oracle():
    rng = np.random.default_rng(3)
    n = 2000
    k = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    s = rng.integers(-2**62, 2**62, n, dtype=np.int64)
    e = s + rng.integers(1, 10**6, n)
    a = [rng.integers(0, 1000, n), rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)]
    cnt, d = rows_digest(*(torch.from_numpy(x) for x in (k, s, e)), [torch.from_numpy(x) for x in a])
    ref = sum(O.row_digest(k[i], s[i], e[i], [a[0][i], a[1][i]]) for i in range(n)) % 2**64
    assert cnt == n and d == ref
    # one changed field changes the digest; the order of the rows does not
    perm = rng.permutation(n)
    assert rows_digest(*(torch.from_numpy(x[perm]) for x in (k, s, e)), [torch.from_numpy(x[perm]) for x in a])[1] == d
    a[0][17] += 1
    assert rows_digest(*(torch.from_numpy(x) for x in (k, s, e)), [torch.from_numpy(x) for x in a])[1] != d


def test_pipeline_digests_equal_sequential_oracle():
    n, batch, nkeys = 600_000, 100_000, 20_000
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                        aggs=[("COUNT", 0), ("SUM_I64", 0)])
    p = A.GenParams(seed_k=11, seed_t=12, seed_v=13, first_index=0, total_records=n, num_keys=nkeys,
                    t0_ms=1_700_000_000_000, span_ms=n // 1000 * 40, max_delay_ms=1000, key_dist=0, val_kind=0)
    _, rows, dig = O.pipeline_digests(cfg, p, n, batch, 3)
    keys, ts, vi, _, _ = O.generate(p, n)
    o = O.Oracle(cfg)
    max_ts = -2**63
    for b in range(n // batch + 1):
        if b < n // batch:
            sl = slice(b * batch, (b + 1) * batch)
            o.push(keys[sl], ts[sl], [vi[sl]])
            max_ts = max(max_ts, int(ts[sl].max()))
            wm = max_ts - 1001
        else:
            wm = A.LONG_MAX
        r = o.advance_watermark(wm)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.int64))  # noqa: E731
        cnt, d = rows_digest(t(r["key"]), t(r["win_start"]), t(r["win_end"]), [t(r["agg0"]), t(r["agg1"])])
        assert (cnt, d) == (int(rows[b]), int(dig[b])), b
    assert rows.sum() > 0 and rows[-1] > 0
    o.close()


def test_pipeline_digests2_equal_sequential_oracle():
    """The general form (or_pipeline_digests2: Zipf keys from a CDF, f32 / f64 columns, threads generating shares of
    each batch) against one sequential oracle over the same stream: HOP over Zipf keys (exact digest) and a Table
    TUMBLE / a DataStream SESSION over the float columns (COUNT and MAX words exact, SUM / AVG as bucket sums)."""
    n, batch, nkeys, nbk = 300_000, 60_000, 5_000, 64
    w = 1.0 / np.arange(1, nkeys + 1, dtype=np.float64) ** 1.1
    cdf = np.cumsum(w) / w.sum()
    fl = [("COUNT", 0), ("SUM_F64", 1), ("AVG_F64", 1), ("MAX_F32", 0), ("MAX_F64", 1)]
    cases = [(dict(window_kind="SLIDE", semantics="TABLE", size_ms=6_000, slide_ms=1_000,
                   aggs=[("COUNT", 0), ("SUM_I64", 0)]), 1, 0, (0, 1), ()),
             (dict(window_kind="TUMBLE", semantics="TABLE", size_ms=10_000, aggs=fl), 0, 1, (0, 3, 4), (1, 2)),
             (dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=500, aggs=fl), 0, 1, (0, 3, 4), (1, 2))]
    for kw, zipf, fp, exact, sums in cases:
        cfg = A.make_config(**kw)
        p = A.GenParams(seed_k=21, seed_t=22, seed_v=23, first_index=0, total_records=n, num_keys=nkeys,
                        t0_ms=1_700_000_000_000, span_ms=n // 1000 * 40, max_delay_ms=1000, key_dist=zipf, val_kind=fp)
        _, rows, dig, bs, ba = O.pipeline_digests2(cfg, p, n, batch, 3, cdf=cdf if zipf else None, float_cols=fp,
                                                   exact=exact, sums=sums, nbuckets=nbk)
        keys, ts, vi, vf, vd = O.generate(p, n, want_floats=bool(fp), cdf=cdf if zipf else None)
        cols = [vf, vd] if fp else [vi]
        o = O.Oracle(cfg)
        max_ts = -2**63
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
        for b in range(n // batch + 1):
            if b < n // batch:
                sl = slice(b * batch, (b + 1) * batch)
                o.push(keys[sl], ts[sl], [c[sl] for c in cols])
                max_ts = max(max_ts, int(ts[sl].max()))
                wm = max_ts - 1001
            else:
                wm = A.LONG_MAX
            r = o.advance_watermark(wm)
            words = {0: lambda a: t(a).to(torch.int64), 1: lambda a: t(a).to(torch.int64),
                     3: lambda a: f32_word(t(a)), 4: lambda a: f64_word(t(a))}
            ex = [words[j](r["agg%d" % j]) for j in exact]
            k64, s64 = t(r["key"]).to(torch.int64), t(r["win_start"]).to(torch.int64)
            cnt, d = rows_digest(k64, s64, t(r["win_end"]).to(torch.int64), ex)
            assert (cnt, d) == (int(rows[b]), int(dig[b])), (kw["window_kind"], b)
            if sums:
                s, a = bucket_sums(k64, s64, [t(r["agg%d" % j]) for j in sums], nbk)
                assert np.allclose(s.numpy(), bs[b], rtol=1e-9, atol=1e-9), (kw["window_kind"], b)
                assert np.allclose(a.numpy(), ba[b], rtol=1e-9, atol=1e-9), (kw["window_kind"], b)
        assert rows.sum() > 0
        o.close()
