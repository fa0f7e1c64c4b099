"""GPU tests of STRING / VARCHAR key fields in the key dictionary (include/flink_amd.h FWA_KEY_FIELD_STRING).

* fwa_binrow_hash of rows with STRING fields equals MurmurHashUtils.hashBytesByWords (the oracle's C restatement) over
  the row's BinaryRowData bytes as oracle.binrow_bytes lays them out (AbstractBinaryWriter.writeString: <= 7 bytes
  inline, longer ones in the variable-length part; tests/test_keydict_cpu.py pins that layout against the reference's
  own BinaryRowDataTest sizes): empty strings, exactly 7 and 8 bytes, multi-byte UTF-8, NULLs, several STRING fields;
* the reference's hash-distribution property (BinaryRowDataTest.java:378-386: 999,999 one-field rows
  "啦啦啦啦啦我是快乐的粉刷匠" + i keep > 99.7 % distinct hashes);
* encode / decode round trips, equal rows one id, ids carrying their row's key group;
* an engine on such ids against the oracle on the same ids, two-phase partials, and the heap-layout snapshot written
  with the key's BinaryRowData (variable-length part included) restored into a fresh dictionary.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu

WORDS = ["", "a", "abcdefg", "abcdefgh", "Flink", "啦啦啦啦啦我是快乐的粉刷匠", "x" * 40, "héllo wörld", "0123456789abcdef"]


def string_rows(rng, types, n, distinct, null_p=0.1):
    """n key rows drawn from `distinct` random rows of the given field types (STRING values of 0..40 bytes)."""
    base = []
    for t in types:
        if t == "STRING":
            vals = list(WORDS)
            while len(vals) < distinct:
                ln = int(rng.integers(0, 41))
                vals.append("".join(chr(int(c)) for c in rng.integers(0x20, 0x250, ln)))
            base.append(np.array(vals[:distinct], dtype=object))
        elif t == "INT":
            base.append(rng.integers(-2**31, 2**31 - 1, distinct).astype(np.int32))
        else:
            base.append(rng.integers(-2**62, 2**62, distinct).astype(np.int64))
    nul = [(rng.random(distinct) < null_p).astype(np.uint8) for _ in types]
    pick = rng.integers(0, distinct, n)
    return [b[pick] for b in base], [z[pick] for z in nul]


def as_rows(types, cols, nulls):
    return [tuple(None if nulls[c][i] else (cols[c][i] if t == "STRING" else int(cols[c][i]))
                  for c, t in enumerate(types)) for i in range(len(cols[0]))]


def oracle_hash(types, row):
    from oracle import oracle as O
    return O.binrow_hash_bytes(O.binrow_bytes(types, row))


def str_col(col, nul):
    return [None if z else v for v, z in zip(col, nul)]


TYPES = [["STRING"], ["STRING", "BIGINT"], ["INT", "STRING", "STRING"], ["STRING", "INT", "BIGINT", "STRING"]]


@pytest.mark.parametrize("types", TYPES, ids=lambda t: "-".join(t))
def test_binrow_hash_with_strings_vs_oracle(types):
    from flink_amd.keydict import binrow_hash
    rng = np.random.default_rng(len(types) + 40)
    cols, nulls = string_rows(rng, types, 4000, 1500)
    args = [str_col(c, z) if t == "STRING" else c for c, z, t in zip(cols, nulls, types)]
    got = binrow_hash(types, args, nulls)
    exp = np.array([oracle_hash(types, r) for r in as_rows(types, cols, nulls)], np.int32)
    assert np.array_equal(got, exp)


def test_string_hash_distribution_like_the_reference():
    """BinaryRowDataTest.testHashAndCopy :378-386: 999,999 rows, > 99.7 % distinct hashCode()s."""
    from flink_amd.keydict import binrow_hash
    n = 999_999
    vals = ["啦啦啦啦啦我是快乐的粉刷匠%d" % i for i in range(n)]
    h = binrow_hash(["STRING"], [vals])
    assert len(np.unique(h)) > int(n * 0.997)
    for i in (0, 1, 77, n - 1):   # spot values against the oracle restatement
        assert h[i] == oracle_hash(["STRING"], (vals[i],))


@pytest.mark.parametrize("types", TYPES, ids=lambda t: "-".join(t))
def test_string_encode_decode_identity(types):
    from flink_amd.keydict import KeyDictionary
    from oracle import oracle as O
    rng = np.random.default_rng(70 + len(types))
    cols, nulls = string_rows(rng, types, 30_000, 4000)
    args = [str_col(c, z) if t == "STRING" else c for c, z, t in zip(cols, nulls, types)]
    d = KeyDictionary(types, max_parallelism=128, capacity=50_000)
    ids, hs = d.encode(args, nulls, hashes=True)
    ids, hs = ids.cpu().numpy(), hs.cpu().numpy()
    rows = as_rows(types, cols, nulls)
    by_row = {}
    for r, i in zip(rows, ids.tolist()):
        by_row.setdefault(r, set()).add(i)
    assert all(len(v) == 1 for v in by_row.values())                     # equal rows -> one id
    assert len({next(iter(v)) for v in by_row.values()}) == len(by_row)  # unequal rows -> different ids
    assert d.size() == len(by_row)
    assert np.array_equal(hs, np.array([oracle_hash(types, r) for r in rows], np.int32))
    assert np.array_equal(ids >> 48, np.array([O.lib().or_murmur_hash(int(x)) % 128 for x in hs]))
    dec, dn = d.decode(ids)
    for c, t in enumerate(types):
        assert np.array_equal(dn[c], nulls[c].astype(bool))
        m = ~dn[c]
        if t == "STRING":
            assert [v for v, k in zip(dec[c], m) if k] == [v for v, k in zip(cols[c], m) if k]
            assert all(v == "" for v, k in zip(dec[c], m) if not k)
        else:
            assert np.array_equal(dec[c][m], np.asarray(cols[c])[m])
    # a second encode with new and old rows: old ids stay, the byte heap grows
    cols2, nulls2 = string_rows(np.random.default_rng(5), types, 8000, 6000)
    args2 = [str_col(c, z) if t == "STRING" else c for c, z, t in zip(cols2, nulls2, types)]
    ids2 = d.encode([list(a) + list(b) if t == "STRING" else np.concatenate([a, b])
                     for a, b, t in zip(args, args2, types)],
                    [np.concatenate([a, b]) for a, b in zip(nulls, nulls2)]).cpu().numpy()
    assert np.array_equal(ids2[:len(ids)], ids)
    d.close()


def test_empty_string_null_and_inline_boundary_are_distinct():
    from flink_amd.keydict import KeyDictionary
    d = KeyDictionary(["STRING"], capacity=64)
    vals = ["", None, "", "abcdefg", "abcdefgh", "abcdefg\x00", "abcdefgh"]
    nul = np.array([v is None for v in vals], np.uint8)
    ids = d.encode([vals], [nul]).cpu().numpy()
    assert ids[0] == ids[2] and ids[4] == ids[6]
    assert len({ids[0], ids[1], ids[3], ids[4], ids[5]}) == 5
    dec, dn = d.decode(ids)
    assert dec[0] == ["", "", "", "abcdefg", "abcdefgh", "abcdefg\x00", "abcdefgh"] and dn[0].tolist() == nul.astype(bool).tolist()
    d.close()


def string_key_stream(seed, n, distinct, span, delay):
    from flink_amd.keydict import KeyDictionary
    from test_gpu_parity import random_stream
    rng = np.random.default_rng(seed)
    _, ts, vi, vf, vd = random_stream(seed, n, 500, span, delay)
    cols, nulls = string_rows(rng, ["STRING", "INT"], n, distinct, null_p=0.05)
    d = KeyDictionary(["STRING", "INT"], max_parallelism=128, capacity=4 * distinct)
    ids = d.encode([str_col(cols[0], nulls[0]), cols[1]], nulls).cpu().numpy()
    return d, ids, ts, [vi, vf, vd], cols, nulls


AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0), ("SUM_F64", 2)]


def test_engine_on_string_keys_vs_oracle_and_partials():
    from flink_amd import engine
    from oracle.oracle import Oracle
    d, ids, ts, cols, kc, kn = string_key_stream(21, 50_000, 2500, 50_000, 1200)
    base = dict(window_kind="SLIDE", semantics="TABLE", size_ms=10_000, slide_ms=5000, aggs=AGGS,
                key_kind=A.KEY_GROUP_PREFIXED, key_capacity=16384)
    names = A.agg_names(A.make_config(**base))
    g, o = engine.WindowAggregator(A.make_config(**base)), Oracle(A.make_config(**base))
    loc = [engine.WindowAggregator(A.make_config(**base)) for _ in range(2)]
    glob = engine.WindowAggregator(A.make_config(**base))
    for a, b in [(0, 20_000), (20_000, 50_000)]:
        cl = [c[a:b] for c in cols]
        assert g.push(ids[a:b], ts[a:b], cl) == o.push(ids[a:b], ts[a:b], cl)
        for s in range(2):
            sl = slice(a + s, b, 2)
            loc[s].push(ids[sl], ts[sl], [c[sl] for c in cols])
        wm = int(ts[:b].max()) - 1201 if b < 50_000 else A.LONG_MAX
        ro = o.advance_watermark(wm)
        assert_rows_equal(g.advance_watermark(wm), ro, names, rtol=1e-9, ctx="wm=%d" % wm)
        for s in range(2):
            p = loc[s].drain_partials(wm)
            glob.push_partials(p["key"], p["slice_start"], p["count"], [p["acc%d" % j] for j in range(len(names))])
        assert_rows_equal(glob.advance_watermark(wm), ro, names, rtol=1e-9, ctx="partials wm=%d" % wm)
    # fired rows decode to the string keys the ids were made from
    dec, dn = d.decode(ids[:100])
    assert [v for v, z in zip(dec[0], dn[0]) if not z] == [v for v, z in zip(kc[0][:100], kn[0][:100]) if not z]
    for x in [g, glob] + loc:
        x.close()
    d.close()


def test_heap_layout_with_string_key_rows():
    """fwa_snapshot_heap_keys writes each key as its BinaryRowData with the variable-length part (checked against
    oracle.binrow_bytes); restored by two subtasks into fresh dictionaries, the run resumes exactly like the oracle."""
    from flink_amd import engine
    from flink_amd.keydict import KeyDictionary
    from oracle import oracle as O
    from oracle.oracle import Oracle
    d, ids, ts, cols, kc, kn = string_key_stream(33, 30_000, 1500, 40_000, 1000)
    base = dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000, aggs=AGGS, key_kind=A.KEY_GROUP_PREFIXED,
                key_capacity=8192)
    names = A.agg_names(A.make_config(**base))
    cut = 18_000
    wm1 = int(ts[:cut].max()) - 1001
    o = Oracle(A.make_config(**base))
    o.push(ids[:cut], ts[:cut], [c[:cut] for c in cols])
    o.advance_watermark(wm1)
    g = engine.WindowAggregator(A.make_config(**base))
    g.push(ids[:cut], ts[:cut], [c[:cut] for c in cols])
    g.advance_watermark(wm1)
    body, offs, wm = g.snapshot_heap(keydict=d)
    g.close()
    # the key row of every key with an unfired window (a record past wm1) is in the body, as BinaryRowSerializer
    # writes it (int length, then the bytes)
    raw = bytes(body)
    uniq = np.unique(ids[:cut][ts[:cut] > wm1])
    (dc, dn) = d.decode(uniq)
    for i in range(0, len(uniq), max(1, len(uniq) // 50)):
        row = (None if dn[0][i] else dc[0][i], None if dn[1][i] else int(dc[1][i]))
        rb = O.binrow_bytes(["STRING", "INT"], row)
        assert len(rb).to_bytes(4, "big") + rb in raw
    o.push(ids[cut:], ts[cut:], [c[cut:] for c in cols])
    final = o.advance_watermark(A.LONG_MAX)
    fk, fn = d.decode(final["key"])
    exp = sorted(zip([None if z else v for v, z in zip(fk[0], fn[0])], [None if z else int(v) for v, z in zip(fk[1], fn[1])],
                     final["win_start"].tolist(), *[final["agg%d" % j].tolist() for j in range(3)]),
                 key=lambda r: tuple((x is None, x) for x in r))
    got = []
    for klo, khi in [(0, 63), (64, 127)]:
        d2 = KeyDictionary(["STRING", "INT"], max_parallelism=128, capacity=8192)
        g2 = engine.WindowAggregator(A.make_config(kg_start=klo, kg_end=khi, **base))
        g2.restore_heap([body], [wm], keydict=d2)
        (rc_, rn_) = d.decode(ids[cut:])
        nid = d2.encode([[None if z else v for v, z in zip(rc_[0], rn_[0])], rc_[1]],
                        [z.astype(np.uint8) for z in rn_]).cpu().numpy()
        assert np.array_equal(nid >> 48, ids[cut:] >> 48)          # same rows, same key groups
        m = ((nid >> 48) >= klo) & ((nid >> 48) <= khi)
        g2.push(nid[m], ts[cut:][m], [c[cut:][m] for c in cols])
        r = g2.advance_watermark(A.LONG_MAX)
        if len(r["key"]):
            k2, n2 = d2.decode(r["key"])
            got += list(zip([None if z else v for v, z in zip(k2[0], n2[0])], [None if z else int(v) for v, z in zip(k2[1], n2[1])],
                            r["win_start"].tolist(), *[r["agg%d" % j].tolist() for j in range(3)]))
        g2.close()
        d2.close()
    assert sorted(got, key=lambda r: tuple((x is None, x) for x in r)) == exp
    d.close()
