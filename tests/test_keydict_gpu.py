"""GPU tests of the key dictionary (multi-column Table keys, include/flink_amd.h fwa_keydict_*).

* fwa_binrow_hash equals the oracle's BinaryRowData.hashCode restatement (tests/test_keydict_cpu.py pins it against a
  byte-level restatement of BinaryRowData.java:68-123 + MurmurHashUtils.hashBytesByWords) for BIGINT / INT / DOUBLE
  fields with NULLs, and the single-BIGINT path the engine uses for FWA_KEY_BINROW_BIGINT;
* encode / decode: equal rows get equal ids and unequal rows (NULL vs 0, -0.0 vs 0.0) different ones, ids carry the
  key group of their row's hash, ids are stable across encodes, decode returns the rows;
* an engine with key_kind FWA_KEY_GROUP_PREFIXED on dictionary ids against the oracle on the same ids: rows, key-group
  ownership (FWA_E_KEYGROUP), two-phase partials, FWASNAP1 snapshot / restore with rescaling.
"""
import ctypes as C
import struct

import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu

TYPES = [["BIGINT", "INT"], ["INT", "DOUBLE", "BIGINT"], ["BIGINT"], ["DOUBLE", "DOUBLE", "INT", "BIGINT"]]
NP_T = {"BIGINT": np.int64, "INT": np.int32, "DOUBLE": np.float64}


def random_key_rows(rng, types, n, distinct, null_p=0.1):
    """n rows drawn from `distinct` random rows (NULLs, -0.0 / 0.0 and INT extremes included)."""
    base = []
    for t in types:
        if t == "BIGINT":
            c = rng.integers(-2**62, 2**62, distinct).astype(np.int64)
        elif t == "INT":
            c = rng.integers(-2**31, 2**31 - 1, distinct).astype(np.int32)
            c[:2] = [-2**31, 2**31 - 1]
        else:
            c = rng.standard_normal(distinct) * 1e6
            c[:3] = [0.0, -0.0, np.inf]
        base.append(c)
    nul = [(rng.random(distinct) < null_p).astype(np.uint8) for _ in types]
    pick = rng.integers(0, distinct, n)
    cols = [b[pick] for b in base]
    nulls = [z[pick] for z in nul]
    for c, z in zip(cols, nulls):          # a NULL field's value is irrelevant: vary it (the row stays the same)
        c[z.astype(bool)] = c[rng.integers(0, n, int(z.sum()))] if z.sum() else c[z.astype(bool)]
    return cols, nulls


def oracle_hashes(types, cols, nulls):
    from oracle import oracle as O
    n = len(cols[0])
    out = np.zeros(n, np.int32)
    for i in range(n):
        slots = np.zeros(len(types), np.int64)
        nb = 0
        for c, t in enumerate(types):
            if nulls[c][i]:
                nb |= 1 << c
            elif t == "INT":
                slots[c] = int(cols[c][i]) & 0xFFFFFFFF
            elif t == "DOUBLE":
                slots[c] = struct.unpack("<q", struct.pack("<d", float(cols[c][i])))[0]
            else:
                slots[c] = int(cols[c][i])
        out[i] = O.lib().or_binrow_hash(slots.ctypes.data, len(types), nb)
    return out


def row_key(types, cols, nulls, i):
    """the row's bytes as the dictionary sees them (NULL fields' values ignored, DOUBLE by bit pattern)"""
    r = []
    for c, t in enumerate(types):
        if nulls[c][i]:
            r.append(None)
        elif t == "DOUBLE":
            r.append(struct.pack("<d", float(cols[c][i])))
        else:
            r.append(int(cols[c][i]))
    return tuple(r)


@pytest.mark.parametrize("types", TYPES, ids=lambda t: "-".join(t))
def test_binrow_hash_vs_oracle(types):
    from flink_amd.keydict import binrow_hash
    rng = np.random.default_rng(len(types))
    cols, nulls = random_key_rows(rng, types, 3000, 1000)
    assert np.array_equal(binrow_hash(types, cols, nulls), oracle_hashes(types, cols, nulls))


def test_binrow_hash_single_bigint_equals_engine_key_hash():
    """one BIGINT field: the same key group as the engine's FWA_KEY_BINROW_BIGINT path (fwa_key_groups)"""
    from flink_amd import engine
    from flink_amd.keydict import binrow_hash
    from oracle import oracle as O
    rng = np.random.default_rng(3)
    k = rng.integers(-2**63, 2**63 - 1, 5000).astype(np.int64)
    h = binrow_hash(["BIGINT"], [k])
    kg_eng, _ = engine.key_groups(k, 128, 1, A.KEY_BINROW_BIGINT)
    kg = np.array([O.lib().or_murmur_hash(int(x)) % 128 for x in h])
    assert np.array_equal(kg, kg_eng)


@pytest.mark.parametrize("types", TYPES, ids=lambda t: "-".join(t))
def test_encode_decode_identity(types):
    from flink_amd.keydict import KeyDictionary
    from oracle import oracle as O
    rng = np.random.default_rng(11 + len(types))
    cols, nulls = random_key_rows(rng, types, 20_000, 3000)
    d = KeyDictionary(types, max_parallelism=128, capacity=100_000)
    ids, hs = d.encode(cols, nulls, hashes=True)
    ids, hs = ids.cpu().numpy(), hs.cpu().numpy()
    keys = [row_key(types, cols, nulls, i) for i in range(len(ids))]
    by_key = {}
    for k, i in zip(keys, ids.tolist()):
        by_key.setdefault(k, set()).add(i)
    assert all(len(v) == 1 for v in by_key.values())                     # equal rows -> one id
    assert len({next(iter(v)) for v in by_key.values()}) == len(by_key)  # unequal rows -> different ids
    assert d.size() == len(by_key)
    assert np.array_equal(hs, oracle_hashes(types, cols, nulls))
    kg = np.array([O.lib().or_murmur_hash(int(x)) % 128 for x in hs])
    assert np.array_equal(ids >> 48, kg)                                 # the id carries its row's key group
    dec, dn = d.decode(ids)
    for c, t in enumerate(types):
        assert np.array_equal(dn[c], nulls[c].astype(bool))
        m = ~dn[c]
        if t == "DOUBLE":
            assert np.array_equal(dec[c][m].view(np.int64), np.asarray(cols[c], np.float64)[m].view(np.int64))
        else:
            assert np.array_equal(dec[c][m], np.asarray(cols[c])[m])
    # a second encode: old rows keep their ids, new rows extend the dictionary
    cols2, nulls2 = random_key_rows(np.random.default_rng(99), types, 5000, 4000)
    allc = [np.concatenate([a, b]) for a, b in zip(cols, cols2)]
    alln = [np.concatenate([a, b]) for a, b in zip(nulls, nulls2)]
    ids2 = d.encode(allc, alln).cpu().numpy()
    assert np.array_equal(ids2[:len(ids)], ids)
    d.close()


def test_negative_zero_and_null_are_distinct_rows():
    from flink_amd.keydict import KeyDictionary
    d = KeyDictionary(["DOUBLE", "BIGINT"], capacity=64)
    ids = d.encode([np.array([0.0, -0.0, 0.0, 0.0]), np.array([1, 1, 0, 7], np.int64)],
                   [np.zeros(4, np.uint8), np.array([0, 0, 1, 1], np.uint8)]).cpu().numpy()
    assert ids[0] != ids[1] and ids[2] == ids[3] and len(set(ids.tolist())) == 3
    d.close()


def test_capacity_exhaustion_is_an_error():
    from flink_amd import engine
    from flink_amd.keydict import KeyDictionary
    d = KeyDictionary(["BIGINT"], capacity=100)
    with pytest.raises(engine.EngineError) as ei:
        d.encode([np.arange(1000, dtype=np.int64)])
    assert A.STATUS[ei.value.code] == "E_OOM"
    # after the failed batch: rows that got an id keep it, rows that were claimed without one still fail as E_OOM (not
    # a garbage id), and a batch of rows that all got ids encodes fine
    ok = None
    for lo in range(0, 1000, 10):
        try:
            ok = d.encode([np.arange(lo, lo + 10, dtype=np.int64)]).cpu().numpy()
            break
        except engine.EngineError as e2:
            assert A.STATUS[e2.code] == "E_OOM"
    assert ok is not None and len(set(ok.tolist())) == 10 and (ok >= 0).all()
    assert d.size() == 100
    with pytest.raises(engine.EngineError) as ei:
        d.encode([np.arange(1000, dtype=np.int64)])
    assert A.STATUS[ei.value.code] == "E_OOM"
    d.close()


def test_torch_key_columns_of_the_wrong_dtype_are_refused():
    import torch
    from flink_amd.keydict import KeyDictionary
    d = KeyDictionary(["BIGINT", "DOUBLE"], capacity=64)
    with pytest.raises(TypeError):
        d.encode([torch.zeros(8, dtype=torch.int32, device="cuda"), torch.zeros(8, dtype=torch.float64, device="cuda")])
    ids = d.encode([torch.zeros(8, dtype=torch.int64, device="cuda"), torch.zeros(8, dtype=torch.float64, device="cuda")])
    assert len(set(ids.cpu().numpy().tolist())) == 1
    d.close()


def test_ids_of_a_dictionary_with_a_larger_max_parallelism_are_rejected():
    """an id whose key group (top 16 bits) is past the engine's max parallelism belongs to no subtask:
    FWA_E_KEYGROUP on every ingest path, also when the engine owns every key group; fwa_key_groups reports -1."""
    import torch
    from flink_amd import engine
    from flink_amd.keydict import KeyDictionary
    d = KeyDictionary(["BIGINT"], max_parallelism=32768, capacity=50_000)
    ids = d.encode([np.arange(50_000, dtype=np.int64)]).cpu().numpy()
    bad = ids[(ids >> 48) >= 128][:64]
    assert len(bad) == 64
    kg, op = engine.key_groups(bad, max_parallelism=128, parallelism=4, key_kind=A.KEY_GROUP_PREFIXED)
    assert (kg == -1).all() and (op == -1).all()
    ts = np.arange(64, dtype=np.int64) * 10
    for kw in (dict(), dict(window_kind="SLIDE", semantics="TABLE", size_ms=4000, slide_ms=1000),
               dict(record_lists=True), dict(window_kind="SESSION", gap_ms=100)):
        cfg = A.make_config(aggs=[("COUNT", 0), ("SUM_I64", 0)], key_kind=A.KEY_GROUP_PREFIXED, key_capacity=4096,
                            **kw)
        g = engine.WindowAggregator(cfg)
        with pytest.raises(engine.EngineError) as ei:
            g.push(bad, ts, [ts])
        assert A.STATUS[ei.value.code] == "E_KEYGROUP", kw
        with pytest.raises(engine.EngineError) as ei:   # device inputs (the two-phase path)
            dk = torch.from_numpy(np.resize(bad, 1 << 16)).cuda()
            dt = torch.arange(1 << 16, dtype=torch.int64, device="cuda")
            g2 = engine.WindowAggregator(cfg)
            g2.push(dk, dt, [dt])
            g2.advance_watermark(A.LONG_MAX)
        assert A.STATUS[ei.value.code] == "E_KEYGROUP", kw
        g.close()
        g2.close()
    d.close()


def multi_key_stream(seed, n, distinct, span, delay):
    """a two-column key (INT, BIGINT) stream: its dictionary ids, timestamps and value columns"""
    from flink_amd.keydict import KeyDictionary
    from test_gpu_parity import random_stream
    rng = np.random.default_rng(seed)
    _, ts, vi, vf, vd = random_stream(seed, n, 500, span, delay)
    cols, nulls = random_key_rows(rng, ["INT", "BIGINT"], n, distinct, null_p=0.05)
    d = KeyDictionary(["INT", "BIGINT"], max_parallelism=128, capacity=4 * distinct)
    ids = d.encode(cols, nulls).cpu().numpy()
    return d, ids, ts, [vi, vf, vd]


AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0), ("SUM_F64", 2)]


def test_engine_on_dictionary_ids_vs_oracle():
    from flink_amd import engine
    from oracle.oracle import Oracle
    d, ids, ts, cols = multi_key_stream(5, 60_000, 2000, 60_000, 1500)
    cfg = A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=10_000, slide_ms=5000, aggs=AGGS,
                        key_kind=A.KEY_GROUP_PREFIXED, key_capacity=8192)
    names = A.agg_names(cfg)
    g, o = engine.WindowAggregator(cfg), Oracle(cfg)
    for a, b in [(0, 20_000), (20_000, 45_000), (45_000, 60_000)]:
        assert g.push(ids[a:b], ts[a:b], [c[a:b] for c in cols]) == o.push(ids[a:b], ts[a:b], [c[a:b] for c in cols])
        wm = int(ts[:b].max()) - 1501 if b < 60_000 else A.LONG_MAX
        rg = g.advance_watermark(wm)
        assert_rows_equal(rg, o.advance_watermark(wm), names, rtol=1e-9, ctx="wm=%d" % wm)
    # fired rows map back to the key columns
    if len(rg["key"]):
        dec, _ = d.decode(rg["key"])
        assert len(dec[0]) == len(rg["key"])
    g.close()
    d.close()


def test_dictionary_ids_key_group_ownership_partials_and_rescale():
    """Ownership by the id's key group; two local pre-aggregators drain partials to the owner (two-phase); a snapshot
    of two subtasks (key groups [0, 63], [64, 127]) restored by one subtask resumes like the oracle."""
    from flink_amd import engine
    from oracle.oracle import Oracle
    d, ids, ts, cols = multi_key_stream(8, 40_000, 1500, 50_000, 1200)
    base = dict(window_kind="TUMBLE", semantics="TABLE", size_ms=5000, aggs=AGGS, key_kind=A.KEY_GROUP_PREFIXED,
                key_capacity=8192)
    names = A.agg_names(A.make_config(**base))
    kg = ids >> 48
    lo = engine.WindowAggregator(A.make_config(kg_start=0, kg_end=63, **base))
    with pytest.raises(engine.EngineError) as ei:
        lo.push(ids[kg >= 64][:10], ts[kg >= 64][:10], [c[kg >= 64][:10] for c in cols])
    assert A.STATUS[ei.value.code] == "E_KEYGROUP"
    lo.close()
    # two-phase
    loc = [engine.WindowAggregator(A.make_config(**base)) for _ in range(2)]
    glob, o = engine.WindowAggregator(A.make_config(**base)), Oracle(A.make_config(**base))
    cut = 25_000
    for a, b in [(0, cut), (cut, 40_000)]:
        o.push(ids[a:b], ts[a:b], [c[a:b] for c in cols])
        for s in range(2):
            sl = slice(a + s, b, 2)
            loc[s].push(ids[sl], ts[sl], [c[sl] for c in cols])
        wm = int(ts[:b].max()) - 1201 if b < 40_000 else A.LONG_MAX
        for s in range(2):
            p = loc[s].drain_partials(wm)
            glob.push_partials(p["key"], p["slice_start"], p["count"], [p["acc%d" % j] for j in range(len(names))])
        assert_rows_equal(glob.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9, ctx="wm=%d" % wm)
    # snapshot / rescale
    o2 = Oracle(A.make_config(**base))
    o2.push(ids[:cut], ts[:cut], [c[:cut] for c in cols])
    wm1 = int(ts[:cut].max()) - 1201
    first = o2.advance_watermark(wm1)
    o2.push(ids[cut:], ts[cut:], [c[cut:] for c in cols])
    final = o2.advance_watermark(A.LONG_MAX)
    blobs, got1 = [], []
    for klo, khi in [(0, 63), (64, 127)]:
        m = np.nonzero((kg[:cut] >= klo) & (kg[:cut] <= khi))[0]
        g = engine.WindowAggregator(A.make_config(kg_start=klo, kg_end=khi, **base))
        g.push(ids[m], ts[m], [c[m] for c in cols])
        got1.append(g.advance_watermark(wm1))
        blobs.append(g.snapshot())
        g.close()
    assert_rows_equal({f: np.concatenate([r[f] for r in got1]) for f in got1[0]}, first, names, rtol=1e-9)
    g = engine.WindowAggregator(A.make_config(**base))
    g.restore(blobs)
    g.push(ids[cut:], ts[cut:], [c[cut:] for c in cols])
    assert_rows_equal(g.advance_watermark(A.LONG_MAX), final, names, rtol=1e-9)
    g.close()
    d.close()


def test_heap_layout_with_multi_column_key_rows():
    """fwa_snapshot_heap_keys: the window state of an engine on dictionary ids in Flink's heap layout with the key as
    its multi-column BinaryRowData row (read back with tests/heap_reader.py); restored by two subtasks into fresh
    dictionaries (rescaling), the run resumes exactly like the oracle."""
    import heap_reader as H
    from flink_amd import engine
    from flink_amd.keydict import KeyDictionary
    from oracle.oracle import Oracle
    d, ids, ts, cols = multi_key_stream(13, 30_000, 1200, 40_000, 1000)
    base = dict(window_kind="SLIDE", semantics="TABLE", size_ms=10_000, slide_ms=5000, aggs=AGGS,
                key_kind=A.KEY_GROUP_PREFIXED, key_capacity=8192)
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
    # the key rows are the dictionary's 2-field rows (INT, BIGINT)
    lay = {0: ("kv", H.ser_long, H.ser_binrow(2), H.ser_binrow(1 + len(AGGS))), 1: ("pq", H.ser_binrow(2), H.ser_long),
           2: ("pq", H.ser_binrow(2), H.ser_long)}
    secs = H.read_key_groups(body, offs, 0, lay)
    seen = set()
    for kg, sec in secs.items():
        for _, key, _ in sec.get(0, []):
            rk, nl, f = key
            assert rk == 0
            seen.add((kg, tuple(nl), tuple(f)))
    dec, dn = d.decode(np.unique(ids[:cut]))
    assert len(seen) > 0 and len({s[1:] for s in seen}) <= len(dec[0])
    # restore into two new subtasks, each with its own dictionary, and finish the run
    o.push(ids[cut:], ts[cut:], [c[cut:] for c in cols])
    final = o.advance_watermark(A.LONG_MAX)
    rows_dec = []
    for klo, khi in [(0, 50), (51, 127)]:
        d2 = KeyDictionary(["INT", "BIGINT"], max_parallelism=128, capacity=8192)
        g2 = engine.WindowAggregator(A.make_config(kg_start=klo, kg_end=khi, **base))
        g2.restore_heap([body], [wm], keydict=d2)
        # the rest of the stream, re-keyed through the new dictionary (the same rows, new ids)
        (kc, kn) = d.decode(ids[cut:])
        nid = d2.encode(kc, [z.astype(np.uint8) for z in kn]).cpu().numpy()
        m = ((nid >> 48) >= klo) & ((nid >> 48) <= khi)
        g2.push(nid[m], ts[cut:][m], [c[cut:][m] for c in cols])
        r = g2.advance_watermark(A.LONG_MAX)
        kc2, kn2 = d2.decode(r["key"]) if len(r["key"]) else ([np.zeros(0, np.int32), np.zeros(0, np.int64)], None)
        rows_dec.append((r, kc2, kn2))
        g2.close()
        d2.close()
    # compare with the oracle's final rows through the original dictionary's rows
    fk, _ = d.decode(final["key"])
    exp = sorted(zip(fk[0].tolist(), fk[1].tolist(), final["win_start"].tolist(), final["win_end"].tolist(),
                     *[final["agg%d" % j].tolist() for j in range(3)]))
    got = []
    for r, kc2, _ in rows_dec:
        got += list(zip(kc2[0].tolist(), kc2[1].tolist(), r["win_start"].tolist(), r["win_end"].tolist(),
                        *[r["agg%d" % j].tolist() for j in range(3)]))
    assert sorted(got) == exp
    d.close()
