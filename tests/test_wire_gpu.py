"""GPU wire decoder (fwa_wire_decode) against the sequential CPU oracle (oracle/wire_oracle.c): bit-exact columns,
events, `consumed` and error positions, on streams the reference's serializers would write
(oracle/wire_encode.py, pinned by tests/test_wire_cpu.py's byte literals)."""
import numpy as np
import pytest

from flink_amd import _abi as A
from flink_amd import wire
from oracle import oracle as O
from oracle import wire_encode as W

pytestmark = pytest.mark.gpu

T3 = ["LONG", "LONG", "LONG"]
C5 = ["LONG", "LONG", "FLOAT", "DOUBLE"]          # key BIGINT, rowtime TIMESTAMP(3), f FLOAT, d DOUBLE


def _stream(rng, n, fields=T3, fmt="TUPLE", with_ts=True, n_events=10, nulls=False, small_keys=False):
    vals = []
    for f in fields:
        if f in ("LONG", "INT"):
            v = rng.integers(-(1 << 40), 1 << 40, n) if not small_keys else rng.integers(0, 64, n)
            vals.append(v.astype(np.int64 if f == "LONG" else np.int32))
        else:
            vals.append(rng.random(n).astype(np.float64 if f == "DOUBLE" else np.float32))
    ts = rng.integers(0, 1 << 45, n).astype(np.int64) if with_ts else None
    pos = np.sort(rng.integers(0, n + 1, n_events))
    tags = rng.choice([2, 3, 4, 5], n_events)
    events = []
    for p, t in zip(pos.tolist(), tags.tolist()):
        v = (int(rng.integers(-(1 << 62), 1 << 62)), int(rng.integers(-(1 << 62), 1 << 62)),
             int(rng.integers(-(1 << 62), 1 << 62)), int(rng.integers(-(1 << 31), 1 << 31)))
        if t == 4:
            v = (int(rng.choice([-1, 0])),)
        if t == 5:
            v = (int(rng.integers(0, 2)),)
        events.append((p, t, v))
    nl = None
    if nulls:
        nl = [None] * len(fields)
        for i in range(2, len(fields)):
            nl[i] = rng.random(n) < 0.1
    return W.encode_stream(fields, vals, ts, fmt, events, nl)


def _check(dec, schema, data, device=False):
    import torch
    rc, ref = O.wire_decode(schema, data)
    assert rc == 0
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda() if device and len(data) else data
    got = dec.decode(x)
    assert got.n_records == ref["n_records"] and got.n_events == ref["n_events"]
    assert got.consumed == ref["consumed"]
    assert np.array_equal(got.key.cpu().numpy(), ref["key"])
    assert np.array_equal(got.ts.cpu().numpy(), ref["ts"])
    for a, b in zip(got.cols, ref["cols"]):
        assert np.array_equal(a.cpu().numpy().view(np.uint8), b.view(np.uint8))   # bit-exact, NaN-safe
    if ref["col_null"] is not None:
        for a, b in zip(got.col_null, ref["col_null"]):
            assert np.array_equal(a.cpu().numpy(), b)
        assert np.array_equal(got.key_null.cpu().numpy(), ref["key_null"])
    assert np.array_equal(got.evt_pos, ref["evt_pos"])
    assert np.array_equal(got.evt_tag, ref["evt_tag"])
    assert np.array_equal(got.evt_val, ref["evt_val"])
    return got, ref


@pytest.mark.parametrize("n", [0, 1, 2, 110, 111, 4096, 33333, 1 << 17])
def test_tuple_streams_vs_oracle(n):
    rng = np.random.default_rng(n)
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[1, 2])
    dec = wire.WireDecoder(s)
    data = _stream(rng, n, n_events=max(1, n // 500))
    _check(dec, s, data)
    _check(dec, s, data, device=True)
    for cut in (1, 4, 5, 36, 37, 4095, 4096, 4097):               # partial element at the end (spanning)
        if cut < len(data):
            _check(dec, s, data[:len(data) - cut])
    dec.close()


def test_exact_chunk_multiples_and_empty_tail():
    rng = np.random.default_rng(1)
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[2])
    dec = wire.WireDecoder(s)
    data = _stream(rng, 20000, n_events=0)
    for nb in (4096, 8192, 4096 * 37, 37 * 4096 - 1):
        _check(dec, s, data[:nb])
    dec.close()


def test_false_chains_small_values():
    """Small field values put valid-looking length/tag pairs inside records (00 00 00 21 00 at a key of 33):
    many candidate chains survive the scan; only the one from offset 0 may be decoded."""
    rng = np.random.default_rng(7)
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[1, 2])
    dec = wire.WireDecoder(s)
    n = 50000
    k = np.full(n, 33, np.int64)
    v = rng.integers(0, 64, n).astype(np.int64)
    ts = np.full(n, 0x21, np.int64)
    data = W.encode_stream(T3, [k, v, k], ts, "TUPLE", [(100, 2, (0x2100000000,)), (7000, 2, (33,))])
    _check(dec, s, data)
    data2 = _stream(rng, 60000, small_keys=True, n_events=40)
    _check(dec, s, data2)
    dec.close()


@pytest.mark.parametrize("with_ts", [True, False])
def test_rowdata_with_nulls_vs_oracle(with_ts):
    rng = np.random.default_rng(11)
    s = wire.make_schema(C5, key_field=0, ts_field=1, cols=[2, 3], fmt="ROWDATA")
    dec = wire.WireDecoder(s)
    data = _stream(rng, 70000, fields=C5, fmt="ROWDATA", with_ts=with_ts, n_events=30, nulls=True)
    got, ref = _check(dec, s, data)
    assert ref["col_null"][0].sum() > 0
    dec.close()


def test_events_beyond_initial_list_capacity():
    """A stream of mostly watermarks (more events than the decoder's first event list) decodes in one call."""
    rng = np.random.default_rng(3)
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[2])
    dec = wire.WireDecoder(s)
    data = _stream(rng, 1000, n_events=40000)
    _check(dec, s, data)
    dec.close()


def test_corrupt_stream_reports_first_bad_element():
    rng = np.random.default_rng(5)
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[2])
    dec = wire.WireDecoder(s)
    data = bytearray(_stream(rng, 30000, n_events=0))
    data[37 * 20000 + 4] = 7                                      # tag byte of record 20000
    rc, ref = O.wire_decode(s, bytes(data))
    assert rc == -9
    with pytest.raises(Exception) as ei:
        dec.decode(bytes(data))
    assert "Corrupt stream, found tag: 7" in str(ei.value) and str(ref["err_pos"]) in str(ei.value)
    _check(dec, s, bytes(data[:37 * 20000]))                      # the decoder is usable afterwards
    dec.close()


def test_large_device_stream_properties():
    """2^22 records (155 MB of wire bytes) in HBM: counts, checksums and the event positions vs the oracle."""
    import torch
    rng = np.random.default_rng(9)
    n = 1 << 22
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[1, 2])
    dec = wire.WireDecoder(s)
    data = _stream(rng, n, n_events=64)
    rc, ref = O.wire_decode(s, data)
    got = dec.decode(torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda())
    assert got.n_records == n and got.consumed == len(data)
    assert np.array_equal(got.key.cpu().numpy(), ref["key"])
    assert int(got.cols[1].sum().item()) == int(ref["cols"][1].sum())
    assert np.array_equal(got.evt_pos, ref["evt_pos"])
    st = dec.stats()
    assert st.records_out == n and st.decode_ms > 0
    dec.close()


def test_network_input_feeds_window_engine():
    """Channel bytes cut into 32 KiB buffers -> NetworkInput (decode, push runs between events, watermarks
    through the one-channel valve) -> GPU engine; the same elements through the window oracle in order."""
    from flink_amd.engine import WindowAggregator
    from oracle.oracle import Oracle
    rng = np.random.default_rng(21)
    n = 200_000
    keys = rng.integers(0, 5000, n).astype(np.int64)
    ts = (np.arange(n) * 3 + rng.integers(0, 2000, n)).astype(np.int64)
    vals = rng.integers(0, 1 << 31, n).astype(np.int64)
    events, wm_seq = [], []
    for p in range(10_000, n, 10_000):
        wm = int(ts[:p].max()) - 2001
        events.append((p, 2, (wm,)))
        if p == 50_000:
            events.append((p, 4, (-1,)))                          # channel idle: the next watermark is ignored
        if p == 60_000:
            events.append((p, 4, (0,)))
        if p == 120_000:
            events.append((p, 2, (wm - 100000,)))                 # non-advancing: ignored by the valve
    data = W.encode_stream(T3, [keys, ts, vals], ts, "TUPLE", events)
    cfg = A.make_config(window_kind="TUMBLE", size_ms=5000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1 << 13)
    eng = WindowAggregator(cfg)
    inp = wire.NetworkInput(wire.make_schema(T3, key_field=0, ts_field=-1, cols=[2]), eng)
    got = []
    for buf in W.split_buffers(data):
        for r in inp.feed(buf):
            got += list(zip(r["key"].tolist(), r["win_end"].tolist(), r["agg0"].tolist(), r["agg1"].tolist()))
    r = eng.advance_watermark(A.LONG_MAX)
    got += list(zip(r["key"].tolist(), r["win_end"].tolist(), r["agg0"].tolist(), r["agg1"].tolist()))
    # reference order: records then events at each position, valve semantics restated
    o = Oracle(cfg)
    exp, at, cur, idle = [], 0, A.LONG_MIN, False
    for pos, tag, v in events + [(n, None, None)]:
        if pos > at:
            o.push(keys[at:pos], ts[at:pos], [vals[at:pos]])
            at = pos
        if tag == 2 and not idle and v[0] > cur:
            cur = v[0]
            r = o.advance_watermark(cur)
            exp += list(zip(r["key"].tolist(), r["win_end"].tolist(), r["agg0"].tolist(), r["agg1"].tolist()))
        elif tag == 4:
            idle = v[0] == -1
    r = o.advance_watermark(A.LONG_MAX)
    exp += list(zip(r["key"].tolist(), r["win_end"].tolist(), r["agg0"].tolist(), r["agg1"].tolist()))
    sg, se = sorted(got), sorted(exp)
    if sg != se:
        from collections import Counter
        cg, ce = Counter(got), Counter(exp)
        only_g, only_e = list((cg - ce).elements()), list((ce - cg).elements())
        raise AssertionError("rows %d vs %d; only GPU %d %s; only oracle %d %s; records_in %d late %d" % (
            len(got), len(exp), len(only_g), sorted(only_g)[:5], len(only_e), sorted(only_e)[:5], inp.records_in,
            inp.late_dropped))
    assert inp.records_in == n and inp.carry == b""
    inp.close()
    eng.close()


def test_network_input_table_rows_with_nulls():
    """Table path from the wire: BinaryRowData rows (key BIGINT, rowtime TIMESTAMP(3), f FLOAT, d DOUBLE) with NULL
    values, without StreamRecord timestamps, cut into 32 KiB buffers -> NetworkInput -> a TABLE engine with nullable
    columns (SQL NULL semantics: SUM/MAX skip NULLs, COUNT(col) counts non-NULL); the oracle gets the same rows and
    NULL flags in order."""
    from flink_amd.engine import WindowAggregator
    from helpers import assert_rows_equal
    from oracle.oracle import Oracle
    rng = np.random.default_rng(33)
    n = 120_000
    keys = rng.integers(0, 4000, n).astype(np.int64)
    ts = (np.arange(n) * 2 + rng.integers(0, 1500, n)).astype(np.int64)
    f = (rng.random(n) * 10).astype(np.float32)
    d = rng.random(n) * 100 - 50
    nf = rng.random(n) < 0.1
    nd = rng.random(n) < 0.2
    events = [(p, 2, (int(ts[:p].max()) - 1501,)) for p in range(15_000, n, 15_000)]
    data = W.encode_stream(C5, [keys, ts, f, d], None, "ROWDATA", events, [None, None, nf, nd])
    aggs = [("COUNT", 0), ("MAX_F32", 0), ("SUM_F64", 1), ("COUNT_COL", 1), ("AVG_F64", 1)]
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=5000, aggs=aggs, key_capacity=1 << 13,
                        nullable_cols=(0, 1))
    names = A.agg_names(cfg)
    eng = WindowAggregator(cfg)
    inp = wire.NetworkInput(wire.make_schema(C5, key_field=0, ts_field=1, cols=[2, 3], fmt="ROWDATA"), eng)
    got = []
    for buf in W.split_buffers(data):
        got += inp.feed(buf)
    got.append(eng.advance_watermark(A.LONG_MAX))
    o = Oracle(cfg)
    exp, at = [], 0
    for pos, _, v in events + [(n, None, (A.LONG_MAX,))]:
        o.push(keys[at:pos], ts[at:pos], [f[at:pos], d[at:pos]], nulls=[nf[at:pos], nd[at:pos]])
        at = pos
        exp.append(o.advance_watermark(v[0]))
    cat = lambda rs: {k: np.concatenate([r[k] for r in rs]) for k in rs[0]}   # noqa: E731
    assert_rows_equal(cat(got), cat(exp), names, rtol=1e-9)
    assert inp.records_in == n
    inp.close()
    eng.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_schemas_and_element_mixes(seed):
    """Random schemas (Tuple of LONG / INT / FLOAT / DOUBLE fields or BinaryRowData, 1-6 fields, with or without
    StreamRecord timestamps), random element mixes (event-heavy to record-only) and random cut points: the GPU
    decode equals the sequential oracle bit for bit."""
    rng = np.random.default_rng(100 + seed)
    fmt = "TUPLE" if seed % 2 == 0 else "ROWDATA"
    arity = int(rng.integers(2, 7))
    fields = ["LONG", "LONG"] + [str(x) for x in rng.choice(["LONG", "INT", "FLOAT", "DOUBLE"], arity - 2)]
    if fmt == "TUPLE" and rng.random() < 0.5:
        fields[0] = "INT"                                          # Integer key (sign-extended)
    ts_field = -1 if rng.random() < 0.5 else 1
    cols = [int(c) for c in rng.choice(np.arange(2, arity), min(3, arity - 2), replace=False)] if arity > 2 else []
    s = wire.make_schema(fields, key_field=0, ts_field=ts_field, cols=cols, fmt=fmt)
    dec = wire.WireDecoder(s)
    n = int(rng.integers(1, 150_000))
    vals = []
    for fl in fields:
        if fl in ("LONG", "INT"):
            v = rng.integers(-(1 << 31), 1 << 31, n)
            vals.append(v.astype(np.int64 if fl == "LONG" else np.int32))
        else:
            vals.append(rng.standard_normal(n).astype(np.float64 if fl == "DOUBLE" else np.float32))
    with_ts = ts_field == -1 or rng.random() < 0.5
    ts = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64) if with_ts else None
    n_ev = int(rng.choice([0, 3, n // 50, n // 2]))
    pos = np.sort(rng.integers(0, n + 1, n_ev))
    events = []
    for p, t in zip(pos.tolist(), rng.choice([2, 3, 4, 5], n_ev).tolist()):
        v = (int(rng.integers(-(1 << 62), 1 << 62)), -1, -1, int(rng.integers(0, 100)))
        events.append((p, t, (v[0] & 1,) if t == 5 else ((-1,) if t == 4 else v)))
    nulls = None
    if fmt == "ROWDATA":
        nulls = [None, None] + [rng.random(n) < 0.05 for _ in fields[2:]]
    data = W.encode_stream(fields, vals, ts, fmt, events, nulls)
    _check(dec, s, data)
    for cut in rng.integers(1, len(data), 5).tolist():           # the head of an element continues later
        _check(dec, s, data[:cut])
    dec.close()
