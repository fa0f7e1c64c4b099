"""Wire format on the CPU: the test-side encoder against byte literals written from the
reference's serializers (big-endian java.io.DataOutput), and the oracle decoder against the elements of
StreamElementSerializerTest.testSerialization (StreamElementSerializerTest.java:73-100: timestamps 77 and
Long.MIN_VALUE, watermarks 13 and -4647654567676555876, a LatencyMarker with OperatorID(-1, -1) and subtask 1,
RecordAttributes backlog = true; the String values there become Tuple3<Long, Long, Long> values here, the
schema this decoder handles)."""
import numpy as np
import pytest

from flink_amd import wire
from oracle import oracle as O
from oracle import wire_encode as W

LONG_MIN = -(1 << 63)
T3 = ["LONG", "LONG", "LONG"]


def be(v, n):
    return (v & ((1 << (8 * n)) - 1)).to_bytes(n, "big")


# element literals: length prefix (RecordWriter.serializeRecord) + StreamElementSerializer.serialize body
KATS = [
    ("record ts 77", be(33, 4) + b"\x00" + be(77, 8) + be(1, 8) + be(2, 8) + be(3, 8)),
    ("record ts Long.MIN_VALUE", be(33, 4) + b"\x00" + be(LONG_MIN, 8) + be(-1, 8) + be(0, 8) + be(5, 8)),
    ("watermark 13", be(9, 4) + b"\x02" + be(13, 8)),
    ("watermark negative", be(9, 4) + b"\x02" + be(-4647654567676555876, 8)),
    ("latency marker", be(29, 4) + b"\x03" + be(1700000000000, 8) + be(-1, 8) + be(-1, 8) + be(1, 4)),
    ("record attributes backlog", be(2, 4) + b"\x05" + b"\x01"),
    ("watermark status idle", be(5, 4) + b"\x04" + be(-1, 4)),
    ("record without timestamp", be(25, 4) + b"\x01" + be(4, 8) + be(5, 8) + be(6, 8)),
]


def test_encoder_matches_literals():
    enc = [
        W.encode_records(T3, [np.array([1]), np.array([2]), np.array([3])], ts=np.array([77])),
        W.encode_records(T3, [np.array([-1]), np.array([0]), np.array([5])], ts=np.array([LONG_MIN])),
        W.encode_event(2, (13,)),
        W.encode_event(2, (-4647654567676555876,)),
        W.encode_event(3, (1700000000000, -1, -1, 1)),
        W.encode_event(5, (1,)),
        W.encode_event(4, (-1,)),
        W.encode_records(T3, [np.array([4]), np.array([5]), np.array([6])], ts=None),
    ]
    for (name, lit), got in zip(KATS, enc):
        assert got == lit, name


def test_rowdata_literal():
    """BinaryRowDataSerializer: int size, then the row (RowKind byte, null bits, little-endian 8-byte slots)."""
    lit = (be(1 + 8 + 4 + 24, 4) + b"\x00" + be(5, 8) + be(24, 4) + bytes(8) + (7).to_bytes(8, "little")
           + bytes.fromhex("000000000000f83f"))
    got = W.encode_records(["LONG", "DOUBLE"], [np.array([7]), np.array([1.5])], ts=np.array([5]), fmt="ROWDATA")
    assert got == lit
    # NULL double: bit 8 + 1 of the header, slot zeroed (BinaryRowWriter.setNullAt)
    got = W.encode_records(["LONG", "DOUBLE"], [np.array([7]), np.array([1.5])], ts=np.array([5]), fmt="ROWDATA",
                           nulls=[None, np.array([True])])
    assert got[17 + 1] == 0x02 and got[17 + 16:17 + 24] == bytes(8)


def test_oracle_decodes_serializer_test_elements():
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[1, 2])
    stream = b"".join(lit for _, lit in KATS)
    rc, r = O.wire_decode(s, stream)
    assert rc == 0 and r["consumed"] == len(stream)
    assert r["n_records"] == 3 and r["n_events"] == 5
    assert r["key"].tolist() == [1, -1, 4]
    assert r["ts"].tolist() == [77, LONG_MIN, LONG_MIN]          # no timestamp -> Long.MIN_VALUE marker
    assert r["cols"][0].tolist() == [2, 0, 5] and r["cols"][1].tolist() == [3, 5, 6]
    assert r["evt_tag"].tolist() == [2, 2, 3, 5, 4]
    assert r["evt_pos"].tolist() == [2, 2, 2, 2, 2]
    assert r["evt_val"][:, 0].tolist() == [13, -4647654567676555876, 1700000000000, 1, -1]
    assert r["evt_val"][2].tolist() == [1700000000000, -1, -1, 1]


def test_oracle_spanning_and_corrupt():
    s = wire.make_schema(T3, key_field=0, ts_field=-1, cols=[2])
    stream = b"".join(lit for _, lit in KATS)
    for cut in range(1, len(stream)):
        rc, a = O.wire_decode(s, stream[:cut])
        assert rc == 0
        rc, b = O.wire_decode(s, stream[a["consumed"]:])
        assert rc == 0 and a["n_records"] + b["n_records"] == 3 and a["n_events"] + b["n_events"] == 5
    bad = bytearray(stream)
    bad[37 + 37 + 4] = 9                                          # tag of the first watermark
    rc, r = O.wire_decode(s, bytes(bad))
    assert rc == -9 and r["err_pos"] == 74 and r["err_tag"] == 9


def test_schema_validation_without_gpu():
    """fwa_wire_create validates before touching the device: bad key field / arity / element length."""
    import ctypes as C
    from flink_amd.engine import lib
    L = wire._bind(lib())
    h = C.c_void_p()
    assert L.fwa_wire_create(C.byref(wire.make_schema(["DOUBLE", "LONG"], key_field=0)), C.byref(h)) == -1
    assert L.fwa_wire_create(C.byref(wire.make_schema(["LONG"] * 3, key_field=5)), C.byref(h)) == -1
    s = wire.make_schema(["LONG", "LONG"], key_field=0)
    s.field[1] = 7                                                # e.g. a String field: variable length
    assert L.fwa_wire_create(C.byref(s), C.byref(h)) == -7


class _OracleDecoder:
    """Stand-in for the GPU decoder in the host-logic test: the oracle's decode, same batch shape."""

    def __init__(self, schema):
        self.schema = schema

    def decode(self, data):
        rc, r = O.wire_decode(self.schema, data)
        assert rc == 0

        class B:
            pass
        b = B()
        b.n_records, b.consumed = r["n_records"], r["consumed"]
        b.key, b.ts, b.cols, b.col_null, b.key_null = r["key"], r["ts"], r["cols"], None, None
        b.evt_pos, b.evt_tag, b.evt_val = r["evt_pos"], r["evt_tag"], r["evt_val"]
        return b

    def close(self):
        pass


def test_network_input_host_logic():
    """NetworkInput (AbstractStreamTaskNetworkInput.processElement + one-channel StatusWatermarkValve) over 32 KiB
    buffers, with the oracle as decoder and as window engine, equals pushing the same elements in order:
    records run up to each event, advancing watermarks fire, idle-channel and non-advancing watermarks do not."""
    from flink_amd import _abi as A
    from oracle.oracle import Oracle
    rng = np.random.default_rng(21)
    n = 60_000
    keys = rng.integers(0, 500, n).astype(np.int64)
    ts = (np.arange(n) * 3 + rng.integers(0, 2000, n)).astype(np.int64)
    vals = rng.integers(0, 1 << 31, n).astype(np.int64)
    events = []
    for p in range(5_000, n, 5_000):
        wm = int(ts[:p].max()) - 2001
        events.append((p, 2, (wm,)))
        if p == 20_000:
            events.append((p, 4, (-1,)))
        if p == 30_000:
            events.append((p, 4, (0,)))
        if p == 40_000:
            events.append((p, 2, (wm - 100000,)))
            events.append((p, 3, (123, -1, -1, 1)))
    data = W.encode_stream(T3, [keys, ts, vals], ts, "TUPLE", events)
    cfg = A.make_config(window_kind="TUMBLE", size_ms=5000, aggs=[("COUNT", 0), ("SUM_I64", 0)])
    eng = Oracle(cfg)
    eng.cfg = cfg
    inp = wire.NetworkInput.__new__(wire.NetworkInput)
    inp.__dict__.update(decoder=_OracleDecoder(wire.make_schema(T3, key_field=0, cols=[2])), engine=eng, carry=b"",
                        watermark=A.LONG_MIN, idle=False, latency_markers=[], record_attributes=[], records_in=0,
                        late_dropped=0)

    def tup(r):
        return list(zip(r["key"].tolist(), r["win_end"].tolist(), r["agg0"].tolist(), r["agg1"].tolist()))
    got = []
    for buf in W.split_buffers(data):
        for r in inp.feed(buf):
            got += tup(r)
    got += tup(eng.advance_watermark(A.LONG_MAX))
    o = Oracle(cfg)
    exp, at, cur, idle, fired = [], 0, A.LONG_MIN, False, 0
    for pos, tag, v in events + [(n, None, None)]:
        if pos > at:
            o.push(keys[at:pos], ts[at:pos], [vals[at:pos]])
            at = pos
        if tag == 2 and not idle and v[0] > cur:
            cur = v[0]
            exp += tup(o.advance_watermark(cur))
            fired += 1
        elif tag == 4:
            idle = v[0] == -1
    exp += tup(o.advance_watermark(A.LONG_MAX))
    assert sorted(got) == sorted(exp) and inp.records_in == n and inp.carry == b""
    assert inp.watermark == cur and inp.latency_markers == [(123, -1, -1, 1)] and fired == 9
