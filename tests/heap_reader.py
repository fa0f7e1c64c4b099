"""Reader of Flink's heap keyed-state checkpoint bytes (test infrastructure).

Independent Python restatement of the reference's readers, used for two things:
  * pinning: it parses the reference's own checkpoint files of `WindowOperator`
    (`flink-streaming-java/src/test/resources/win-op-migration-test-*-snapshot`, written by
    `WindowOperatorMigrationTest.java` through `OperatorSnapshotUtil.writeStateHandle`), see
    tests/test_heap_reference_cpu.py;
  * checking: the engine's `fwa_snapshot_heap` bytes are parsed with the same section reader
    (tests/test_heap_snapshot_gpu.py).

Layers (all java.io.DataOutput, big-endian):
  OperatorSnapshotUtil.writeStateHandle (OperatorSnapshotUtil.java:48-123): int version; null stream handle byte;
    raw / managed operator state counts; raw keyed handles; managed keyed handles -- each a KeyGroupsStateHandle
    (MetadataV2V3SerializerBase.serializeKeyedStateHandle :309-331): byte 12 (KEY_GROUPS_HANDLE_V2), int first key
    group, int number of key groups, long offset per key group, the delegate ByteStreamStateHandle (:670-690:
    byte 1, UTF handle name, int length, the bytes), UTF state handle id.
  The delegate bytes: the KeyedBackendSerializationProxy header (state meta infos; ids are assigned in the order the
    states are listed, HeapSnapshotResources.java:100-139), then per key group (HeapSnapshotStrategy.java:154-175)
    int keyGroupId and, per state, short stateId + the state's entries:
      key/value state: int n, n x (namespace, key, value)      CopyOnWriteStateMapSnapshot.writeState :138-148
      priority queue (timers): int n, n x (long flipSignBit(ts), key, namespace)   TimerSerializer.serialize :147-152
Serializers: StringSerializer (StringValue.writeString: varint length + 1, then chars), LongSerializer,
IntSerializer, TimeWindow.Serializer (long start, long end), VoidNamespaceSerializer (one byte), TupleSerializer
(fields in order), ListSerializer (int size, elements), BinaryRowDataSerializer (int size, row bytes: header + null
bits, little-endian 8-byte slots).
"""
import re
import struct


class Reader:
    def __init__(self, b, at=0, end=None):
        self.b, self.at = b, at
        self.end = len(b) if end is None else end

    def get(self, fmt):
        v = struct.unpack_from(fmt, self.b, self.at)
        self.at += struct.calcsize(fmt)
        assert self.at <= self.end, "read past the section"
        return v[0] if len(v) == 1 else v

    def utf(self):
        n = self.get(">H")
        s = self.b[self.at:self.at + n].decode("utf-8")
        self.at += n
        return s

    def raw(self, n):
        s = self.b[self.at:self.at + n]
        self.at += n
        return s


# ------------------------------------------------------------------------------------------------
# serializers: each is a function Reader -> value

def ser_long(r):
    return r.get(">q")


def ser_ulong(r):
    return r.get(">Q")


def ser_int(r):
    return r.get(">i")


def ser_string(r):
    """StringValue.readString: variable-length (len + 1) in 7-bit groups, low group first, then each char the same
    way (ASCII in one byte); 0 = null."""
    def varint():
        v, sh = 0, 0
        while True:
            c = r.get(">B")
            v |= (c & 0x7F) << sh
            if c < 0x80:
                return v
            sh += 7
    n = varint()
    if n == 0:
        return None
    return "".join(chr(varint()) for _ in range(n - 1))


def ser_time_window(r):
    return (r.get(">q"), r.get(">q"))


def ser_void(r):
    assert r.get(">b") == 0
    return None


def ser_tuple(*fields):
    return lambda r: tuple(f(r) for f in fields)


def ser_list(elem):
    def rd(r):
        n = r.get(">i")
        return [elem(r) for _ in range(n)]
    return rd


def ser_map(key, value):
    """MapSerializer: int size, then per entry the key, a null flag byte and (if not null) the value"""
    def rd(r):
        out = []
        for _ in range(r.get(">i")):
            k = key(r)
            out.append((k, None if r.get(">b") else value(r)))
        return out
    return rd


def ser_binrow(arity):
    """BinaryRowDataSerializer of a row with `arity` fixed-length 8-byte fields -> (RowKind byte, null flags, fields)"""
    def rd(r):
        size = r.get(">i")
        nb = ((arity + 63 + 8) // 64) * 8
        assert size == nb + 8 * arity, (size, arity)
        hdr = r.raw(nb)
        nulls = [bool((hdr[(i + 8) // 8] >> ((i + 8) % 8)) & 1) for i in range(arity)]
        return hdr[0], nulls, [r.get("<Q") for _ in range(arity)]
    return rd


def ser_binrow_dec(arity, dec):
    """BinaryRowDataSerializer of an accumulator row whose fields in `dec` are non-compact DECIMALs (precision > 18):
    AbstractBinaryWriter.writeDecimal reserves 16 bytes per non-NULL one in the variable-length part, slot = offset <<
    32 | length, the bytes DecimalData.toUnscaledBytes (minimal big-endian two's complement; the reader asserts the
    minimal form); a NULL one is setNullAt (slot 0). -> (RowKind, null flags, fields; DECIMALs as Python ints)"""
    def rd(r):
        size = r.get(">i")
        nb = ((arity + 63 + 8) // 64) * 8
        row = r.raw(size)
        assert size == nb + 8 * arity + 16 * sum(1 for i in dec if not (row[(i + 8) // 8] >> ((i + 8) % 8)) & 1)
        nulls = [bool((row[(i + 8) // 8] >> ((i + 8) % 8)) & 1) for i in range(arity)]
        f = [struct.unpack_from("<Q", row, nb + 8 * i)[0] for i in range(arity)]
        for i in dec:
            if nulls[i]:
                assert f[i] == 0
                continue
            off, ln = f[i] >> 32, f[i] & 0xFFFFFFFF
            assert nb + 8 * arity <= off and off + 16 <= size and 1 <= ln <= 16
            assert not any(row[off + ln:off + 16]), "the reserved 16 bytes are zero past the value"
            v = int.from_bytes(row[off:off + ln], "big", signed=True)
            jbl = v.bit_length() if v >= 0 else (~v).bit_length()      # BigInteger.bitLength
            assert ln == jbl // 8 + 1, "toUnscaledBytes is BigInteger.toByteArray (minimal)"
            f[i] = v
        return row[0], nulls, f
    return rd


# ------------------------------------------------------------------------------------------------
# OperatorSnapshotUtil wrapper -> managed keyed state handles

def read_operator_snapshot(b):
    """[(first key group, offsets[], delegate bytes)] of the managed keyed state in an OperatorSnapshotUtil file."""
    r = Reader(b)
    assert r.get(">i") in (2, 3, 4, 5)                     # MetadataV3Serializer.VERSION (compatibility)
    assert r.get(">b") == 0                                # null stream handle
    for _ in range(2):                                     # raw and managed operator state
        assert r.get(">i") in (0, -1), "operator state handles are not expected here"
    assert r.get(">i") in (0, -1)                          # raw keyed state
    out = []
    for _ in range(max(0, r.get(">i"))):                   # managed keyed state
        kind = r.get(">b")
        assert kind in (3, 12), kind                       # KEY_GROUPS_HANDLE(_V2)
        first, num = r.get(">i"), r.get(">i")
        offs = [r.get(">q") for _ in range(num)]
        assert r.get(">b") == 1                            # ByteStreamStateHandle
        r.utf()
        data = r.raw(r.get(">i"))
        if kind == 12:
            r.utf()                                        # StateHandleID
        out.append((first, offs, data))
    return out


def state_ids(header, names):
    """State id of each known state name: ids follow the order the meta infos list the states in the proxy header
    (each name written once with DataOutput.writeUTF)."""
    pos = {}
    for n in names:
        m = re.search(re.escape(struct.pack(">H", len(n)) + n.encode()), header)
        if m:
            pos[n] = m.start()
    return {n: i for i, n in enumerate(sorted(pos, key=pos.get))}


# ------------------------------------------------------------------------------------------------
# key-group sections

def read_key_groups(data, offsets, first_kg, layouts, end=None):
    """Parse the key-group sections of one keyed state handle.

    layouts: state id -> ("kv", namespace_ser, key_ser, value_ser) or ("pq", key_ser, namespace_ser).
    Returns {kg: {state id: [entries]}}: kv entries (namespace, key, value), pq entries (ts, key, namespace)."""
    out = {}
    end = len(data) if end is None else end
    bounds = list(offsets) + [end]
    for i, off in enumerate(offsets):
        r = Reader(data, off, bounds[i + 1] if bounds[i + 1] >= off else end)
        kg = r.get(">i")
        assert kg == first_kg + i, (kg, first_kg + i)
        sections = {}
        while r.at < r.end:
            sid = r.get(">h")
            assert sid in layouts, "unknown state id %d" % sid
            lay = layouts[sid]
            n = r.get(">i")
            ents = []
            for _ in range(n):
                if lay[0] == "kv":
                    ns = lay[1](r)
                    key = lay[2](r)
                    ents.append((ns, key, lay[3](r)))
                else:
                    ts = r.get(">Q") ^ (1 << 63)
                    ts = ts - (1 << 64) if ts >= 1 << 63 else ts
                    key = lay[1](r)
                    ents.append((ts, key, lay[2](r)))
            sections[sid] = ents
        out[kg] = sections
    return out


def s64(x):
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= 1 << 63 else x


def parse_engine_heap(body, offsets, ds, naggs, sess=False, first_kg=0):
    """The engine's fwa_snapshot_heap body (the layout the Java shim puts behind its own proxy header):
    DataStream: 0 window-contents (TimeWindow, Long, Tuple of 1 + naggs longs), [sessions: 1 merging-window-set
    (VoidNamespace, Long, List<Tuple2<TimeWindow, TimeWindow>>)], then processing and event timers (Long key,
    TimeWindow); Table: 0 window state (Long slice end, BinaryRowData key, BinaryRowData acc), 1 processing and 2 event
    timers (BinaryRowData key, Long). The ids are the heap backend's (heap_snapshot.cpp ids_of).
    Returns (key group -> [(key, start, end, acc fields, null flags)], timers, merging sets)."""
    if ds:
        lay = {0: ("kv", ser_time_window, ser_long, ser_tuple(*[ser_ulong] * (1 + naggs)))}
        if sess:
            lay[1] = ("kv", ser_void, ser_long, ser_list(ser_tuple(ser_time_window, ser_time_window)))
        nxt = 2 if sess else 1
        lay[nxt] = ("pq", ser_long, ser_time_window)             # processing-time timers (none on this path)
        lay[nxt + 1] = ("pq", ser_long, ser_time_window)         # event-time timers
    elif sess:                                                   # legacy Table WindowOperator (GROUP BY SESSION)
        lay = {0: ("kv", ser_void, ser_binrow(1), ser_map(ser_time_window, ser_time_window)),
               1: ("kv", ser_time_window, ser_binrow(1), ser_binrow(1 + naggs)),
               2: ("pq", ser_binrow(1), ser_time_window), 3: ("pq", ser_binrow(1), ser_time_window)}
    else:
        lay = {0: ("kv", ser_long, ser_binrow(1), ser_binrow(1 + naggs)), 1: ("pq", ser_binrow(1), ser_long),
               2: ("pq", ser_binrow(1), ser_long)}
    secs = read_key_groups(body, offsets, first_kg, lay)
    ents, timers, msets = {}, {}, {}
    tid = max(lay)
    cid, mid = (1, 0) if sess and not ds else (0, 1)            # window contents / merging set state ids
    for kg, s in secs.items():
        assert sorted(s) == sorted(lay), "every state section is written, in id order"
        e = []
        for ns, key, val in s.get(cid, []):
            if ds:
                e.append((key, ns[0], ns[1], list(val), [False] * (1 + naggs)))
            else:
                rk, kn, kf = key
                assert rk == 0 and not kn[0]                 # RowKind INSERT, non-NULL key
                vk, vn, vf = val
                assert vk == 0
                if sess:
                    e.append((kf[0], ns[0], ns[1], vf, vn))
                else:
                    e.append((kf[0], None, ns, vf, vn))
        ents[kg] = e
        if sess:
            if ds:
                msets[kg] = {key: [(a[0], a[1], b[0], b[1]) for a, b in val] for _, key, val in s.get(mid, [])}
            else:
                msets[kg] = {key[2][0]: [(a[0], a[1], b[0], b[1]) for a, b in val] for _, key, val in s.get(mid, [])}
        if ds:
            timers[kg] = [(ts, key, ns[0], ns[1]) for ts, key, ns in s.get(tid, [])]
        elif sess:
            timers[kg] = [(ts, key[2][0], ns[0], ns[1]) for ts, key, ns in s.get(tid, [])]
        else:
            timers[kg] = [(ts, key[2][0], ns) for ts, key, ns in s.get(tid, [])]
    return ents, timers, msets
