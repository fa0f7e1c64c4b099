"""TEST INFRASTRUCTURE ONLY: the sender side of Flink's wire format, to build decoder inputs.

Restates (numpy, vectorised per run of records):
  RecordWriter.serializeRecord                  RecordWriter.java:145-157 (4-byte big-endian length prefix,
                                                DataOutputSerializer.writeIntUnsafe :209-214)
  StreamElementSerializer.serialize             StreamElementSerializer.java:158-187 (tags :48-53)
  TupleSerializer -> Long/Double/Float/IntSerializer (java.io.DataOutput: big-endian)
  BinaryRowDataSerializer.serialize             BinaryRowDataSerializer.java:85-93 (int size + row bytes)
  BinaryRowWriter layout                        BinaryRowData.java:68-75,114-116: RowKind in byte 0, null bit
                                                of field i at bit i + 8, 8-byte little-endian fixed slots
Buffers: a channel's elements are written back to back across 32 KiB network buffers
(TaskManagerOptions.java:304-307, memory segment size); `split_buffers` cuts a stream the same way.
"""
import struct

import numpy as np

TUPLE_BE = {"LONG": ">i8", "DOUBLE": ">f8", "FLOAT": ">f4", "INT": ">i4"}
ROW_LE = {"LONG": "<i8", "DOUBLE": "<f8", "FLOAT": "<f4", "INT": "<i4"}
FIELD_NP = {"LONG": np.int64, "DOUBLE": np.float64, "FLOAT": np.float32, "INT": np.int32}


def nullbits_width(arity):
    return ((arity + 63 + 8) // 64) * 8                      # BinaryRowData.calculateBitSetWidthInBytes


def _record_dtype(fields, fmt, with_ts):
    d = [("len", ">i4"), ("tag", "u1")]
    if with_ts:
        d.append(("ts", ">i8"))
    if fmt == "TUPLE":
        d += [("f%d" % i, TUPLE_BE[f]) for i, f in enumerate(fields)]
    else:
        d += [("rowsize", ">i4"), ("hdr", "u1", (nullbits_width(len(fields)),))]
        for i, f in enumerate(fields):
            d.append(("f%d" % i, ROW_LE[f]))
            if f in ("FLOAT", "INT"):
                d.append(("p%d" % i, "u1", (4,)))
    return np.dtype(d)


def encode_records(fields, values, ts=None, fmt="TUPLE", nulls=None):
    """values: one array per field; ts: StreamRecord timestamps (None: TAG_REC_WITHOUT_TIMESTAMP);
    nulls (ROWDATA): one bool array or None per field. Returns the elements' bytes back to back."""
    n = len(values[0])
    dt = _record_dtype(fields, fmt, ts is not None)
    a = np.zeros(n, dt)
    a["len"] = dt.itemsize - 4
    a["tag"] = 0 if ts is not None else 1
    if ts is not None:
        a["ts"] = ts
    for i, f in enumerate(fields):
        v = np.asarray(values[i]).astype(FIELD_NP[f])
        if fmt == "ROWDATA" and nulls is not None and nulls[i] is not None:
            v = np.where(nulls[i], 0, v).astype(FIELD_NP[f])     # BinaryRowWriter.setNullAt zeroes the slot
        a["f%d" % i] = v
    if fmt == "ROWDATA":
        nb = nullbits_width(len(fields))
        a["rowsize"] = nb + 8 * len(fields)
        hdr = np.zeros((n, nb), np.uint8)                        # byte 0: RowKind.INSERT = 0
        if nulls is not None:
            for i, m in enumerate(nulls):
                if m is not None:
                    bit = i + 8
                    hdr[:, bit >> 3] |= (np.asarray(m, bool).astype(np.uint8) << (bit & 7))
        a["hdr"] = hdr
    return a.tobytes()


def encode_event(tag, vals=(0,)):
    """Non-record elements (StreamElementSerializer.serialize :169-184)."""
    if tag == 2:
        body = struct.pack(">bq", 2, vals[0])                    # Watermark
    elif tag == 3:
        body = struct.pack(">bqqqi", 3, vals[0], vals[1], vals[2], vals[3])   # LatencyMarker
    elif tag == 4:
        body = struct.pack(">bi", 4, vals[0])                    # WatermarkStatus
    elif tag == 5:
        body = struct.pack(">b?", 5, bool(vals[0]))              # RecordAttributes (writeBoolean)
    else:
        raise ValueError(tag)
    return struct.pack(">i", len(body)) + body


def encode_stream(fields, values, ts=None, fmt="TUPLE", events=(), nulls=None):
    """events: (pos, tag, vals) sorted by pos: the event is written before record `pos`."""
    n = len(values[0])
    out, at = [], 0
    for pos, tag, vals in list(events) + [(n, None, None)]:
        if pos > at:
            sl = slice(at, pos)
            out.append(encode_records(fields, [v[sl] for v in values], None if ts is None else ts[sl], fmt,
                                      None if nulls is None else [None if m is None else m[sl] for m in nulls]))
            at = pos
        if tag is not None:
            out.append(encode_event(tag, vals))
    return b"".join(out)


def split_buffers(stream, size=32 * 1024):
    return [stream[i:i + size] for i in range(0, len(stream), size)]
