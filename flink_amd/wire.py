"""On-GPU decoding of Flink's network wire format (include/flink_amd_wire.h).

`WireDecoder` binds fwa_wire_decode: the concatenated data-buffer payloads of one input channel go in, SoA
columns in HBM (zero-copy torch views, valid until the next decode) and the ordered non-record elements come
out. `NetworkInput` is the host-side mirror of the channel loop in front of the operator:
  AbstractStreamTaskNetworkInput.emitNext / processElement   flink-streaming-java/.../runtime/io/
                                                             AbstractStreamTaskNetworkInput.java:100-181
  StatusWatermarkValve (one channel)                         .../watermarkstatus/StatusWatermarkValve.java:93-115
It pushes each run of records between two events straight from HBM into the window engine and applies the
events in stream order: a watermark that advances the channel's watermark fires windows
(processWatermark), WatermarkStatus IDLE / ACTIVE toggles the channel, latency markers and record attributes
are forwarded. No CPU fallback: the HIP library must be present.
"""
import ctypes as C

import numpy as np

from . import _abi as A
from .engine import EngineError, _is_torch_cuda, dev_view, lib

MAX_FIELDS = 16
FORMATS = {"TUPLE": 0, "ROWDATA": 1}
FIELDS = {"LONG": 0, "DOUBLE": 1, "FLOAT": 2, "INT": 3}
FIELD_DTYPE = {0: "i8", 1: "f8", 2: "f4", 3: "i8"}           # value-column dtype per field type
TAG_REC_WITH_TIMESTAMP, TAG_REC_WITHOUT_TIMESTAMP, TAG_WATERMARK, TAG_LATENCY_MARKER, TAG_STREAM_STATUS, \
    TAG_RECORD_ATTRIBUTES = range(6)
WIRE_DEVICE_BYTES = 0x1
WATERMARK_STATUS_IDLE, WATERMARK_STATUS_ACTIVE = -1, 0     # WatermarkStatus.IDLE_STATUS / ACTIVE_STATUS


class Schema(C.Structure):
    _fields_ = [("format", C.c_int32), ("arity", C.c_int32), ("field", C.c_int32 * MAX_FIELDS),
                ("key_field", C.c_int32), ("ts_field", C.c_int32), ("num_cols", C.c_int32),
                ("col_field", C.c_int32 * 8), ("device", C.c_int32), ("max_bytes", C.c_int64)]


class Batch(C.Structure):
    _fields_ = [("n_records", C.c_int64), ("n_events", C.c_int64), ("consumed", C.c_int64),
                ("key", C.c_void_p), ("ts", C.c_void_p), ("col", C.c_void_p * 8), ("col_null", C.c_void_p * 8),
                ("key_null", C.c_void_p), ("evt_pos", C.c_void_p), ("evt_tag", C.c_void_p), ("evt_val", C.c_void_p)]


class WireStats(C.Structure):
    _fields_ = [("calls", C.c_int64), ("bytes_in", C.c_int64), ("records_out", C.c_int64),
                ("decode_ms", C.c_double), ("scan_ms", C.c_double)]


def make_schema(fields, key_field, ts_field=-1, cols=(), fmt="TUPLE", device=0, max_bytes=0):
    """fields: field type names in value order ("LONG", "DOUBLE", "FLOAT", "INT"); ts_field -1 = the
    StreamRecord timestamp; cols: the fields that become value columns 0, 1, ..."""
    s = Schema()
    s.format = FORMATS[fmt]
    s.arity = len(fields)
    for i, f in enumerate(fields):
        s.field[i] = FIELDS[f]
    s.key_field, s.ts_field = key_field, ts_field
    s.num_cols = len(cols)
    for j, f in enumerate(cols):
        s.col_field[j] = f
    s.device, s.max_bytes = device, max_bytes
    return s


def _bind(L):
    if getattr(L, "_wire_bound", False):
        return L
    L.fwa_wire_create.argtypes = [C.POINTER(Schema), C.POINTER(C.c_void_p)]
    L.fwa_wire_create.restype = C.c_int
    L.fwa_wire_destroy.argtypes = [C.c_void_p]
    L.fwa_wire_destroy.restype = None
    L.fwa_wire_last_error.argtypes = [C.c_void_p]
    L.fwa_wire_last_error.restype = C.c_char_p
    L.fwa_wire_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.POINTER(Batch)]
    L.fwa_wire_decode.restype = C.c_int
    L.fwa_wire_get_stats.argtypes = [C.c_void_p, C.POINTER(WireStats)]
    L.fwa_wire_get_stats.restype = C.c_int
    L._wire_bound = True
    return L


class DecodedBatch:
    """Columns of one decode (torch CUDA views into decoder-owned HBM, valid until its next decode)."""

    def __init__(self, schema, b):
        self.n_records, self.n_events, self.consumed = b.n_records, b.n_events, b.consumed
        n = self.n_records
        self.key = dev_view(b.key, n, np.dtype("i8"))
        self.ts = dev_view(b.ts, n, np.dtype("i8"))
        self.cols = [dev_view(b.col[j], n, np.dtype(FIELD_DTYPE[schema.field[schema.col_field[j]]]))
                     for j in range(schema.num_cols)]
        rowdata = schema.format == FORMATS["ROWDATA"]
        self.col_null = [dev_view(b.col_null[j], n, np.dtype("u1")) for j in range(schema.num_cols)] if rowdata else None
        self.key_null = dev_view(b.key_null, n, np.dtype("u1")) if rowdata else None
        ne = self.n_events
        if ne:
            self.evt_pos = np.ctypeslib.as_array(C.cast(b.evt_pos, C.POINTER(C.c_int64)), (ne,)).copy()
            self.evt_tag = np.ctypeslib.as_array(C.cast(b.evt_tag, C.POINTER(C.c_int32)), (ne,)).copy()
            self.evt_val = np.ctypeslib.as_array(C.cast(b.evt_val, C.POINTER(C.c_int64)), (ne, 4)).copy()
        else:
            self.evt_pos = np.zeros(0, np.int64)
            self.evt_tag = np.zeros(0, np.int32)
            self.evt_val = np.zeros((0, 4), np.int64)


class WireDecoder:
    """One decoder per input channel (single-threaded, like the channel's record deserializer)."""

    def __init__(self, schema):
        self.schema = schema
        self.L = _bind(lib())
        self.h = C.c_void_p()
        rc = self.L.fwa_wire_create(C.byref(schema), C.byref(self.h))
        if rc:
            raise EngineError(rc, "fwa_wire_create")

    def decode(self, data):
        """data: bytes / numpy uint8 (host, staged by the decoder) or a torch CUDA uint8 tensor (HBM)."""
        b = Batch()
        if _is_torch_cuda(data):
            import torch
            torch.cuda.current_stream(data.device).synchronize()   # the bytes' producer ran on torch's stream
            ptr, n, flags = C.c_void_p(data.data_ptr()), data.numel(), WIRE_DEVICE_BYTES
            keep = data
        else:
            arr = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, np.uint8)
            ptr, n, flags = arr.ctypes.data_as(C.c_void_p), arr.size, 0
            keep = arr
        rc = self.L.fwa_wire_decode(self.h, ptr, n, flags, C.byref(b))
        del keep
        if rc:
            raise EngineError(rc, self.L.fwa_wire_last_error(self.h).decode())
        return DecodedBatch(self.schema, b)

    def stats(self):
        s = WireStats()
        self.L.fwa_wire_get_stats(self.h, C.byref(s))
        return s

    def close(self):
        if self.h:
            self.L.fwa_wire_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NetworkInput:
    """One input channel in front of a window engine handle (flink_amd.engine.WindowAggregator).

    feed(buffer) takes the next data-buffer payload of the channel; an element that continues in the next
    buffer is carried over (SpanningWrapper). Returns the window rows fired by the watermarks in it.
    """

    def __init__(self, schema, engine):
        self.decoder = WireDecoder(schema)
        self.engine = engine
        self.carry = b""
        self.watermark = A.LONG_MIN                 # the channel's last forwarded watermark (valve)
        self.idle = False
        self.latency_markers = []                   # (markedTime, operatorId lower, upper, subtaskIndex)
        self.record_attributes = []                 # isBacklog flags, in order
        self.records_in = 0
        self.late_dropped = 0

    def _push(self, batch, a, b):
        if b <= a:
            return
        if batch.key_null is not None and bool(batch.key_null[a:b].any()):
            raise EngineError(-7, "NULL grouping key: pass the key hash with FWA_KEY_PREHASHED instead")
        nulls = None
        if batch.col_null is not None:
            nulls = [c[a:b] for c in batch.col_null]
        self.late_dropped += self.engine.push(batch.key[a:b], batch.ts[a:b], [c[a:b] for c in batch.cols],
                                              nulls=nulls if nulls and self.engine.cfg.nullable_cols else None)
        self.records_in += b - a

    def feed(self, buffer):
        import torch
        if self.carry:
            if _is_torch_cuda(buffer):
                buffer = torch.cat([torch.frombuffer(bytearray(self.carry), dtype=torch.uint8).to(buffer.device), buffer])
            else:
                buffer = self.carry + bytes(buffer)
        batch = self.decoder.decode(buffer)
        rows = []
        at = 0
        for pos, tag, val in zip(batch.evt_pos.tolist(), batch.evt_tag.tolist(), batch.evt_val.tolist()):
            self._push(batch, at, pos)
            at = pos
            if tag == TAG_WATERMARK:
                # StatusWatermarkValve.inputWatermark: an idle channel's or a non-advancing watermark is ignored
                if not self.idle and val[0] > self.watermark:
                    self.watermark = val[0]
                    rows.append(self.engine.advance_watermark(val[0]))
            elif tag == TAG_STREAM_STATUS:
                self.idle = val[0] == WATERMARK_STATUS_IDLE
            elif tag == TAG_LATENCY_MARKER:
                self.latency_markers.append(tuple(val))
            else:
                self.record_attributes.append(bool(val[0]))
        self._push(batch, at, batch.n_records)
        tail = len(buffer) - batch.consumed if not _is_torch_cuda(buffer) else buffer.numel() - batch.consumed
        if tail:
            rest = buffer[batch.consumed:]
            self.carry = bytes(rest.cpu().numpy()) if _is_torch_cuda(rest) else bytes(rest)
        else:
            self.carry = b""
        return rows

    def close(self):
        self.decoder.close()
