"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle/liboracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
The product (flink_amd/) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from flink_amd import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        A.bind_common(L, "or_")
        L.or_push.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                              C.c_int64, C.POINTER(C.c_int64)]
        L.or_push.restype = C.c_int
        for f in ("or_murmur_hash", "or_bit_mix"):
            getattr(L, f).argtypes = [C.c_int32]
            getattr(L, f).restype = C.c_int32
        L.or_long_hash.argtypes = [C.c_int64]
        L.or_long_hash.restype = C.c_int32
        L.or_binrow_bigint_hash.argtypes = [C.c_int64]
        L.or_binrow_bigint_hash.restype = C.c_int32
        L.or_binrow_hash.argtypes = [C.c_void_p, C.c_int32, C.c_uint64]
        L.or_binrow_hash.restype = C.c_int32
        L.or_hash_bytes_by_words.argtypes = [C.c_char_p, C.c_int32]
        L.or_hash_bytes_by_words.restype = C.c_int32
        L.or_key_group.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32]
        L.or_key_group.restype = C.c_int32
        L.or_operator_index.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        L.or_operator_index.restype = C.c_int32
        L.or_key_group_range.argtypes = [C.c_int32, C.c_int32, C.c_int32,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.or_window_start.argtypes = [C.c_int64, C.c_int64, C.c_int64]
        L.or_window_start.restype = C.c_int64
        L.or_assign_windows.argtypes = [C.POINTER(A.Config), C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
        L.or_assign_windows.restype = C.c_int
        L.or_assign_slice_end.argtypes = [C.POINTER(A.Config), C.c_int64]
        L.or_assign_slice_end.restype = C.c_int64
        L.or_push_nullable.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.POINTER(C.c_int64)]
        L.or_push_nullable.restype = C.c_int
        L.or_late_records.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.or_late_records.restype = C.c_int
        for f in ("or_to_local", "or_tz_timer"):
            getattr(L, f).argtypes = [C.POINTER(A.Config), C.c_int64]
            getattr(L, f).restype = C.c_int64
        L.or_splitmix64.argtypes = [C.c_uint64]
        L.or_splitmix64.restype = C.c_uint64
        L.or_generate.argtypes = [C.POINTER(A.GenParams), C.c_int64, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_generate.restype = None
        L.or_bench_pipeline.argtypes = [C.POINTER(A.Config), C.POINTER(A.GenParams), C.c_int64,
                                        C.c_int64, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
        L.or_bench_pipeline.restype = C.c_double
        L.or_pipeline_digests.argtypes = [C.POINTER(A.Config), C.POINTER(A.GenParams), C.c_int64, C.c_int64, C.c_int,
                                          C.c_void_p, C.c_void_p]
        L.or_pipeline_digests.restype = C.c_double
        L.or_pipeline_digests2.argtypes = [C.POINTER(A.Config), C.POINTER(A.GenParams), C.c_void_p, C.c_int,
                                           C.c_uint32, C.c_uint32, C.c_int, C.c_int64, C.c_int64, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_pipeline_digests2.restype = C.c_double
        L.or_row_digest.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_int]
        L.or_row_digest.restype = C.c_uint64
        _LIB = L
    return _LIB


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def binrow_bytes(types, row):
    """The bytes of a BinaryRowData key row as BinaryRowWriter writes it (a restatement for the tests: header with
    RowKind INSERT and null bits from bit 8, 8-byte little-endian slots -- BIGINT / DOUBLE bits, INT in the low 4 bytes,
    NULL zeroed; a STRING of <= 7 UTF-8 bytes inline (first byte 0x80 | length), a longer one in the variable-length part,
    8-byte aligned with zero padding, slot = offset << 32 | length (AbstractBinaryWriter.java:80-105,279-334))."""
    import struct
    arity = len(types)
    nb = ((arity + 63 + 8) // 64) * 8
    head = bytearray(nb)
    slots, var = [], bytearray()
    for c, (t, v) in enumerate(zip(types, row)):
        if v is None:
            head[(c + 8) // 8] |= 1 << ((c + 8) % 8)
            slots.append(0)
        elif t == "STRING":
            b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
            if len(b) <= 7:
                slots.append(((0x80 | len(b)) << 56) | int.from_bytes(b, "little"))
            else:
                slots.append(((nb + 8 * arity + len(var)) << 32) | len(b))
                var += b + bytes((-len(b)) % 8)
        elif t == "INT":
            slots.append(v & 0xFFFFFFFF)
        elif t == "DOUBLE":
            slots.append(struct.unpack("<Q", struct.pack("<d", v))[0])
        else:
            slots.append(v & 0xFFFFFFFFFFFFFFFF)
    return bytes(head) + b"".join(x.to_bytes(8, "little") for x in slots) + bytes(var)


def binrow_hash_bytes(row_bytes):
    """BinaryRowData.hashCode() of a row's bytes (MurmurHashUtils.hashBytesByWords, the oracle's C restatement)."""
    return lib().or_hash_bytes_by_words(row_bytes, len(row_bytes))


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (A.STATUS.get(code, code), msg))
        self.code = code


def rows_from_out(out, names):
    """Copy an fwa_out (host pointers) into a dict of numpy arrays."""
    n = out.n_rows
    res = {}
    for field, dt in (("key", np.int64), ("win_start", np.int64), ("win_end", np.int64)):
        p = getattr(out, field)
        res[field] = (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int64)), (n,)).copy()
                      if n else np.zeros(0, dt))
    for j, name in enumerate(names):
        dt = np.dtype(A.AGG_RESULT_DTYPE[name])
        if n == 0:
            res["agg%d" % j] = np.zeros(0, object if name in A.DEC_KINDS else dt)
            continue
        # oracle stores each result in a 16-byte slot (union); i64/f64 results in the low 8 bytes, f32 in the low 4,
        # DECIMAL ones fill it
        raw16 = np.ctypeslib.as_array(C.cast(out.agg[j], C.POINTER(C.c_uint64)), (2 * n,)).copy()
        if name in A.DEC_KINDS:
            res["agg%d" % j] = A.dec128_values(raw16)
            if out.agg_null[j]:
                res["null%d" % j] = np.ctypeslib.as_array(C.cast(out.agg_null[j], C.POINTER(C.c_uint8)), (n,)).copy()
            continue
        raw = raw16[0::2].copy()
        if dt.itemsize == 4:
            res["agg%d" % j] = (raw & 0xffffffff).astype(np.uint32).view(dt)
        else:
            res["agg%d" % j] = raw.view(dt)
        if out.agg_null[j]:
            res["null%d" % j] = np.ctypeslib.as_array(C.cast(out.agg_null[j], C.POINTER(C.c_uint8)), (n,)).copy()
    return res


class Oracle:
    """Same contract as flink_amd.WindowAggregator, computed on the CPU by the restatement."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.names = A.agg_names(cfg)
        self.h = C.c_void_p()
        rc = lib().or_create(C.byref(cfg), C.byref(self.h))
        if rc:
            raise OracleError(rc, "or_create")

    def push(self, keys, ts, cols=(), key_hash=None, nulls=None):
        keys = np.ascontiguousarray(keys, np.int64)
        ts = np.ascontiguousarray(ts, np.int64)
        cols = [np.ascontiguousarray(c) for c in cols]
        arr = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        kh = None if key_hash is None else np.ascontiguousarray(key_hash, np.int32)
        narr = None
        if nulls is not None:
            nulls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in nulls]
            narr = (C.c_void_p * max(1, len(nulls)))(*[None if x is None else x.ctypes.data for x in nulls])
        dropped = C.c_int64(0)
        rc = lib().or_push_nullable(self.h, _ptr(keys), _ptr(ts), arr, narr, _ptr(kh), len(keys), C.byref(dropped))
        if rc:
            raise OracleError(rc, lib().or_last_error(self.h).decode())
        return dropped.value

    def late_records(self):
        """Indices of the records the last push dropped as late (ascending)."""
        p, n = C.c_void_p(), C.c_int64()
        lib().or_late_records(self.h, C.byref(p), C.byref(n))
        if n.value == 0:
            return np.zeros(0, np.int32)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(n.value,)).copy()

    def advance_watermark(self, wm):
        out = A.Out()
        rc = lib().or_advance_watermark(self.h, wm, C.byref(out))
        if rc:
            raise OracleError(rc, lib().or_last_error(self.h).decode())
        return rows_from_out(out, self.names)

    def flush(self):
        """The oracle applies every record immediately; nothing is buffered."""

    def stats(self):
        st = A.Stats()
        lib().or_get_stats(self.h, C.byref(st))
        return st

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def generate(params, n, want_floats=False, cdf=None):
    """CPU generator of the synthetic stream (bit-identical to the device generator)."""
    keys = np.empty(n, np.int64)
    ts = np.empty(n, np.int64)
    vi = np.empty(n, np.int64)
    vf = np.empty(n, np.float32) if want_floats else None
    vd = np.empty(n, np.float64) if want_floats else None
    cdf_a = None if cdf is None else np.ascontiguousarray(cdf, np.float64)
    lib().or_generate(C.byref(params), n, _ptr(keys), _ptr(ts), _ptr(vi), _ptr(vf), _ptr(vd), _ptr(cdf_a))
    return keys, ts, vi, vf, vd


def bench_pipeline(cfg, params, n, batch, threads):
    rows = C.c_int64(0)
    cs = C.c_uint64(0)
    secs = lib().or_bench_pipeline(C.byref(cfg), C.byref(params), n, batch, threads, C.byref(rows), C.byref(cs))
    return secs, rows.value, cs.value


def pipeline_digests2(cfg, params, n, batch, threads, cdf=None, float_cols=False, exact=(), sums=(), nbuckets=4096):
    """or_pipeline_digests2: per watermark the row count, the digest of (key, start, end, the aggregates listed in
    `exact`: their 8-byte result words) and, for the aggregates in `sums` (double results), per row bucket the sum of
    the values and of their magnitudes. Returns (secs, rows[nb+1], digests[nb+1], bsum[nb+1][len(sums)][nbuckets],
    babs[...])."""
    nb = (n + batch - 1) // batch
    rows = np.zeros(nb + 1, np.int64)
    dig = np.zeros(nb + 1, np.uint64)
    bsum = np.zeros((nb + 1, len(sums), nbuckets), np.float64)
    babs = np.zeros_like(bsum)
    em = sum(1 << j for j in exact)
    sm = sum(1 << j for j in sums)
    cdf_a = None if cdf is None else np.ascontiguousarray(cdf, np.float64)
    secs = lib().or_pipeline_digests2(C.byref(cfg), C.byref(params), _ptr(cdf_a), int(bool(float_cols)), em, sm,
                                      nbuckets, n, batch, threads, _ptr(rows), _ptr(dig), _ptr(bsum), _ptr(babs))
    if secs < 0:
        raise OracleError(int(secs), "or_pipeline_digests2")
    return secs, rows, dig, bsum, babs


def pipeline_digests(cfg, params, n, batch, threads):
    """Threaded oracle over the generated stream: per batch watermark (max_ts - D - 1) and the final Long.MAX_VALUE
    one, the fired row count and the order-free row digest (or_row_digest summed mod 2^64). Returns (secs, rows[nb+1],
    digests[nb+1] as uint64)."""
    nb = (n + batch - 1) // batch
    rows = np.zeros(nb + 1, np.int64)
    dig = np.zeros(nb + 1, np.uint64)
    secs = lib().or_pipeline_digests(C.byref(cfg), C.byref(params), n, batch, threads, _ptr(rows), _ptr(dig))
    if secs < 0:
        raise OracleError(int(secs), "or_pipeline_digests")
    return secs, rows, dig


def row_digest(key, start, end, aggs):
    a = np.ascontiguousarray(aggs, np.int64)
    return lib().or_row_digest(int(key), int(start), int(end), _ptr(a), len(a))


def wire_decode(schema, data):
    """Sequential CPU decode of a channel's bytes (oracle/wire_oracle.c). schema: flink_amd.wire.Schema.
    Returns (status, dict) with numpy columns, events and `consumed`."""
    L = lib()
    if not getattr(L, "_wire_bound", False):
        P = C.c_void_p
        L.or_wire_decode.argtypes = [P, P, C.c_int64, P, P, P, P, P, P, P, P, P, P, P, P, P]
        L.or_wire_decode.restype = C.c_int
        L._wire_bound = True
    arr = np.frombuffer(bytes(data), np.uint8)
    nb = arr.size
    cap_r, cap_e = nb // 6 + 1, nb // 6 + 1
    fdt = {0: np.int64, 1: np.float64, 2: np.float32, 3: np.int64}
    key = np.zeros(cap_r, np.int64)
    ts = np.zeros(cap_r, np.int64)
    cols = [np.zeros(cap_r, fdt[schema.field[schema.col_field[j]]]) for j in range(schema.num_cols)]
    rowdata = schema.format == 1
    cnull = [np.zeros(cap_r, np.uint8) for _ in range(schema.num_cols)] if rowdata else []
    knull = np.zeros(cap_r, np.uint8) if rowdata else None
    epos = np.zeros(cap_e, np.int64)
    etag = np.zeros(cap_e, np.int32)
    evals = np.zeros((cap_e, 4), np.int64)
    colp = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
    nullp = (C.c_void_p * max(1, len(cnull)))(*[c.ctypes.data for c in cnull]) if rowdata else None
    nr, ne, cons, etg, eps = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32(), C.c_int64()
    rc = L.or_wire_decode(C.byref(schema), _ptr(arr), nb, _ptr(key), _ptr(ts), colp, nullp, _ptr(knull), _ptr(epos),
                          _ptr(etag), _ptr(evals), C.byref(nr), C.byref(ne), C.byref(cons), C.byref(etg), C.byref(eps))
    n, m = nr.value, ne.value
    res = {"n_records": n, "n_events": m, "consumed": cons.value, "key": key[:n], "ts": ts[:n],
           "cols": [c[:n] for c in cols], "col_null": [c[:n] for c in cnull] if rowdata else None,
           "key_null": knull[:n] if rowdata else None, "evt_pos": epos[:m], "evt_tag": etag[:m],
           "evt_val": evals[:m], "err_tag": etg.value, "err_pos": eps.value}
    return rc, res
