"""ctypes mirror of include/flink_amd.h (the C-ABI of the engine).

Kept in one place so the product wrapper (flink_amd.engine) and the test-side oracle wrapper bind
the exact same struct layouts.
"""
import ctypes as C

import numpy as np

FWA_ABI_VERSION = 5
FWA_MAX_AGGS = 8
FWA_MAX_COLS = 8

# enum fwa_window_kind
TUMBLE, SLIDE, CUMULATE, SESSION = 0, 1, 2, 3
WINDOW_KINDS = {"TUMBLE": TUMBLE, "SLIDE": SLIDE, "HOP": SLIDE, "CUMULATE": CUMULATE, "SESSION": SESSION}
# enum fwa_semantics
SEM_DATASTREAM, SEM_TABLE = 0, 1
SEMANTICS = {"DATASTREAM": SEM_DATASTREAM, "TABLE": SEM_TABLE}
# enum fwa_key_kind
KEY_JAVA_LONG, KEY_BINROW_BIGINT, KEY_PREHASHED, KEY_GROUP_PREFIXED = 0, 1, 2, 3

AGG_KINDS = {
    "COUNT": 0, "SUM_I64": 1, "SUM_F32": 2, "SUM_F64": 3, "MIN_I64": 4, "MAX_I64": 5,
    "MIN_F32": 6, "MAX_F32": 7, "MIN_F64": 8, "MAX_F64": 9, "AVG_I64": 10, "AVG_F32": 11,
    "AVG_F64": 12, "COUNT_COL": 13,
    "SUM_DEC": 14, "AVG_DEC": 15, "SUM_DEC128": 16, "AVG_DEC128": 17,
    # DataStream built-in reductions (FWA_CFG_REDUCE)
    "SUM_I32": 18, "MIN_I32": 19, "MAX_I32": 20, "FIRST_64": 21, "FIRST_32": 22,
    "MINBY_I64": 23, "MAXBY_I64": 24, "MINBY_I32": 25, "MAXBY_I32": 26, "MINBY_F64": 27, "MAXBY_F64": 28,
    "MINBY_F32": 29, "MAXBY_F32": 30, "SEL_64": 31, "SEL_32": 32,
}
DEC_KINDS = ("SUM_DEC", "AVG_DEC", "SUM_DEC128", "AVG_DEC128")
AGG_NAMES = {v: k for k, v in AGG_KINDS.items()}
# numpy dtype of each aggregate's RESULT column
AGG_RESULT_DTYPE = {
    "COUNT": "i8", "SUM_I64": "i8", "SUM_F32": "f4", "SUM_F64": "f8", "MIN_I64": "i8",
    "MAX_I64": "i8", "MIN_F32": "f4", "MAX_F32": "f4", "MIN_F64": "f8", "MAX_F64": "f8",
    "AVG_I64": "i8", "AVG_F32": "f4", "AVG_F64": "f8", "COUNT_COL": "i8",
    # DECIMAL: 16-byte unscaled two's complement; the wrappers return Python ints (object arrays)
    "SUM_DEC": "V16", "AVG_DEC": "V16", "SUM_DEC128": "V16", "AVG_DEC128": "V16",
    # FIRST_* / SEL_*: the field's raw bits (view them as the field's type)
    "SUM_I32": "i4", "MIN_I32": "i4", "MAX_I32": "i4", "FIRST_64": "i8", "FIRST_32": "i4",
    "MINBY_I64": "i8", "MAXBY_I64": "i8", "MINBY_I32": "i4", "MAXBY_I32": "i4", "MINBY_F64": "f8", "MAXBY_F64": "f8",
    "MINBY_F32": "f4", "MAXBY_F32": "f4", "SEL_64": "i8", "SEL_32": "i4",
}
# numpy dtype of each aggregate's INPUT column (None: no input)
AGG_INPUT_DTYPE = {
    "COUNT": None, "SUM_I64": "i8", "SUM_F32": "f4", "SUM_F64": "f8", "MIN_I64": "i8",
    "MAX_I64": "i8", "MIN_F32": "f4", "MAX_F32": "f4", "MIN_F64": "f8", "MAX_F64": "f8",
    "AVG_I64": "i8", "AVG_F32": "f4", "AVG_F64": "f8", "COUNT_COL": None,
    "SUM_DEC": "i8", "AVG_DEC": "i8", "SUM_DEC128": "V16", "AVG_DEC128": "V16",
    "SUM_I32": "i4", "MIN_I32": "i4", "MAX_I32": "i4", "FIRST_64": "i8", "FIRST_32": "i4",
    "MINBY_I64": "i8", "MAXBY_I64": "i8", "MINBY_I32": "i4", "MAXBY_I32": "i4", "MINBY_F64": "f8", "MAXBY_F64": "f8",
    "MINBY_F32": "f4", "MAXBY_F32": "f4", "SEL_64": "i8", "SEL_32": "i4",
}


def dec128_column(values):
    """Unscaled DECIMAL values (Python ints, |v| < 2^127) -> the engine's 16-byte column: int64 [n, 2] (low, high)."""
    out = np.empty((len(values), 2), np.int64)
    for i, v in enumerate(values):
        u = int(v) & ((1 << 128) - 1)
        lo, hi = u & ((1 << 64) - 1), u >> 64
        out[i, 0] = lo - (1 << 64) if lo >= 1 << 63 else lo
        out[i, 1] = hi - (1 << 64) if hi >= 1 << 63 else hi
    return out


def dec128_values(raw):
    """16-byte two's-complement values (any buffer of n * 16 bytes) -> numpy object array of Python ints."""
    w = np.frombuffer(memoryview(raw).cast("B"), np.uint64).reshape(-1, 2)
    out = np.empty(w.shape[0], object)
    for i in range(w.shape[0]):
        u = int(w[i, 0]) | (int(w[i, 1]) << 64)
        out[i] = u - (1 << 128) if u >= 1 << 127 else u
    return out

STATUS = {0: "OK", -1: "E_ARG", -2: "E_TS_MIN", -3: "E_KEYGROUP", -4: "E_MERGE_LATE", -5: "E_OOM",
          -6: "E_DEVICE", -7: "E_UNSUPPORTED", -8: "E_STATE", -9: "E_CORRUPT"}

CFG_DYNAMIC_GAP = 0x1
CFG_LATE_INDICES = 0x2
CFG_RECORD_LISTS = 0x4
CFG_REDUCE = 0x8
CFG_BY_LAST = 0x10

PUSH_DEVICE_PTRS = 0x1
PUSH_ASYNC = 0x2

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


class AggSpec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("col", C.c_int32)]


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("window_kind", C.c_int32), ("semantics", C.c_int32),
        ("key_kind", C.c_int32), ("size_ms", C.c_int64), ("slide_ms", C.c_int64),
        ("offset_ms", C.c_int64), ("gap_ms", C.c_int64), ("allowed_lateness_ms", C.c_int64),
        ("max_parallelism", C.c_int32), ("kg_start", C.c_int32), ("kg_end", C.c_int32),
        ("num_aggs", C.c_int32), ("aggs", AggSpec * FWA_MAX_AGGS), ("device", C.c_int32),
        ("output_on_device", C.c_int32), ("key_capacity", C.c_int64), ("max_batch", C.c_int64),
        ("flags", C.c_int32), ("gap_col", C.c_int32), ("tz_n", C.c_int32), ("nullable_cols", C.c_int32),
        ("tz", C.c_void_p),
        ("dec_scale", C.c_int32 * FWA_MAX_AGGS),    # ABI 4: DECIMAL aggregate j's input scale
    ]


class Out(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64), ("on_device", C.c_int32), ("num_aggs", C.c_int32),
        ("key", C.c_void_p), ("win_start", C.c_void_p), ("win_end", C.c_void_p),
        ("agg", C.c_void_p * FWA_MAX_AGGS), ("agg_null", C.c_void_p * FWA_MAX_AGGS),
    ]


FWA_MAX_DEST = 64


class Routed(C.Structure):
    """fwa_routed (include/flink_amd.h): fwa_drain_route's per-destination packed rows."""
    _fields_ = [("n", C.c_int64), ("parallelism", C.c_int32), ("cells", C.c_int32), ("on_device", C.c_int32),
                ("pad", C.c_int32), ("rows", C.c_void_p * FWA_MAX_DEST), ("count", C.c_int64 * FWA_MAX_DEST)]


class Partials(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("on_device", C.c_int32), ("num_aggs", C.c_int32),
        ("key", C.c_void_p), ("slice_start", C.c_void_p), ("count", C.c_void_p),
        ("acc", C.c_void_p * FWA_MAX_AGGS), ("num_hidden", C.c_int32), ("pad", C.c_int32),
        ("hidden", C.c_void_p * FWA_MAX_COLS),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("records_in", C.c_int64), ("late_dropped", C.c_int64), ("rows_out", C.c_int64),
        ("live_keys", C.c_int64), ("live_slices", C.c_int64), ("current_watermark", C.c_int64),
        ("ingest_launches", C.c_int64), ("ingest_ms", C.c_double), ("ingest_records", C.c_int64),
        ("fire_launches", C.c_int64), ("fire_ms", C.c_double), ("fire_rows", C.c_int64),
        ("partition_ms", C.c_double), ("combine_ms", C.c_double), ("replay_records", C.c_int64),
        ("dec_inexact", C.c_int64),
    ]


class GenParams(C.Structure):
    _fields_ = [
        ("seed_k", C.c_uint64), ("seed_t", C.c_uint64), ("seed_v", C.c_uint64),
        ("first_index", C.c_int64), ("total_records", C.c_int64), ("num_keys", C.c_int64),
        ("t0_ms", C.c_int64), ("span_ms", C.c_int64), ("max_delay_ms", C.c_int64),
        ("key_dist", C.c_int32), ("val_kind", C.c_int32), ("zipf_cdf", C.c_void_p),
    ]


def make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000, slide_ms=0,
                offset_ms=0, gap_ms=0, allowed_lateness_ms=0, aggs=(("COUNT", 0), ("SUM_I64", 0)),
                key_kind=KEY_JAVA_LONG, max_parallelism=128, kg_start=0, kg_end=None, device=0,
                output_on_device=0, key_capacity=0, max_batch=0, gap_col=None, tz=None, late_indices=False,
                nullable_cols=(), record_lists=False, reduce=False, by_last=False):
    """Build a Config struct. aggs: sequence of (agg name, value-column index). gap_col: value column of
    per-record session gaps (DynamicEventTimeSessionWindows). tz: [(utc_instant_ms, offset_ms), ...] shift
    time zone of a TIMESTAMP_LTZ rowtime (the struct keeps a pointer to a buffer held on the struct). reduce: a
    DataStream built-in reduction (FWA_CFG_REDUCE, WindowedStream.sum/min/max/minBy/maxBy); by_last: minBy / maxBy
    ties go to the last element (FWA_CFG_BY_LAST)."""
    c = Config()
    c.abi_version = FWA_ABI_VERSION
    c.window_kind = WINDOW_KINDS[window_kind] if isinstance(window_kind, str) else int(window_kind)
    c.semantics = SEMANTICS[semantics] if isinstance(semantics, str) else int(semantics)
    c.key_kind = key_kind
    c.size_ms, c.slide_ms, c.offset_ms = size_ms, slide_ms, offset_ms
    c.gap_ms, c.allowed_lateness_ms = gap_ms, allowed_lateness_ms
    c.max_parallelism = max_parallelism
    c.kg_start = kg_start
    c.kg_end = (max_parallelism - 1) if kg_end is None else kg_end
    if len(aggs) > FWA_MAX_AGGS:
        raise ValueError("at most %d aggregates" % FWA_MAX_AGGS)
    c.num_aggs = len(aggs)
    for i, spec in enumerate(aggs):                       # (name, col) or, for DECIMAL, (name, col, scale)
        name, col = spec[0], spec[1]
        c.aggs[i].kind = AGG_KINDS[name]
        c.aggs[i].col = col
        if len(spec) > 2:
            c.dec_scale[i] = int(spec[2])
    c.device = device
    c.output_on_device = output_on_device
    c.key_capacity = key_capacity
    c.max_batch = max_batch
    if late_indices:
        c.flags |= CFG_LATE_INDICES
    if record_lists:                                      # TUMBLE state as record lists (huge key spaces)
        c.flags |= CFG_RECORD_LISTS
    if reduce:
        c.flags |= CFG_REDUCE
    if by_last:
        c.flags |= CFG_BY_LAST
    for col in nullable_cols:                             # value columns that may hold SQL NULLs
        c.nullable_cols |= 1 << col
    if gap_col is not None:
        c.flags |= CFG_DYNAMIC_GAP
        c.gap_col = gap_col
    if tz:
        buf = (C.c_int64 * (2 * len(tz)))(*[int(x) for pair in tz for x in pair])
        c._tz_buf = buf                                  # keep the pairs alive as long as the struct
        c.tz_n = len(tz)
        c.tz = C.cast(buf, C.c_void_p)
    return c


def agg_names(cfg):
    return [AGG_NAMES[cfg.aggs[i].kind] for i in range(cfg.num_aggs)]


def bind_common(lib, prefix):
    """Declare argtypes for the engine-shaped API exported under `prefix` (fwa_ or or_)."""
    P = C.c_void_p
    getattr(lib, prefix + "create").argtypes = [C.POINTER(Config), C.POINTER(P)]
    getattr(lib, prefix + "create").restype = C.c_int
    getattr(lib, prefix + "destroy").argtypes = [P]
    getattr(lib, prefix + "destroy").restype = None
    getattr(lib, prefix + "advance_watermark").argtypes = [P, C.c_int64, C.POINTER(Out)]
    getattr(lib, prefix + "advance_watermark").restype = C.c_int
    getattr(lib, prefix + "get_stats").argtypes = [P, C.POINTER(Stats)]
    getattr(lib, prefix + "get_stats").restype = C.c_int
    getattr(lib, prefix + "last_error").argtypes = [P]
    getattr(lib, prefix + "last_error").restype = C.c_char_p
