/*
 * flink_amd.h -- C-ABI of the MI355X keyed event-time window-aggregation engine.
 *
 * This is the drop-in boundary for Flink's keyed windowed-aggregation hot path
 * (SURVEY.md §8(b)). A Java shim (JNI, or Panama FFM on JDK >= 22) sitting behind
 * the unchanged Flink operator surface calls these entry points; see INTEGRATION.md
 * for the binding stubs. No torch types cross this boundary: plain pointers + sizes.
 *
 * Entry point -> reference interface it replaces:
 *   fwa_create             WindowOperator ctor + open()
 *                            flink-streaming-java/.../runtime/operators/windowing/WindowOperator.java:179-266
 *                          SlicingWindowAggOperatorBuilder.build + AbstractWindowAggProcessor.open
 *                            flink-table-runtime/.../aggregate/window/SlicingWindowAggOperatorBuilder.java:127-171
 *   fwa_push               WindowOperator.processElement (per record, batched here)
 *                            WindowOperator.java:278-434
 *                          SlicingWindowProcessor.processElement  SlicingWindowProcessor.java:53
 *                            (AbstractWindowAggProcessor.java:142-182)
 *   fwa_advance_watermark  AbstractStreamOperator.processWatermark -> InternalTimerServiceImpl.advanceWatermark
 *                            -> WindowOperator.onEventTime      (InternalTimerServiceImpl.java:302-314,
 *                                                                 WindowOperator.java:437-481)
 *                          SlicingWindowOperator.processWatermark/onTimer (SlicingWindowOperator.java:230-264)
 *                            -> fireWindow/clearWindow (SliceSharedWindowAggProcessor.java:64-118,
 *                               SliceUnsharedWindowAggProcessor.java:46-55)
 *   fwa_flush              SlicingWindowProcessor.prepareCheckpoint (RecordsWindowBuffer.flush :107-118)
 *   fwa_drain_partials     LocalSlicingWindowAggOperator -> RecordsWindowBuffer.flush (local half of two-phase)
 *                            LocalSlicingWindowAggOperator.java:111-137
 *   fwa_push_partials      GlobalAggCombiner.combine (global half)  GlobalAggCombiner.java:77-110
 *   fwa_drain_route        fwa_drain_partials + the keyBy send side in one pass (packed rows per owning subtask)
 *   fwa_fire_partials      the owner's GlobalAggCombiner.combine + window fire over the received packed rows
 *   fwa_route_rows         KeyGroupStreamPartitioner.selectChannel + per-channel packing (the keyBy send side)
 *   fwa_key_groups         KeyGroupRangeAssignment.assignToKeyGroup + computeOperatorIndexForKeyGroup
 *                            flink-runtime/.../state/KeyGroupRangeAssignment.java:63-127
 *                          (the keyBy partitioner KeyGroupStreamPartitioner.selectChannel :55-65)
 *   fwa_snapshot           HeapSnapshotStrategy (keyed window state by key group) + the watermark union
 *                            state of SlicingWindowOperator.snapshotState (:204-209)
 *   fwa_restore            HeapRestoreOperation / SlicingWindowOperator.initializeState (:186-202)
 *   fwa_snapshot_heap      HeapSnapshotStrategy key-group sections (HeapSnapshotStrategy.java:154-175) in Flink's bytes
 *   fwa_restore_heap       HeapRestoreOperation over those sections
 *   fwa_destroy            WindowOperator.close / SlicingWindowProcessor.close
 *
 * Status codes mirror the Java exceptions the reference throws.
 * Late records are not errors: they are counted (numLateRecordsDropped,
 * WindowOperator.java:140,431; SlicingWindowOperator.java:108-110).
 */
#ifndef FLINK_AMD_H
#define FLINK_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FWA_ABI_VERSION 5   /* 5: fwa_stats.dec_inexact, fwa_stats_size, FWA_OPT_DEC_WRAP_NULL; 4: fwa_config.dec_scale
                             * (DECIMAL aggregates). Version-3 and -4 configurations are still accepted (same layout);
                             * a caller built against an older header must size its fwa_stats by fwa_stats_size(). */
#define FWA_MAX_AGGS 8
#define FWA_MAX_COLS 8

/* Window kinds. TUMBLE: TumblingEventTimeWindows / TUMBLE TVF. SLIDE: SlidingEventTimeWindows
 * (DataStream, any size/slide) / HOP TVF (Table, size % slide == 0). CUMULATE: CUMULATE TVF
 * (Table only). SESSION: EventTimeSessionWindows / legacy GROUP BY SESSION (merging). */
enum fwa_window_kind { FWA_TUMBLE = 0, FWA_SLIDE = 1, FWA_CUMULATE = 2, FWA_SESSION = 3 };

/* Which operator's observable semantics to reproduce.
 * DATASTREAM: WindowOperator + EventTimeTrigger (allowed lateness supported, late firings).
 * TABLE:      SlicingWindowOperator + Slice{Shared,Unshared}WindowAggProcessor (HOP/CUMULATE
 *             emit only if COUNT(*) > 0, late records routed to unfired windows). */
enum fwa_semantics { FWA_SEM_DATASTREAM = 0, FWA_SEM_TABLE = 1 };

/* How the key-group hash is computed from the int64 key column.
 * JAVA_LONG:      Long.hashCode(key) = (int)(key ^ (key >>> 32))            (DataStream keyBy on a Long)
 * BINROW_BIGINT:  BinaryRowData.hashCode of a 1-field BIGINT key row         (Table GROUP BY a BIGINT)
 *                 = MurmurHashUtils.hashBytesByWords over [0, 0, lo32, hi32], seed 42
 * PREHASHED:      the caller passes key.hashCode() in the low 32 bits of a separate column
 *                 (fwa_push key_hash argument); the int64 key is an opaque dictionary id. */
enum fwa_key_kind { FWA_KEY_JAVA_LONG = 0, FWA_KEY_BINROW_BIGINT = 1, FWA_KEY_PREHASHED = 2,
                    FWA_KEY_GROUP_PREFIXED = 3 /* ids of a key dictionary (fwa_keydict): bits 48-63 = key group */ };

/* Aggregates. Result column type in brackets. */
enum fwa_agg_kind {
    FWA_COUNT = 0,   /* COUNT(*)                                   [i64] */
    FWA_SUM_I64 = 1, /* SUM(BIGINT), two's-complement wrap          [i64] */
    FWA_SUM_F32 = 2, /* SUM(FLOAT)                                  [f32] */
    FWA_SUM_F64 = 3, /* SUM(DOUBLE)                                 [f64] */
    FWA_MIN_I64 = 4, /*                                             [i64] */
    FWA_MAX_I64 = 5, /*                                             [i64] */
    FWA_MIN_F32 = 6, /*                                             [f32] */
    FWA_MAX_F32 = 7, /*                                             [f32] */
    FWA_MIN_F64 = 8, /*                                             [f64] */
    FWA_MAX_F64 = 9, /*                                             [f64] */
    FWA_AVG_I64 = 10,/* AVG(BIGINT): sum/count, truncating division [i64] */
    FWA_AVG_F32 = 11,/* AVG(FLOAT): double sum / count, cast float  [f32] */
    FWA_AVG_F64 = 12,/* AVG(DOUBLE)                                 [f64] */
    FWA_COUNT_COL = 13,/* COUNT(col): non-NULL values of col (Count aggregate over a nullable column;
                          COUNT(*) when col is not nullable)       [i64] */
    FWA_SUM_DEC = 14,  /* SUM(DECIMAL(p, s)), p <= 18: int64 unscaled input (DecimalData's compact form);
                          result DECIMAL(38, s)                      [i128] */
    FWA_AVG_DEC = 15,  /* AVG(DECIMAL(p, s)), p <= 18: result DECIMAL(38, max(6, s))  [i128] */
    FWA_SUM_DEC128 = 16,/* SUM(DECIMAL(p, s)), p <= 38: 16-byte unscaled input        [i128] */
    FWA_AVG_DEC128 = 17,/* AVG(DECIMAL(p, s)), p <= 38                               [i128] */
    /* DataStream built-in reductions (FWA_CFG_REDUCE handles, below) */
    FWA_SUM_I32 = 18,  /* Integer field: Java int addition, 32-bit wrap (SumFunction.IntSum)  [i32] */
    FWA_MIN_I32 = 19,  /* Integer field, ComparableAggregator MIN                          [i32] */
    FWA_MAX_I32 = 20,  /* Integer field, ComparableAggregator MAX                          [i32] */
    FWA_FIRST_64 = 21, /* 8-byte field of the window's first element (arrival order)      [i64 bits] */
    FWA_FIRST_32 = 22, /* 4-byte field of the window's first element                        [i32 bits] */
    FWA_MINBY_I64 = 23,/* minBy over a Long field: that field of the selected element       [i64] */
    FWA_MAXBY_I64 = 24,/* maxBy over a Long field                                           [i64] */
    FWA_MINBY_I32 = 25,/* minBy / maxBy over an Integer field                              [i32] */
    FWA_MAXBY_I32 = 26,
    FWA_MINBY_F64 = 27,/* minBy / maxBy over a Double field (Double.compareTo order)        [f64] */
    FWA_MAXBY_F64 = 28,
    FWA_MINBY_F32 = 29,/* minBy / maxBy over a Float field (Float.compareTo order)          [f32] */
    FWA_MAXBY_F32 = 30,
    FWA_SEL_64 = 31,   /* 8-byte field of the element minBy / maxBy selected                [i64 bits] */
    FWA_SEL_32 = 32,   /* 4-byte field of the element minBy / maxBy selected                [i32 bits] */
    FWA_AGG_KIND_COUNT = 33
};
/* Built-in DataStream reductions (FWA_CFG_REDUCE): WindowedStream.sum / min / max / minBy / maxBy(pos)
 * (WindowedStream.java:680-890) reduce the window's elements in arrival order with SumAggregator
 * (SumAggregator.java:66-76) or ComparableAggregator (ComparableAggregator.java:83-107): the result is a copy of the
 * accumulated value1 with field pos replaced, so every other field comes from the window's FIRST element
 * (FWA_FIRST_*), while minBy / maxBy keep a whole element -- the one with the smallest / largest pos field, ties to
 * the first element, or to the last with FWA_CFG_BY_LAST (minBy(pos, false)) -- whose other fields are FWA_SEL_*.
 * Comparisons are Java compareTo (Long / Integer / Double.compare / Float.compare: -0.0 < 0.0, NaN above +Inf; a MIN
 * or MAX result NaN is returned canonical). SUM over Float is accumulated in double and rounded once (the reference
 * adds in float, in arrival order), over Double in device order (within the tolerance of SUM_F64).
 * A reduce handle is DATASTREAM, TUMBLE or SLIDE, or SESSION over a Tuple2<key, f1> (exactly one aggregate, SUM / MIN /
 * MAX / MINBY / MAXBY of f1: MergingWindowSet merges state namespaces in java.util.HashSet order, which leaves any
 * other field of a merged session, and the by-tie among them, to hash order; the reduced field itself is
 * order-free, float sums aside), with any allowed lateness
 * (late firings emit the reduced element after each late element, in arrival order); every aggregate is a field
 * of the reduced tuple: at most one MINBY / MAXBY, FWA_SEL_* only with it and FWA_FIRST_* only without it, SUM / MIN /
 * MAX over any type; COUNT, AVG, DECIMAL, NULLs, record lists, partials and the heap layout are FWA_E_UNSUPPORTED.
 * fwa_snapshot / fwa_restore work: an entry per (key, slice) holds the slice's reduced fields (acc_j: the field value,
 * a 4-byte field zero-extended) and, in its count column, the arrival rank of the element it selected; a restore
 * (any key-group split) pushes the entries back as elements in that order, so later windows equal an uninterrupted
 * run. A tuple (key, f1, ..., fn) with sum(k) maps to FIRST_* for every fi, i != k, and SUM_* for fk; minBy(k) to
 * SEL_* and MINBY_* (flink_amd/operators.py reduction_aggs). */
/* DECIMAL aggregates (Table semantics; the input column's scale s in fwa_config.dec_scale[j]). Values are unscaled
 * integers in 16-byte little-endian two's complement ([i128]: low 8 bytes, then high 8 bytes).
 *  SUM: DecimalSumAggFunction (SumAggFunction.java:150-168): the exact sum at the result type of
 *       LogicalTypeMerging.findSumAggType (:280-294), DECIMAL(38, s); NULL when it has more than 38 digits
 *       (DecimalDataUtils.add -> DecimalData.fromBigDecimal, DecimalData.java:184-195), or no non-NULL input.
 *  AVG: DecimalAvgAggFunction (AvgAggFunction.java:213-251): that sum over the non-NULL count, divided as
 *       DecimalDataUtils.divide (DecimalDataUtils.java:40,145-148) into findAvgAggType's DECIMAL(38, max(6, s))
 *       (LogicalTypeMerging.java:261-277): the quotient rounded HALF_UP to 38 significant digits, then HALF_UP to the
 *       result scale; NULL past 38 digits or with no non-NULL input.
 * Overflow is decided on the window's exact total. The reference decides it on each running sum in arrival order,
 * and SUM and AVG differ there:
 *  SUM: a running sum that overflowed is NULL and restarts from the next value (ifThenElse(isNull(sum), operand, ..)),
 *       so the reference's result is the sum of the values after the last overflow; the engine's is the exact total,
 *       NULL if that has more than 38 digits.
 *  AVG: DecimalAvgAggFunction has no restart (AvgAggFunction.java:79 aggDecimalPlus): once a running sum passes 38
 *       digits the window's AVG is NULL; the engine's is the exact total over the count, non-NULL when that total
 *       is back within 38 digits (tests/test_decimal_gpu.py::test_documented_overflow_difference pins both).
 * Results differ only for windows in which a running sum passes 38 digits. A (key, window) may hold up to 2^32 - 1
 * records, past which the piece sums may wrap: the watermark step that fires such a window fails with
 * FWA_E_UNSUPPORTED, or, with fwa_set_option(FWA_OPT_DEC_WRAP_NULL, 1), emits that window's DECIMAL results as NULL
 * and counts them in fwa_stats.dec_inexact (the other rows of that watermark are unaffected). Internally each DECIMAL source column is summed as 2 (int64 input)
 * or 4 (16-byte) 32-bit pieces, each one of the handle's FWA_MAX_AGGS aggregates, plus a count; a list past that
 * budget is FWA_E_UNSUPPORTED at fwa_create. Not available for fwa_drain_partials / fwa_push_partials
 * (FWA_E_UNSUPPORTED); fwa_snapshot_heap writes the exact total as the DECIMAL(38, s) buffer, a NULL buffer when it
 * has more than 38 digits, and fwa_restore_heap reads a NULL buffer back as a zero sum with the window's counts kept:
 * after a restore of such a window its SUM restarts from the later values (the reference's SUM behaviour) and so does
 * its AVG, where the reference's AVG would stay NULL (parity across a restore of an overflowed window is unpinned). */
/* SQL NULL semantics (fwa_config.nullable_cols, Table semantics): SUM/MIN/MAX/AVG skip NULL inputs and are
 * NULL when a window holds no non-NULL input (SumAggFunction.java:54-110, MaxAggFunction.java:63-73,
 * MinAggFunction.java:63-, AvgAggFunction.java:65-106: AVG = sum / count of non-NULL inputs); COUNT(*) counts
 * rows, COUNT(col) non-NULL values. SUM(FLOAT) is accumulated in double and rounded to float once at the
 * fire (the reference keeps a float buffer: the results differ by at most that buffer's own rounding,
 * n * 2^-24 * sum|x| for n inputs). */

enum fwa_status {
    FWA_OK = 0,
    FWA_E_ARG = -1,         /* IllegalArgumentException (e.g. abs(offset) >= size, TumblingEventTimeWindows.java:58-62) */
    FWA_E_TS_MIN = -2,      /* Long.MIN_VALUE timestamp (TumblingEventTimeWindows.java:83-86) */
    FWA_E_KEYGROUP = -3,    /* key group outside the owned range (StateTable.java:300-307) */
    FWA_E_MERGE_LATE = -4,  /* merged session window ends before the watermark (WindowOperator.java:308-319) */
    FWA_E_OOM = -5,         /* device memory exhausted */
    FWA_E_DEVICE = -6,      /* HIP runtime error */
    FWA_E_UNSUPPORTED = -7, /* configuration not supported by this engine build */
    FWA_E_STATE = -8,       /* API misuse (e.g. call on a destroyed handle) */
    FWA_E_CORRUPT = -9      /* malformed wire bytes (IOException "Corrupt stream", StreamElementSerializer.java:208-210) */
};

/* Flags for fwa_push */
#define FWA_PUSH_DEVICE_PTRS 0x1 /* key/ts/value pointers are device (HBM) pointers */
#define FWA_PUSH_ASYNC 0x2       /* enqueue and return without a host synchronisation: the batch is
                                  * settled (status read, miss replay, lookahead) at the start of the
                                  * next call on the handle, which also reports its errors. Device
                                  * input buffers must stay valid until that next call returns;
                                  * late_dropped_out is not written (see fwa_stats.late_dropped). */

typedef struct fwa_agg_spec {
    int32_t kind; /* enum fwa_agg_kind */
    int32_t col;  /* index into the value-column array of fwa_push (ignored for COUNT) */
} fwa_agg_spec;

typedef struct fwa_config {
    int32_t abi_version;         /* must be FWA_ABI_VERSION */
    int32_t window_kind;         /* enum fwa_window_kind */
    int32_t semantics;           /* enum fwa_semantics */
    int32_t key_kind;            /* enum fwa_key_kind */
    int64_t size_ms;             /* TUMBLE size; SLIDE size; CUMULATE max size */
    int64_t slide_ms;            /* SLIDE slide; CUMULATE step; unused otherwise */
    int64_t offset_ms;           /* window offset (assigner 'offset'); 0 = epoch aligned */
    int64_t gap_ms;              /* SESSION gap */
    int64_t allowed_lateness_ms; /* DATASTREAM only (WindowOperator allowedLateness) */
    int32_t max_parallelism;     /* number of key groups (pipeline.max-parallelism), default 128 */
    int32_t kg_start;            /* owned key-group range [kg_start, kg_end] (inclusive) */
    int32_t kg_end;
    int32_t num_aggs;
    fwa_agg_spec aggs[FWA_MAX_AGGS];
    int32_t device;              /* HIP device ordinal */
    int32_t output_on_device;    /* 1: fwa_out points into HBM; 0: engine copies rows to host */
    int64_t key_capacity;        /* sizing hint: max distinct live keys (0 = default 1<<20) */
    int64_t max_batch;           /* sizing hint: max records per fwa_push (0 = default 1<<26) */
    /* ABI 2 */
    int32_t flags;               /* FWA_CFG_* */
    int32_t gap_col;             /* FWA_CFG_DYNAMIC_GAP: value column holding each record's session gap (int64 ms) */
    int32_t tz_n;                /* shift time zone of a Table TIMESTAMP_LTZ rowtime: number of (instant, offset)
                                    pairs in tz; 0 = UTC (TimeWindowUtil.toUtcTimestampMills :52-60) */
    int32_t nullable_cols;       /* Table: bit c set = value column c may hold SQL NULLs (fwa_push_nullable) */
    const int64_t* tz;           /* [2 * tz_n]: from UTC instant tz[2i] (ms, ascending) on, the zone's offset is
                                    tz[2i+1] ms (java.time ZoneRules transitions); copied by fwa_create */
    /* ABI 4 */
    int32_t dec_scale[FWA_MAX_AGGS];   /* DECIMAL aggregate j: the scale s of its input column (0..38) */
} fwa_config;

/* fwa_config.flags */
#define FWA_CFG_DYNAMIC_GAP 0x1  /* SESSION: per-record gap from value column gap_col -- DynamicEventTimeSessionWindows
                                  * with a SessionWindowTimeGapExtractor (DynamicEventTimeSessionWindows.java:57-68);
                                  * a gap <= 0 raises FWA_E_ARG like the assigner's IllegalArgumentException */
#define FWA_CFG_LATE_INDICES 0x2 /* collect, per push, the indices of the records dropped as late (fwa_late_records):
                                  * WindowOperator's lateDataOutputTag side output (WindowOperator.java:425-433) and the
                                  * per-record processElement() == true of SlicingWindowProcessor
                                  * (SlicingWindowOperator.java:222-226, lateRecordsDroppedRate) */
#define FWA_CFG_REDUCE 0x8       /* DataStream built-in reduction (WindowedStream.sum/min/max/minBy/maxBy): Java
                                  * compareTo order for MIN / MAX, FWA_FIRST_* / FWA_SEL_* / FWA_MINBY_* kinds (above) */
#define FWA_CFG_BY_LAST 0x10     /* minBy / maxBy(pos, first = false): ties select the LAST element */
#define FWA_CFG_RECORD_LISTS 0x4 /* TUMBLE, lateness 0, no NULLs, UTC: keep each window's state as its accepted records
                                  * (key + accumulator words) bucketed by hash partition, aggregated once when the window
                                  * fires -- for key spaces where keys barely repeat within a window (C4: 1e8 keys).
                                  * Selected automatically when key_capacity >= 2^25; fwa_get_config reports it.
                                  * Same results, snapshots and partials as the dense layout. Other configurations:
                                  * FWA_E_UNSUPPORTED. */

typedef struct fwa_out {
    int64_t n_rows;
    int32_t on_device;           /* pointers below are device pointers if 1 */
    int32_t num_aggs;
    const int64_t* key;
    const int64_t* win_start;
    const int64_t* win_end;      /* DataStream record timestamp = win_end - 1 (TimeWindow.maxTimestamp) */
    const void* agg[FWA_MAX_AGGS];
    const uint8_t* agg_null[FWA_MAX_AGGS]; /* per aggregate: 1 = the result is SQL NULL; NULL pointer when the
                                              aggregate can never be NULL (no nullable input) */
} fwa_out;

typedef struct fwa_stats {
    int64_t records_in;
    int64_t late_dropped;        /* numLateRecordsDropped */
    int64_t rows_out;
    int64_t live_keys;
    int64_t live_slices;
    int64_t current_watermark;
    /* device time of the engine's kernels, measured with HIP events on the handle's stream */
    int64_t ingest_launches;
    double ingest_ms;            /* sum over ingest-kernel launches */
    int64_t ingest_records;      /* distinct records pushed through those launches (replays excluded) */
    int64_t fire_launches;
    double fire_ms;
    int64_t fire_rows;
    double partition_ms;         /* two-phase ingest split: phase P (key lookup + partition) */
    double combine_ms;           /* phase A (LDS combine + HBM merge) */
    int64_t replay_records;      /* records re-visited by slice-miss / bucket-overflow replays (not in ingest_records) */
    int64_t dec_inexact;         /* DECIMAL results emitted NULL because their window held 2^32 or more records (the
                                    32-bit piece sums may have wrapped; below that they are exact) */
} fwa_stats;


typedef struct fwa_engine fwa_engine;

/* Engine lifecycle. Handles are single-threaded (one Flink subtask / mailbox thread each);
 * distinct handles may be used concurrently (one HIP stream per handle). */
int fwa_create(const fwa_config* cfg, fwa_engine** out);
void fwa_destroy(fwa_engine* e);
const char* fwa_last_error(const fwa_engine* e);
const char* fwa_version(void);

/* Columnar batch of n records: keys[n], ts[n], val_cols[c][n] (type implied by the aggs reading c).
 * key_hash may be NULL unless key_kind == FWA_KEY_PREHASHED (then int32 key.hashCode() per record).
 * Input buffers are borrowed for the duration of the call only (FWA_PUSH_ASYNC: until the next call). */
int fwa_push(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
             const int32_t* key_hash, int64_t n, int32_t flags, int64_t* late_dropped_out);

/* fwa_push with SQL NULLs: null_cols[c] (NULL = no NULLs in column c) holds n bytes, nonzero = the value of
 * value column c is NULL in that record (Flink's columnar isNullAt / heap-vector isNull[]). Columns that
 * carry NULLs must be declared in fwa_config.nullable_cols; only the entries of declared columns are read
 * (the array needs at least 1 + the highest declared column entries). Replaces the null handling of the generated
 * accumulate code (AggsHandleFunction, e.g. SumAggFunction.accumulateExpressions). */
int fwa_push_nullable(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
                      const uint8_t* const* null_cols, const int32_t* key_hash, int64_t n, int32_t flags,
                      int64_t* late_dropped_out);

/* Stream ordering of device inputs (FWA_PUSH_DEVICE_PTRS): the caller's HIP stream that produces the
 * input columns (e.g. the framework's current stream). Every later device-pointer push makes the engine's
 * own stream wait for the work enqueued on `stream` so far before reading the columns. NULL (default):
 * the caller guarantees the inputs are complete (e.g. it synchronised). Outputs are complete when the
 * entry point that returns them returns. fwa_drain_partials and fwa_drain_route wait for the stream too before
 * they rewrite the device buffers their previous call returned, so a consumer that reads those buffers on
 * `stream` (the keyBy exchange's all-to-all) is never overtaken by the next drain. */
int fwa_set_input_stream(fwa_engine* e, void* stream);

/* Advance the event-time watermark; fires every window whose maxTimestamp (end-1) <= wm.
 * Non-advancing watermarks fire nothing (SlicingWindowOperator.java:231, StatusWatermarkValve).
 * DataStream late firings (allowed lateness > 0: a record for a fired window that is not past cleanup,
 * EventTimeTrigger.onElement :37-45) are computed during fwa_push, one row per (element, fired window)
 * in arrival order, and returned at the head of the next fwa_advance_watermark's rows (also when wm
 * does not advance).
 * Output rows (fired (key, window) results) stay valid until the next call on this handle. */
int fwa_advance_watermark(fwa_engine* e, int64_t wm, fwa_out* out);

/* fwa_advance_watermark split in two so the caller can hand the next batch to the engine while the fire runs (the
 * mailbox thread emitting the fired rows downstream while the next network buffer is processed, StreamTask
 * processInput -> WindowOperator.processWatermark -> output.collect). fwa_advance_watermark_async takes the same
 * watermark step and returns without waiting for the fire when it can (a TUMBLE handle after an FWA_PUSH_ASYNC push:
 * the fire is enqueued and the host waits only for the push's status); the rows are taken with fwa_fired_output,
 * which waits for them. Between the two, fwa_push / fwa_push_partials may be called (their ingest runs behind the
 * fire); any other call completes the fire first. The output stays valid until the next watermark call. Results are
 * those of fwa_advance_watermark at the same point. */
int fwa_advance_watermark_async(fwa_engine* e, int64_t wm);
int fwa_fired_output(fwa_engine* e, fwa_out* out);

/* Make every pushed record visible in state (checkpoint barrier, SlicingWindowOperator.java:267-269). */
int fwa_flush(fwa_engine* e);

int fwa_get_stats(fwa_engine* e, fwa_stats* out);
/* sizeof(fwa_stats) of this library (it grew in ABI 5): a caller checks it against its own before fwa_get_stats. */
int64_t fwa_stats_size(void);

/* ---- two-phase (local / global) aggregation ----
 * Flink's two-phase window plan (TwoStageOptimizedWindowAggregateRule.java:88-103):
 *   LocalSlicingWindowAggOperator (LocalSlicingWindowAggOperator.java:111-131) pre-aggregates each
 *   source subtask's records per (key, slice) and emits partial accumulators, which are shuffled by key
 *   group to GlobalAggCombiner (GlobalAggCombiner.java:77-110), which merges them into the window state.
 * Used by the multi-GPU keyBy exchange to ship per-(key, slice) partials instead of raw records.
 * Not available for SESSION windows (FWA_E_UNSUPPORTED). */
typedef struct fwa_partials {
    int64_t n;
    int32_t on_device;           /* pointers below are device pointers if 1 */
    int32_t num_aggs;
    const int64_t* key;
    const int64_t* slice_start;  /* start timestamp of the (key, slice) accumulator */
    const int64_t* count;        /* COUNT(*) of the records it holds */
    const void* acc[FWA_MAX_AGGS]; /* 8-byte accumulator of agg j: i64 sum, f64 sum bits, or the engine's
                                      order-preserving MIN/MAX key (the accumulator's identity when the
                                      aggregate saw no non-NULL input); COUNT aggregates repeat count */
    int32_t num_hidden;          /* handles with nullable_cols: hidden non-NULL counters (one per nullable
                                    input column an aggregate reads, in first-use order), else 0 */
    int32_t pad;
    const int64_t* hidden[FWA_MAX_COLS]; /* the non-NULL input count of each hidden counter (AvgAggFunction's
                                            count, the null flag of Sum/Min/MaxAggFunction's buffer) */
} fwa_partials;

/* Local pre-aggregator watermark step (LocalSlicingWindowAggOperator: flush the buffer, forward the
 * watermark). Exports, instead of firing, the (key, slice) accumulators of every slice that received
 * records and is complete at wm (slice end - 1 <= wm; every such slice when wm == INT64_MAX), resets
 * them, then advances this handle's watermark to wm (records for fired windows are late from then on;
 * slices past cleanup are released). A handle drained this way never emits window rows itself: the
 * owner merges the partials with fwa_push_partials before advancing its own watermark to wm. */
int fwa_drain_partials(fwa_engine* e, int64_t wm, fwa_partials* out);

/* fwa_drain_route's export: the drained (key, slice) partials as packed rows grouped by owning subtask. */
#define FWA_MAX_DEST 64
typedef struct fwa_routed {
    int64_t n;                        /* rows drained, all destinations */
    int32_t parallelism, cells;       /* destinations; 8-byte cells per row */
    int32_t on_device, pad;           /* 1: rows are device pointers (always) */
    const int64_t* rows[FWA_MAX_DEST];/* destination d's rows, [count[d]][cells], engine-owned, valid until the next
                                         call on the handle */
    int64_t count[FWA_MAX_DEST];
} fwa_routed;

/* fwa_drain_partials and the keyBy send side (fwa_route_rows) in one pass: the same (key, slice) partials, each
 * written as a packed row -- cell 0 key, 1 slice start, 2 COUNT(*), then one cell per user aggregate other than
 * COUNT(*) (its accumulator, or COUNT(*) for an aggregate that keeps none), then one per hidden non-NULL counter --
 * into the region of the subtask owning its key group (computeOperatorIndexForKeyGroup(max_parallelism,
 * parallelism, assignToKeyGroup(key)), KeyGroupStreamPartitioner.selectChannel). The per-destination counts are host
 * values: the exchange's split sizes need no device read. Dense slicing-window handles with output_on_device
 * (FWA_E_UNSUPPORTED otherwise: use fwa_drain_partials + fwa_route_rows). The rows feed fwa_fire_partials on the
 * owner with acc_cell[j] = the cell of aggregate j as laid out here. */
int fwa_drain_route(fwa_engine* e, int64_t wm, int32_t parallelism, fwa_routed* out);

/* Merge partial accumulators (as produced by fwa_drain_partials on another handle with the same
 * window and aggregate configuration) into this handle's state. slice_ts may be any timestamp inside
 * the slice. Late partials are dropped like records (their counts are added to late_dropped_out).
 * acc holds one column per aggregate; a handle with nullable_cols reads fwa_partials.num_hidden more
 * entries after them, acc[num_aggs + h] = hidden[h] (GlobalAggCombiner merges the nullable buffers,
 * GlobalAggCombiner.java:77-110). */
int fwa_push_partials(fwa_engine* e, const int64_t* keys, const int64_t* slice_ts, const int64_t* count,
                      const void* const* acc, int64_t n, int32_t flags, int64_t* late_dropped_out);

/* The owner's watermark step of the two-phase plan over the exchange's receive buffer: the same result as
 * fwa_push_partials of the rows' cells followed by fwa_advance_watermark(wm, out) (GlobalAggCombiner.combine
 * then WindowOperator.onEventTime). rows: n packed rows of m 8-byte cells -- cell 0 the key, 1 a timestamp inside
 * the slice, 2 COUNT(*), and acc_cell[j] the cell of aggregate j's accumulator for every aggregate and hidden
 * counter that keeps one (fwa_drain_partials' acc / hidden; ignored for the others). With FWA_PUSH_DEVICE_PTRS
 * (rows in HBM, ordered after fwa_set_input_stream's stream) on a TUMBLE handle without allowed lateness that holds
 * no window data, the rows are grouped per (key, window) on chip and fired directly (no slot state in between;
 * FWA_OPT_FIRE_PARTIALS counts those calls); otherwise, and for a row whose window would not fire at wm, the call
 * runs as the two calls above. The replacement of fwa_push_partials + fwa_advance_watermark in the owner's loop
 * (RecordsWindowBuffer.flush -> GlobalAggCombiner -> fire, SlicingWindowOperator.processWatermark). */
int fwa_fire_partials(fwa_engine* e, const int64_t* rows, int64_t n, int32_t m, const int32_t* acc_cell, int64_t wm,
                      int32_t flags, fwa_out* out, int64_t* late_dropped_out);

/* ---- checkpoint / restore ----
 * fwa_snapshot replaces the keyed-state half of the operator snapshot: HeapSnapshotStrategy writes the
 * window state per key group with a KeyGroupRangeOffsets index (HeapSnapshotStrategy.java:154-179,
 * CopyOnWriteStateMapSnapshot.java:142-147) and SlicingWindowOperator.snapshotState stores the current
 * watermark in union list state (SlicingWindowOperator.java:204-209). The blob holds, in one buffer
 * (little-endian int64 words): a header (magic "FWASNAP1", window/aggregate configuration,
 * watermark, entry count), a key-group offset table off[max_parallelism + 1] (entries of key group g
 * are [off[g], off[g+1])), then SoA columns key[n], slice_start[n], count[n], acc_j[n] (one per
 * aggregate, same encoding as fwa_partials), then for a handle with nullable_cols one hidden[h][n]
 * column per hidden non-NULL counter (header word 25 = their number, word 24 = nullable_cols). Per-key timers are not stored: the engine's timers are
 * derived from the live slices and the watermark, as the reference re-registers them from state.
 * SESSION windows: the entries are the in-flight sessions (the MergingWindowSet mapping + window state,
 * WindowOperator.java:224-238) with slice_start = session start and one more column end[n] after the
 * acc_j columns. FWA_KEY_PREHASHED handles (keys of any Java type as 64-bit ids beside their key.hashCode()): one
 * more last column hash[n], the hashCode() each key was pushed with (the engine keeps it per key), by which the
 * entries are placed in key groups and a restore places them again; record-list handles keep no per-key hash and
 * refuse (FWA_E_UNSUPPORTED). The blob is engine-allocated; free it with fwa_blob_free. */
typedef struct fwa_blob {
    void* data;
    int64_t size;   /* bytes */
} fwa_blob;

int fwa_snapshot(fwa_engine* e, fwa_blob* out);
void fwa_blob_free(fwa_blob* b);

/* Restore a fresh handle (nothing pushed yet) from one or more snapshots of handles with the same
 * window and aggregate configuration: only the key groups of this handle's [kg_start, kg_end] are
 * read (rescaling, StateAssignmentOperation / KeyGroupRangeOffsets), and the watermark becomes the
 * MIN of the snapshots' watermarks (SlicingWindowOperator.initializeState :186-202). Windows that
 * fired before the snapshot do not fire again. */
int fwa_restore(fwa_engine* e, const void* const* blobs, const int64_t* sizes, int32_t n_blobs);

/* The same keyed state in the byte layout of Flink's heap keyed-state backend (HeapSnapshotStrategy.java:154-175):
 * for each owned key group g = kg_start..kg_end, in order: int g, then one section per state the reference operator
 * registers -- short state id, int n, n entries -- with the ids a heap backend gives them (HeapSnapshotResources
 * .java:100-139: key/value states, then the timer queues, each in java.util.HashMap order of the names; pinned by the
 * reference's own snapshots, tests/test_heap_reference_cpu.py):
 *   DATASTREAM TUMBLE  (WindowOperator): 0 "window-contents", 1 "_timer_state/processing_window-timers" (empty),
 *                      2 "_timer_state/event_window-timers"
 *   DATASTREAM SESSION (WindowOperator): 0 "window-contents", 1 "merging-window-set", 2 processing timers (empty),
 *                      3 event timers
 *   TABLE TUMBLE / HOP / CUMULATE (SlicingWindowOperator): 0 "window-aggs", 1 processing timers (empty), 2 event timers
 * Key/value entries are (namespace, key, value) (CopyOnWriteStateMapSnapshot.writeState :138-148), timer entries
 * (long flipSignBit(ts), key, namespace) (TimerSerializer.serialize :147-152); big-endian java.io.DataOutput.
 *   DataStream: namespace TimeWindow (long start, long end), key Long, value a Tuple of Long COUNT(*) then one field
 *     per aggregate (Long for COUNT / BIGINT SUM / AVG / MIN / MAX, Double for floating SUM / AVG / MIN / MAX). Timers:
 *     window.maxTimestamp() while the window has not fired (EventTimeTrigger) and the cleanup time maxTimestamp +
 *     allowedLateness (WindowOperator.registerCleanupTimer :608-620). Sessions: the merging-window-set holds, per
 *     key under VoidNamespace (one byte), the List of (actual, state) TimeWindow pairs; each in-flight session is
 *     written as its own state window.
 *   Table: namespace Long slice end (local time under a shift time zone), key BinaryRowData(BIGINT), value a
 *     BinaryRowData of COUNT(*), one field per aggregate (NULL bit set when the aggregate saw only NULLs) and one
 *     BIGINT per hidden non-NULL counter of a nullable handle; a DECIMAL SUM / AVG field is the DECIMAL(38, s)
 *     running sum as a non-compact DecimalData (AbstractBinaryWriter.writeDecimal: 16 bytes in the variable-length
 *     part, BigInteger.toByteArray), NULL past 38 digits; a CUMULATE window's fired slices are folded into its
 *     first slice (the shared state SliceSharedWindowAggProcessor keeps); one timer per (key, first unfired window
 *     end of each live slice) at toEpochMillsForTimer(window end - 1) (UTC: window end - 1).
 *   DATASTREAM SLIDE (WindowOperator per-window state, merged from the engine's slices) and TABLE SESSION (the legacy
 *     Table WindowOperator: 0 "session-window-mapping", 1 "window-aggs", 2 / 3 timers) are written as
 *     flink_amd/csrc/heap_snapshot.cpp describes.
 * kg_offsets[g - kg_start] receives the byte offset of key group g's section (KeyGroupRangeOffsets; the Java shim
 * writes its KeyedBackendSerializationProxy header in front and shifts them), *watermark the operator watermark
 * (union list state, SlicingWindowOperator.java:204-209). PREHASHED keys (their Java serialization is the caller's)
 * and DataStream reductions (FWA_CFG_REDUCE): FWA_E_UNSUPPORTED -- fwa_snapshot / fwa_restore carry both, PREHASHED
 * keys with their hashes (dense and session handles). The blob is freed with fwa_blob_free. */
int fwa_snapshot_heap(fwa_engine* e, fwa_blob* out, int64_t* kg_offsets, int64_t* watermark);

/* Restore a fresh handle from heap-layout bodies (as written by fwa_snapshot_heap on handles with the same window
 * and aggregate configuration, any key-group ranges): the key groups of [kg_start, kg_end] are read, timers are
 * re-derived from the window state, session contents are re-keyed from their state window to the actual window
 * the merging-window-set maps to it, the watermark is the MIN of watermarks[] (HeapRestoreOperation /
 * SlicingWindowOperator.initializeState :186-202). */
int fwa_restore_heap(fwa_engine* e, const void* const* bodies, const int64_t* sizes, const int64_t* watermarks,
                     int32_t n_bodies);

/* FWA_CFG_LATE_INDICES: indices (ascending, into the last push's batch) of the records that push dropped as
 * late -- the records WindowOperator would send to its lateDataOutputTag side output, and those for which
 * SlicingWindowProcessor.processElement returns true. Valid until the next call on the handle; for an
 * FWA_PUSH_ASYNC push, available once it is settled (this call settles it). Replaces
 * WindowOperator.sideOutput (WindowOperator.java:425-433, :559-567). */
int fwa_late_records(fwa_engine* e, const int32_t** idx, int64_t* n);

/* Reset the kernel timing counters of fwa_stats (bench warm-up). */
int fwa_reset_timers(fwa_engine* e);

/* Per-handle tuning / test options (no reference counterpart: the engine's own adaptive choices, which the defaults
 * make). The library reads no environment variables; a TaskManager sets these per operator instance if at all.
 * value -1 = adaptive (default), 0 = never, 1 = always for the tri-state options. FWA_E_ARG for an unknown option,
 * FWA_E_UNSUPPORTED for an option that does not apply to the handle's state layout, FWA_E_STATE when the option can
 * no longer change (FWA_OPT_SP_TABLE after the first push). */
enum fwa_option {
    FWA_OPT_SKEW_MERGE = 1,      /* Phase P tile pre-aggregation of equal (key, slice) records (skewed keys) */
    FWA_OPT_WINDOW_PASSES = 2,   /* combiner window passes (chunks spanning more slices than the LDS window) */
    FWA_OPT_NARROW_ENTRIES = 3,  /* 10-byte bucket entries for COUNT + SUM(BIGINT) while keys / values fit 32 bits */
    FWA_OPT_SESSION_CELLS = 4,   /* sessions: the cell path for order-free pushes with a fixed gap (0 / -1) */
    FWA_OPT_OUT_MIN_ROWS = 5,    /* first sizing of the fire's output columns in rows (0: 4M); tests force regrowth */
    FWA_OPT_PARTIALS_ONE_PASS = 6, /* 1: fwa_push_partials merges through the one-pass atomic ingest */
    FWA_OPT_SP_TABLE = 7,        /* record lists: LDS aggregation table slots (power of two >= 64, before any push) */
    FWA_OPT_SP_FMAX = 8,         /* record lists: max fine buckets per (window, partition) at fire */
    FWA_OPT_SP_BUDGET = 9,       /* record lists: live list bytes above which windows are compacted */
    FWA_OPT_PROFILE = 10,        /* 1: per-phase clock profile of Phase P / A, printed to stderr (diagnostic) */
    FWA_OPT_SESSION_PATH = 11,   /* read only: the path of the last session push -- 0 general, 1 sort-based cells,
                                    2 cell pre-aggregation (fwa_get_option) */
    FWA_OPT_INGEST_VARIANT = 12, /* diagnostic A/B switches of the ingest kernels (0 default); bit 0: the combiner
                                    reads a slot it merges into even when no record reached it yet */
    FWA_OPT_SLIDE_CARRIED = 13,  /* read only: sliding fires whose first window reused the previous run's carried
                                    window sums (fwa_get_option; set: 0 disables the reuse, 1 enables it, default) */
    FWA_OPT_FIRE_PARTIALS = 14,  /* read only: fwa_fire_partials calls that merged and fired on chip (fwa_get_option;
                                    set: 0 sends every call through fwa_push_partials + fwa_advance_watermark) */
    FWA_OPT_DEC_WRAP_NULL = 15   /* 1: a DECIMAL SUM / AVG over 2^32 or more records of one window is emitted NULL and
                                  * counted (fwa_stats.dec_inexact); 0 (default): that watermark step fails
                                  * (FWA_E_UNSUPPORTED) instead of a silently different result */
};
int fwa_set_option(fwa_engine* e, int32_t option, int64_t value);
/* The option's effective value: for the tri-state options 1 if the handle currently takes that path (forced, or
 * switched on by the adaptive rule after a push), else 0; the sizes as set (or the default in use). */
int fwa_get_option(const fwa_engine* e, int32_t option, int64_t* value);

/* Stateless key-group assignment of n keys (device or host pointers per flags):
 * kg_out[i] = murmurHash(hash(key_i)) % max_parallelism; op_out[i] = kg*parallelism/max_parallelism
 * (FWA_KEY_GROUP_PREFIXED: kg = the id's top 16 bits; both -1 for an id whose key group is >= max_parallelism).
 * op_out may be NULL. */
int fwa_key_groups(const int64_t* keys, const int32_t* key_hash, int64_t n, int32_t key_kind,
                   int32_t max_parallelism, int32_t parallelism, int32_t* kg_out, int32_t* op_out,
                   int32_t flags, int32_t device);

/* keyBy send side of a columnar batch (KeyGroupStreamPartitioner.selectChannel :55-65 + the RecordWriter's
 * per-channel serialisation, RecordWriter.java:104-157), on the device: dest(i) = computeOperatorIndexForKeyGroup(
 * max_parallelism, parallelism, assignToKeyGroup(key_i)); the ncols columns (cols[c]: col_bytes[c] = 4 or 8 bytes
 * per row, 4-byte columns zero-extended) are packed into out[n][ncols] int64 rows grouped by destination, in arrival
 * order within a destination, and counts[d] receives the rows for destination d (parallelism <= 64, ncols <= 16).
 * All pointers are device pointers; work is enqueued on `stream` (NULL: the default stream) without a host
 * synchronisation: outputs are complete once that stream's work is (a consumer on another stream waits on it). */
int fwa_route_rows(const int64_t* keys, const int32_t* key_hash, int64_t n, int32_t key_kind, int32_t max_parallelism,
                   int32_t parallelism, const void* const* cols, const int32_t* col_bytes, int32_t ncols, int64_t* out,
                   int64_t* counts, int32_t device, void* stream);

/* The receive side of that exchange: rows[n][ncols] (int64 cells) -> cols[c][n], device pointers, enqueued on `stream`
 * (no host synchronisation). */
int fwa_unpack_rows(const int64_t* rows, int64_t n, int32_t ncols, int64_t* const* cols, int32_t device, void* stream);

/* ---- key dictionary: multi-column Table keys ----
 * A Table job keyed by several columns has BinaryRowData keys of `arity` fields whose hashCode()
 * (BinaryRowData.java:452-454 -> MurmurHashUtils.hashBytesByWords :92-170) places them in key groups
 * (KeyGroupRangeAssignment.assignToKeyGroup :63-77). The dictionary computes that hash on the GPU and maps each
 * distinct key row to a 64-bit id whose bits 48-63 are the row's key group and bits 0-47 a dense sequence number;
 * an engine created with key_kind FWA_KEY_GROUP_PREFIXED runs on those ids -- key-group ownership, partials,
 * FWASNAP1 snapshots and rescaling work unchanged (the key group is read from the id) -- and fired rows are mapped
 * back to the key columns with fwa_keydict_decode. Rows are equal iff their bytes are (BinaryRowData.equals), so
 * -0.0 and 0.0 are different DOUBLE keys, as in the reference. Identity is a 64-bit hash of the row's bytes checked
 * against the stored row: two rows with the same 64-bit hash (never observed) fail the encode with FWA_E_STATE
 * instead of merging. One dictionary serves one engine handle (ids are local to it). */
enum fwa_key_field_type { FWA_KEY_FIELD_BIGINT = 0, FWA_KEY_FIELD_INT = 1, FWA_KEY_FIELD_DOUBLE = 2,
                          FWA_KEY_FIELD_STRING = 3 };
#define FWA_KEYDICT_MAX_ARITY 8
/* A STRING / VARCHAR key field (FWA_KEY_FIELD_STRING): the UTF-8 bytes of row i are bytes[offsets[i] .. offsets[i+1])
 * (Arrow layout, device pointers; at most 2^23 - 1 bytes per value). The key row is laid out as BinaryRowWriter
 * writes it (AbstractBinaryWriter.writeString / writeBytesToFixLenPart / writeBytesToVarLenPart :80-105,279-334): up to
 * 7 bytes inline in the field's slot (first byte 0x80 | length, the bytes in the low 7), longer ones appended to the
 * row's variable-length part rounded up to 8 bytes (zero padding) with slot = offset << 32 | length; hashCode()
 * covers the whole row (BinarySegmentUtils.hashByWords :374-380). For such a field, cols[c] of fwa_keydict_encode /
 * fwa_binrow_hash points to a (host) fwa_key_strings; fwa_keydict_decode writes through a (host) fwa_key_strings_out:
 * offsets[0..n] always, and the bytes when `bytes` is non-NULL and `capacity` holds them (else FWA_E_ARG); `needed`
 * receives the byte count either way (call once with bytes = NULL to size the buffer). */
typedef struct fwa_key_strings { const int32_t* offsets; const uint8_t* bytes; } fwa_key_strings;
typedef struct fwa_key_strings_out { int32_t* offsets; uint8_t* bytes; int64_t capacity; int64_t needed; } fwa_key_strings_out;
typedef struct fwa_keydict fwa_keydict;
/* capacity: the most distinct key rows the dictionary will hold (FWA_E_OOM past it) */
int fwa_keydict_create(int32_t arity, const int32_t* field_types, int32_t max_parallelism, int64_t capacity,
                       int32_t device, fwa_keydict** out);
void fwa_keydict_destroy(fwa_keydict* d);
const char* fwa_keydict_last_error(const fwa_keydict* d);
int64_t fwa_keydict_size(const fwa_keydict* d);            /* distinct rows so far */
/* Device pointers: cols[c][i] is field c of row i (int64 BIGINT, int32 INT, double DOUBLE); nulls[c] (or nulls
 * itself) may be NULL = no NULLs in field c. Writes ids[i] and, if hashes != NULL, hashes[i] = the row's hashCode(). */
int fwa_keydict_encode(fwa_keydict* d, const void* const* cols, const uint8_t* const* nulls, int64_t n, int64_t* ids,
                       int32_t* hashes);
/* Device pointers: the key columns (and NULL flags, if nulls != NULL) of n ids from this dictionary. */
int fwa_keydict_decode(fwa_keydict* d, const int64_t* ids, int64_t n, void* const* cols, uint8_t* const* nulls);
/* fwa_snapshot_heap / fwa_restore_heap for an engine on dictionary ids (Table semantics): key rows are written and
 * read as the dictionary's BinaryRowData rows of `arity` fields (restored rows are encoded into `dict`). */
int fwa_snapshot_heap_keys(fwa_engine* e, fwa_keydict* dict, fwa_blob* out, int64_t* kg_offsets, int64_t* watermark);
int fwa_restore_heap_keys(fwa_engine* e, fwa_keydict* dict, const void* const* bodies, const int64_t* sizes,
                          const int64_t* watermarks, int32_t n_bodies);
/* BinaryRowData.hashCode() of n rows of fixed-length fields, device pointers (no dictionary). */
int fwa_binrow_hash(int32_t arity, const int32_t* field_types, const void* const* cols, const uint8_t* const* nulls,
                    int64_t n, int32_t* out, int32_t device);

/* ---- bench / test support (synthetic streams of SURVEY.md §8(d), generated in HBM) ---- */
typedef struct fwa_gen_params {
    uint64_t seed_k, seed_t, seed_v;
    int64_t first_index;   /* global record index of element 0 (multi-GPU: rank's slice) */
    int64_t total_records; /* N of the whole stream (drives the ts ramp) */
    int64_t num_keys;      /* K */
    int64_t t0_ms;         /* T0 */
    int64_t span_ms;       /* event-time span of the whole stream */
    int64_t max_delay_ms;  /* D (bounded out-of-orderness) */
    int32_t key_dist;      /* 0 uniform, 1 zipf (needs cdf) */
    int32_t val_kind;      /* 0: i64 non-negative 31-bit; 1: f32+f64 in [0,1) */
    const double* zipf_cdf;/* device pointer, num_keys entries (key_dist==1) */
} fwa_gen_params;

int fwa_generate(const fwa_gen_params* p, int64_t n, int64_t* keys, int64_t* ts, int64_t* v_i64,
                 float* v_f32, double* v_f64, int32_t device, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FLINK_AMD_H */
