/*
 * flink_amd_wire.h -- on-GPU decoding of Flink's network wire format.
 *
 * Upstream of the window operator, Flink's StreamTask input deserialises every StreamElement of a channel
 * from its network buffers on the task thread, one virtual call chain per record:
 *   SpillingAdaptiveSpanningRecordDeserializer.getNextRecord  (.../io/network/api/serialization/
 *     SpillingAdaptiveSpanningRecordDeserializer.java:88-131: a 4-byte big-endian length, then the
 *     element; an element may span buffers, SpanningWrapper)
 *   -> StreamElementSerializer.deserialize  (flink-streaming-java/.../streamrecord/StreamElementSerializer.java:
 *     tag byte :48-53, then TAG_REC_WITH_TIMESTAMP: long ts + value, TAG_REC_WITHOUT_TIMESTAMP: value,
 *     TAG_WATERMARK: long, TAG_STREAM_STATUS: int, TAG_LATENCY_MARKER: long, long, long, int,
 *     TAG_RECORD_ATTRIBUTES: boolean -- :190-211; written by serialize :158-187 behind
 *     RecordWriter.serializeRecord's length prefix, RecordWriter.java:145-157)
 *   -> the value serializer: TupleSerializer of Long/Double/Float/Integer fields (java.io.DataOutput
 *     big-endian), or RowDataSerializer -> BinaryRowDataSerializer.serialize (BinaryRowDataSerializer.java:
 *     85-93: int size, then the BinaryRowData bytes: null bit set with the RowKind in byte 0, 8-byte
 *     little-endian fixed-length slots, BinaryRowData.java:68-75,114-116)
 *   -> AbstractStreamTaskNetworkInput.processElement (:154-181) dispatches records to the operator and
 *     watermarks / status / latency markers / record attributes to their handlers.
 *
 * fwa_wire_decode replaces that loop for the records of one input channel: the channel's data-buffer
 * payloads, concatenated in arrival order, are parsed on the GPU into the SoA columns fwa_push takes
 * (FWA_PUSH_DEVICE_PTRS, zero copy), and the non-record elements come back as an ordered event list
 * carrying the record position they sit at, so the caller interleaves fwa_push / fwa_advance_watermark
 * exactly as processElement would. Element boundaries are found on the GPU (every chunk parses all its
 * candidate entry offsets; the chunk maps are composed hierarchically), so no host pass touches the bytes.
 *
 * Supported value types: fixed-length fields only (BIGINT / TIMESTAMP(p<=3) / TIMESTAMP_LTZ(p<=3) as
 * FWA_FIELD_LONG, DOUBLE, FLOAT, INT). Rows with variable-length fields, non-INSERT RowKinds and LZ4-compressed
 * buffers (taskmanager.network.compression) return FWA_E_UNSUPPORTED. Status codes: include/flink_amd.h.
 */
#ifndef FLINK_AMD_WIRE_H
#define FLINK_AMD_WIRE_H

#include <stdint.h>

#include "flink_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FWA_WIRE_MAX_FIELDS 16

/* StreamElementSerializer tags (StreamElementSerializer.java:48-53) */
enum fwa_wire_tag {
    FWA_TAG_REC_WITH_TIMESTAMP = 0,
    FWA_TAG_REC_WITHOUT_TIMESTAMP = 1,
    FWA_TAG_WATERMARK = 2,
    FWA_TAG_LATENCY_MARKER = 3,
    FWA_TAG_STREAM_STATUS = 4,
    FWA_TAG_RECORD_ATTRIBUTES = 5
};

/* Value serializer of the channel's StreamRecords. */
enum fwa_wire_format {
    FWA_WIRE_TUPLE = 0,    /* TupleSerializer (DataStream Tuple2..Tuple16): fields back to back, big-endian
                              (LongSerializer / DoubleSerializer / FloatSerializer / IntSerializer) */
    FWA_WIRE_ROWDATA = 1   /* RowDataSerializer -> BinaryRowDataSerializer (Table runtime rows) */
};

/* Field types (java.lang.Long / BIGINT / compact TIMESTAMP, Double / DOUBLE, Float / FLOAT, Integer / INT). */
enum fwa_wire_field { FWA_FIELD_LONG = 0, FWA_FIELD_DOUBLE = 1, FWA_FIELD_FLOAT = 2, FWA_FIELD_INT = 3 };

typedef struct fwa_wire_schema {
    int32_t format;                          /* enum fwa_wire_format */
    int32_t arity;                           /* fields per value, 1..FWA_WIRE_MAX_FIELDS */
    int32_t field[FWA_WIRE_MAX_FIELDS];      /* enum fwa_wire_field of each field */
    int32_t key_field;                       /* field -> key column (int64; INT sign-extended) */
    int32_t ts_field;                        /* field -> ts column; -1: the StreamRecord timestamp (records
                                                written without one get INT64_MIN, StreamRecord.hasTimestamp
                                                false, which fwa_push rejects with FWA_E_TS_MIN like
                                                TumblingEventTimeWindows.java:83-86) */
    int32_t num_cols;                        /* value columns */
    int32_t col_field[FWA_MAX_COLS];         /* field -> value column c: LONG/INT -> int64, DOUBLE -> double,
                                                FLOAT -> float (the input types fwa_push's aggregates read) */
    int32_t device;                          /* HIP device ordinal */
    int64_t max_bytes;                       /* sizing hint: largest nbytes per call (0 = 64 MiB; grows) */
} fwa_wire_schema;

typedef struct fwa_wire_decoder fwa_wire_decoder;

/* One decoded span of a channel. Device columns are decoder-owned and valid until the next call on it. */
typedef struct fwa_wire_batch {
    int64_t n_records;                       /* StreamRecords decoded, in stream order */
    int64_t n_events;                        /* non-record elements decoded */
    int64_t consumed;                        /* bytes of whole elements; [consumed, nbytes) is the head of an
                                                element continuing in the next buffer (SpanningWrapper): pass
                                                those bytes first in the next call */
    const int64_t* key;                      /* device [n_records] */
    const int64_t* ts;                       /* device [n_records] */
    const void* col[FWA_MAX_COLS];           /* device [n_records] per value column */
    const uint8_t* col_null[FWA_MAX_COLS];   /* ROWDATA: device [n_records], 1 = the field is NULL (the row's
                                                null bit; fwa_push_nullable's null_cols); NULL for TUPLE */
    const uint8_t* key_null;                 /* ROWDATA: device [n_records], 1 = NULL key field */
    /* events, host memory, in stream order */
    const int64_t* evt_pos;                  /* records of this batch that precede the event */
    const int32_t* evt_tag;                  /* enum fwa_wire_tag (2..5) */
    const int64_t* evt_val;                  /* [4 * n_events]: WATERMARK {timestamp}; STREAM_STATUS {status};
                                                LATENCY_MARKER {markedTime, operatorId.lower, operatorId.upper,
                                                subtaskIndex}; RECORD_ATTRIBUTES {isBacklog} */
} fwa_wire_batch;

/* Input location flag (same value as FWA_PUSH_DEVICE_PTRS): bytes is a device (HBM) pointer. */
#define FWA_WIRE_DEVICE_BYTES 0x1

int fwa_wire_create(const fwa_wire_schema* schema, fwa_wire_decoder** out);
void fwa_wire_destroy(fwa_wire_decoder* d);
const char* fwa_wire_last_error(const fwa_wire_decoder* d);

/* Decode the elements of bytes[0, nbytes) (concatenated buffer payloads of one channel, starting at an
 * element boundary). Device bytes (FWA_WIRE_DEVICE_BYTES) must be complete when the call is made: the decoder
 * runs on its own stream (the caller synchronises the producer's stream first); everything is complete on
 * return. A malformed element (unknown tag, or a length that does not match its tag and the schema) returns
 * FWA_E_CORRUPT ("Corrupt stream, found tag", StreamElementSerializer.java:208-210).
 * Device timing of the decode kernels accumulates in fwa_wire_stats. */
int fwa_wire_decode(fwa_wire_decoder* d, const uint8_t* bytes, int64_t nbytes, int32_t flags,
                    fwa_wire_batch* out);

typedef struct fwa_wire_stats {
    int64_t calls;
    int64_t bytes_in;
    int64_t records_out;
    double decode_ms;                        /* HIP-event device time of the decode kernels */
    double scan_ms;                          /* of which: the chunk-map pass (boundary candidates) */
} fwa_wire_stats;

int fwa_wire_get_stats(fwa_wire_decoder* d, fwa_wire_stats* out);

#ifdef __cplusplus
}
#endif
#endif /* FLINK_AMD_WIRE_H */
