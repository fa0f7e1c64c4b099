/*
 * wire_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker of the GPU wire decoder, never the product path).
 *
 * Sequential CPU restatement of how a Flink input channel turns its buffer bytes into StreamElements:
 *   SpillingAdaptiveSpanningRecordDeserializer.getNextRecord   SpillingAdaptiveSpanningRecordDeserializer.java:88-131
 *     (4-byte big-endian length, NonSpanningWrapper.readInt :142; an incomplete element waits for the next
 *      buffer, SpanningWrapper -- here: parsing stops and `consumed` marks where it starts)
 *   StreamElementSerializer.deserialize                          StreamElementSerializer.java:190-211 (tags :48-53)
 *   TupleSerializer.deserialize -> Long/Double/Float/IntSerializer (java.io.DataInput, big-endian)
 *   BinaryRowDataSerializer.deserialize                         BinaryRowDataSerializer.java:85-93 (int size + row)
 *     BinaryRowData getters: null bits after the RowKind byte (BinaryRowData.java:68-75, HEADER_SIZE_IN_BITS 8),
 *     8-byte fixed-length slots at nullBits + 8 * pos (:114-116), little-endian (BinaryRowData.LITTLE_ENDIAN)
 * Element lengths are checked against the tag the way the GPU decoder checks them (a length that disagrees with
 * the tag's body is what the reference would hit as an EOFException / "Corrupt stream" IOException).
 */
#include <stdint.h>
#include <string.h>

#include "../include/flink_amd_wire.h"

static uint32_t rd_be32(const uint8_t* b) {
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | (uint32_t)b[3];
}
static uint64_t rd_be64(const uint8_t* b) { return ((uint64_t)rd_be32(b) << 32) | rd_be32(b + 4); }
static uint64_t rd_le(const uint8_t* b, int n) {
    uint64_t v = 0;
    for (int i = n - 1; i >= 0; --i) v = (v << 8) | b[i];
    return v;
}

static int fbytes(int t) { return (t == FWA_FIELD_LONG || t == FWA_FIELD_DOUBLE) ? 8 : 4; }

/* value of field f as 64 bits (INT sign-extended, FLOAT bits in the low word) */
static uint64_t field_value(const fwa_wire_schema* s, const uint8_t* v, int f, int nullbits) {
    const int t = s->field[f];
    if (s->format == FWA_WIRE_TUPLE) {
        int off = 0;
        for (int i = 0; i < f; ++i) off += fbytes(s->field[i]);
        if (fbytes(t) == 8) return rd_be64(v + off);
        uint32_t x = rd_be32(v + off);
        return t == FWA_FIELD_INT ? (uint64_t)(int64_t)(int32_t)x : (uint64_t)x;
    }
    const uint8_t* slot = v + nullbits + 8 * f;
    if (fbytes(t) == 8) return rd_le(slot, 8);
    uint32_t x = (uint32_t)rd_le(slot, 4);
    return t == FWA_FIELD_INT ? (uint64_t)(int64_t)(int32_t)x : (uint64_t)x;
}

static int is_null(const uint8_t* row, int f) { return (row[(f + 8) >> 3] >> ((f + 8) & 7)) & 1; }

/* Decode bytes[0, nbytes). Outputs sized by the caller (records <= nbytes / 10, events <= nbytes / 6).
 * cols[j]: int64 / double (8 B) or float (4 B) per the field type. col_null / key_null may be NULL (TUPLE).
 * Returns 0 or a negative fwa_status (err_tag / err_pos describe it). */
int or_wire_decode(const fwa_wire_schema* s, const uint8_t* bytes, int64_t nbytes, int64_t* key, int64_t* ts,
                   void* const* cols, uint8_t* const* col_null, uint8_t* key_null, int64_t* evt_pos, int32_t* evt_tag,
                   int64_t* evt_val, int64_t* n_rec, int64_t* n_evt, int64_t* consumed, int32_t* err_tag,
                   int64_t* err_pos) {
    const int nullbits = ((s->arity + 63 + 8) / 64) * 8;
    int value_len = 0;
    if (s->format == FWA_WIRE_TUPLE)
        for (int f = 0; f < s->arity; ++f) value_len += fbytes(s->field[f]);
    else
        value_len = 4 + nullbits + 8 * s->arity;
    const int64_t body[6] = {1 + 8 + value_len, 1 + value_len, 9, 29, 5, 2};
    int64_t p = 0, nr = 0, ne = 0;
    *err_tag = 0;
    *err_pos = 0;
    for (;;) {
        if (p + 4 > nbytes) break;                         /* length not complete: wait for the next buffer */
        const int64_t len = rd_be32(bytes + p);
        if (p + 5 > nbytes) break;
        const int tag = bytes[p + 4];
        if (tag > 5 || len != body[tag]) { *err_tag = tag; *err_pos = p; *n_rec = nr; *n_evt = ne; *consumed = p; return FWA_E_CORRUPT; }
        if (p + 4 + len > nbytes) break;                   /* element continues in the next buffer */
        const uint8_t* q = bytes + p + 5;
        if (tag == FWA_TAG_REC_WITH_TIMESTAMP || tag == FWA_TAG_REC_WITHOUT_TIMESTAMP) {
            int64_t rts = INT64_MIN;
            if (tag == FWA_TAG_REC_WITH_TIMESTAMP) { rts = (int64_t)rd_be64(q); q += 8; }
            int knull = 0;
            if (s->format == FWA_WIRE_ROWDATA) {
                if ((int32_t)rd_be32(q) != nullbits + 8 * s->arity) { *err_tag = tag; *err_pos = p; return FWA_E_UNSUPPORTED; }
                q += 4;
                if (q[0] != 0) { *err_tag = 256 + q[0]; *err_pos = p; return FWA_E_UNSUPPORTED; }
                if (s->ts_field >= 0 && is_null(q, s->ts_field)) { *err_tag = tag; *err_pos = p; return FWA_E_ARG; }
                knull = is_null(q, s->key_field);
                if (key_null) key_null[nr] = (uint8_t)knull;
                for (int j = 0; j < s->num_cols; ++j)
                    if (col_null && col_null[j]) col_null[j][nr] = (uint8_t)is_null(q, s->col_field[j]);
            }
            key[nr] = knull ? 0 : (int64_t)field_value(s, q, s->key_field, nullbits);
            ts[nr] = s->ts_field >= 0 ? (int64_t)field_value(s, q, s->ts_field, nullbits) : rts;
            for (int j = 0; j < s->num_cols; ++j) {
                const int f = s->col_field[j];
                const uint64_t v = field_value(s, q, f, nullbits);
                if (s->field[f] == FWA_FIELD_FLOAT) ((uint32_t*)cols[j])[nr] = (uint32_t)v;
                else ((uint64_t*)cols[j])[nr] = v;
            }
            ++nr;
        } else {
            int64_t v[4] = {0, 0, 0, 0};
            if (tag == FWA_TAG_WATERMARK) v[0] = (int64_t)rd_be64(q);                 /* new Watermark(readLong) */
            else if (tag == FWA_TAG_STREAM_STATUS) v[0] = (int32_t)rd_be32(q);        /* new WatermarkStatus(readInt) */
            else if (tag == FWA_TAG_LATENCY_MARKER) {                                 /* LatencyMarker(long, OperatorID(long, long), int) */
                v[0] = (int64_t)rd_be64(q);
                v[1] = (int64_t)rd_be64(q + 8);
                v[2] = (int64_t)rd_be64(q + 16);
                v[3] = (int32_t)rd_be32(q + 24);
            } else v[0] = q[0] != 0;                                                   /* RecordAttributes(readBoolean) */
            evt_pos[ne] = nr;
            evt_tag[ne] = tag;
            memcpy(evt_val + 4 * ne, v, sizeof v);
            ++ne;
        }
        p += 4 + len;
    }
    *n_rec = nr;
    *n_evt = ne;
    *consumed = p;
    return 0;
}
