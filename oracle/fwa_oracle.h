/*
 * fwa_oracle.h -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference Flink algorithms for
 * the keyed event-time window-aggregation path. Used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the CHECKER; never linked into or called by the product path
 * (flink_amd/ + libflink_amd.so).
 *
 * Parity pin: see oracle/README in DESIGN.md §Oracle -- window/operator semantics are pinned by the
 * reference's own known-answer tests transcribed into tests/golden/ (assigner KATs, WindowOperatorTest,
 * SlicingWindowAggOperatorTest event sequences); murmur/key-group integers are pinned by
 * specification only (no reference test holds literal values, SURVEY.md §4 "Gap").
 */
#ifndef FWA_ORACLE_H
#define FWA_ORACLE_H
#include <stdint.h>
#include "../include/flink_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Java arithmetic restatements ---- */
int32_t or_murmur_hash(int32_t code);                      /* MathUtils.java:137-155 */
int32_t or_bit_mix(int32_t in);                            /* MathUtils.java:194-201 */
int32_t or_long_hash(int64_t v);                           /* java.lang.Long.hashCode (JLS spec) */
int32_t or_binrow_bigint_hash(int64_t v);                  /* BinaryRowData.hashCode, 1 BIGINT field */
int32_t or_key_group(int64_t key, int32_t key_kind, int32_t key_hash, int32_t max_par);
int32_t or_operator_index(int32_t max_par, int32_t par, int32_t kg);
void or_key_group_range(int32_t max_par, int32_t par, int32_t idx, int32_t* start, int32_t* end);
int64_t or_window_start(int64_t ts, int64_t offset, int64_t size);   /* TimeWindow.java:264-272 */
int32_t or_long_to_int_with_bit_mixing(int64_t in);        /* MathUtils.java:170-175 */

/* Assign windows for a DataStream assigner: writes up to cap (start,end) pairs; returns count
 * or a negative fwa_status. Order = the reference assigner's list order. */
int or_assign_windows(const fwa_config* cfg, int64_t ts, int64_t* starts, int64_t* ends, int cap);
/* Table slice assigner: sliceEnd for ts (SliceAssigners.java:165-168/232-235/319-322). */
int64_t or_assign_slice_end(const fwa_config* cfg, int64_t ts);
/* Shift time zone (cfg->tz): TimeWindowUtil.toUtcTimestampMills / toEpochMillsForTimer. */
int64_t or_to_local(const fwa_config* cfg, int64_t epoch);
int64_t or_tz_timer(const fwa_config* cfg, int64_t local);

/* ---- streaming operator restatement ---- */
typedef struct or_engine or_engine;
int or_create(const fwa_config* cfg, or_engine** out);
int or_late_records(or_engine* e, const int32_t** idx, int64_t* n);
int or_push_nullable(or_engine* e, const int64_t* keys, const int64_t* ts, const void* const* cols,
                     const uint8_t* const* nulls, const int32_t* key_hash, int64_t n, int64_t* late_dropped_out);
void or_destroy(or_engine* e);
/* Same contract as fwa_push / fwa_advance_watermark (host pointers only). */
int or_push(or_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
            const int32_t* key_hash, int64_t n, int64_t* late_dropped_out);
int or_advance_watermark(or_engine* e, int64_t wm, fwa_out* out);
int or_get_stats(or_engine* e, fwa_stats* st);
const char* or_last_error(or_engine* e);

/* ---- synthetic stream of SURVEY.md §8(d) (bit-identical to the device generator) ---- */
uint64_t or_splitmix64(uint64_t x);
void or_generate(const fwa_gen_params* p, int64_t n, int64_t* keys, int64_t* ts, int64_t* v_i64,
                 float* v_f32, double* v_f64, const double* zipf_cdf_host);

/* ---- multi-threaded CPU baseline (Flink subtasks = threads owning key-group ranges) ----
 * Generates records [first, first+n) of the stream with p, runs the keyBy partition step and
 * `threads` operator instances (each owning computeKeyGroupRangeForOperatorIndex(maxP, threads, i)),
 * pushes in batches of `batch` with wm = max_ts - D - 1 after each batch, final wm = Long.MAX.
 * Returns seconds spent in the operator pipeline (generation excluded); rows/checksum out. */
double or_bench_pipeline(const fwa_config* cfg, const fwa_gen_params* p, int64_t n, int64_t batch,
                         int threads, int64_t* rows_out, uint64_t* checksum_out);
uint64_t or_row_digest(int64_t key, int64_t start, int64_t end, const int64_t* aggs, int naggs);
double or_pipeline_digests(const fwa_config* cfg, const fwa_gen_params* p, int64_t n, int64_t batch, int threads,
                           int64_t* wm_rows, uint64_t* wm_dig);
/* Full-size digests of the benched configurations beyond C2 (Zipf keys via cdf, float columns, any window kind):
   fwa_oracle.c, "full-size digests, general form". wm_bsum / wm_babs: [(n / batch + 2)][popcount(sum_mask)][nbuckets]. */
double or_pipeline_digests2(const fwa_config* cfg, const fwa_gen_params* p, const double* cdf, int float_cols,
                            uint32_t exact_mask, uint32_t sum_mask, int nbuckets, int64_t n, int64_t batch, int threads,
                            int64_t* wm_rows, uint64_t* wm_dig, double* wm_bsum, double* wm_babs);

#ifdef __cplusplus
}
#endif
#endif
