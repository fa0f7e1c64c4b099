// engine.hip -- MI355X (gfx950) keyed event-time window aggregation engine behind include/flink_amd.h.
//
// State model: every window kind is a union of fixed-size SLICES (Flink's slicing
// design, SliceAssigners.java:134-385): tumbling g = size, sliding/hop g = gcd(size, slide),
// cumulate g = step. Slice q covers [off + q*g, off + (q+1)*g). Per (key, slice) accumulators live
// in HBM as dense SoA columns indexed by (slot, kid): kid = the key's position in an open-addressing
// key table, slot = a pool entry that the host assigns to slice q and publishes in a READ-ONLY (per
// launch) slice directory. Records whose slice has no slot yet are appended to a miss list and
// replayed after the host allocated slots (a lookahead keeps that rare on ordered streams), so no
// kernel needs intra-launch cross-CU hand-offs except the atomics themselves.
//
//   ingest kernel : one pass over the columnar batch: Java key-group check, slice assignment,
//                   lateness test against the current watermark, key lookup/insert, accumulate.
//   fire kernel   : on a watermark, for every newly fired window (end-1 <= wm) merge its slices per
//                   key and emit (key, start, end, aggs) for keys with COUNT > 0.
//
// Semantics restated (not copied) from WindowOperator.java:278-481 (DataStream; late firings within
// allowed lateness go to late_fire_kernel) and AbstractWindowAggProcessor.java:142-182 +
// Slice{Shared,Unshared}WindowAggProcessor (Table): a record contributes to every window containing
// it that has not fired when it arrives; it is dropped (numLateRecordsDropped) iff that set is
// empty; a window is emitted for a key iff at least one record contributed to it.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/flink_amd.h"
#include "java_math.h"
#include "dec_view.h"

#define LONG_MIN_J ((int64_t)0x8000000000000000LL)
#define LONG_MAX_J ((int64_t)0x7fffffffffffffffLL)

namespace {

#include "ingest.inc"


// ------------------------------------------------------------------------------------------------
// fire

struct FireWindow {
    int64_t start, end;         // emitted window bounds
    int32_t slot_off, nslots;
};

struct FireArgs {
    const unsigned long long* key_table;
    int64_t capacity;           // key table capacity (side slot at capacity)
    int64_t stride;
    unsigned long long* const* slot_base;
    const FireWindow* win;
    const int32_t* win_slots;
    int32_t nwin;
    int32_t blocks_per_win;
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    void* o_agg[FWA_MAX_AGGS];
    uint8_t* o_null[FWA_MAX_AGGS];   // SQL NULL flags per nullable aggregate (nullptr otherwise)
    int64_t* o_count;           // partial mode: COUNT(*) per row
    int64_t* o_hid[FWA_MAX_COLS];   // partial mode of a nullable handle: hidden non-NULL counter h per row
    int32_t raw;                // 1: emit accumulators (fwa_drain_partials), not results
    int64_t out_cap;            // rows past it are counted but not written (the host grows and relaunches)
    DevStatus* st;
};

constexpr int kFireJ = 16;                        // keys per thread per block: 4096-key chunks

// Final value of one aggregate (AggregateFunction.getResult / SQL getValueExpression) from its
// accumulator column value x (i64 sum bits, f64 sum bits or an ordered MIN/MAX key) and COUNT.
__device__ __forceinline__ int type_size_dev(int kind) {
    return (kind == FWA_SUM_F32 || kind == FWA_MIN_F32 || kind == FWA_MAX_F32 || kind == FWA_AVG_F32 ||
            kind == FWA_SUM_I32 || kind == FWA_MIN_I32 || kind == FWA_MAX_I32 || kind == FWA_FIRST_32 || kind == FWA_SEL_32 ||
            kind == FWA_MINBY_I32 || kind == FWA_MAXBY_I32 || kind == FWA_MINBY_F32 || kind == FWA_MAXBY_F32) ? 4 : 8;
}

// SQL NULLs (nn = the window's non-NULL input count of a nullable aggregate, d.nn > 0): SUM/MIN/MAX/AVG of
// no non-NULL input is NULL (nul[row] = 1, value 0); AVG divides by the non-NULL count (AvgAggFunction).
__device__ __forceinline__ void write_agg(const AggDesc& d, uint64_t cnt, unsigned long long x, uint64_t nn, void* out,
                                          uint8_t* nul, int64_t row) {
    const bool isnull = d.nn > 0 && d.kind != FWA_COUNT && d.kind != FWA_COUNT_COL && nn == 0;
    if (nul) nul[row] = isnull ? 1 : 0;
    if (isnull) {
        if (type_size_dev(d.kind) == 4) ((uint32_t*)out)[row] = 0u; else ((unsigned long long*)out)[row] = 0ull;
        return;
    }
    if (d.nn > 0 && (d.kind == FWA_AVG_I64 || d.kind == FWA_AVG_F32 || d.kind == FWA_AVG_F64)) cnt = nn;
    const int64_t iv = (int64_t)x;
    const double dv = __longlong_as_double((long long)x);
    switch (d.kind) {
        case FWA_COUNT: ((int64_t*)out)[row] = (int64_t)cnt; break;
        case FWA_COUNT_COL: ((int64_t*)out)[row] = d.acc > 0 ? (int64_t)x : (int64_t)cnt; break;
        case FWA_SUM_I64: ((int64_t*)out)[row] = iv; break;
        case FWA_SUM_F32: ((float*)out)[row] = (float)dv; break;
        case FWA_SUM_F64: ((double*)out)[row] = dv; break;
        case FWA_AVG_I64: {
            const int64_t n = (int64_t)cnt;  // AvgAggFunction: sum / count (Java long division)
            ((int64_t*)out)[row] = (n == -1 && iv == LONG_MIN_J) ? LONG_MIN_J : iv / n;
            break;
        }
        case FWA_AVG_F32: ((float*)out)[row] = (float)(dv / (double)(int64_t)cnt); break;
        case FWA_AVG_F64: ((double*)out)[row] = dv / (double)(int64_t)cnt; break;
        case FWA_MIN_I64: case FWA_MAX_I64: ((int64_t*)out)[row] = jm::unord_i64(x); break;
        case FWA_MIN_F32: case FWA_MAX_F32:
            ((float*)out)[row] = (float)__longlong_as_double((long long)jm::unord_bits64(x));
            break;
        case FWA_MIN_F64: case FWA_MAX_F64:
            ((double*)out)[row] = __longlong_as_double((long long)jm::unord_bits64(x));
            break;
        // the reduced field of a session reduction (FWA_CFG_REDUCE over session windows; reduce.inc red_write otherwise)
        case FWA_SUM_I32: ((uint32_t*)out)[row] = (uint32_t)x; break;
        case FWA_MIN_I32: case FWA_MAX_I32: case FWA_MINBY_I32: case FWA_MAXBY_I32:
            ((int32_t*)out)[row] = (int32_t)jm::unord_i64(x); break;
        case FWA_MINBY_I64: case FWA_MAXBY_I64: ((int64_t*)out)[row] = jm::unord_i64(x); break;
        case FWA_MINBY_F32: case FWA_MAXBY_F32:
            ((float*)out)[row] = (float)__longlong_as_double((long long)jm::unord_bits64(x)); break;
        case FWA_MINBY_F64: case FWA_MAXBY_F64:
            ((double*)out)[row] = __longlong_as_double((long long)jm::unord_bits64(x)); break;
        default: break;
    }
}

// Accumulator algebra: combine two accumulator values of one column (AggregateFunction.merge).
__device__ __forceinline__ unsigned long long acc_combine(int acc_kind, unsigned long long x, unsigned long long y) {
    switch (acc_kind) {
        case ACC_ADD_I64: return x + y;
        case ACC_ADD_F64:
            return (unsigned long long)__double_as_longlong(__longlong_as_double((long long)x) + __longlong_as_double((long long)y));
        case ACC_MIN_ORD: return y < x ? y : x;
        case ACC_MAX_ORD: return y > x ? y : x;
        default: return x;
    }
}

__device__ __forceinline__ void emit_row(const FireArgs& f, const EngineConst& c, const FireWindow& win, int64_t k,
                                         unsigned long long kv, uint64_t cnt, int64_t row) {
    f.o_key[row] = (k < f.capacity) ? (int64_t)kv : LONG_MIN_J;
    f.o_start[row] = win.start;
    f.o_end[row] = win.end;
    if (f.o_count) f.o_count[row] = (int64_t)cnt;
    for (int j = 0; j < c.nout; ++j) {
        const AggDesc d = c.agg[j];
        unsigned long long x = ident_of(d.acc_kind);
        uint64_t nn = 0;
        if (d.acc > 0)
            for (int s = 0; s < win.nslots; ++s)
                x = acc_combine(d.acc_kind, x, f.slot_base[f.win_slots[win.slot_off + s]][(int64_t)d.acc * f.stride + k]);
        if (d.nn > 0)
            for (int s = 0; s < win.nslots; ++s) nn += f.slot_base[f.win_slots[win.slot_off + s]][(int64_t)d.nn * f.stride + k];
        if (f.raw) {   // partial accumulators (fwa_drain_partials): the accumulator value itself
            ((unsigned long long*)f.o_agg[j])[row] = d.acc > 0 ? x : cnt;
            continue;
        }
        write_agg(d, cnt, x, nn, f.o_agg[j], f.o_null[j], row);
    }
    if (f.raw)   // SQL NULLs: the hidden non-NULL counters travel with the partial accumulators
        for (int h = c.nout; h < c.naggs; ++h) {
            const AggDesc d = c.agg[h];
            uint64_t nn = 0;
            for (int s = 0; s < win.nslots; ++s) nn += f.slot_base[f.win_slots[win.slot_off + s]][(int64_t)d.acc * f.stride + k];
            f.o_hid[h - c.nout][row] = (int64_t)nn;
        }
}

// TUMBLE fire of a handle with 3..5 accumulator columns (COUNT included; every window one slot, not raw): every column
// of the block's kids is loaded before the first row store -- the generic emit_row reloads each column behind the
// previous row's stores (a possible alias), which held C5's fire (five aggregates over four columns) near 1.5 TB/s.
// One block = one window x kBlock * 4 kids; one row reservation per block as fire_kernel.
template <int NA>
__global__ void __launch_bounds__(kBlock) fire_multi_kernel(FireArgs f, const EngineConst* __restrict__ cp) {
    constexpr int J = 4;
    const EngineConst& c = *cp;
    const int32_t w = blockIdx.x / f.blocks_per_win;
    const int64_t k0 = (int64_t)(blockIdx.x % f.blocks_per_win) * kBlock * J;
    const FireWindow win = f.win[w];
    const int64_t nk = f.capacity + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int kWaves = kBlock / 64;
    __shared__ uint32_t woff[J][kWaves];
    __shared__ unsigned long long s_base;
    const unsigned long long* slot = f.slot_base[f.win_slots[win.slot_off]];
    unsigned long long kvs[J], x[J][NA], masks[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {                       // clamped index: unconditional loads
        const int64_t k = min(k0 + (int64_t)j * kBlock + tid, nk - 1);
        kvs[j] = f.key_table[k];
#pragma unroll
        for (int a = 0; a < NA; ++a) x[j][a] = slot[(int64_t)a * f.stride + k];
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t k = k0 + (int64_t)j * kBlock + tid;
        const bool present = k < nk && ((k < f.capacity) ? (kvs[j] != kEmptyKey) : (kvs[j] == 1ull));
        masks[j] = __ballot(present && x[j][0] != 0);
        if (lane == 0) woff[j][wid] = (uint32_t)__popcll(masks[j]);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int j = 0; j < J; ++j)
            for (int v = 0; v < kWaves; ++v) { const uint32_t t = woff[j][v]; woff[j][v] = run; run += t; }
        s_base = run ? atomicAdd(&f.st->rows, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        if (!((masks[j] >> lane) & 1ull)) continue;
        const int64_t k = k0 + (int64_t)j * kBlock + tid;
        const int64_t row = (int64_t)s_base + woff[j][wid] + __popcll(masks[j] & lt);
        if (row >= f.out_cap) continue;
        f.o_key[row] = (k < f.capacity) ? (int64_t)kvs[j] : LONG_MIN_J;
        f.o_start[row] = win.start;
        f.o_end[row] = win.end;
        for (int a = 0; a < c.nout; ++a) {
            const AggDesc d = c.agg[a];
            unsigned long long xv = ident_of(d.acc_kind), nn = 0;
#pragma unroll
            for (int q = 1; q < NA; ++q) {                 // register selects, no dynamic index
                if (q == d.acc) xv = x[j][q];
                if (q == d.nn) nn = x[j][q];
            }
            write_agg(d, x[j][0], xv, nn, f.o_agg[a], f.o_null[a], row);
        }
    }
}

// One block = one window x one chunk of kBlock*kFireJ consecutive kids. Pass 1 sums COUNT over the
// window's slices and ballots the emitting keys; one atomic reserves the block's rows; pass 2 writes
// rows j-major so every wave store is contiguous.
// PRE = 1 (one stateful accumulator column, e.g. COUNT + SUM(long), single-slot windows): pass 1
// also loads that column, so pass 2 only stores (the generic emit re-reads it behind every store).
template <int PRE>
__global__ void __launch_bounds__(kBlock) fire_kernel(FireArgs f, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int32_t w = blockIdx.x / f.blocks_per_win;
    const int64_t chunk = blockIdx.x % f.blocks_per_win;
    const FireWindow win = f.win[w];
    const int64_t nk = f.capacity + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int kWaves = kBlock / 64;
    __shared__ uint32_t woff[kFireJ][kWaves];
    __shared__ unsigned long long s_base;
    const int64_t k0 = chunk * (int64_t)kBlock * kFireJ;
    uint64_t cnt[kFireJ];
    unsigned long long kvs[kFireJ];
    unsigned long long masks[kFireJ];
    unsigned long long xs[PRE ? kFireJ : 1];
    const unsigned long long* slot0 = PRE ? f.slot_base[f.win_slots[win.slot_off]] : nullptr;
    if (PRE) {   // issue every load of the chunk before the first use
#pragma unroll
        for (int j = 0; j < kFireJ; ++j) {
            const int64_t k = k0 + (int64_t)j * kBlock + tid;
            kvs[j] = k < nk ? f.key_table[k] : kEmptyKey;
            cnt[j] = k < nk ? slot0[k] : 0;
            xs[PRE ? j : 0] = k < nk ? slot0[f.stride + k] : 0;
        }
    }
#pragma unroll
    for (int j = 0; j < kFireJ; ++j) {
        const int64_t k = k0 + (int64_t)j * kBlock + tid;
        bool present = false;
        unsigned long long kv = PRE ? kvs[j] : 0;
        if (k < nk) {
            if (!PRE) kv = f.key_table[k];
            present = (k < f.capacity) ? (kv != kEmptyKey) : (kv == 1ull);
        }
        uint64_t cc = 0;
        if (PRE) cc = present ? cnt[j] : 0;
        else if (present)
            for (int s = 0; s < win.nslots; ++s) cc += f.slot_base[f.win_slots[win.slot_off + s]][k];
        cnt[j] = cc;
        kvs[j] = kv;
        const unsigned long long m = __ballot(present && cc != 0);
        masks[j] = m;
        if (lane == 0) woff[j][wid] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int j = 0; j < kFireJ; ++j)
            for (int v = 0; v < kWaves; ++v) { const uint32_t t = woff[j][v]; woff[j][v] = run; run += t; }
        s_base = run ? atomicAdd(&f.st->rows, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < kFireJ; ++j) {
        if (!((masks[j] >> lane) & 1ull)) continue;
        const int64_t k = k0 + (int64_t)j * kBlock + tid;
        const int64_t row = (int64_t)s_base + woff[j][wid] + __popcll(masks[j] & lt);
        if (row >= f.out_cap) continue;
        if (PRE) {
            f.o_key[row] = (k < f.capacity) ? (int64_t)kvs[j] : LONG_MIN_J;
            f.o_start[row] = win.start;
            f.o_end[row] = win.end;
            if (f.o_count) f.o_count[row] = (int64_t)cnt[j];
            for (int a = 0; a < c.nout; ++a) {   // one stateful column: a nullable aggregate's counter is that column
                const AggDesc d = c.agg[a];
                const unsigned long long x = d.acc > 0 ? xs[PRE ? j : 0] : ident_of(d.acc_kind);
                if (f.raw) ((unsigned long long*)f.o_agg[a])[row] = d.acc > 0 ? x : cnt[j];
                else write_agg(d, cnt[j], x, d.nn > 0 ? xs[PRE ? j : 0] : 0ull, f.o_agg[a], f.o_null[a], row);
            }
        } else {
            emit_row(f, c, win, k, kvs[j], cnt[j], row);
        }
    }
}

// drain_route (fwa_drain_route): the raw fire of complete slices (fwa_drain_partials) written straight into the
// exchange's send layout -- packed partial rows grouped by owning subtask (KeyGroupStreamPartitioner.selectChannel,
// KeyGroupStreamPartitioner.java:55-65) -- so the drain and the keyBy routing are one pass over the slot columns. One
// block = one slice x one chunk of kBlock*kFireJ kids (fire_kernel's grid); one cursor reservation per (block,
// destination), LDS positions inside it.
constexpr int kMaxDest = 64;
struct DrainRouteArgs {
    FireArgs f;                        // key table, slots, the slices (one slot each)
    int32_t par, m, ncell, pad;        // destinations, cells per row, accumulator cells (cells 3..m-1)
    int32_t cell_acc[kMaxAggsInt];     // accumulator column feeding cell 3 + i (0: COUNT(*), an aggregate without one)
    int64_t cap;                       // rows per destination region
    int64_t* rows;                     // [par][cap][m]
    unsigned long long* dcnt;          // [par] rows per destination (past cap: counted, not written; host relaunches)
};

constexpr int kDrJ = 8;                           // kids per thread: 2048-kid chunks per block
// One block per kid chunk walks every drained slice: the key table is read and each key's owner computed once per
// chunk, not once per (chunk, slice); one cursor reservation per (slice, destination).
__global__ void __launch_bounds__(kBlock) drain_route_kernel(DrainRouteArgs r, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int64_t chunk = blockIdx.x;
    const unsigned long long* __restrict__ keys = r.f.key_table;
    const int64_t cap_k = r.f.capacity, nk = cap_k + 1, stride = r.f.stride;
    const int tid = threadIdx.x;
    const int par = r.par, m = r.m, ncell = r.ncell;
    __shared__ uint32_t s_cnt[kMaxDest], s_pos[kMaxDest];
    __shared__ unsigned long long s_base[kMaxDest];
    __shared__ int32_t s_cell[kMaxAggsInt];
    for (int i = tid; i < ncell; i += kBlock) s_cell[i] = r.cell_acc[i];
    const int64_t k0 = chunk * (int64_t)kBlock * kDrJ;
    int64_t key[kDrJ];
    int32_t dst[kDrJ];                                 // -1: no key at this kid
#pragma unroll
    for (int j = 0; j < kDrJ; ++j) {
        const int64_t k = k0 + (int64_t)j * kBlock + tid;
        key[j] = 0;
        dst[j] = -1;
        if (k < nk) {
            const unsigned long long kv = keys[k];
            if ((k < cap_k) ? (kv != kEmptyKey) : (kv == 1ull)) {
                key[j] = (k < cap_k) ? (int64_t)kv : LONG_MIN_J;
                const int32_t kg = jm::key_group_of(key[j], c.key_kind, 0, c.max_par);
                dst[j] = kg < 0 ? 0 : jm::operator_index(c.max_par, par, kg);
            }
        }
    }
    for (int w = 0; w < r.f.nwin; ++w) {
        const FireWindow win = r.f.win[w];
        const unsigned long long* __restrict__ slot0 = r.f.slot_base[r.f.win_slots[win.slot_off]];
        for (int d = tid; d < par; d += kBlock) { s_cnt[d] = 0; s_pos[d] = 0; }
        __syncthreads();
        uint64_t cnt[kDrJ];
#pragma unroll
        for (int j = 0; j < kDrJ; ++j) {
            const int64_t k = k0 + (int64_t)j * kBlock + tid;
            cnt[j] = dst[j] >= 0 ? slot0[k] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < kDrJ; ++j) if (cnt[j]) atomicAdd(&s_cnt[dst[j]], 1u);
        __syncthreads();
        for (int d = tid; d < par; d += kBlock) s_base[d] = s_cnt[d] ? atomicAdd(&r.dcnt[d], (unsigned long long)s_cnt[d]) : 0ull;
        __syncthreads();
        for (int j = 0; j < kDrJ; ++j) {
            if (!cnt[j]) continue;
            const int64_t k = k0 + (int64_t)j * kBlock + tid;
            const int d = dst[j];
            const unsigned long long pos = s_base[d] + atomicAdd(&s_pos[d], 1u);
            if ((int64_t)pos >= r.cap) continue;
            int64_t* row = r.rows + ((int64_t)d * r.cap + (int64_t)pos) * m;
            row[0] = key[j];
            row[1] = win.start;
            row[2] = (int64_t)cnt[j];
            for (int i = 0; i < ncell; ++i) {
                const int a = s_cell[i];
                row[3 + i] = a > 0 ? (int64_t)slot0[(int64_t)a * stride + k] : (int64_t)cnt[j];
            }
        }
        __syncthreads();                               // s_cnt / s_pos / s_base reused by the next slice
    }
}

// ------------------------------------------------------------------------------------------------
// fire_slide: one watermark fires a RUN of consecutive hop windows (HOP 60 s / 1 s over a batch of
// 67 s of event time fires 67 windows of 60 slices each). The generic fire re-merges every window
// from its slices (67 x 60 slice reads per key and column); here each key walks the run once with a
// running sum, S_w = S_{w-1} + (slices entering) - (slices leaving): 2r slice reads per window
// (r = slide / slice). Only for invertible accumulators -- COUNT and 64-bit integer sums, which wrap
// exactly like Java long arithmetic, so the running sum equals the direct sum bit for bit; float
// sums and MIN/MAX keep the generic fire. Rows are emitted window by window with one row
// reservation per block and window.
constexpr int kSlideMaxU = 2048;                  // union slices per launch (LDS slot table)
constexpr int kSlideBlock = 1024;                 // threads per block
constexpr int kSlideJ = 2;                        // keys per thread (2048 keys per block)
constexpr int kSlideAcc = 4;                      // COUNT + up to 3 integer-sum columns

struct FireSlideArgs {
    const unsigned long long* key_table;
    int64_t capacity, stride;
    const unsigned long long* const* upos;   // [m] slot base per union slice (a slice without records points at a
                                             // zero slice); bit 0 set: the slice retires at this watermark -- its last
                                             // read restores the identity
    int32_t m, nw, L, r;                     // union slices, windows, slices per window, per slide
    int64_t start0, slide, size;             // first window start, window step, window size
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    void* o_agg[FWA_MAX_AGGS];
    int64_t out_cap;                         // rows past it are counted, not written (host grows, relaunches)
    DevStatus* st;
    // carried window sums (rsum, [NA][stride]): r_u0 > 0 -- window 0 is rsum (its slices 0 .. r_u0 - 1, unchanged since
    // the previous fire stored them) plus slices r_u0 .. L - 1; r_k > 0 -- store for the next run the sums over the
    // slices the next run's window 0 shares with this run's last window, minus that window's last r_k slices
    unsigned long long* rsum;
    int32_t r_u0, r_k;
};

// NA = the handle's accumulator count (compile time: the running sums and the next window's slice values stay in
// registers). Every slice load is unconditional -- absent keys read their (zero) slot through a clamped index and are
// masked after the load, a slice without records reads the zero slice -- since a load under a per-element condition
// makes hipcc branch around it and wait for each load separately. With one slice per slide (r = 1) the slices entering
// / leaving window w + 1 are loaded before window w's rows are reserved and written, so their latency overlaps the
// ballot, the row reservation and the stores.
// Slices that retire at this watermark (tagged upos entries) are cleared here instead of by reset_slots_kernel: the
// read that subtracts a leaving slice is its last, and only the non-zero values are written back (a Zipf stream
// leaves most keys absent from most slices, so this writes a fraction of the dense column reset_slots_kernel wrote).
// Measured (r04, C3, ms per fire at 67 windows x ~1M keys): 2.24 the r03 kernel (8 keys per lane, conditional loads,
// two barriers and one reservation per window); 2.19-2.33 this one over 256..1024-thread blocks and 2..8 keys per lane,
// with or without non-temporal row stores -- the fire moves ~9 GB per launch (window 0's 60 slices, 2 slices x 2 columns
// per window over the whole 2M-slot table, 40-byte rows) at ~4 TB/s, so it is bandwidth-bound on the dense slot layout.
// Clearing: the conditional clear here 2.25 ms + no reset, an unconditional (full-line) clear 2.44, no clear 1.99 +
// reset_slots_kernel -- 5.83 / 6.20 / 6.00 ms per C3 step.
__device__ __forceinline__ unsigned long long* slide_ptr(const unsigned long long* p) {
    return (unsigned long long*)((uintptr_t)p & ~(uintptr_t)1);
}
__device__ __forceinline__ bool slide_zero(const unsigned long long* p) { return ((uintptr_t)p & 1) != 0; }

template <int NA, int J = kSlideJ, int TB = kSlideBlock>
__global__ void __launch_bounds__(TB) fire_slide_kernel(FireSlideArgs f, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    constexpr int kWaves = TB / 64;
    __shared__ const unsigned long long* s_u[kSlideMaxU];
    __shared__ uint32_t woff[3][J][kWaves];           // three generations: counted, scanned, read by the writers
    __shared__ unsigned long long s_base[3];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int i = tid; i < f.m; i += TB) s_u[i] = f.upos[i];
    const int64_t nk = f.capacity + 1;
    const int64_t k0 = (int64_t)blockIdx.x * TB * J;
    const int64_t st = f.stride;
    unsigned long long kv[J];
    int64_t kc[J];                                    // slot index, clamped into the table
    bool present[J];
    unsigned long long S[J][NA];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t k = k0 + (int64_t)j * TB + tid;
        kc[j] = k < nk ? k : nk - 1;
        kv[j] = f.key_table[kc[j]];
        present[j] = k < nk && ((k < f.capacity) ? (kv[j] != kEmptyKey) : (kv[j] == 1ull));
#pragma unroll
        for (int a = 0; a < NA; ++a) S[j][a] = 0;
    }
    __syncthreads();
    // window 0: the sum of its L slices (or the carried sums of its first r_u0 slices plus the others)
    if (f.r_u0 > 0) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) S[j][a] = present[j] ? f.rsum[a * st + kc[j]] : 0ull;
    }
    for (int u = f.r_u0; u < f.L; ++u) {
        const unsigned long long* b = slide_ptr(s_u[u]);
        unsigned long long x[J][NA];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) x[j][a] = b[a * st + kc[j]];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) S[j][a] += present[j] ? x[j][a] : 0ull;
    }
    unsigned long long Xi[J][NA], Xo[J][NA];
    unsigned long long* po = nullptr;
    bool pz = false;
    auto load2 = [&](const unsigned long long* bi, const unsigned long long* to) {
        po = slide_ptr(to);
        pz = slide_zero(to);
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                Xi[j][a] = bi[a * st + kc[j]];
                Xo[j][a] = po[a * st + kc[j]];
            }
    };
    auto apply = [&]() {   // S(w) = S(w - 1) + entering - leaving; a retiring leaving slice is cleared
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (!present[j]) continue;
                S[j][a] = S[j][a] + Xi[j][a] - Xo[j][a];
                if (pz && Xo[j][a]) po[a * st + kc[j]] = 0ull;
            }
    };
    const unsigned long long lt = (1ull << lane) - 1ull;
    // rows of window w (sums Sw, masks mw) at the block's reservation of generation g
    auto write_rows = [&](int w, const unsigned long long (&Sw)[J][NA], const unsigned long long (&mw)[J], int g) {
        const int64_t ws = f.start0 + (int64_t)w * f.slide;
        const int64_t we = ws + f.size;
        const int64_t rb = (int64_t)s_base[g];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (!((mw[j] >> lane) & 1ull)) continue;
            const int64_t row = rb + woff[g][j][wid] + __popcll(mw[j] & lt);
            if (row >= f.out_cap) continue;
            f.o_key[row] = kc[j] < f.capacity ? (int64_t)kv[j] : LONG_MIN_J;
            f.o_start[row] = ws;
            f.o_end[row] = we;
            for (int a = 0; a < c.nout; ++a) {   // (no nullable aggregates on this path: the host checks)
                const AggDesc d = c.agg[a];
                unsigned long long x = 0;
#pragma unroll
                for (int q = 1; q < NA; ++q) if (q == d.acc) x = Sw[j][q];
                const int64_t cnt = (int64_t)Sw[j][0], iv = (int64_t)x;
                int64_t v;
                switch (d.kind) {   // every aggregate of an invertible handle has a 64-bit integer result
                    case FWA_COUNT: v = cnt; break;
                    case FWA_COUNT_COL: v = d.acc > 0 ? iv : cnt; break;
                    case FWA_SUM_I64: v = iv; break;
                    case FWA_AVG_I64: v = (cnt == -1 && iv == LONG_MIN_J) ? LONG_MIN_J : iv / cnt; break;
                    default: write_agg(d, Sw[j][0], x, 0, f.o_agg[a], nullptr, row); continue;
                }
                ((int64_t*)f.o_agg[a])[row] = v;
            }
        }
    };
    // One barrier per window: window w's rows are counted and its reservation issued (thread 0) while the other waves
    // write window w - 1's rows at the reservation made one iteration earlier.
    const bool one = f.r == 1;
    if (one && f.nw > 1) load2(slide_ptr(s_u[f.L]), s_u[0]);
    unsigned long long Sp[J][NA], mp[J];
    for (int w = 0; w < f.nw; ++w) {
        if (w > 0 && one) {
            apply();
            if (w + 1 < f.nw) load2(slide_ptr(s_u[w + f.L]), s_u[w]);   // in flight while window w - 1 is written
        } else if (w > 0) {
            for (int t = 0; t < f.r; ++t) {
                load2(slide_ptr(s_u[(w - 1) * f.r + f.L + t]), s_u[(w - 1) * f.r + t]);
                apply();
            }
        }
        const int g = w % 3;
        unsigned long long masks[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            masks[j] = __ballot(present[j] && S[j][0] != 0);
            if (lane == 0) woff[g][j][wid] = (uint32_t)__popcll(masks[j]);
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t run = 0;
            for (int j = 0; j < J; ++j)
                for (int v = 0; v < kWaves; ++v) { const uint32_t t = woff[g][j][v]; woff[g][j][v] = run; run += t; }
            s_base[g] = run ? atomicAdd(&f.st->rows, (unsigned long long)run) : 0ull;
        }
        if (w > 0) write_rows(w - 1, Sp, mp, (w - 1) % 3);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            mp[j] = masks[j];
#pragma unroll
            for (int a = 0; a < NA; ++a) Sp[j][a] = S[j][a];
        }
    }
    __syncthreads();
    if (f.nw > 0) write_rows(f.nw - 1, Sp, mp, (f.nw - 1) % 3);
    if (f.r_k > 0 && f.nw > 0) {   // the next run's carried sums (before the retiring slices below are cleared)
        const int lw = (f.nw - 1) * f.r;               // first slice of the last window
        auto sub = [&](int u) {
            const unsigned long long* b = slide_ptr(s_u[u]);
#pragma unroll
            for (int j = 0; j < J; ++j)
#pragma unroll
                for (int a = 0; a < NA; ++a) Sp[j][a] -= present[j] ? b[a * st + kc[j]] : 0ull;
        };
        for (int u = lw; u < lw + f.r; ++u) sub(u);              // leave before the next window
        for (int u = f.m - f.r_k; u < f.m; ++u) sub(u);          // may still change before the next fire
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (k0 + (int64_t)j * TB + tid >= nk) continue;      // (clamped lanes would overwrite the last kid)
#pragma unroll
            for (int a = 0; a < NA; ++a) f.rsum[a * st + kc[j]] = present[j] ? Sp[j][a] : 0ull;
        }
    }
    // retiring slices whose last window is the run's last one never left it: clear them now
    for (int u = (f.nw - 1) * f.r; u < f.m; ++u) {
        if (!slide_zero(s_u[u])) continue;
        unsigned long long* b = slide_ptr(s_u[u]);
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a) Xo[j][a] = b[a * st + kc[j]];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a)
                if (present[j] && Xo[j][a]) b[a * st + kc[j]] = 0ull;
    }
}

// ------------------------------------------------------------------------------------------------
// sessions (merging windows): DataStream EventTimeSessionWindows + EventTimeTrigger (allowed lateness
// L >= 0) and the Table legacy GROUP BY SESSION (TR/operators/window/WindowOperator.java:331-398 with
// MergingWindowProcessFunction and EventTimeTriggers.afterEndOfWindow).
//
// State: a flat list of in-flight sessions {kid, start, end, acc[nacc]} (column 0 = COUNT), in no
// particular order; no per-key cap. A push rebuilds it (DESIGN.md §2 "Sessions"):
//  * Order-free records -- the lone window [ts, ts+gap) ends after the watermark (ts + gap - 1 > wm).
//    Such a record is never dropped, never fires on arrival, and merging is a union of intersecting
//    intervals, so the key's session set after the push is the connected components of (its in-flight
//    sessions + its new windows) regardless of arrival order (MergingWindowSet.addWindow :153-236,
//    TimeWindow.intersects/cover :116-124 -- touching windows merge). Bulk path: one radix sort by
//    (kid, start), a segmented max-scan of the ends (a new session starts where start > every earlier
//    end of the key), a cluster-id scan, and a wave-segmented reduction of the accumulators.
//  * A key with at least one order-sensitive record in the push (lone window already ends at or before
//    the watermark: it may be dropped, may fire on arrival with the session contents, or may be saved by
//    a session an earlier record of the push created) goes through an arrival-order walk instead: its
//    sessions and records sorted by (kid, arrival), one lane per key applying addWindow / isWindowLate /
//    EventTimeTrigger.onElement in order (WindowOperator.java:288-389). Late firings are written to the
//    late-row buffer (returned at the head of the next fwa_advance_watermark).
//  * Fire at a watermark advance prev -> wm: every session with prev < end - 1 <= wm emits a row
//    (EventTimeTrigger.onEventTime: sessions whose maxTimestamp <= prev already fired -- at a timer or
//    on an element); every session with cleanup = end - 1 + L <= wm is cleared (clearAllState).

struct SessCtr {                 // per-push device counters (zeroed by the host before a push / fire)
    unsigned long long ts_min, ts_max;   // ord-encoded, over records and in-flight session starts (cell pre-aggregation:
                                         // the smallest / largest cell number of the push)
    unsigned long long n_special;        // records whose lone window ends at or before the watermark
    unsigned long long n_bulk, n_sp;     // elements routed to the bulk / the arrival-order path
    unsigned long long n_out_sp;         // sessions written by the arrival-order path
    unsigned long long n_keep;           // fire: sessions kept
    unsigned long long n_redo;           // cell path: elements outside the cell range (the push is redone)
};

struct SessList {                // one in-flight session list (SoA)
    uint32_t* kid;
    int64_t* start;
    int64_t* end;
    unsigned long long* acc;     // [nacc][stride]
    int64_t stride;
};

struct Sess2Args {
    const int64_t* keys;
    const int64_t* ts;
    const void* cols[FWA_MAX_COLS];
    const int32_t* key_hash;
    const int64_t* gapc;         // per-record gaps (DynamicEventTimeSessionWindows) or nullptr: fixed `gap`
    const uint8_t* nulls[FWA_MAX_COLS];   // SQL NULL flags per value column (nullptr: no NULLs)
    int64_t n;
    int64_t wm, gap, lateness;
    unsigned long long* key_table;
    uint64_t key_mask;
    int32_t seg_log, part_bits;
    int64_t capacity;            // key-table capacity (side slot at capacity)
    uint32_t* rkid;              // [n] kid per record (0xffffffff: rejected)
    uint8_t* kflag;              // [capacity + 1] key has an order-sensitive record in this push
    SessList in;                 // in-flight sessions before the push
    int64_t n_in;
    SessList out;                // after the push
    // bulk path
    int64_t base;                // smallest start of the push (records and in-flight sessions)
    int32_t tb;                  // bits of (start - base) in the sort key (kid << tb | start - base)
    int32_t all_sp;              // 1: route everything through the arrival-order path
    unsigned long long* bkey;    // [nb] sort keys (then sorted)
    uint32_t* bval;              // [nb] payload: bulk position, | 0x80000000 when its end is in pe (sessions,
                                 // dynamic gaps)
    unsigned long long* pk;      // [nb][pkw] the element's COUNT + accumulator words, in bulk order (one row per
                                 // element gathered once after the sort, not one value column per accumulator)
    int64_t* pe;                 // [nb] end of a flagged element
    uint32_t* sg_kid;            // segment kernel staging: wave w's clusters at [h0(w), h0(w) + count(w)) (no atomics)
    int64_t* sg_start;
    int64_t* sg_end;
    unsigned long long* sg_acc;  // [nacc][cap]
    int64_t sg_cap;
    uint32_t* sg_cnt;            // [nw + 1] clusters per wave
    uint32_t* sg_off;            // [nw + 1] their exclusive sum
    int64_t* sg_h0;              // [nw] first owned position per wave
    int32_t pkw;
    jm::UDiv64 gap_div;          // cell path: cell = (start - base) / gap, base = ctr->ts_min
    int32_t seg_out;             // bulk sessions appended on ctr->n_out_sp by sess2_segment_kernel (the arrival-order
                                 // path appends after them on the same counter)
    int64_t* bend;               // [nb] window / session end per sorted element
    int64_t* bmax;               // [nb] inclusive max of bend over the key so far (segmented scan)
    uint32_t* bcid;              // [nb] head flags, then 1-based cluster ids (inclusive sum)
    int64_t nb;
    int32_t col_owner[1 + kMaxAggsInt];    // aggregate that feeds accumulator column c (-1: COUNT)
    // arrival-order path
    unsigned long long* skey;    // [ns] (kid << 32) | (0 for a session, 1 + record index)
    uint32_t* sval;
    int64_t nsp;
    int64_t* sc_start;           // [ns] scratch session lists, one region per key run
    int64_t* sc_end;
    unsigned long long* sc_acc;  // [nacc][ns]
    // late-firing rows
    int64_t* lr_key;
    int64_t* lr_start;
    int64_t* lr_end;
    void* lr_agg[FWA_MAX_AGGS];
    unsigned long long* lr_n;
    int64_t lr_cap;
    SessCtr* ctr;
    int32_t* dropidx;            // FWA_CFG_LATE_INDICES list (nullptr: not collected)
    DevStatus* st;
};

__device__ __forceinline__ int64_t sess_cleanup(int64_t max_ts, int64_t lateness) {   // WindowOperator.cleanupTime :647-654
    const int64_t ct = jm::wadd(max_ts, lateness);
    return ct >= max_ts ? ct : LONG_MAX_J;
}

__device__ __forceinline__ void wave_minmax(unsigned long long lo, unsigned long long hi, unsigned long long* dlo,
                                            unsigned long long* dhi) {
    for (int sh = 32; sh >= 1; sh >>= 1) {
        const unsigned long long a = __shfl_xor(lo, sh), b = __shfl_xor(hi, sh);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0 && lo <= hi) { atomicMin(dlo, lo); atomicMax(dhi, hi); }
}

// Pass 1 over the records: key-group check, kid, order-sensitivity flag per key, start range.
__global__ void __launch_bounds__(kBlock) sess2_classify_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    unsigned long long lo = ~0ull, hi = 0ull, nsp = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t key = a.keys[i];
        const int64_t ts = a.ts[i];
        a.rkid[i] = 0xffffffffu;
        const int32_t kg = jm::key_group_of(key, c.key_kind, a.key_hash ? a.key_hash[i] : 0, c.max_par);
        if (kg < c.kg_lo || kg > c.kg_hi) { raise_error(a.st, FWA_E_KEYGROUP); continue; }   // StateTable :300-307
        const int64_t gap = a.gapc ? a.gapc[i] : a.gap;
        if (gap <= 0) { raise_error(a.st, FWA_E_ARG); continue; }   // DynamicEventTimeSessionWindows.java:60-64
        const int64_t kid = key_slot(a.key_table, a.key_mask, a.seg_log, a.part_bits, key, a.st);
        if (kid < 0) { a.st->key_full = 1; raise_error(a.st, FWA_E_OOM); continue; }
        a.rkid[i] = (uint32_t)kid;
        if (jm::wsub(jm::wadd(ts, gap), 1) <= a.wm) { a.kflag[kid] = 1; ++nsp; }   // lone window maxTs <= wm
        const unsigned long long o = jm::ord_i64(ts);
        lo = o < lo ? o : lo;
        hi = o > hi ? o : hi;
    }
    wave_minmax(lo, hi, &a.ctr->ts_min, &a.ctr->ts_max);
    for (int sh = 32; sh >= 1; sh >>= 1) nsp += __shfl_xor(nsp, sh);
    if ((threadIdx.x & 63) == 0 && nsp) atomicAdd(&a.ctr->n_special, nsp);
}

__global__ void __launch_bounds__(kBlock) sess2_range_kernel(Sess2Args a) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n_in; j += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long o = jm::ord_i64(a.in.start[j]);
        lo = o < lo ? o : lo;
        hi = o > hi ? o : hi;
    }
    wave_minmax(lo, hi, &a.ctr->ts_min, &a.ctr->ts_max);
}

// Pass 2: route every record and in-flight session to the bulk sort or the arrival-order sort. A block
// owns a contiguous chunk of kRouteItems * blockDim elements and reserves its two output runs with one
// atomic per list (a per-wave reservation on one counter serialised 1M waves per push: 12.8 ms on C5s).
constexpr int kRouteItems = 16;
__device__ __forceinline__ void route_elem(const Sess2Args& a, int64_t t, bool& valid, bool& sp, unsigned long long& bk,
                                           unsigned long long& sk, uint32_t& pay) {
    valid = false; sp = false; bk = 0; sk = 0; pay = 0;
    if (t < a.n) {
        const uint32_t kid = a.rkid[t];
        if (kid == 0xffffffffu) return;
        valid = true;
        sp = a.all_sp || a.kflag[kid];
        pay = (uint32_t)t;
        bk = ((unsigned long long)kid << a.tb) | (uint64_t)(a.ts[t] - a.base);
        sk = ((unsigned long long)kid << 32) | (uint64_t)(t + 1);
    } else if (t < a.n + a.n_in) {
        const int64_t j = t - a.n;
        const uint32_t kid = a.in.kid[j];
        valid = true;
        sp = a.all_sp || a.kflag[kid];
        pay = (uint32_t)j | 0x80000000u;
        bk = ((unsigned long long)kid << a.tb) | (uint64_t)(a.in.start[j] - a.base);
        sk = (unsigned long long)kid << 32;
    }
}

__global__ void __launch_bounds__(kBlock) sess2_route_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    constexpr int kW = kBlock / 64;
    __shared__ uint32_t s_wb[kW], s_ws[kW];
    __shared__ unsigned long long s_base[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * kBlock * kRouteItems;
    uint32_t nbk = 0, nsp = 0;
    for (int j = 0; j < kRouteItems; ++j) {
        bool valid, sp; unsigned long long bk, sk; uint32_t pay;
        route_elem(a, c0 + (int64_t)j * kBlock + threadIdx.x, valid, sp, bk, sk, pay);
        nbk += (uint32_t)__popcll(__ballot(valid && !sp));
        nsp += (uint32_t)__popcll(__ballot(valid && sp));
    }
    if (lane == 0) { s_wb[wv] = nbk; s_ws[wv] = nsp; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tb = 0, ts = 0;
        for (int w = 0; w < kW; ++w) { const uint32_t x = s_wb[w], y = s_ws[w]; s_wb[w] = tb; s_ws[w] = ts; tb += x; ts += y; }
        s_base[0] = tb ? atomicAdd(&a.ctr->n_bulk, (unsigned long long)tb) : 0ull;
        s_base[1] = ts ? atomicAdd(&a.ctr->n_sp, (unsigned long long)ts) : 0ull;
    }
    __syncthreads();
    unsigned long long pb = s_base[0] + s_wb[wv], ps = s_base[1] + s_ws[wv];
    const unsigned long long lt = (1ull << lane) - 1;
    for (int j = 0; j < kRouteItems; ++j) {
        bool valid, sp; unsigned long long bk, sk; uint32_t pay;
        route_elem(a, c0 + (int64_t)j * kBlock + threadIdx.x, valid, sp, bk, sk, pay);
        const unsigned long long mb = __ballot(valid && !sp), ms = __ballot(valid && sp);
        if (valid && !sp) {
            const unsigned long long o = pb + __popcll(mb & lt);
            a.bkey[o] = bk;
            const bool sess = (pay & 0x80000000u) != 0;
            const bool flag = sess || a.gapc;
            a.bval[o] = (uint32_t)o | (flag ? 0x80000000u : 0u);
            unsigned long long* row = a.pk + (int64_t)o * a.pkw;
            const int64_t x = (int64_t)(pay & 0x7fffffffu);
            const EngineConst& c = *cp;
            auto word = [&](int cc) -> unsigned long long {
                if (sess) return a.in.acc[(int64_t)cc * a.in.stride + x];
                if (cc == 0) return 1ull;
                const AggDesc& d = c.agg[a.col_owner[cc]];
                return acc_input(d, a.cols[d.col], x, a.nulls[d.col]);
            };
            int cc = 0;
            if ((a.pkw & 1) == 0)                                  // 16-byte stores (rows stay 16-byte aligned)
                for (; cc < a.pkw; cc += 2) *reinterpret_cast<ulonglong2*>(row + cc) = make_ulonglong2(word(cc), word(cc + 1));
            for (; cc < a.pkw; ++cc) row[cc] = word(cc);
            if (sess) a.pe[o] = a.in.end[x];
            else if (a.gapc) a.pe[o] = jm::wadd(a.ts[x], a.gapc[x]);
        }
        if (valid && sp) { const unsigned long long o = ps + __popcll(ms & lt); a.skey[o] = sk; a.sval[o] = pay; }
        pb += __popcll(mb);
        ps += __popcll(ms);
    }
}

// Bulk: end of every sorted element (records: start + gap; sessions: their end).
__global__ void __launch_bounds__(kBlock) sess2_ends_kernel(Sess2Args a) {
    const uint64_t smask = a.tb >= 64 ? ~0ull : (((uint64_t)1 << a.tb) - 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.nb; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = a.bval[i];
        const int64_t start = a.base + (int64_t)(a.bkey[i] & smask);
        a.bend[i] = (p & 0x80000000u) ? a.pe[p & 0x7fffffffu] : jm::wadd(start, a.gap);
    }
}

// Bulk: head flag = first element of a key, or start after every earlier end of the key.
__global__ void __launch_bounds__(kBlock) sess2_heads_kernel(Sess2Args a) {
    const uint64_t smask = (((uint64_t)1 << a.tb) - 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.nb; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = 1;
        if (i > 0) {
            const unsigned long long k = a.bkey[i], kp = a.bkey[i - 1];
            h = ((k >> a.tb) != (kp >> a.tb) || a.base + (int64_t)(k & smask) > a.bmax[i - 1]) ? 1u : 0u;
        }
        a.bcid[i] = h;
    }
}


__device__ __forceinline__ void acc_atomic(int acc_kind, unsigned long long* p, unsigned long long v) {
    switch (acc_kind) {
        case ACC_NONE: case ACC_ADD_I64: atomicAdd(p, v); break;
        case ACC_ADD_F64: atomicAdd((double*)p, __longlong_as_double((long long)v)); break;
        case ACC_MIN_ORD: atomicMin(p, v); break;
        case ACC_MAX_ORD: atomicMax(p, v); break;
        default: break;
    }
}

__global__ void __launch_bounds__(kBlock) sess2_init_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int64_t ncl = a.nb > 0 ? (int64_t)a.bcid[a.nb - 1] : 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ncl; j += (int64_t)gridDim.x * blockDim.x)
        for (int cc = 0; cc < c.nacc; ++cc) a.out.acc[(int64_t)cc * a.out.stride + j] = cc == 0 ? 0ull : ident_of(c.acc_kind[cc]);
}

// Bulk: wave-segmented reduction of each cluster (COUNT + accumulator columns). The cluster's true
// head writes kid and start, its true tail the end (= the key's running max end there); accumulators
// of a cluster that lies inside one wave are written with plain stores, a cluster spanning waves is
// combined into identity-initialised columns with atomics.
__global__ void __launch_bounds__(kBlock) sess2_reduce_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int lane = threadIdx.x & 63;
    const uint64_t smask = (((uint64_t)1 << a.tb) - 1);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w0 = (int64_t)blockIdx.x * blockDim.x; w0 < a.nb; w0 += stride) {   // uniform trips per wave
        const int64_t wb = w0 + (threadIdx.x & ~63);     // this wave's first element
        const int64_t i = w0 + threadIdx.x;
        const bool act = i < a.nb;
        const int64_t cid = act ? (int64_t)a.bcid[i] : -1 - lane;   // inactive lanes: distinct ids
        const uint32_t p = act ? a.bval[i] : 0u;
        const int64_t cid0 = __shfl(cid, 0);
        const bool head0 = wb < a.nb && (wb == 0 || a.bcid[wb] != a.bcid[wb - 1]);
        const int64_t cn = __shfl_down(cid, 1);
        const bool last = act && (i + 1 >= a.nb || a.bcid[i + 1] != (uint32_t)cid);   // cluster's true tail
        const bool tail = act && (lane == 63 || cn != cid);                          // its last lane here
        const bool whole = (cid != cid0 || head0) && (lane != 63 || last);
        const int64_t cl = cid - 1;
        if (act && (i == 0 || a.bcid[i - 1] != (uint32_t)cid)) {
            a.out.kid[cl] = (uint32_t)(a.bkey[i] >> a.tb);
            a.out.start[cl] = a.base + (int64_t)(a.bkey[i] & smask);
        }
        if (last) a.out.end[cl] = a.bmax[i];
        for (int cc = 0; cc < c.nacc; ++cc) {
            const int ak = cc == 0 ? ACC_ADD_I64 : c.acc_kind[cc];
            unsigned long long v = act ? a.pk[(int64_t)(p & 0x7fffffffu) * a.pkw + cc] : 0ull;
            for (int d = 1; d < 64; d <<= 1) {
                const unsigned long long y = __shfl_up(v, d);
                const int64_t yc = __shfl_up(cid, d);
                if (lane >= d && yc == cid) v = acc_combine(ak, v, y);
            }
            if (!tail) continue;
            unsigned long long* dst = &a.out.acc[(int64_t)cc * a.out.stride + cl];
            if (whole) *dst = v;
            else acc_atomic(ak, dst, v);
        }
    }
}

// Bulk sessions after the (kid, start) sort in one pass, replacing ends / scan-by-key / heads / cluster-id scan /
// reduce: wave w owns the keys whose first sorted element lies in positions [64w, 64w + 64) and walks each owned key
// to its end in 64-element chunks, carrying the open cluster (the session being built) from chunk to chunk. Per chunk:
// the ends (start + gap, or the element's own end), the key's running max end (segmented shuffle scan; lane 0 joins
// the carried key), cluster heads (a new key, or a start after every earlier end of the key: TimeWindow.intersects is
// inclusive, so touching windows merge), the accumulators per cluster (segmented shuffle scans over the packed
// rows) and the completed clusters appended to the output list (one reservation per wave and chunk).
template <int NA>
__global__ void __launch_bounds__(kBlock) sess2_segment_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int lane = threadIdx.x & 63;
    const uint64_t smask = ((uint64_t)1 << a.tb) - 1;              // tb <= 63 - kid bits on this path
    const int64_t nb = a.nb;
    const int64_t nw = (nb + 63) >> 6;
    const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
    int ak[NA];
#pragma unroll
    for (int cc = 0; cc < NA; ++cc) ak[cc] = cc == 0 ? ACC_ADD_I64 : c.acc_kind[cc];
    const unsigned long long below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // lanes <= this one
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const int64_t p0 = w << 6;
        // a window of 128 sorted positions (this wave's 64 and the next 64) and the element before, loaded at once:
        // the heads, the end of the last owned key and the first two chunks come from it (one round trip)
        const int64_t pa = p0 + lane, pb = p0 + 64 + lane;
        const unsigned long long kA = pa < nb ? a.bkey[pa] : 0ull, kB = pb < nb ? a.bkey[pb] : 0ull;
        const uint32_t vA = pa < nb ? a.bval[pa] : 0u, vB = pb < nb ? a.bval[pb] : 0u;
        const unsigned long long kprev = p0 > 0 ? a.bkey[p0 - 1] : 0ull;
        const uint32_t kidA = (uint32_t)(kA >> a.tb), kidB = (uint32_t)(kB >> a.tb);
        const uint32_t kup = __shfl_up(kidA, 1);
        const bool hd = pa < nb && (lane == 0 ? (p0 == 0 || (uint32_t)(kprev >> a.tb) != kidA) : kidA != kup);
        const unsigned long long hm = __ballot(hd);
        if (!hm) {                                                  // inside a key owned by an earlier wave
            if (lane == 0) a.sg_cnt[w] = 0u;
            continue;
        }
        const int64_t h0 = p0 + (__ffsll((long long)hm) - 1);
        uint32_t wc = 0;                                            // clusters this wave wrote (staging h0 + i)
        int64_t h1 = min(p0 + 64, nb);
        if (h1 < nb) {                                              // the last owned key may run past the range
            const uint32_t kl = __shfl(kidA, 63);
            const unsigned long long dm = __ballot(pb >= nb || kidB != kl);
            if (dm) h1 = p0 + 64 + (__ffsll((long long)dm) - 1);
            else
                for (int64_t q = p0 + 128;; q += 64) {
                    const int64_t pp = q + lane;
                    const unsigned long long dq = __ballot(pp >= nb || (uint32_t)(a.bkey[pp] >> a.tb) != kl);
                    if (dq) { h1 = q + (__ffsll((long long)dq) - 1); break; }
                }
        }
        // chunk loads: key, payload, end, accumulator row of position base + lane (window or memory)
        auto fetch = [&](int64_t base, unsigned long long& bk, uint32_t& pay, int64_t& en, unsigned long long* x) {
            const int64_t q = base + lane;
            const int64_t d = q - p0;
            if (base + 63 - p0 < 128) {                             // inside the window
                const int src = (int)(d & 63);
                const unsigned long long ka = __shfl(kA, src), kb = __shfl(kB, src);
                const uint32_t va = __shfl(vA, src), vb = __shfl(vB, src);
                bk = d < 64 ? ka : kb;
                pay = d < 64 ? va : vb;
            } else {
                bk = q < h1 ? a.bkey[q] : 0ull;
                pay = q < h1 ? a.bval[q] : 0u;
            }
            const bool v = q < h1;
            const int64_t st = a.base + (int64_t)(bk & smask);
            en = !v ? LONG_MIN_J : (pay & 0x80000000u) ? a.pe[pay & 0x7fffffffu] : jm::wadd(st, a.gap);
            const uint32_t o = pay & 0x7fffffffu;
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) x[cc] = v ? a.pk[(int64_t)o * a.pkw + cc] : 0ull;
        };
        uint32_t ck = 0u;                                           // the carried open cluster
        int64_t cmax = LONG_MIN_J, cst = 0;
        unsigned long long cacc[NA];
#pragma unroll
        for (int cc = 0; cc < NA; ++cc) cacc[cc] = 0ull;
        bool copen = false;
        unsigned long long nbk, nx[NA];                             // the next chunk, in flight (software pipeline)
        uint32_t npay;
        int64_t nen;
        fetch(h0, nbk, npay, nen, nx);
        for (int64_t base = h0; base < h1; base += 64) {
            const int64_t q = base + lane;
            const bool v = q < h1;
            const unsigned long long bk = nbk;
            const int64_t en = nen;
            unsigned long long acc[NA];
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) acc[cc] = nx[cc];
            if (base + 64 < h1) fetch(base + 64, nbk, npay, nen, nx);
            const uint32_t kk = (uint32_t)(bk >> a.tb);
            const int64_t st = a.base + (int64_t)(bk & smask);
            const uint32_t kp = __shfl_up(kk, 1);
            const bool kc = v && (lane == 0 ? (!copen || kk != ck) : kk != kp);
            const unsigned long long km = __ballot(kc) & below;
            const int ks = km ? 63 - __clzll((long long)km) : 0;   // first lane of this lane's key in the chunk
            int64_t m = en;                                         // running max end of the key (inclusive)
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t y = __shfl_up(m, d);
                if (lane - d >= ks && y > m) m = y;
            }
            if (km == 0 && copen && cmax > m) m = cmax;            // the key continues from the previous chunk
            int64_t mprev = __shfl_up(m, 1);
            if (lane == 0) mprev = cmax;
            const bool head = v && (kc || st > mprev);
            const unsigned long long hb = __ballot(head) & below;
            const int cs = hb ? 63 - __clzll((long long)hb) : 0;   // first lane of this lane's cluster in the chunk
            const bool ccont = hb == 0;                            // still the carried cluster
            const int64_t hst = __shfl(st, cs);
            const int64_t cstart = ccont ? cst : hst;
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) {
                unsigned long long x = acc[cc];
                for (int d = 1; d < 64; d <<= 1) {
                    const unsigned long long y = __shfl_up(x, d);
                    if (lane - d >= cs) x = acc_combine(ak[cc], x, y);
                }
                if (ccont && copen) x = acc_combine(ak[cc], cacc[cc], x);
                acc[cc] = x;
            }
            const bool nxt = __shfl_down(head ? 1 : 0, 1) != 0;
            const bool tail = v && (q + 1 == h1 || (lane < 63 && nxt));
            const bool emit_c = copen && __shfl(head ? 1 : 0, 0) != 0;   // the carried cluster ended before lane 0
            if (emit_c && lane == 0) {
                const int64_t sc = h0 + (int64_t)wc;
                a.sg_kid[sc] = ck;
                a.sg_start[sc] = cst;
                a.sg_end[sc] = cmax;
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) a.sg_acc[(int64_t)cc * a.sg_cap + sc] = cacc[cc];
            }
            wc += emit_c ? 1u : 0u;
            const unsigned long long tm = __ballot(tail);
            if (tail) {
                const int64_t so = h0 + (int64_t)wc + __popcll(tm & ((1ull << lane) - 1ull));
                a.sg_kid[so] = kk;
                a.sg_start[so] = cstart;
                a.sg_end[so] = m;                                   // the key's max end at the cluster's last element
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) a.sg_acc[(int64_t)cc * a.sg_cap + so] = acc[cc];
            }
            wc += (uint32_t)__popcll(tm);
            ck = __shfl(kk, 63);
            cmax = __shfl(m, 63);
            cst = __shfl(cstart, 63);
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) cacc[cc] = __shfl(acc[cc], 63);
            copen = true;
        }
        if (lane == 0) { a.sg_cnt[w] = wc; a.sg_h0[w] = h0; }
    }
}

// The segment kernel's clusters, moved from each wave's staging range to the output list at the exclusive sum of the
// per-wave counts (one thread per wave; the arrival-order path appends after them on ctr->n_out_sp).
// One thread per output session (coalesced stores): the staging wave w that owns output dst is the last one with
// sg_off[w] <= dst (a binary search over the scanned counts, which stay cache-resident); a thread per wave copying its
// ~1.4 clusters serially took 0.24 ms per C5s push.
__global__ void __launch_bounds__(kBlock) sess2_compact_kernel(Sess2Args a, int64_t nw, int nacc) {
    const int64_t tot = a.sg_off[nw];
    for (int64_t dst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; dst < tot; dst += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = nw;                          // invariant: sg_off[lo] <= dst < sg_off[hi]
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)a.sg_off[mid] <= dst) lo = mid; else hi = mid;
        }
        const int64_t src = a.sg_h0[lo] + (dst - (int64_t)a.sg_off[lo]);
        a.out.kid[dst] = a.sg_kid[src];
        a.out.start[dst] = a.sg_start[src];
        a.out.end[dst] = a.sg_end[src];
        for (int cc = 0; cc < nacc; ++cc) a.out.acc[(int64_t)cc * a.out.stride + dst] = a.sg_acc[(int64_t)cc * a.sg_cap + src];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctr->n_out_sp = (unsigned long long)tot;
}

// ---- Cell path: fixed gap, every record of the push order-free ------------------------------------------------------
// The time axis is cut into cells of width gap starting at base = the smallest start of the push. Two windows whose
// starts lie in one cell intersect (s2 - s1 < gap <= end1 - s1, TimeWindow.intersects), so the elements of one
// (kid, cell) group end in one session whatever their order: sorting by the 32-bit key kid << cb | cell (cb = 32 -
// kid_bits) replaces the (kid, start) sort (4 one-byte passes over 8-byte pairs instead of 5 over 12-byte pairs), and
// the segment walk reduces each group (min start, max end, accumulators) before chaining the key's groups in cell
// order. Records go to the sort at their input position (no compaction); a record that is not order-free or a start
// outside the cell range is counted and the host redoes the push on the general path (sess2_*).
constexpr uint32_t kCellSent = 0xffffffffu;        // sorts last; its kid (all ones in kid_bits) is never a real kid

__global__ void __launch_bounds__(kBlock) sess3_min_kernel(Sess2Args a) {
    __shared__ unsigned long long s_lo[kBlock / 64];
    unsigned long long lo = ~0ull;
    const int64_t tot = a.n + a.n_in;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long o = jm::ord_i64(t < a.n ? a.ts[t] : a.in.start[t - a.n]);
        lo = o < lo ? o : lo;
    }
    for (int sh = 32; sh >= 1; sh >>= 1) { const unsigned long long y = __shfl_xor(lo, sh); lo = y < lo ? y : lo; }
    if ((threadIdx.x & 63) == 0) s_lo[threadIdx.x >> 6] = lo;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) lo = s_lo[w] < lo ? s_lo[w] : lo;
        if (lo != ~0ull) atomicMin(&a.ctr->ts_min, lo);
    }
}

// Probe of the key's first 8-slot bucket (one 64-byte read); -1 when the key is not there (then key_slot, which also
// inserts). Loads only: the caller issues several before using any.
__device__ __forceinline__ int64_t key_probe8(const unsigned long long* table, int seg_log, int part_bits, int64_t key,
                                             ulonglong2 (&bk)[4], uint64_t& i0) {
    const uint64_t h = jm::mix64((uint64_t)key);
    const uint64_t smask = ((uint64_t)1 << seg_log) - 1;
    i0 = seg_base(h, seg_log, part_bits) | (h & smask & ~(uint64_t)(kBucket - 1));
    const ulonglong2* p = reinterpret_cast<const ulonglong2*>(table + i0);
#pragma unroll
    for (int j = 0; j < 4; ++j) bk[j] = p[j];
    return 0;
}
__device__ __forceinline__ int64_t key_probe8_find(const ulonglong2 (&bk)[4], uint64_t i0, int64_t key) {
    const unsigned long long k = (unsigned long long)key;
    int64_t r = -1;
#pragma unroll
    for (int j = 3; j >= 0; --j) {
        if (bk[j].y == k) r = (int64_t)(i0 + 2 * j + 1);
        if (bk[j].x == k) r = (int64_t)(i0 + 2 * j);
    }
    return r;
}

// Records: block b routes its chunk [b * chunk, (b + 1) * chunk): key-group check, kid (U records' bucket probes in
// flight at once), 32-bit cell key and payload (the row position) at the record's input position, and the packed row
// [ts, acc_1 .. acc_{nacc-1}] (COUNT is 1 for a record) at the same position.
template <int U>
__global__ void __launch_bounds__(kBlock) sess3_route_kernel(Sess2Args a, const EngineConst* __restrict__ cp, int64_t chunk) {
    __shared__ uint32_t s_c[2];
    const EngineConst& c = *cp;
    if (threadIdx.x == 0) { s_c[0] = 0u; s_c[1] = 0u; }
    __syncthreads();
    const int cb = a.tb;
    const uint64_t ncell = (uint64_t)1 << cb;
    const uint64_t base = (uint64_t)jm::unord_i64(a.ctr->ts_min);
    uint32_t nsp = 0, nredo = 0;
    uint32_t* bkey = reinterpret_cast<uint32_t*>(a.bkey);
    const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(a.n, r0 + chunk);
    for (int64_t t0 = r0 + threadIdx.x; t0 < r1; t0 += (int64_t)blockDim.x * U) {
        int64_t key[U], ts[U], kid[U];
        ulonglong2 bk[U][4];
        uint64_t i0[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t = t0 + (int64_t)u * blockDim.x;
            key[u] = t < r1 ? a.keys[t] : 0;
            ts[u] = t < r1 ? a.ts[t] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) key_probe8(a.key_table, a.seg_log, a.part_bits, key[u], bk[u], i0[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t = t0 + (int64_t)u * blockDim.x;
            if (t >= r1) continue;
            uint32_t k32 = kCellSent;
            kid[u] = -1;
            const int32_t kg = jm::key_group_of(key[u], c.key_kind, a.key_hash ? a.key_hash[t] : 0, c.max_par);
            if (kg < c.kg_lo || kg > c.kg_hi) {
                raise_error(a.st, FWA_E_KEYGROUP);                     // StateTable :300-307
            } else {
                kid[u] = (uint64_t)key[u] == kEmptyKey ? -1 : key_probe8_find(bk[u], i0[u], key[u]);
                if (kid[u] < 0) kid[u] = key_slot(a.key_table, a.key_mask, a.seg_log, a.part_bits, key[u], a.st);
                if (kid[u] < 0) {
                    a.st->key_full = 1;
                    raise_error(a.st, FWA_E_OOM);
                } else if (jm::wsub(jm::wadd(ts[u], a.gap), 1) <= a.wm) {   // order-sensitive: the general path
                    a.kflag[kid[u]] = 1;
                    ++nsp;
                } else {
                    const uint64_t cell = jm::udiv64((uint64_t)ts[u] - base, a.gap_div);
                    if (cell >= ncell) ++nredo;
                    else k32 = ((uint32_t)kid[u] << cb) | (uint32_t)cell;
                }
            }
            uint32_t pos = 0u;
            if (k32 != kCellSent) {
                pos = (uint32_t)t;
                unsigned long long* row = a.pk + (int64_t)pos * a.pkw;
                const int64_t tsu = ts[u];
                auto word = [&](int cc) -> unsigned long long {
                    if (cc == 0) return (unsigned long long)tsu;
                    const AggDesc& d = c.agg[a.col_owner[cc]];
                    return acc_input(d, a.cols[d.col], t, a.nulls[d.col]);
                };
                int cc = 0;
                if ((a.pkw & 1) == 0)
                    for (; cc < a.pkw; cc += 2) *reinterpret_cast<ulonglong2*>(row + cc) = make_ulonglong2(word(cc), word(cc + 1));
                for (; cc < a.pkw; ++cc) row[cc] = word(cc);
            }
            bkey[t] = k32;
            a.bval[t] = pos;
        }
    }
    for (int sh = 32; sh >= 1; sh >>= 1) { nsp += __shfl_xor(nsp, sh); nredo += __shfl_xor(nredo, sh); }
    if ((threadIdx.x & 63) == 0 && (nsp | nredo)) { atomicAdd(&s_c[0], nsp); atomicAdd(&s_c[1], nredo); }
    __syncthreads();
    if (threadIdx.x == 0 && s_c[0]) atomicAdd(&a.ctr->n_special, (unsigned long long)s_c[0]);
    if (threadIdx.x == 0 && s_c[1]) atomicAdd(&a.ctr->n_redo, (unsigned long long)s_c[1]);
}

// In-flight sessions at sort positions n + j: cell key of their start, payload j | 0x80000000.
__global__ void __launch_bounds__(kBlock) sess3_route_sessions_kernel(Sess2Args a) {
    const int cb = a.tb;
    const uint64_t ncell = (uint64_t)1 << cb;
    const uint64_t base = (uint64_t)jm::unord_i64(a.ctr->ts_min);
    uint32_t* bkey = reinterpret_cast<uint32_t*>(a.bkey);
    uint32_t nredo = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n_in; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t cell = jm::udiv64((uint64_t)a.in.start[j] - base, a.gap_div);
        uint32_t k32 = kCellSent;
        if (cell >= ncell) ++nredo;
        else k32 = (a.in.kid[j] << cb) | (uint32_t)cell;
        bkey[a.n + j] = k32;
        a.bval[a.n + j] = (uint32_t)j | 0x80000000u;
    }
    for (int sh = 32; sh >= 1; sh >>= 1) nredo += __shfl_xor(nredo, sh);
    if ((threadIdx.x & 63) == 0 && nredo) atomicAdd(&a.ctr->n_redo, (unsigned long long)nredo);
}

__device__ __forceinline__ uint32_t perm32(int dst4, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_permute(dst4, (int)v); }
__device__ __forceinline__ unsigned long long perm64(int dst4, unsigned long long v) {
    const uint32_t lo = perm32(dst4, (uint32_t)v), hi = perm32(dst4, (uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// Cross-lane moves on the VALU (DPP) instead of the LDS crossbar: row_shr:n = 0x110 + n, row_bcast:15 = 0x142,
// row_bcast:31 = 0x143, wave_shl:1 = 0x130, wave_shr:1 = 0x138 (lanes without a source get 0)
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ unsigned long long dpp64(unsigned long long v) {
    return ((unsigned long long)dpp32<CTRL, RM>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL, RM>((uint32_t)v);
}
__device__ __forceinline__ unsigned long long rdlane64(unsigned long long v, int l) {   // wave-uniform l
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rdlane32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// Segmented inclusive scans: lane L combines the lanes [gs(L), L] (gs = first lane of L's segment) with the earlier
// part as the second operand. Hillis-Steele inside rows of 16 (row_shr 1, 2, 4, 8), then the row totals (row_bcast 15
// / 31); one accumulator kind per scan, branch-free (selects; the kind switch is taken once per scan, not per step).
template <int K>
__device__ __forceinline__ unsigned long long comb_k(unsigned long long x, unsigned long long y) {
    if constexpr (K == ACC_ADD_I64) return x + y;
    else if constexpr (K == ACC_ADD_F64)
        return (unsigned long long)__double_as_longlong(__longlong_as_double((long long)x) + __longlong_as_double((long long)y));
    else if constexpr (K == ACC_MIN_ORD) return y < x ? y : x;
    else if constexpr (K == ACC_MAX_ORD) return y > x ? y : x;
    else return x;
}
template <int K>
__device__ __forceinline__ unsigned long long seg_scan_k(unsigned long long x, int lane, int gs) {
    unsigned long long y, r;
    y = dpp64<0x111>(x); r = comb_k<K>(x, y); x = ((lane & 15) >= 1 && lane - 1 >= gs) ? r : x;
    y = dpp64<0x112>(x); r = comb_k<K>(x, y); x = ((lane & 15) >= 2 && lane - 2 >= gs) ? r : x;
    y = dpp64<0x114>(x); r = comb_k<K>(x, y); x = ((lane & 15) >= 4 && lane - 4 >= gs) ? r : x;
    y = dpp64<0x118>(x); r = comb_k<K>(x, y); x = ((lane & 15) >= 8 && lane - 8 >= gs) ? r : x;
    y = dpp64<0x142, 0xa>(x); r = comb_k<K>(x, y); x = ((lane & 16) != 0 && gs < (lane & ~15)) ? r : x;
    y = dpp64<0x143, 0xc>(x); r = comb_k<K>(x, y); x = (lane >= 32 && gs < 32) ? r : x;
    return x;
}
__device__ __forceinline__ unsigned long long seg_scan_acc(int k, unsigned long long x, int lane, int gs) {
    switch (k) {
        case ACC_ADD_I64: return seg_scan_k<ACC_ADD_I64>(x, lane, gs);
        case ACC_ADD_F64: return seg_scan_k<ACC_ADD_F64>(x, lane, gs);
        case ACC_MIN_ORD: return seg_scan_k<ACC_MIN_ORD>(x, lane, gs);
        case ACC_MAX_ORD: return seg_scan_k<ACC_MAX_ORD>(x, lane, gs);
        default: return x;
    }
}
__device__ __forceinline__ int64_t seg_min64(int64_t x, int lane, int gs) {   // ord encoding: unsigned min
    return jm::unord_i64(seg_scan_k<ACC_MIN_ORD>(jm::ord_i64(x), lane, gs));
}
__device__ __forceinline__ int64_t seg_max64(int64_t x, int lane, int gs) {
    return jm::unord_i64(seg_scan_k<ACC_MAX_ORD>(jm::ord_i64(x), lane, gs));
}

// The cell-sorted elements in one pass. Ownership as in sess2_segment_kernel (wave w owns the keys whose first sorted
// element lies in [64w, 64w + 64) and walks each to its end). Per 64-element chunk: (1) segmented scans over the
// (kid, cell) groups -- min start, max end, accumulators -- joined with the group carried from the previous chunk;
// (2) the groups that end in the chunk are packed to the low lanes (ds_permute) and chained as sess2_segment_kernel
// chains elements: a group opens a session if it starts a key or starts after the key's running max end.
template <int NA>
__global__ void __launch_bounds__(kBlock) sess3_segment_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int lane = threadIdx.x & 63;
    const int cb = a.tb;
    const uint32_t* bkey = reinterpret_cast<const uint32_t*>(a.bkey);
    const int64_t nb = a.nb;
    const int64_t nw = (nb + 63) >> 6;
    const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
    int ak[NA];
    unsigned long long idn[NA];
#pragma unroll
    for (int cc = 0; cc < NA; ++cc) { ak[cc] = cc == 0 ? ACC_ADD_I64 : c.acc_kind[cc]; idn[cc] = ident_of(ak[cc]); }
    const unsigned long long below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // lanes <= this one
    const unsigned long long before = (1ull << lane) - 1ull;                          // lanes < this one
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const int64_t p0 = w << 6;
        const int64_t pa = p0 + lane, pb = p0 + 64 + lane;
        const uint32_t kA = pa < nb ? bkey[pa] : kCellSent, kB = pb < nb ? bkey[pb] : kCellSent;
        const uint32_t vA = pa < nb ? a.bval[pa] : 0u, vB = pb < nb ? a.bval[pb] : 0u;
        const uint32_t kprev = p0 > 0 ? bkey[p0 - 1] : kCellSent;
        const uint32_t kidA = kA >> cb;
        const uint32_t kup = __shfl_up(kidA, 1);
        const bool okA = kA != kCellSent;
        const bool hd = okA && (lane == 0 ? (p0 == 0 || (kprev >> cb) != kidA) : kidA != kup);
        const unsigned long long hm = __ballot(hd);
        if (!hm) {
            if (lane == 0) a.sg_cnt[w] = 0u;
            continue;
        }
        const int64_t h0 = p0 + (__ffsll((long long)hm) - 1);
        int64_t h1;
        const unsigned long long sa = __ballot(!okA);               // sentinels / the end inside this range
        if (sa) {
            h1 = p0 + (__ffsll((long long)sa) - 1);
        } else {                                                    // the last owned key may run past the range
            const uint32_t kl = __shfl(kidA, 63);
            const unsigned long long dm = __ballot((kB >> cb) != kl);   // a sentinel's kid differs from every kid
            if (dm) h1 = p0 + 64 + (__ffsll((long long)dm) - 1);
            else
                for (int64_t q = p0 + 128;; q += 64) {
                    const int64_t pp = q + lane;
                    const uint32_t kq = pp < nb ? bkey[pp] : kCellSent;
                    const unsigned long long dq = __ballot((kq >> cb) != kl);
                    if (dq) { h1 = q + (__ffsll((long long)dq) - 1); break; }
                }
        }
        auto fetch = [&](int64_t base, uint32_t& bk, int64_t& st, int64_t& en, unsigned long long* x) {
            const int64_t q = base + lane;
            const int64_t d = q - p0;
            uint32_t pay;
            if (base + 63 - p0 < 128) {                             // inside the loaded window
                const int src = (int)(d & 63);
                const uint32_t ka = __shfl(kA, src), kb = __shfl(kB, src);
                const uint32_t va = __shfl(vA, src), vb = __shfl(vB, src);
                bk = d < 64 ? ka : kb;
                pay = d < 64 ? va : vb;
            } else {
                bk = q < h1 ? bkey[q] : kCellSent;
                pay = q < h1 ? a.bval[q] : 0u;
            }
            const uint32_t o = pay & 0x7fffffffu;
            if (q >= h1) {
                bk = kCellSent;
                st = LONG_MAX_J;
                en = LONG_MIN_J;
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) x[cc] = idn[cc];
            } else if (pay & 0x80000000u) {                         // in-flight session
                st = a.in.start[o];
                en = a.in.end[o];
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) x[cc] = a.in.acc[(int64_t)cc * a.in.stride + o];
            } else {                                                // record: packed row [ts, acc_1 ..]
                const unsigned long long* row = a.pk + (int64_t)o * NA;
                unsigned long long wv[NA];
                if constexpr ((NA & 1) == 0) {
#pragma unroll
                    for (int cc = 0; cc < NA; cc += 2) {
                        const ulonglong2 p = reinterpret_cast<const ulonglong2*>(row)[cc >> 1];
                        wv[cc] = p.x;
                        wv[cc + 1] = p.y;
                    }
                } else {
#pragma unroll
                    for (int cc = 0; cc < NA; ++cc) wv[cc] = row[cc];
                }
                st = (int64_t)wv[0];
                en = jm::wadd(st, a.gap);
                x[0] = 1ull;
#pragma unroll
                for (int cc = 1; cc < NA; ++cc) x[cc] = wv[cc];
            }
        };
        // Carries (wave-uniform): the pending group (its last element not seen yet: its session is undecided) and the
        // open session (every group before the pending one that belongs to it).
        bool gopen = false, copen = false;
        uint32_t gkey = 0u, ck = 0u;
        int64_t gmin = 0, gmax = 0, cmaxe = LONG_MIN_J, cst = 0;
        unsigned long long gacc[NA], cacc[NA];
#pragma unroll
        for (int cc = 0; cc < NA; ++cc) { gacc[cc] = 0ull; cacc[cc] = 0ull; }
        uint32_t wc = 0;                                            // sessions this wave wrote (staging h0 + i)
        uint32_t nbk;
        int64_t nst, nen;
        unsigned long long nx[NA];
        fetch(h0, nbk, nst, nen, nx);
        for (int64_t base = h0; base < h1; base += 64) {
            const int64_t q = base + lane;
            const bool v = q < h1;
            const uint32_t bk = nbk;
            int64_t st = nst, en = nen;
            unsigned long long x[NA];
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) x[cc] = nx[cc];
            const bool more = base + 64 < h1;
            if (more) fetch(base + 64, nbk, nst, nen, nx);
            // (1) groups: min start / max end per (kid, cell) run, joined with the pending group at lane 0
            const uint32_t gup = dpp32<0x138>(bk);                  // lane - 1
            const bool cont0 = gopen && rdlane32(bk, 0) == gkey;    // lane 0 continues the pending group
            const bool gf = v && (lane == 0 ? !cont0 : bk != gup);
            const unsigned long long GF = __ballot(gf);
            const unsigned long long gm = GF & below;
            const int gs = gm ? 63 - __clzll((long long)gm) : 0;
            st = seg_min64(st, lane, gs);
            en = seg_max64(en, lane, gs);
            if (gm == 0 && cont0) {
                st = gmin < st ? gmin : st;
                en = gmax > en ? gmax : en;
            }
            const uint32_t nk0 = rdlane32(nbk, 0);                  // the next chunk's first key (when `more`)
            const uint32_t gdn = dpp32<0x130>(bk);                  // lane + 1
            const bool gt = v && (q + 1 == h1 || (lane < 63 ? gdn != bk : nk0 != bk));   // the group's last element
            const int lv = (int)min<int64_t>(63, h1 - 1 - base);   // last valid lane
            const unsigned long long P = __ballot(gt);
            const bool pend = ((P >> lv) & 1ull) == 0;              // the last group continues in the next chunk
            // (2) chain the groups that end here, packed to lanes [0, np): heads and session tails
            const int np = __popcll(P);
            uint32_t kk = 0u;
            int64_t gst = 0, m = LONG_MIN_J, cstart = 0;
            bool head = false, ptail = false;
            unsigned long long H = 0ull;
            if (np) {
                const int dst = gt ? __popcll(P & before) : np + __popcll(~P & before);
                kk = perm32(dst * 4, bk >> cb);
                gst = (int64_t)perm64(dst * 4, (unsigned long long)st);
                const int64_t gen = (int64_t)perm64(dst * 4, (unsigned long long)en);
                const bool range_end = base + lv + 1 == h1;         // the last packed group closes the walk
                const bool pv = lane < np;
                const uint32_t kp = dpp32<0x138>(kk);
                const bool kc = pv && (lane == 0 ? (!copen || kk != ck) : kk != kp);
                const unsigned long long km = __ballot(kc) & below;
                const int ks = km ? 63 - __clzll((long long)km) : 0;
                m = seg_max64(pv ? gen : LONG_MIN_J, lane, ks);     // running max end of the key (inclusive)
                if (km == 0 && copen && cmaxe > m) m = cmaxe;       // the key continues from the open session
                int64_t mprev = (int64_t)dpp64<0x138>((unsigned long long)m);
                if (lane == 0) mprev = cmaxe;
                head = pv && (kc || gst > mprev);
                H = __ballot(head);
                const unsigned long long hb = H & below;
                const int cs = hb ? 63 - __clzll((long long)hb) : 0;
                const int64_t hst = __shfl(gst, cs);
                cstart = hb == 0 ? cst : hst;
                ptail = pv && (lane == np - 1 ? range_end : (lane < 63 && ((H >> ((lane + 1) & 63)) & 1ull) != 0));
            }
            // (3) accumulators once, per element, segmented by session: a segment starts at lane 0, at the first
            // element of every head group, and at the first element of the pending group
            const unsigned long long Pge = P & ~before;             // groups ending at or after this lane
            const int tl = Pge ? __ffsll((long long)Pge) - 1 : 64;  // this lane's group tail (64: pending group)
            const int rk = __popcll(P & ((tl < 64) ? ((1ull << tl) - 1ull) : ~0ull));   // its packed rank
            const bool ghead = tl < 64 && ((H >> rk) & 1ull) != 0;
            const unsigned long long SS = __ballot(v && gf && (tl == 64 || ghead)) | 1ull;
            const unsigned long long sm = SS & below;
            const int ss = 63 - __clzll((long long)sm);
            // prefix of the first segment: the open session unless its first group is a head, then the pending group
            // that lane 0 continues
            const bool g0end = (P & ~0ull) != 0;                    // the group at lane 0 ends in this chunk
            const bool pre_c = copen && g0end && (H & 1ull) == 0;
            const bool pre_g = cont0;
#pragma unroll
            for (int cc = 0; cc < NA; ++cc) {
                unsigned long long xx = seg_scan_acc(ak[cc], x[cc], lane, ss);
                if (ss == 0 && pre_g) xx = acc_combine(ak[cc], xx, gacc[cc]);
                if (ss == 0 && pre_c) xx = acc_combine(ak[cc], xx, cacc[cc]);
                x[cc] = xx;
            }
            // the open session ended before the first group here
            const bool emit_c = copen && np > 0 && (H & 1ull) != 0;
            if (emit_c && lane == 0) {
                const int64_t sc = h0 + (int64_t)wc;
                a.sg_kid[sc] = ck;
                a.sg_start[sc] = cst;
                a.sg_end[sc] = cmaxe;
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) a.sg_acc[(int64_t)cc * a.sg_cap + sc] = cacc[cc];
            }
            wc += emit_c ? 1u : 0u;
            // sessions ending at an element lane (the tail of a packed group whose session ends)
            const int rsrc = gt ? __popcll(P & before) : 0;
            const int ptl = __shfl(ptail ? 1 : 0, rsrc);           // every lane takes part in the shuffle
            const bool etail = gt && ptl != 0;
            const int64_t e_start = __shfl(cstart, rsrc);
            const int64_t e_end = __shfl(m, rsrc);
            const unsigned long long tm = __ballot(etail);
            if (etail) {
                const int64_t so = h0 + (int64_t)wc + __popcll(tm & before);
                a.sg_kid[so] = bk >> cb;
                a.sg_start[so] = e_start;
                a.sg_end[so] = e_end;
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) a.sg_acc[(int64_t)cc * a.sg_cap + so] = x[cc];
            }
            wc += (uint32_t)__popcll(tm);
            // carries
            if (np) {
                const int tlast = 63 - __clzll((long long)P);       // element lane of the last ended group
                ck = rdlane32(kk, np - 1);
                cmaxe = (int64_t)rdlane64((unsigned long long)m, np - 1);
                cst = (int64_t)rdlane64((unsigned long long)cstart, np - 1);
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) cacc[cc] = rdlane64(x[cc], tlast);
                copen = true;
            }
            gopen = pend;
            if (pend) {
                gkey = rdlane32(bk, lv);
                gmin = (int64_t)rdlane64((unsigned long long)st, lv);
                gmax = (int64_t)rdlane64((unsigned long long)en, lv);
#pragma unroll
                for (int cc = 0; cc < NA; ++cc) gacc[cc] = rdlane64(x[cc], lv);
            }
        }
        if (lane == 0) { a.sg_cnt[w] = wc; a.sg_h0[w] = h0; }
    }
}

__device__ __forceinline__ int64_t sess_key_of(const unsigned long long* key_table, int64_t capacity, uint32_t kid) {
    return (int64_t)kid < capacity ? (int64_t)key_table[kid] : LONG_MIN_J;   // side slot: the sentinel key
}

// Arrival-order path: one lane per key run of the (kid, arrival)-sorted list; its in-flight sessions
// come first (low word 0), then its records in arrival order. The run's scratch region [t, t + len)
// holds its session list (a run of len elements never has more than len sessions).
__global__ void __launch_bounds__(kBlock) sess2_ordered_kernel(Sess2Args a, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int nacc = c.nacc;
    const bool table = c.sem == FWA_SEM_TABLE;
    const int64_t ncl = (a.seg_out || a.nb == 0) ? 0 : (int64_t)a.bcid[a.nb - 1];
    unsigned long long dropped = 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < a.nsp; t += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t kid = (uint32_t)(a.skey[t] >> 32);
        if (t > 0 && (uint32_t)(a.skey[t - 1] >> 32) == kid) continue;   // not the head of the key's run
        int64_t* ss = a.sc_start + t;
        int64_t* se = a.sc_end + t;
        auto acc = [&](int cc, int64_t s) -> unsigned long long& { return a.sc_acc[(int64_t)cc * a.nsp + t + s]; };
        int64_t ns = 0;
        bool failed = false;
        for (int64_t j = t; j < a.nsp && (uint32_t)(a.skey[j] >> 32) == kid && !failed; ++j) {
            const uint32_t p = a.sval[j];
            if (p & 0x80000000u) {                              // an in-flight session of this key
                const int64_t q = p & 0x7fffffffu;
                ss[ns] = a.in.start[q];
                se[ns] = a.in.end[q];
                for (int cc = 0; cc < nacc; ++cc) acc(cc, ns) = a.in.acc[(int64_t)cc * a.in.stride + q];
                ++ns;
                continue;
            }
            const int64_t r = p;
            const int64_t ts = a.ts[r];
            const int64_t ws = ts, we = jm::wadd(ts, a.gapc ? a.gapc[r] : a.gap);   // EventTimeSessionWindows.assignWindows :61-63
            // MergingWindowSet.addWindow: the in-flight sessions intersecting the new window
            int64_t first = -1, nm = 0, cs = ws, ce = we;
            bool covers = false;
            for (int64_t s = 0; s < ns; ++s) {
                if (!(ss[s] <= we && se[s] >= ws)) continue;    // TimeWindow.intersects
                ++nm;
                if (first < 0) first = s;
                cs = ss[s] < cs ? ss[s] : cs;                   // TimeWindow.cover
                ce = se[s] > ce ? se[s] : ce;
                covers = covers || (ss[s] <= ws && se[s] >= we);
            }
            int64_t act = first;
            if (nm > 1 || (nm == 1 && !covers)) {               // MergeFunction.merge (WindowOperator.java:296-349)
                if (jm::wadd(jm::wsub(ce, 1), a.lateness) <= a.wm) { raise_error(a.st, FWA_E_MERGE_LATE); failed = true; break; }
                for (int64_t s = ns - 1; s >= 0; --s) {         // mergeNamespaces into the first, drop the rest
                    if (s == first || !(ss[s] <= we && se[s] >= ws)) continue;
                    for (int cc = 0; cc < nacc; ++cc)
                        acc(cc, first) = acc_combine(cc == 0 ? ACC_ADD_I64 : c.acc_kind[cc], acc(cc, first), acc(cc, s));
                    --ns;
                    if (s != ns) {
                        ss[s] = ss[ns]; se[s] = se[ns];
                        for (int cc = 0; cc < nacc; ++cc) acc(cc, s) = acc(cc, ns);
                        if (first == ns) first = s;
                    }
                }
                act = first;
                ss[act] = cs;
                se[act] = ce;
            }
            const int64_t aw_end = act >= 0 ? se[act] : we;
            if (sess_cleanup(jm::wsub(aw_end, 1), a.lateness) <= a.wm) {   // isWindowLate -> retireWindow, skip
                if (act >= 0) {
                    --ns;
                    if (act != ns) { ss[act] = ss[ns]; se[act] = se[ns]; for (int cc = 0; cc < nacc; ++cc) acc(cc, act) = acc(cc, ns); }
                }
                // Table: every skipped record counts (WindowOperator.java:386-389); DataStream: only if
                // isElementLate (WindowOperator.java:425-433, :597-601)
                if (table || jm::wadd(ts, a.lateness) <= a.wm) {
                    ++dropped;
                    if (a.dropidx) a.dropidx[atomicAdd(&a.st->drop_n, 1ull)] = (int32_t)r;
                }
                continue;
            }
            if (act < 0) {                                      // new self-contained session
                act = ns++;
                ss[act] = ws;
                se[act] = we;
                acc(0, act) = 0ull;
                for (int cc = 1; cc < nacc; ++cc) acc(cc, act) = ident_of(c.acc_kind[cc]);
            }
            acc(0, act) += 1ull;                                // windowState.add (AggregateFunction.add)
            for (int cc = 1; cc < nacc; ++cc)
                acc(cc, act) = acc_combine(c.acc_kind[cc], acc(cc, act),
                                           acc_input(c.agg[a.col_owner[cc]], a.cols[c.agg[a.col_owner[cc]].col], r,
                                                     a.nulls[c.agg[a.col_owner[cc]].col]));
            if (jm::wsub(se[act], 1) <= a.wm) {                 // EventTimeTrigger.onElement: FIRE at once
                const unsigned long long row = atomicAdd(a.lr_n, 1ull);
                if ((int64_t)row >= a.lr_cap) { raise_error(a.st, FWA_E_STATE); continue; }
                a.lr_key[row] = sess_key_of(a.key_table, a.capacity, kid);
                a.lr_start[row] = ss[act];
                a.lr_end[row] = se[act];
                for (int jj = 0; jj < c.nout; ++jj) {
                    const AggDesc d = c.agg[jj];
                    write_agg(d, acc(0, act), d.acc > 0 ? acc(d.acc, act) : 0ull, d.nn > 0 ? acc(d.nn, act) : 0ull,
                              a.lr_agg[jj], nullptr, (int64_t)row);
                }
            }
        }
        for (int64_t s = 0; s < ns; ++s) {                      // the key's sessions after the push
            const int64_t o = ncl + (int64_t)atomicAdd(&a.ctr->n_out_sp, 1ull);
            a.out.kid[o] = kid;
            a.out.start[o] = ss[s];
            a.out.end[o] = se[s];
            for (int cc = 0; cc < nacc; ++cc) a.out.acc[(int64_t)cc * a.out.stride + o] = acc(cc, s);
        }
    }
    for (int sh = 32; sh >= 1; sh >>= 1) dropped += __shfl_xor(dropped, sh);
    if ((threadIdx.x & 63) == 0 && dropped) atomicAdd(&a.st->dropped, dropped);
}

struct Sess2FireArgs {
    SessList in, out;
    int64_t n_in;
    int64_t prev_wm, wm, lateness;
    const unsigned long long* key_table;
    int64_t capacity;
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    void* o_agg[FWA_MAX_AGGS];
    uint8_t* o_null[FWA_MAX_AGGS];
    int64_t out_cap;
    SessCtr* ctr;
    DevStatus* st;
};

// Watermark advance prev -> wm: emit every session with prev < end - 1 <= wm (EventTimeTrigger.onEventTime
// / AfterEndOfWindow); keep every session whose cleanup time is still after wm (clearAllState otherwise).
// A block owns a contiguous chunk of kSessFireItems * kBlock sessions and reserves its emitted rows and kept sessions
// with one atomic per counter (a per-wave reservation on the two counters serialised ~23 K waves per fire: 0.33 ms on
// C5s); the flags are computed twice, once to count and once to write.
constexpr int kSessFireItems = 16;
__global__ void __launch_bounds__(kBlock) sess2_fire_kernel(Sess2FireArgs f, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    constexpr int kW = kBlock / 64;
    __shared__ uint32_t s_wr[kW], s_wk[kW];
    __shared__ unsigned long long s_base[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * kBlock * kSessFireItems;
    auto flags = [&](int64_t j, int64_t& end, bool& fire, bool& keep) {
        const bool act = j < f.n_in;
        end = act ? f.in.end[j] : 0;
        const int64_t mt = jm::wsub(end, 1);
        fire = act && mt > f.prev_wm && mt <= f.wm;
        keep = act && !(sess_cleanup(mt, f.lateness) <= f.wm);
    };
    uint32_t nr = 0, nk = 0;
    for (int it = 0; it < kSessFireItems; ++it) {
        int64_t end; bool fire, keep;
        flags(c0 + (int64_t)it * kBlock + threadIdx.x, end, fire, keep);
        nr += (uint32_t)__popcll(__ballot(fire));
        nk += (uint32_t)__popcll(__ballot(keep));
    }
    if (lane == 0) { s_wr[wv] = nr; s_wk[wv] = nk; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tr = 0, tk = 0;
        for (int w = 0; w < kW; ++w) { const uint32_t x = s_wr[w], y = s_wk[w]; s_wr[w] = tr; s_wk[w] = tk; tr += x; tk += y; }
        s_base[0] = tr ? atomicAdd(&f.st->rows, (unsigned long long)tr) : 0ull;
        s_base[1] = tk ? atomicAdd(&f.ctr->n_keep, (unsigned long long)tk) : 0ull;
    }
    __syncthreads();
    unsigned long long pr = s_base[0] + s_wr[wv], pk = s_base[1] + s_wk[wv];
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int it = 0; it < kSessFireItems; ++it) {
        const int64_t j = c0 + (int64_t)it * kBlock + threadIdx.x;
        int64_t end; bool fire, keep;
        flags(j, end, fire, keep);
        const unsigned long long mf = __ballot(fire), mk = __ballot(keep);
        if (fire) {
            const unsigned long long row = pr + __popcll(mf & lt);
            if ((int64_t)row >= f.out_cap) raise_error(f.st, FWA_E_STATE);
            else {
                const uint32_t kid = f.in.kid[j];
                f.o_key[row] = sess_key_of(f.key_table, f.capacity, kid);
                f.o_start[row] = f.in.start[j];
                f.o_end[row] = end;
                const uint64_t cnt = f.in.acc[j];
                for (int jj = 0; jj < c.nout; ++jj) {
                    const AggDesc d = c.agg[jj];
                    write_agg(d, cnt, d.acc > 0 ? f.in.acc[(int64_t)d.acc * f.in.stride + j] : 0ull,
                              d.nn > 0 ? f.in.acc[(int64_t)d.nn * f.in.stride + j] : 0ull, f.o_agg[jj], f.o_null[jj], (int64_t)row);
                }
            }
        }
        if (keep) {
            const unsigned long long k = pk + __popcll(mk & lt);
            f.out.kid[k] = f.in.kid[j];
            f.out.start[k] = f.in.start[j];
            f.out.end[k] = end;
            for (int cc = 0; cc < c.nacc; ++cc) f.out.acc[(int64_t)cc * f.out.stride + k] = f.in.acc[(int64_t)cc * f.in.stride + j];
        }
        pr += __popcll(mf);
        pk += __popcll(mk);
    }
}

// ------------------------------------------------------------------------------------------------
// utility kernels

// Per-push reset of the device status (all but n_keys / rows; min_q = ~0), the want-set and, for the
// Late firings (DataStream, allowed lateness > 0): WindowOperator.processElement :391-420 adds the element to
// every window that is not late (cleanupTime > wm, isWindowLate :586-589) and EventTimeTrigger.onElement
// (:37-45) FIREs at once when maxTimestamp <= wm, emitting the window's whole (non-purged) contents.
// Element order matters (each firing shows the state after that element), so the deferred records are
// applied in arrival order by one lane; such records are rare (they need a watermark past the window).
struct LateArgs {
    IngestArgs in;              // the push's columns + key table / directory / slots
    const int32_t* order;       // deferred record indices, ascending (arrival order)
    int64_t n;
    int32_t kind;               // FWA_TUMBLE or FWA_SLIDE
    int64_t size, slide, lateness;
    jm::UDiv64 slide_div;
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    void* o_agg[FWA_MAX_AGGS];
    unsigned long long* rows;   // row counter
};

__global__ void __launch_bounds__(64) late_fire_kernel(LateArgs L, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const IngestArgs& a = L.in;
    unsigned long long nrow = *L.rows;
    for (int64_t t = 0; t < L.n; ++t) {
        const int64_t i = L.order[t];
        const int64_t key = a.keys[i];
        const int64_t ts = a.ts[i];
        const int64_t d = jm::wsub(assign_ts(c, ts), c.off);
        const uint64_t ud = d < 0 ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
        const uint64_t uq = jm::udiv64(ud, c.g_div);
        const int64_t q = d >= 0 ? (int64_t)uq : ((uq * c.g_div.d == ud) ? -(int64_t)uq : -(int64_t)uq - 1);
        const DirEntry* e = dir_find(a.dir, a.dir_mask, q);
        if (e == nullptr || e->slot < 0) { raise_error(a.st, FWA_E_STATE); return; }   // host allocated it
        const int64_t kid = key_slot(a.key_table, a.key_mask, a.seg_log, a.part_bits, key, a.st);
        if (kid < 0) { a.st->key_full = 1; raise_error(a.st, FWA_E_OOM); return; }
        unsigned long long* base = a.slot_base[e->slot];
        a.touched[e->slot] = 1;
        const unsigned long long cadd = a.pcount ? a.pcount[i] : 1ull;
        base[kid] += cadd;                                           // state.add (slice accumulator)
        for (int j = 0; j < c.naggs; ++j) {
            const AggDesc dsc = c.agg[j];
            if (dsc.acc == 0 || dsc.alias) continue;
            unsigned long long* col = base + (int64_t)dsc.acc * a.stride + kid;
            const unsigned long long x = a.pcount ? ((const unsigned long long*)a.cols[j])[i]
                                                  : acc_input(dsc, a.cols[dsc.col], i);
            *col = acc_combine(dsc.acc_kind, *col, x);
        }
        // windows of the record (TimeWindow.getWindowStartWithOffset + Tumbling/SlidingEventTimeWindows)
        const int64_t sa = jm::wadd(c.off, (int64_t)((uint64_t)q * (uint64_t)c.g));
        for (int64_t ws = jm::window_start(sa, c.off, L.slide_div); ws > jm::wsub(sa, L.size); ws = jm::wsub(ws, L.slide)) {
            const int64_t we = jm::wadd(ws, L.size);
            const int64_t mt = jm::wsub(we, 1);
            int64_t cleanup = jm::wadd(mt, L.lateness);
            if (cleanup < mt) cleanup = LONG_MAX_J;
            if (cleanup <= a.wm || mt > a.wm) continue;              // late window / timer still pending
            // FIRE: merge the window's slices for this key (getResult over the window state)
            uint64_t cnt = 0;
            unsigned long long acc[FWA_MAX_AGGS];
            for (int j = 0; j < c.naggs; ++j) acc[j] = ident_of(c.agg[j].acc_kind);
            for (int64_t s0 = ws; s0 < we; s0 = jm::wadd(s0, c.g)) {
                const int64_t dd = jm::wsub(s0, c.off);
                const uint64_t udd = dd < 0 ? (uint64_t)0 - (uint64_t)dd : (uint64_t)dd;
                const uint64_t uqq = jm::udiv64(udd, c.g_div);
                const int64_t qq = dd >= 0 ? (int64_t)uqq : ((uqq * c.g_div.d == udd) ? -(int64_t)uqq : -(int64_t)uqq - 1);
                const DirEntry* ee = dir_find(a.dir, a.dir_mask, qq);
                if (ee == nullptr || ee->slot < 0) continue;
                const unsigned long long* b2 = a.slot_base[ee->slot];
                cnt += b2[kid];
                for (int j = 0; j < c.naggs; ++j) {
                    const AggDesc dj = c.agg[j];
                    if (dj.acc > 0) acc[j] = acc_combine(dj.acc_kind, acc[j], b2[(int64_t)dj.acc * a.stride + kid]);
                }
            }
            L.o_key[nrow] = key;
            L.o_start[nrow] = ws;
            L.o_end[nrow] = we;
            for (int j = 0; j < c.nout; ++j) write_agg(c.agg[j], cnt, acc[j], 0, L.o_agg[j], nullptr, (int64_t)nrow);   // DataStream: no NULLs
            ++nrow;
        }
    }
    *L.rows = nrow;
}

// two-phase path, the bucket cursors: one launch instead of a string of memsets.
__global__ void push_reset_kernel(DevStatus* st, unsigned long long* want, int32_t nwant, uint32_t* bcnt, int32_t nbcnt) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t nt = gridDim.x * blockDim.x;
    if (t == 0) {
        st->error = 0; st->spill_n = 0; st->want_n = 0; st->key_full = 0;
        st->dropped = 0; st->late_fire = 0; st->max_q = 0; st->min_q = ~0ull; st->ovf_n = 0; st->strag_n = 0; st->wide_n = 0;
    }
    for (int32_t i = t; i < nwant; i += nt) want[i] = 0ull;
    for (int32_t i = t; i < nbcnt; i += nt) bcnt[i] = 0u;
}

// Restore the identities of a list of slots (every accumulator column; MIN columns 0xFF..) and clear
// their touched flags: one launch for all slices a watermark retires (was 3 memsets per slot). An entry ~slot
// (negative) was cleared by fire_slide_kernel: only its touched flag is reset.
struct SlotList { int32_t n, id[15]; };   // up to 15 slot ids by value (no upload); more: the device list
__global__ void reset_slots_kernel(unsigned long long* const* slot_base, const int32_t* list, SlotList inl, int64_t stride,
                                   int32_t* touched, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    const int32_t sid = inl.n ? inl.id[blockIdx.y] : list[blockIdx.y];
    const int32_t slot = sid < 0 ? ~sid : sid;
    if (sid < 0) {   // cleared by the fire that read it last: the touched flag only
        if (blockIdx.x == 0 && threadIdx.x == 0) touched[slot] = 0;
        return;
    }
    unsigned long long* base = slot_base[slot];
    // 4 x 16-byte stores in flight per thread and trip (one store per thread and launch made a 32 MB C2 slot reset a
    // 30 us launch-overhead-bound kernel)
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int64_t m = stride / 2;                                      // stride % 64 == 0: 16 B stores
    for (int col = 0; col < c.nacc; ++col) {
        const unsigned long long v = (col > 0 && c.acc_kind[col] == ACC_MIN_ORD) ? ~0ull : 0ull;
        ulonglong2* p = (ulonglong2*)(base + (int64_t)col * stride);
        const ulonglong2 v2 = make_ulonglong2(v, v);
        int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        for (; i + 3 * step < m; i += 4 * step) { p[i] = v2; p[i + step] = v2; p[i + 2 * step] = v2; p[i + 3 * step] = v2; }
        for (; i < m; i += step) p[i] = v2;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) touched[slot] = 0;
}

__global__ void to_local_kernel(const int64_t* ts, int64_t* out, int64_t n, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = assign_ts(c, ts[i]);   // TR WindowOperator.processElement :340 toUtcTimestampMills
}

__global__ void fill_u64_kernel(unsigned long long* p, unsigned long long v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void key_groups_kernel(const int64_t* keys, const int32_t* kh, int64_t n, int32_t kind, int32_t maxp,
                                  int32_t par, int32_t* kg_out, int32_t* op_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t kg = jm::key_group_of(keys[i], kind, kh ? kh[i] : 0, maxp);
        kg_out[i] = kg;
        if (op_out) op_out[i] = jm::operator_index(maxp, par, kg);
    }
}

__global__ void generate_kernel(fwa_gen_params p, int64_t n, int64_t* keys, int64_t* ts, int64_t* vi, float* vf,
                                double* vd) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t i = (uint64_t)(p.first_index + j);
        const uint64_t hk = jm::splitmix64(p.seed_k ^ i);
        int64_t key;
        if (p.key_dist == 0) {
            key = (int64_t)(hk % (uint64_t)p.num_keys);
        } else {
            const double u = (double)(hk >> 11) * (1.0 / 9007199254740992.0);
            int64_t lo = 0, hi = p.num_keys - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (p.zipf_cdf[mid] > u) hi = mid; else lo = mid + 1;
            }
            key = lo;
        }
        if (keys) keys[j] = key;
        const __int128 prod = (__int128)(int64_t)i * (__int128)p.span_ms;  // floor(i * span / N), exact
        const int64_t ramp = (int64_t)(prod / (__int128)p.total_records);
        if (ts) ts[j] = p.t0_ms + ramp - (int64_t)(jm::splitmix64(p.seed_t ^ i) % (uint64_t)(p.max_delay_ms + 1));
        const uint64_t hv = jm::splitmix64(p.seed_v ^ i);
        if (vi) vi[j] = (int64_t)(hv >> 33);
        if (vf) vf[j] = (float)(hv >> 40) * (1.0f / 16777216.0f);
        if (vd) vd[j] = (double)(jm::splitmix64(hv) >> 11) * (1.0 / 9007199254740992.0);
    }
}

int grid_for(int64_t n, int64_t cap = 256 * 16) {
    int64_t g = (n + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a < 0 ? -a : a;
}

#include "sessions4.inc"
#include "merge_fire.inc"

}  // namespace

// ==================================================================================================
// host engine

struct SpState;                       // record-list window state (sparse.inc)
struct DecPlan;                       // DECIMAL aggregates over 32-bit piece sums (decimal.inc)

struct fwa_engine {
    fwa_config cfg;                   // the engine's configuration (DECIMAL handles: the internal one, see decimal.inc)
    DecPlan* dec = nullptr;
    const void* dev_override[FWA_MAX_COLS] = {};   // stage_inputs: value columns already on the device
    bool restoring = false;           // fwa_restore feeding fwa_push_partials
    // FWA_KEY_PREHASHED: the caller's key.hashCode() of every key, by kid (the key table's slot), so a snapshot can
    // place the keys in their key groups; filled after each push that inserted keys (khash_fill_kernel)
    int32_t* d_khash = nullptr;
    unsigned long long khash_nkeys = 0;   // n_keys when d_khash was last filled
    const int32_t* rs_hash = nullptr;     // fwa_restore -> fwa_push_partials: the snapshot's hash column (host)
    int32_t* d_rs_hash = nullptr;         // its device copy
    int64_t rs_hash_cap = 0;
    EngineConst ec;
    EngineConst* d_ec = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // window geometry (host)
    int32_t kind = 0, sem = 0;
    int64_t g = 0, off = 0, size = 0, slide = 0, lateness = 0;
    std::vector<int64_t> tz;          // shift time zone (instant, offset) pairs (fwa_config.tz, copied)
    int64_t* d_tz = nullptr;
    jm::UDiv64 slide_div, size_div;
    // key table
    int64_t capacity = 0;
    unsigned long long* d_keys = nullptr;
    // accumulators
    int64_t stride = 0;
    int32_t nacc = 1;
    int32_t nacc_comb = 1;                // EngineConst::nacc_comb
    std::vector<void*> chunks;
    std::vector<unsigned long long*> slot_ptr;
    unsigned long long** d_slot_base = nullptr;
    int32_t slot_base_cap = 0;
    std::vector<int32_t> free_slots;
    int32_t* d_touched = nullptr;
    std::vector<int32_t> pending_reset;   // slots whose identities reset_slots_kernel restores next
    int32_t* d_reset_list = nullptr;
    int32_t reset_cap = 0;
    std::vector<int32_t> touched;     // host mirror
    std::vector<uint8_t> slot_clean;  // 1: a fire already restored the slot's identities (fire_slide)
    // slice directory
    DirEntry* d_dir = nullptr;
    bool dir_dirty = false;         // the host directory changed since the last publish (published before v1 ingest)
    uint32_t dir_cap = 0;
    std::map<int64_t, int32_t> live;  // slice number -> slot (allocated slices)
    std::set<int64_t> negative;       // slices known late during the current push (published with slot -1)
    bool have_q = false;
    int64_t max_q = 0;                // max slice number that received data
    int64_t lookahead = 4;
    unsigned long long* d_want = nullptr;
    int32_t* d_spill = nullptr;
    int64_t spill_cap = 0;
    int32_t* d_replay = nullptr;
    int64_t replay_cap = 0;
    int32_t* d_late = nullptr;        // deferred late-firing record indices (spill_cap entries)
    // FWA_CFG_LATE_INDICES: indices of the records the last settled push dropped as late
    int32_t* d_dropidx = nullptr;
    int64_t dropidx_cap = 0;
    std::vector<int32_t> late_idx;
    // rows fired inside fwa_push (late firings), returned by the next fwa_advance_watermark
    int64_t late_rows = 0, lr_cap = 0;
    int64_t* lr_col[3 + FWA_MAX_AGGS] = {};
    unsigned long long* d_lr_n = nullptr;
    // status
    DevStatus* d_st = nullptr;
    DevStatus* h_st = nullptr;
    // host-pointer input staging
    void* d_in = nullptr;
    size_t d_in_bytes = 0;
    // output
    int64_t out_cap = 0;
    int64_t* o_key = nullptr;
    int64_t* o_start = nullptr;
    int64_t* o_end = nullptr;
    void* o_agg[FWA_MAX_AGGS] = {};
    uint8_t* o_null[FWA_MAX_AGGS] = {};   // SQL NULL flags of the nullable aggregates' output columns
    int64_t* o_hid[FWA_MAX_COLS] = {};    // raw exports of a nullable handle: hidden non-NULL counters
    int64_t* d_lts = nullptr;             // Table sessions under a shift time zone: the push's local timestamps
    int64_t lts_cap = 0;
    std::vector<char> h_out;
    FireWindow* d_win = nullptr;
    int32_t win_cap = 0;
    int32_t* d_win_slots = nullptr;
    int32_t win_slots_cap = 0;
    void* d_upos = nullptr;            // fire_slide union slot table
    void* d_zslice = nullptr;          // fire_slide: the slot columns of a slice without records (zeros)
    size_t zslice_bytes = 0;
    // watermark / stats
    int64_t wm = LONG_MIN_J;
    int64_t records_in = 0, late_dropped = 0, rows_out = 0;
    size_t mem_budget = 0;
    // v2 (two-phase) ingest
    bool v2 = false;
    int32_t seg_log = 12, part_bits = 0, np = 0, sl = 2, nv = 0, vcol[2] = {0, 0}, vsize[2] = {8, 8};
    int64_t capb = 0;
    unsigned long long* d_bkey = nullptr;
    uint16_t* d_brel = nullptr;
    uint16_t* d_bn = nullptr;         // PRE buckets: records per entry
    bool pre = false;                 // skew seen (sub-bucket overflow): Phase P pre-aggregates equal (key, slice)
    bool mp = false;                  // many stragglers seen: the combiner takes window passes (combine3 MP)
    unsigned long long* d_bval[2] = {nullptr, nullptr};
    uint32_t* d_bcnt = nullptr;
    int32_t* d_rel2slot = nullptr;
    bool v2_timing_pending = false;   // Phase P / A events recorded, read after the next sync
    // FWA_PUSH_ASYNC: the last push is enqueued but not yet settled (status, miss replay, lookahead)
    bool pend = false, pend_v2 = false;
    int64_t pend_n = 0;
    IngestArgs pend_a;
    size_t combine_lds = 0;
    int32_t partition_grid = 256;
    // kernel timing (HIP events on this handle's stream)
    hipEvent_t ev[10] = {};
    double partition_ms = 0, combine_ms = 0;
    int64_t ingest_launches = 0, ingest_records = 0, replay_records = 0, fire_launches = 0, fire_rows = 0;
    // producer stream of device inputs (fwa_set_input_stream): every push waits for it (stream order)
    hipStream_t in_stream = nullptr;
    hipEvent_t ev_in = nullptr;
    double ingest_ms = 0, fire_ms = 0;
    // sessions (merging windows): in-flight session lists (double-buffered) and per-push scratch
    SessList ss[2] = {};
    int32_t ss_cur = 0;
    int64_t ss_cap = 0, n_ss = 0;
    uint32_t* d_rkid = nullptr;
    uint8_t* d_kflag = nullptr;
    SessCtr* d_sctr = nullptr;
    SessCtr* h_sctr = nullptr;
    int64_t sb_cap = 0;                // bulk / ordered sort buffers (elements)
    unsigned long long* d_skey[4] = {};   // bulk in/out, ordered in/out
    uint32_t* d_sval[4] = {};
    int64_t* d_send2 = nullptr;
    unsigned long long* d_spk = nullptr;   // session bulk rows (Sess2Args::pk)
    void* d_sg = nullptr;                  // segment kernel staging (Sess2Args::sg_*)
    void* d_s4 = nullptr;                  // cell pre-aggregation scratch (sessions4.inc)
    size_t s4_bytes = 0;
    bool s4_attr = false;
    int64_t sg_cap = 0, sgw_cap = 0;
    int32_t cell_skip = 0;
    int32_t sess_path = 0;                 // path of the last session push (FWA_OPT_SESSION_PATH)
    bool narrow = true, narrow_used = false;   // Phase P / A narrow bucket entries (sticky off after a wide push)
    int64_t* d_spe = nullptr;
    int64_t* d_smax = nullptr;
    uint32_t* d_scid = nullptr;
    int64_t sc_cap = 0;                // ordered-path scratch session lists
    int64_t* d_sc = nullptr;           // start[sc_cap] | end[sc_cap] | acc[nacc][sc_cap]
    void* d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    int32_t kid_bits = 0;
    // partial accumulators (fwa_drain_partials)
    int64_t* o_count = nullptr;
    // pinned upload arena: small host->device uploads (directory, code table, fire lists) are copied into
    // it and enqueued without a host sync; it is recycled at every stream synchronisation
    char* h_arena = nullptr;
    size_t arena_cap = 0, arena_used = 0;
    // the arena is used in two halves: when one is full the other is taken over once the GPU consumed its copies
    // (ev_arena[h], recorded when half h was left), so a pipelined caller that never drains the stream never stalls
    int32_t arena_half = 0;
    hipEvent_t ev_arena[2] = {};
    hipEvent_t ev_st = nullptr;       // recorded after every status copy (enqueue_status)
    bool st_ready = false;            // h_st already holds the pending push's status (waited on ev_st)
    // fwa_advance_watermark_async: the fired rows of the last async advance, not yet taken by fwa_fired_output
    bool af_pend = false;             // an output is waiting to be taken
    bool af_gpu = false;              // ... and its fire is still in flight (row count on the device)
    int64_t af_rows = 0;
    int64_t* h_af_rows = nullptr;     // pinned landing of the in-flight fire's row count
    hipEvent_t ev_af = nullptr;
    int32_t* h_touched = nullptr;     // pinned landing buffer of the touched-flag mirror
    int32_t h_touched_cap = 0;
    // FWA_CFG_RECORD_LISTS: TUMBLE window state as hash-partitioned record lists, aggregated at fire (sparse.inc)
    bool sparse = false;
    // FWA_CFG_REDUCE: DataStream built-in reductions (reduce.inc): per-record (kid, slot) of the last push
    bool red = false;
    unsigned long long* d_rk = nullptr;
    int32_t* d_iota = nullptr;            // red_iota: the push's record index column (kIotaCol)
    int64_t iota_cap = 0;
    int64_t iota_n = 0;                   // its length; filled on first use (ensure_iota): partition3 computes the index
    bool iota_pending = false, iota_ran = false;
    int32_t* d_rslots = nullptr;          // red_iota: slots the payload pass scans
    int64_t rslots_cap = 0;
    int64_t rk_cap = 0;
    int64_t red_seq_base = 0;             // arrival sequence of the restored elements (red_restore)
    SpState* sp = nullptr;
    // per-handle options (fwa_set_option; the defaults are the production behaviour)
    int32_t opt_pre = -1, opt_mp = -1, opt_narrow = -1, opt_cells = -1;   // -1 adaptive, 0 never, 1 always
    int32_t opt_variant = 0;                                              // FWA_OPT_INGEST_VARIANT (A/B builds)
    int32_t push_epoch = 0;             // epoch of the current / last push (touched flags hold the last one per slot)
    // fire_slide's carried window sums: valid for a run whose first window starts at slice rs_q0 while the slices
    // [rs_q0, rs_q0 + rs_u0) have not been touched by a push after epoch rs_epoch
    unsigned long long* d_rsum = nullptr;
    bool rs_valid = false;
    int64_t rs_q0 = 0;
    int32_t rs_u0 = 0, rs_epoch = 0;
    int32_t rs_k = 4;                   // trailing slices left out of the carried sums (doubles when a push hits them)
    bool rs_on = true;                  // FWA_OPT_SLIDE_CARRIED
    int64_t rs_used = 0;                // fires that reused them
    int64_t opt_out_min = 0;
    bool opt_partials_v1 = false;
    int32_t opt_profile = 0;
    // fwa_fire_partials scratch: [3] u64 counters | b_cnt u32[NB] | bucket regions; groups per row seen last call
    void* d_mf = nullptr;
    size_t mf_bytes = 0;
    double mf_groups_per_row = 1.0;
    double mf_capx = 2.0;                 // bucket region = mean rows per bucket x this (+ slack); grows on overflow
    int32_t opt_fire_partials = -1;       // FWA_OPT_FIRE_PARTIALS: -1 / 1 the merge-fire path where eligible, 0 never
    int32_t opt_dec_wrap_null = 0;        // FWA_OPT_DEC_WRAP_NULL: 1 emits NULL for a wrapped DECIMAL window, 0 fails
    int64_t mf_calls = 0, mf_fallbacks = 0;
    // fwa_drain_route: send regions [par][dr_cap][cells] and the per-destination row counters (d_dr_cnt)
    int64_t* d_dr = nullptr;
    unsigned long long* d_dr_cnt = nullptr;
    size_t dr_bytes = 0;
    int64_t dr_cap = 0, dr_cap_used = 0;
    long long* d_prof = nullptr;          // FWA_OPT_PROFILE: per-block phase cycle counters of Phase P / A
};

namespace {

int upload(fwa_engine* e, void* dst, const void* src, size_t bytes);
int stream_sync(fwa_engine* e);

int fail(fwa_engine* e, int code, const std::string& msg) {
    if (e) e->err = msg;
    return code;
}

#define HIPCHK(e, call)                                                                       \
    do {                                                                                      \
        hipError_t _r = (call);                                                               \
        if (_r != hipSuccess) {                                                               \
            if (_r == hipErrorOutOfMemory) return fail(e, FWA_E_OOM, "out of device memory"); \
            return fail(e, FWA_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(_r));  \
        }                                                                                     \
    } while (0)

int acc_kind_of(int kind) {
    switch (kind) {
        case FWA_COUNT: case FWA_COUNT_COL: return ACC_NONE;
        case FWA_SUM_I64: case FWA_AVG_I64: case FWA_SUM_I32: return ACC_ADD_I64;
        case FWA_FIRST_64: case FWA_FIRST_32: case FWA_SEL_64: case FWA_SEL_32: return ACC_PAYLOAD;
        case FWA_MIN_I32: case FWA_MINBY_I64: case FWA_MINBY_I32: case FWA_MINBY_F64: case FWA_MINBY_F32: return ACC_MIN_ORD;
        case FWA_SUM_F32: case FWA_SUM_F64: case FWA_AVG_F32: case FWA_AVG_F64: return ACC_ADD_F64;
        case FWA_MIN_I64: case FWA_MIN_F32: case FWA_MIN_F64: return ACC_MIN_ORD;
        default: return ACC_MAX_ORD;
    }
}

int input_class(int kind) {   // 0: BIGINT input, 1: FLOAT, 2: DOUBLE, 3: INT, 4 / 5: raw 4 / 8 bytes (payload fields)
    switch (kind) {
        case FWA_SUM_F32: case FWA_MIN_F32: case FWA_MAX_F32: case FWA_AVG_F32: case FWA_MINBY_F32: case FWA_MAXBY_F32: return 1;
        case FWA_SUM_F64: case FWA_MIN_F64: case FWA_MAX_F64: case FWA_AVG_F64: case FWA_MINBY_F64: case FWA_MAXBY_F64: return 2;
        case FWA_SUM_I32: case FWA_MIN_I32: case FWA_MAX_I32: case FWA_MINBY_I32: case FWA_MAXBY_I32: return 3;
        case FWA_FIRST_32: case FWA_SEL_32: return 4;
        case FWA_FIRST_64: case FWA_SEL_64: return 5;
        default: return 0;
    }
}

bool is_reduce_kind(int k) { return k >= FWA_SUM_I32 && k <= FWA_SEL_32; }
bool is_by_kind(int k) { return k >= FWA_MINBY_I64 && k <= FWA_MAXBY_F32; }

size_t type_size(int kind) {  // input width == result width for every kind except COUNT
    switch (kind) {
        case FWA_SUM_F32: case FWA_MIN_F32: case FWA_MAX_F32: case FWA_AVG_F32: return 4;
        case FWA_SUM_I32: case FWA_MIN_I32: case FWA_MAX_I32: case FWA_FIRST_32: case FWA_SEL_32:
        case FWA_MINBY_I32: case FWA_MAXBY_I32: case FWA_MINBY_F32: case FWA_MAXBY_F32: return 4;
        default: return 8;
    }
}

int validate(const fwa_config* c) {
    if (c->abi_version != FWA_ABI_VERSION && c->abi_version != 4 && c->abi_version != 3) return FWA_E_ARG;
    if (c->num_aggs < 0 || c->num_aggs > FWA_MAX_AGGS) return FWA_E_ARG;
    for (int j = 0; j < c->num_aggs; ++j) {
        if (c->aggs[j].kind < 0 || c->aggs[j].kind >= FWA_AGG_KIND_COUNT) return FWA_E_ARG;
        if (c->aggs[j].kind != FWA_COUNT && (c->aggs[j].col < 0 || c->aggs[j].col >= FWA_MAX_COLS)) return FWA_E_ARG;
    }
    const int64_t absoff = c->offset_ms < 0 ? -c->offset_ms : c->offset_ms;
    switch (c->window_kind) {
        case FWA_TUMBLE:
            if (c->size_ms <= 0 || absoff >= c->size_ms) return FWA_E_ARG;  // TumblingEventTimeWindows.java:58-62
            break;
        case FWA_SLIDE:                                                      // SlidingEventTimeWindows.java:58-64
            if (c->size_ms <= 0 || c->slide_ms <= 0) return FWA_E_ARG;
            if (c->semantics == FWA_SEM_DATASTREAM && absoff >= c->slide_ms) return FWA_E_ARG;
            if (c->semantics == FWA_SEM_TABLE && c->size_ms % c->slide_ms != 0) return FWA_E_ARG;  // SliceAssigners.java:214-220
            break;
        case FWA_CUMULATE:
            if (c->semantics != FWA_SEM_TABLE || c->size_ms <= 0 || c->slide_ms <= 0 || c->size_ms % c->slide_ms)
                return FWA_E_ARG;
            break;
        case FWA_SESSION:                                                    // EventTimeSessionWindows.java:45-50
            if (c->gap_ms <= 0 && !(c->flags & FWA_CFG_DYNAMIC_GAP)) return FWA_E_ARG;
            break;
        default:
            return FWA_E_ARG;
    }
    if (c->flags & ~(FWA_CFG_DYNAMIC_GAP | FWA_CFG_LATE_INDICES | FWA_CFG_RECORD_LISTS | FWA_CFG_REDUCE | FWA_CFG_BY_LAST))
        return FWA_E_ARG;
    {   // DataStream built-in reductions (include/flink_amd.h FWA_CFG_REDUCE)
        int nby = 0, nsel = 0, nfirst = 0, nred = 0, nother = 0;
        for (int j = 0; j < c->num_aggs; ++j) {
            const int k = c->aggs[j].kind;
            nby += is_by_kind(k);
            nsel += k == FWA_SEL_64 || k == FWA_SEL_32;
            nfirst += k == FWA_FIRST_64 || k == FWA_FIRST_32;
            nred += is_reduce_kind(k);
            nother += (k >= FWA_AVG_I64 && k <= FWA_AVG_DEC128) || k == FWA_COUNT;   // AVG, COUNT, DECIMAL: not fields
        }
        if (nred && !(c->flags & FWA_CFG_REDUCE)) return FWA_E_ARG;
        if ((c->flags & FWA_CFG_BY_LAST) && !(c->flags & FWA_CFG_REDUCE)) return FWA_E_ARG;
        if (c->flags & FWA_CFG_REDUCE) {
            if (nby > 1 || (nsel && !nby) || (nfirst && nby)) return FWA_E_ARG;
            // session windows: only a tuple whose one value field is the reduced one (Tuple2<key, f1>): merging
            // sessions then cannot pick another element's fields, which the reference leaves to HashSet order (§2)
            const bool sess_ok = c->window_kind == FWA_SESSION && c->num_aggs == 1 && !nsel && !nfirst;
            if (nother || c->semantics != FWA_SEM_DATASTREAM ||
                (c->window_kind != FWA_TUMBLE && c->window_kind != FWA_SLIDE && !sess_ok) ||
                (c->flags & FWA_CFG_RECORD_LISTS) || ((c->flags & FWA_CFG_DYNAMIC_GAP) && !sess_ok))
                return FWA_E_UNSUPPORTED;
        }
    }
    if ((c->flags & FWA_CFG_RECORD_LISTS) && !(c->window_kind == FWA_TUMBLE && c->nullable_cols == 0 && c->tz_n == 0 &&
                                              (c->semantics == FWA_SEM_TABLE || c->allowed_lateness_ms == 0)))
        return FWA_E_UNSUPPORTED;
    if ((c->flags & FWA_CFG_DYNAMIC_GAP) && (c->window_kind != FWA_SESSION || c->gap_col < 0 || c->gap_col >= FWA_MAX_COLS))
        return FWA_E_ARG;
    if (c->nullable_cols && c->semantics != FWA_SEM_TABLE) return FWA_E_ARG;   // SQL NULLs: Table semantics
    if (c->tz_n < 0 || (c->tz_n > 0 && !c->tz)) return FWA_E_ARG;
    if (c->tz_n > 0) {                       // TIMESTAMP_LTZ rowtime: Table slicing windows only
        if (c->semantics != FWA_SEM_TABLE) return FWA_E_ARG;
        for (int32_t i = 1; i < c->tz_n; ++i) if (c->tz[2 * i] <= c->tz[2 * (i - 1)]) return FWA_E_ARG;
    }
    if (c->semantics != FWA_SEM_DATASTREAM && c->semantics != FWA_SEM_TABLE) return FWA_E_ARG;
    if (c->semantics == FWA_SEM_TABLE && c->allowed_lateness_ms != 0) return FWA_E_ARG;
    if (c->allowed_lateness_ms < 0) return FWA_E_ARG;
    if (c->key_kind < 0 || c->key_kind > 3) return FWA_E_ARG;
    if (c->max_parallelism <= 0 || c->max_parallelism > 32768) return FWA_E_ARG;
    if (c->kg_start < 0 || c->kg_end >= c->max_parallelism || c->kg_start > c->kg_end) return FWA_E_ARG;
    return FWA_OK;
}

// ---- slice geometry (host) ----

int64_t slice_start(const fwa_engine* e, int64_t q) { return jm::wadd(e->off, (int64_t)((uint64_t)q * (uint64_t)e->g)); }

// Epoch time at which a window whose last local timestamp is `max_ts` fires (TimeWindowUtil.
// toEpochMillsForTimer / isWindowFired :162-183); identity without a shift time zone.
int64_t trig(const fwa_engine* e, int64_t max_ts) {
    return e->tz.empty() ? max_ts : jm::tz_timer(e->tz.data(), (int)(e->tz.size() / 2), max_ts);
}

// Table sessions under a shift time zone: every instant the operator compares with the watermark is
// toEpochMillsForTimer(local) (InternalWindowProcessFunction.isWindowLate :119-123, MergingWindowProcessFunction
// :137-141, EventTimeTriggers.AfterEndOfWindow), a non-decreasing function of the local time. So trig(x) <= wm
// <=> x <= local_wm(wm) = the largest local time whose timer instant is <= wm, and the session kernels compare
// local window times with that local watermark unchanged.
int64_t local_wm(const fwa_engine* e, int64_t wm) {
    if (e->tz.empty() || wm == LONG_MAX_J || wm == LONG_MIN_J) return wm;
    const int64_t kLim = (int64_t)1 << 61;                  // past the zone table: a fixed offset (hi - lo fits int64)
    const int64_t thi = trig(e, kLim), tlo = trig(e, -kLim);
    if (thi <= wm) return jm::wadd(kLim, jm::wsub(wm, thi));
    if (tlo > wm) return jm::wsub(-kLim, jm::wsub(tlo, wm));
    int64_t lo = -kLim, hi = kLim;                          // trig(lo) <= wm < trig(hi)
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (trig(e, mid) <= wm) lo = mid; else hi = mid;
    }
    return lo;
}

int64_t slice_q(const fwa_engine* e, int64_t t) {  // slice number of a timestamp / slice start
    const int64_t d = jm::wsub(t, e->off);
    const uint64_t ud = d < 0 ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
    const uint64_t uq = ud / (uint64_t)e->g;
    if (d >= 0) return (int64_t)uq;
    return (uq * (uint64_t)e->g == ud) ? -(int64_t)uq : -(int64_t)uq - 1;
}

// windows containing slice q as (start, end), per kind (assigner restatements)
void windows_of_slice(const fwa_engine* e, int64_t q, std::vector<std::pair<int64_t, int64_t>>& out) {
    const int64_t a = slice_start(e, q);
    if (e->kind == FWA_TUMBLE) { out.push_back({a, jm::wadd(a, e->g)}); return; }
    if (e->kind == FWA_SLIDE) {  // SlidingEventTimeWindows.assignWindows :70-82 applied to the slice start
        for (int64_t st = jm::window_start(a, e->off, e->slide_div); st > jm::wsub(a, e->size); st = jm::wsub(st, e->slide))
            out.push_back({st, jm::wadd(st, e->size)});
        return;
    }
    const int64_t m = jm::window_start(a, e->off, e->size_div);  // CUMULATE: max window start
    const int64_t last = jm::wadd(m, e->size);
    for (int64_t en = jm::wadd(a, e->g); en <= last && en > m; en = jm::wadd(en, e->g)) out.push_back({m, en});
}

int64_t last_window_end(const fwa_engine* e, int64_t q) {
    const int64_t a = slice_start(e, q);
    if (e->kind == FWA_TUMBLE) return jm::wadd(a, e->g);
    if (e->kind == FWA_SLIDE) {
        if (e->sem == FWA_SEM_TABLE) return jm::wadd(a, e->size);          // sliceEnd - sliceSize + size
        return jm::wadd(jm::window_start(a, e->off, e->slide_div), e->size);
    }
    return jm::wadd(jm::window_start(a, e->off, e->size_div), e->size);    // windowStart(sliceEnd) + maxSize
}

int64_t first_window_end(const fwa_engine* e, int64_t q) {
    std::vector<std::pair<int64_t, int64_t>> w;
    windows_of_slice(e, q, w);
    int64_t best = LONG_MAX_J;
    for (auto& x : w) best = std::min(best, x.second);
    return best;
}

// acceptance threshold: accepted iff wm < thr, or always
void accept_threshold(const fwa_engine* e, int64_t q, int64_t* thr, bool* always) {
    const int64_t last_end = last_window_end(e, q);
    const int64_t mt = trig(e, jm::wsub(last_end, 1));
    *always = false;
    if (e->sem == FWA_SEM_TABLE) {                     // !TimeWindowUtil.isWindowFired(lastWindowEnd, wm)
        if (last_end == LONG_MAX_J) *always = true;
        *thr = mt;
        return;
    }
    int64_t cleanup = jm::wadd(mt, e->lateness);       // WindowOperator.cleanupTime :647-654
    if (cleanup < mt) cleanup = LONG_MAX_J;
    *thr = cleanup;                                    // !isWindowLate: cleanup > wm
}

// ---- slot pool ----

int grow_slots(fwa_engine* e, int32_t add) {
    const size_t col_bytes = (size_t)e->stride * 8;
    const size_t slot_bytes = col_bytes * e->nacc;
    void* chunk = nullptr;
    HIPCHK(e, hipMalloc(&chunk, slot_bytes * add));
    e->chunks.push_back(chunk);
    for (int32_t s = 0; s < add; ++s) {
        unsigned long long* base = (unsigned long long*)((char*)chunk + slot_bytes * s);
        e->free_slots.push_back((int32_t)e->slot_ptr.size());
        e->slot_ptr.push_back(base);
        e->touched.push_back(0);
        e->slot_clean.push_back(0);
        HIPCHK(e, hipMemsetAsync(base, 0, slot_bytes, e->stream));  // identities: 0; MIN columns 0xFF..
        for (int c = 1; c < e->nacc; ++c)
            if (e->ec.acc_kind[c] == ACC_MIN_ORD) HIPCHK(e, hipMemsetAsync(base + (int64_t)c * e->stride, 0xFF, col_bytes, e->stream));
    }
    const int32_t n = (int32_t)e->slot_ptr.size();
    if (n > e->slot_base_cap) {
        if (e->d_slot_base) HIPCHK(e, hipFree(e->d_slot_base));
        if (e->d_touched) HIPCHK(e, hipFree(e->d_touched));
        e->slot_base_cap = std::max<int32_t>(64, n * 2);
        HIPCHK(e, hipMalloc(&e->d_slot_base, sizeof(void*) * e->slot_base_cap));
        HIPCHK(e, hipMalloc(&e->d_touched, sizeof(int32_t) * e->slot_base_cap));
    }
    int rc = upload(e, e->d_slot_base, e->slot_ptr.data(), sizeof(void*) * n);
    if (rc) return rc;
    return upload(e, e->d_touched, e->touched.data(), sizeof(int32_t) * n);
}

int alloc_slice(fwa_engine* e, int64_t q) {
    if (e->live.count(q)) return FWA_OK;
    if (e->free_slots.empty()) {
        int rc = grow_slots(e, std::max<int32_t>(4, (int32_t)e->slot_ptr.size() / 2));
        if (rc) return rc;
    }
    const int32_t s = e->free_slots.back();
    e->free_slots.pop_back();
    e->live[q] = s;
    return FWA_OK;
}

// Queue a slot for identity restoration (untouched slots are still clean); flush_resets launches it.
int reset_slot(fwa_engine* e, int32_t slot) {
    if (e->touched[slot]) {   // ~slot: identities already restored, only the touched flag is cleared
        e->pending_reset.push_back(e->slot_clean[slot] ? ~slot : slot);
        e->touched[slot] = 0;
    }
    e->slot_clean[slot] = 0;
    return FWA_OK;
}

// Enqueue the queued resets (one kernel) before anything can reuse those slots.
int flush_resets(fwa_engine* e) {
    const int32_t n = (int32_t)e->pending_reset.size();
    if (n == 0) return FWA_OK;
    if (n > e->reset_cap) {
        if (e->d_reset_list) HIPCHK(e, hipFree(e->d_reset_list));
        e->d_reset_list = nullptr;
        e->reset_cap = std::max<int32_t>(64, 2 * n);
        HIPCHK(e, hipMalloc(&e->d_reset_list, sizeof(int32_t) * e->reset_cap));
    }
    SlotList inl;
    memset(&inl, 0, sizeof(inl));
    if (n <= 15) {                                  // slot ids in the kernel arguments: no upload, no copy on the stream
        inl.n = n;
        for (int32_t i = 0; i < n; ++i) inl.id[i] = e->pending_reset[i];
    } else {
        int rc = upload(e, e->d_reset_list, e->pending_reset.data(), sizeof(int32_t) * n);
        if (rc) return rc;
    }
    // about two 256-thread blocks per CU over all the slots, each thread storing 4 x 16 B per trip
    const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, 512 / n), (e->stride / 2 + 4095) / 4096);
    reset_slots_kernel<<<dim3((unsigned)blocks, (unsigned)n), 256, 0, e->stream>>>(e->d_slot_base, e->d_reset_list, inl,
                                                                                  e->stride, e->d_touched, e->d_ec);
    HIPCHK(e, hipGetLastError());
    e->pending_reset.clear();
    return FWA_OK;
}

int release_slot(fwa_engine* e, int32_t slot) {
    int rc = reset_slot(e, slot);
    if (rc) return rc;
    e->free_slots.push_back(slot);
    return FWA_OK;
}

// Publish the directory: every allocated slice (with slot) plus a negative entry for nothing else.
int publish_dir(fwa_engine* e) {
    uint32_t need = 256;
    while (need < 2 * (e->live.size() + e->negative.size() + 16)) need <<= 1;
    if (need > e->dir_cap) {
        if (e->d_dir) HIPCHK(e, hipFree(e->d_dir));
        HIPCHK(e, hipMalloc(&e->d_dir, sizeof(DirEntry) * need));
        e->dir_cap = need;
    }
    std::vector<DirEntry> h(e->dir_cap);
    memset(h.data(), 0, sizeof(DirEntry) * h.size());
    for (auto& kv : e->live) {
        uint32_t i = (uint32_t)jm::mix64((uint64_t)kv.first) & (e->dir_cap - 1);
        while (h[i].flags & 1) i = (i + 1) & (e->dir_cap - 1);
        DirEntry& d = h[i];
        d.q = kv.first;
        d.slot = kv.second;
        bool always;
        accept_threshold(e, kv.first, &d.thr, &always);
        d.flags = 1 | (always ? 2 : 0);
        d.first_maxts = trig(e, jm::wsub(first_window_end(e, kv.first), 1));
    }
    for (int64_t q : e->negative) {
        uint32_t i = (uint32_t)jm::mix64((uint64_t)q) & (e->dir_cap - 1);
        while (h[i].flags & 1) i = (i + 1) & (e->dir_cap - 1);
        DirEntry& d = h[i];
        d.q = q;
        d.slot = -1;
        bool always;
        accept_threshold(e, q, &d.thr, &always);
        d.flags = 1 | (always ? 2 : 0);
        d.first_maxts = LONG_MAX_J;
    }
    e->dir_dirty = false;
    return upload(e, e->d_dir, h.data(), sizeof(DirEntry) * h.size());
}

int ensure_out(fwa_engine* e, int64_t rows) {
    if (rows <= e->out_cap) return FWA_OK;
    const int64_t cap = std::max<int64_t>(rows + rows / 4, 1024);
    for (void* p : {(void*)e->o_key, (void*)e->o_start, (void*)e->o_end}) if (p) HIPCHK(e, hipFree(p));
    for (int j = 0; j < FWA_MAX_AGGS; ++j) { if (e->o_agg[j]) HIPCHK(e, hipFree(e->o_agg[j])); e->o_agg[j] = nullptr; }
    HIPCHK(e, hipMalloc(&e->o_key, 8 * cap));
    HIPCHK(e, hipMalloc(&e->o_start, 8 * cap));
    HIPCHK(e, hipMalloc(&e->o_end, 8 * cap));
    for (int j = 0; j < e->cfg.num_aggs; ++j) HIPCHK(e, hipMalloc(&e->o_agg[j], 8 * cap));
    for (int j = 0; j < FWA_MAX_AGGS; ++j) { if (e->o_null[j]) HIPCHK(e, hipFree(e->o_null[j])); e->o_null[j] = nullptr; }
    for (int j = 0; j < e->cfg.num_aggs; ++j)
        if (e->ec.agg[j].nn > 0 && e->ec.agg[j].kind != FWA_COUNT_COL) HIPCHK(e, hipMalloc(&e->o_null[j], (size_t)cap));
    if (e->o_count) HIPCHK(e, hipFree(e->o_count));
    HIPCHK(e, hipMalloc(&e->o_count, 8 * cap));
    for (int h = 0; h < FWA_MAX_COLS; ++h) { if (e->o_hid[h]) HIPCHK(e, hipFree(e->o_hid[h])); e->o_hid[h] = nullptr; }
    for (int h = 0; h < e->ec.naggs - e->ec.nout; ++h) HIPCHK(e, hipMalloc(&e->o_hid[h], 8 * cap));
    e->out_cap = cap;
    return FWA_OK;
}

int stream_sync(fwa_engine* e) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->arena_used = 0;
    return FWA_OK;
}

// The one host synchronisation of a push / fire: device status + touched-flag mirror in one round trip.
int enqueue_status(fwa_engine* e) {
    e->st_ready = false;
    HIPCHK(e, hipMemcpyAsync(e->h_st, e->d_st, sizeof(DevStatus), hipMemcpyDeviceToHost, e->stream));
    const int32_t ns = (int32_t)e->touched.size();
    if (ns > 0 && e->d_touched) {
        if (ns > e->h_touched_cap) {
            HIPCHK(e, hipStreamSynchronize(e->stream));
            if (e->h_touched) HIPCHK(e, hipHostFree(e->h_touched));
            e->h_touched = nullptr;
            e->h_touched_cap = std::max<int32_t>(256, ns * 2);
            HIPCHK(e, hipHostMalloc(&e->h_touched, sizeof(int32_t) * e->h_touched_cap));
        }
        HIPCHK(e, hipMemcpyAsync(e->h_touched, e->d_touched, sizeof(int32_t) * ns, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(e, hipEventRecord(e->ev_st, e->stream));
    return FWA_OK;
}

// Wait for the last status copy only (work enqueued after it keeps running): h_st and the touched mirror are then
// the pending push's; push_settle then skips its own wait (st_ready).
int wait_status_event(fwa_engine* e) {
    HIPCHK(e, hipEventSynchronize(e->ev_st));
    const int32_t ns = (int32_t)e->touched.size();
    if (ns > 0 && e->d_touched) memcpy(e->touched.data(), e->h_touched, sizeof(int32_t) * ns);
    e->st_ready = true;
    return FWA_OK;
}

// Wait for a status copy enqueued by enqueue_status (nothing may resize `touched` in between).
int wait_status(fwa_engine* e) {
    int rc = stream_sync(e);
    if (rc) return rc;
    const int32_t ns = (int32_t)e->touched.size();
    if (ns > 0 && e->d_touched) memcpy(e->touched.data(), e->h_touched, sizeof(int32_t) * ns);
    return FWA_OK;
}

int sync_status(fwa_engine* e) {
    int rc = enqueue_status(e);
    if (rc) return rc;
    return wait_status(e);
}

// Enqueue a host->device copy of a small host buffer through the pinned arena (no host sync; the
// source may be reused as soon as this returns).
int upload(fwa_engine* e, void* dst, const void* src, size_t bytes) {
    if (!bytes) return FWA_OK;
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (2 * need > e->arena_cap) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (e->h_arena) HIPCHK(e, hipHostFree(e->h_arena));
        e->h_arena = nullptr;
        e->arena_cap = std::max<size_t>(need * 4, (size_t)4 << 20);
        HIPCHK(e, hipHostMalloc((void**)&e->h_arena, e->arena_cap));
        e->arena_used = 0;
        e->arena_half = 0;
    }
    const size_t half = e->arena_cap / 2;
    if (e->arena_used + need > half) {   // this half is full: move to the other once its copies are done
        HIPCHK(e, hipEventRecord(e->ev_arena[e->arena_half], e->stream));
        e->arena_half ^= 1;
        HIPCHK(e, hipEventSynchronize(e->ev_arena[e->arena_half]));
        e->arena_used = 0;
    }
    char* p = e->h_arena + (size_t)e->arena_half * half + e->arena_used;
    memcpy(p, src, bytes);
    HIPCHK(e, hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, e->stream));
    e->arena_used += need;
    return FWA_OK;
}

int reset_push_status(fwa_engine* e, bool v2bufs = false) {
    // zero everything but n_keys / rows; min_q starts at ~0; want-set; v2: bucket cursors
    push_reset_kernel<<<64, kBlock, 0, e->stream>>>(e->d_st, e->d_want, e->d_want ? kWantCap : 0,
                                                    v2bufs ? e->d_bcnt : nullptr, v2bufs ? kMaxPart * kSub : 0);
    HIPCHK(e, hipGetLastError());
    return FWA_OK;
}

}  // namespace

#include "sparse.inc"
#include "decimal.inc"
static const uint64_t kSnapMagic = 0x3150414E53415746ull;   // "FWASNAP1"
enum { kSnapHdr = 32 };                                       // header words
#include "reduce.inc"

// ==================================================================================================
// C-ABI

extern "C" {

const char* fwa_version(void) { return "flink_amd 0.1 (gfx950)"; }

const char* fwa_last_error(const fwa_engine* e) { return e ? e->err.c_str() : "null engine"; }

// internal accessors for the host-only layers compiled into the same library (heap_snapshot.cpp)
int fwa_get_config(const fwa_engine* e, fwa_config* out) {
    if (!e || !out) return FWA_E_ARG;
    *out = e->dec ? e->dec->ucfg : e->cfg;
    if (e->sparse) out->flags |= FWA_CFG_RECORD_LISTS;   // reports the auto-selected mode too
    out->tz = e->tz.empty() ? nullptr : e->tz.data();    // the handle's own copy (valid while it lives)
    return FWA_OK;
}
int fwa_set_error(fwa_engine* e, int code, const char* msg) { return fail(e, code, msg); }
int fwa_dec_view(const fwa_engine* e, FwaDecView* v) {
    if (!e || !v) return FWA_E_ARG;
    memset(v, 0, sizeof(*v));
    if (!e->dec) return FWA_OK;
    v->active = 1;
    v->icfg = e->cfg;
    v->icfg.tz = e->tz.empty() ? nullptr : e->tz.data();
    for (int j = 0; j < e->dec->ucfg.num_aggs; ++j) {
        const DecAggMap& m = e->dec->d[j];
        v->umap[j] = m.kind ? -1 : e->dec->umap[j];
        v->npc[j] = m.kind ? m.npc : 0;
        for (int k = 0; k < 4; ++k) v->pc[j][k] = m.pc_agg[k];
        v->cnt[j] = m.kind ? m.cnt_agg : -1;
    }
    return FWA_OK;
}

void fwa_destroy(fwa_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->cfg.device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    sp_destroy(e);
    dec_free(e->dec);
    for (int c = 0; c < 3 + FWA_MAX_AGGS; ++c) if (e->lr_col[c]) (void)hipFree(e->lr_col[c]);
    if (e->d_late) (void)hipFree(e->d_late);
    if (e->d_lr_n) (void)hipFree(e->d_lr_n);
    void* bufs[] = {e->d_ec, e->d_keys, e->d_slot_base, e->d_touched, e->d_dir, e->d_want, e->d_spill, e->d_replay,
                    e->d_st, e->d_in, e->o_key, e->o_start, e->o_end, e->d_win, e->d_bkey, e->d_brel, e->d_bn,
                    e->d_bval[0], e->d_bval[1], e->d_bcnt, e->d_rel2slot, e->d_reset_list, e->d_upos, e->d_zslice, e->d_rsum,
                    e->d_rkid, e->d_kflag, e->d_sctr, e->d_tz, e->d_dropidx, e->d_send2, e->d_smax, e->d_scid, e->d_sc, e->d_sort_tmp, e->o_count, e->d_spk, e->d_spe, e->d_sg, e->d_prof, e->d_s4, e->d_rk, e->d_iota, e->d_rslots, e->d_mf, e->d_dr, e->d_dr_cnt,
                    e->d_khash, e->d_rs_hash};
    for (void* p : bufs) if (p) (void)hipFree(p);
    for (int q = 0; q < 4; ++q) { if (e->d_skey[q]) (void)hipFree(e->d_skey[q]); if (e->d_sval[q]) (void)hipFree(e->d_sval[q]); }
    for (int q = 0; q < 2; ++q) for (void* p : {(void*)e->ss[q].kid, (void*)e->ss[q].start, (void*)e->ss[q].end, (void*)e->ss[q].acc}) if (p) (void)hipFree(p);
    if (e->h_sctr) (void)hipHostFree(e->h_sctr);
    for (int j = 0; j < FWA_MAX_AGGS; ++j) if (e->o_agg[j]) (void)hipFree(e->o_agg[j]);
    for (int j = 0; j < FWA_MAX_AGGS; ++j) if (e->o_null[j]) (void)hipFree(e->o_null[j]);
    for (int h = 0; h < FWA_MAX_COLS; ++h) if (e->o_hid[h]) (void)hipFree(e->o_hid[h]);
    if (e->d_lts) (void)hipFree(e->d_lts);
    for (void* p : e->chunks) (void)hipFree(p);
    if (e->h_st) (void)hipHostFree(e->h_st);
    if (e->h_arena) (void)hipHostFree(e->h_arena);
    if (e->h_touched) (void)hipHostFree(e->h_touched);
    for (hipEvent_t ev : e->ev) if (ev) (void)hipEventDestroy(ev);
    if (e->ev_in) (void)hipEventDestroy(e->ev_in);
    for (hipEvent_t ev : e->ev_arena) if (ev) (void)hipEventDestroy(ev);
    if (e->ev_st) (void)hipEventDestroy(e->ev_st);
    if (e->ev_af) (void)hipEventDestroy(e->ev_af);
    if (e->h_af_rows) (void)hipHostFree(e->h_af_rows);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

static int create_engine(const fwa_config* cfg, fwa_engine** out);

int fwa_create(const fwa_config* ucfg, fwa_engine** out) {
    if (!ucfg || !out) return FWA_E_ARG;
    *out = nullptr;
    if (ucfg->abi_version != FWA_ABI_VERSION && ucfg->abi_version != 4 && ucfg->abi_version != 3) return FWA_E_ARG;
    fwa_config uc;                               // a version-3 caller's struct ends before dec_scale
    memset(&uc, 0, sizeof(uc));
    memcpy(&uc, ucfg, ucfg->abi_version == 3 ? offsetof(fwa_config, dec_scale) : sizeof(fwa_config));
    const int v = validate(&uc);
    if (v) return v;
    bool dec = false;
    for (int j = 0; j < uc.num_aggs; ++j) dec |= is_dec_kind(uc.aggs[j].kind);
    if (!dec) return create_engine(&uc, out);
    if (uc.abi_version == 3) return FWA_E_ARG;   // no scales
    DecPlan* P = new DecPlan();
    fwa_config ic;
    int rc = dec_plan(&uc, P, &ic);
    if (!rc) rc = validate(&ic);
    if (!rc) rc = create_engine(&ic, out);
    if (rc) { delete P; return rc; }
    (*out)->dec = P;
    return FWA_OK;
}

static int create_engine(const fwa_config* cfg, fwa_engine** out) {
    fwa_engine* e = new fwa_engine();
    e->cfg = *cfg;
    if (cfg->tz_n > 0) e->tz.assign(cfg->tz, cfg->tz + 2 * (size_t)cfg->tz_n);
    e->cfg.tz = nullptr;                         // the caller's table is not kept (copied above)
    e->kind = cfg->window_kind;
    e->sem = cfg->semantics;
    e->size = cfg->size_ms;
    e->slide = cfg->slide_ms;
    e->lateness = cfg->semantics == FWA_SEM_DATASTREAM ? cfg->allowed_lateness_ms : 0;
    if (e->kind == FWA_TUMBLE) {
        e->g = cfg->size_ms;
        e->off = cfg->offset_ms % cfg->size_ms;  // (globalOffset + staggerOffset) % size, ALIGNED stagger
    } else if (e->kind == FWA_SLIDE) {
        e->g = gcd64(cfg->size_ms, cfg->slide_ms);
        e->off = cfg->offset_ms;
    } else if (e->kind == FWA_CUMULATE) {
        e->g = cfg->slide_ms;
        e->off = cfg->offset_ms;
    } else {                                     // SESSION: no slices
        e->g = 1;
        e->off = 0;
    }
    e->slide_div = jm::udiv64_make((uint64_t)(e->slide > 0 ? e->slide : 1));
    e->size_div = jm::udiv64_make((uint64_t)e->size);
    EngineConst& c = e->ec;
    memset(&c, 0, sizeof(c));
    c.g_div = jm::udiv64_make((uint64_t)e->g);
    c.g = e->g;
    c.off = e->off;
    c.sem = e->sem;
    c.lateness_pos = e->lateness > 0;
    c.key_kind = cfg->key_kind;
    c.max_par = cfg->max_parallelism;
    c.kg_lo = cfg->kg_start;
    c.kg_hi = cfg->kg_end;
    c.naggs = cfg->num_aggs;
    c.nacc = 1;
    c.acc_kind[0] = ACC_ADD_I64;
    // a reduce handle's payload fields get their columns after the accumulating ones (the combiner merges only those);
    // a first- / last-element reduction (no MINBY / MAXBY) selects through an accumulator: MIN (MAX) over the
    // push's record index, a hidden aggregate (SCR) over the engine's index column kIotaCol (reduce.inc), placed before
    // them; the payload pass turns it into the arrival sequence SELQ
    bool red_iota = (cfg->flags & FWA_CFG_REDUCE) != 0 && cfg->window_kind != FWA_SESSION;
    for (int j = 0; j < cfg->num_aggs; ++j)
        if (is_by_kind(cfg->aggs[j].kind) || cfg->aggs[j].col == kIotaCol) red_iota = false;
    c.red_iota = red_iota;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1 && red_iota) {
            const bool last = (cfg->flags & FWA_CFG_BY_LAST) != 0;
            AggDesc& h = c.agg[c.naggs++];
            memset(&h, 0, sizeof(h));
            h.kind = last ? FWA_MAX_I32 : FWA_MIN_I32;    // over the push's record index (4-byte column)
            h.col = kIotaCol;
            h.acc_kind = last ? ACC_MAX_ORD : ACC_MIN_ORD;
            h.acc = c.nacc;
            c.acc_kind[c.nacc] = h.acc_kind;
            c.red_scr = c.nacc++;
        }
        for (int j = 0; j < cfg->num_aggs; ++j) {
            AggDesc& d = c.agg[j];
            d.kind = cfg->aggs[j].kind;
            d.col = cfg->aggs[j].col;
            d.acc_kind = acc_kind_of(d.kind);
            if ((d.acc_kind == ACC_PAYLOAD) != (pass == 1)) continue;
            d.alias = 0;
            d.acc = 0;
            if (d.acc_kind == ACC_NONE) continue;
            int share = -1;   // same accumulator kind over the same input column and input type: one column
            for (int i = 0; i < cfg->num_aggs && share < 0; ++i)
                if (i != j && c.agg[i].acc > 0 && !c.agg[i].alias && c.agg[i].acc_kind == d.acc_kind &&
                    c.agg[i].col == d.col && input_class(c.agg[i].kind) == input_class(d.kind) &&
                    ((pass == 0 && i < j) || (pass == 1 && c.agg[i].acc_kind == ACC_PAYLOAD && i < j)))
                    share = i;
            if (share >= 0) { d.acc = c.agg[share].acc; d.alias = 1; continue; }
            d.acc = c.nacc;
            c.acc_kind[c.nacc] = d.acc_kind;
            c.nacc++;
        }
    }
    // SQL NULLs: one hidden non-NULL counter per nullable input column (an ADD_I64 column fed 1 per
    // non-NULL value, AvgAggFunction's count / the null flag of Sum/Min/MaxAggFunction's buffer); COUNT(col)
    // over a nullable column reads it, over a non-nullable one it is COUNT(*)
    c.nout = cfg->num_aggs;
    c.nullable = cfg->nullable_cols;
    int nn_acc[FWA_MAX_COLS] = {};
    for (int j = 0; j < cfg->num_aggs; ++j) {
        AggDesc& d = c.agg[j];
        d.nn = 0;
        if (d.kind == FWA_COUNT || !((cfg->nullable_cols >> d.col) & 1)) continue;
        if (!nn_acc[d.col]) {
            AggDesc& h = c.agg[c.naggs++];
            memset(&h, 0, sizeof(h));
            h.kind = FWA_COUNT_COL;
            h.col = d.col;
            h.acc_kind = ACC_ADD_I64;
            h.acc = c.nacc;
            c.acc_kind[c.nacc] = ACC_ADD_I64;
            nn_acc[d.col] = c.nacc++;
        }
        d.nn = nn_acc[d.col];
        if (d.kind == FWA_COUNT_COL) { d.acc = d.nn; d.alias = 1; d.acc_kind = ACC_ADD_I64; }
    }
    // DataStream built-in reductions: the selected element's arrival sequence (SELQ: identity ~0 to select the first
    // element, 0 the last) and the by-value it was selected at (SELK) as two more slot columns (reduce.inc)
    e->red = (cfg->flags & FWA_CFG_REDUCE) != 0;
    c.red = e->red;
    c.red_by = -1;
    if (e->red) {
        for (int j = 0; j < cfg->num_aggs; ++j) {
            c.agg[j].jcmp = 1;
            if (is_by_kind(cfg->aggs[j].kind)) {
                c.red_by = j;
                c.red_max = cfg->aggs[j].kind == FWA_MAXBY_I64 || cfg->aggs[j].kind == FWA_MAXBY_I32 ||
                            cfg->aggs[j].kind == FWA_MAXBY_F64 || cfg->aggs[j].kind == FWA_MAXBY_F32;
            }
        }
        c.red_last = (cfg->flags & FWA_CFG_BY_LAST) != 0;
        if (cfg->window_kind != FWA_SESSION) {   // (a session reduction's one field is its only column: no selection)
            c.red_selq = c.nacc;                   // (red_iota: the payload pass moves the push's selection here)
            c.acc_kind[c.nacc++] = c.red_last ? ACC_MAX_ORD : ACC_MIN_ORD;
            c.red_selk = c.nacc;
            c.acc_kind[c.nacc++] = ACC_PAYLOAD;
            if (c.red_by >= 0) {   // scratch: identity between pushes (red_by_payload_kernel restores it)
                c.red_scr = c.nacc;
                c.acc_kind[c.nacc++] = c.red_last ? ACC_MAX_ORD : ACC_MIN_ORD;
            }
        }
    }
    e->nacc = c.nacc;
    c.nacc_comb = c.nacc;
    if (e->red) {
        c.nacc_comb = 1;
        for (int j = 0; j < c.naggs; ++j)
            if (c.agg[j].acc > 0 && c.agg[j].acc_kind != ACC_PAYLOAD) c.nacc_comb = std::max(c.nacc_comb, c.agg[j].acc + 1);
    }
    e->nacc_comb = c.nacc_comb;
    // key-table segmentation (all paths) and v2 eligibility: <= 2 distinct carried value columns,
    // an LDS window of >= 2 slices next to the SEG-key LDS segment, <= kMaxPart partitions
    {
        const int64_t kc0 = cfg->key_capacity > 0 ? cfg->key_capacity : (1 << 20);
        int cap_log = 10;
        while (((int64_t)1 << cap_log) < 2 * kc0) ++cap_log;
        // (session handles: 8192-key segments, half the partitions for the s5 route -- sessions4.inc)
        int seg_log = std::max(6, std::min(e->kind == FWA_SESSION ? 13 : 12, cap_log));
        e->seg_log = seg_log;
        e->part_bits = cap_log - seg_log;
        int cols[2] = {-1, -1}, sizes[2] = {8, 8}, nv = 0;
        bool ok = true;
        for (int j = 0; j < c.naggs; ++j) {
            AggDesc& d = c.agg[j];
            if (d.acc == 0 || d.acc_kind == ACC_PAYLOAD) continue;   // payload: written by the selection passes
            if (d.kind == FWA_COUNT_COL) { d.vslot = 0; continue; }   // counts rows: no value carried
            int slot = -1;
            for (int v = 0; v < nv; ++v) if (cols[v] == d.col) slot = v;
            if (slot < 0) {
                if (nv == 2) { ok = false; break; }
                slot = nv;
                cols[nv] = d.col;
                sizes[nv] = (int)type_size(d.kind);
                nv++;
            } else if (sizes[slot] != (int)type_size(d.kind)) ok = false;
            d.vslot = slot;
        }
        // segment size: the largest SEG whose LDS key segment + 2-slice accumulator window fits next to
        // each other in 160 KB (wide aggregate lists, e.g. C5's 4 float accumulators, need SEG < 4096)
        // while the partition count stays <= kMaxPart
        auto lds_need = [&](int sg) {
            const int64_t sgz = (int64_t)1 << sg;
            return sgz * 8 + 2 * sgz * 4 + (int64_t)(c.nacc_comb - 1) * 2 * sgz * 8 + 4 * 4 * kSub + 16 +
                   (int64_t)sizeof(StragL) * kStragL + 256;   // + static LDS (straggler list, descriptors)
        };
        // (session handles never run the combiner: their segments stay at 4096 keys, which the s5 route of the cell
        // pre-aggregation resolves in LDS -- sessions4.inc)
        while (e->kind != FWA_SESSION && seg_log > 9 && lds_need(seg_log) > 160 * 1024 &&
               ((int64_t)1 << (cap_log - seg_log + 1)) <= kMaxPart)
            --seg_log;
        e->seg_log = seg_log;
        e->part_bits = cap_log - seg_log;
        const int64_t seg = (int64_t)1 << seg_log;
        const int64_t bps = 4 + 8 * (int64_t)(c.nacc_comb - 1);
        const int64_t avail = 160 * 1024 - 512 - (int64_t)sizeof(StragL) * kStragL - seg * 8;
        int sl = (int)std::min<int64_t>(8, avail > 0 ? avail / (bps * seg) : 0);
        if (lds_need(seg_log) > 160 * 1024) sl = 0;
        const int64_t np = (int64_t)1 << e->part_bits;
        // record lists (sparse.inc): asked for, or a key space of >= 2^25 keys
        const bool want_sp = (cfg->flags & FWA_CFG_RECORD_LISTS) || kc0 >= ((int64_t)1 << 25);
        e->sparse = want_sp && sp_eligible(cfg);
        // reductions: two-phase accumulators when every reduced field is a BIGINT SUM / MIN / MAX / MINBY / MAXBY or a
        // DOUBLE SUM over an 8-byte column (the combiner's carried-value arithmetic; other fields keep the v1 ingest)
        bool red_ok = true;
        for (int j = 0; e->red && j < c.naggs; ++j) {
            const int k = c.agg[j].kind;
            if (c.agg[j].acc_kind == ACC_PAYLOAD || c.agg[j].acc == 0) continue;
            red_ok = red_ok && (k == FWA_SUM_I64 || k == FWA_SUM_F64 || k == FWA_MIN_I64 || k == FWA_MAX_I64 ||
                                k == FWA_MINBY_I64 || k == FWA_MAXBY_I64 ||
                                (c.agg[j].col == kIotaCol && (k == FWA_MIN_I32 || k == FWA_MAX_I32)));
        }
        ok = ok && np <= kMaxPart && sl >= 2 && e->kind != FWA_SESSION && !e->sparse && (!e->red || red_ok);
        e->v2 = ok;
        if (ok) {
            e->np = (int32_t)np;
            e->sl = sl;
            e->nv = nv;
            for (int v = 0; v < 2; ++v) { e->vcol[v] = cols[v] < 0 ? 0 : cols[v]; e->vsize[v] = sizes[v]; }
            e->combine_lds = (size_t)seg * 8 + (((size_t)sl * seg * 4 + 15) & ~(size_t)15) +
                             (size_t)(c.nacc_comb - 1) * sl * seg * 8 + 16;
        }
    }
    if (hipSetDevice(cfg->device) != hipSuccess) { delete e; return FWA_E_DEVICE; }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return FWA_E_DEVICE; }
    const int64_t kc = e->sparse ? 512 : (cfg->key_capacity > 0 ? cfg->key_capacity : (1 << 20));   // no key table
    int64_t cap = 1024;
    while (cap < 2 * kc) cap <<= 1;
    e->capacity = cap;
    e->stride = ((cap + 1 + 63) / 64) * 64;
    int rc = FWA_OK;
    do {
        if (!e->tz.empty()) {
            if (hipMalloc(&e->d_tz, 8 * e->tz.size()) != hipSuccess) { rc = FWA_E_OOM; break; }
            if (hipMemcpy(e->d_tz, e->tz.data(), 8 * e->tz.size(), hipMemcpyHostToDevice) != hipSuccess) { rc = FWA_E_DEVICE; break; }
            c.tz = e->d_tz;
            c.tz_n = (int32_t)(e->tz.size() / 2);
        }
        if (hipMalloc(&e->d_ec, sizeof(EngineConst)) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (hipMemcpy(e->d_ec, &c, sizeof(EngineConst), hipMemcpyHostToDevice) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        if (hipMalloc(&e->d_keys, sizeof(unsigned long long) * (cap + 1)) != hipSuccess) { rc = FWA_E_OOM; break; }
        fill_u64_kernel<<<grid_for(cap), kBlock, 0, e->stream>>>(e->d_keys, kEmptyKey, cap);
        if (hipMemsetAsync(e->d_keys + cap, 0, 8, e->stream) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        if (cfg->key_kind == FWA_KEY_PREHASHED && !e->sparse) {
            if (hipMalloc(&e->d_khash, sizeof(int32_t) * (cap + 1)) != hipSuccess) { rc = FWA_E_OOM; break; }
            if (hipMemsetAsync(e->d_khash, 0, sizeof(int32_t) * (cap + 1), e->stream) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        }
        if (hipMalloc(&e->d_st, sizeof(DevStatus)) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (hipHostMalloc(&e->h_st, sizeof(DevStatus)) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (hipHostMalloc(&e->h_af_rows, sizeof(int64_t)) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (hipMemsetAsync(e->d_st, 0, sizeof(DevStatus), e->stream) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        bool evok = true;
        for (hipEvent_t& ev : e->ev) evok = evok && hipEventCreate(&ev) == hipSuccess;
        evok = evok && hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming) == hipSuccess;
        for (hipEvent_t& ev : e->ev_arena) evok = evok && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
        evok = evok && hipEventCreateWithFlags(&e->ev_st, hipEventDisableTiming) == hipSuccess;
        evok = evok && hipEventCreateWithFlags(&e->ev_af, hipEventDisableTiming) == hipSuccess;
        if (!evok) { rc = FWA_E_DEVICE; break; }
        if (hipMalloc(&e->d_want, sizeof(unsigned long long) * kWantCap) != hipSuccess) { rc = FWA_E_OOM; break; }
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        e->mem_budget = fr / 2;
        if (e->kind == FWA_SESSION) {            // flat in-flight session lists
            e->kid_bits = 1;
            while (((int64_t)1 << e->kid_bits) < cap + 1) ++e->kid_bits;
            if (hipMalloc(&e->d_kflag, (size_t)cap + 1) != hipSuccess) { rc = FWA_E_OOM; break; }
            if (hipMalloc(&e->d_sctr, sizeof(SessCtr)) != hipSuccess) { rc = FWA_E_OOM; break; }
            if (hipHostMalloc(&e->h_sctr, sizeof(SessCtr)) != hipSuccess) { rc = FWA_E_OOM; break; }
        } else if (e->sparse) {
            if ((rc = sp_init(e))) break;
        } else {
            if ((rc = grow_slots(e, 4))) break;
            if ((rc = publish_dir(e))) break;
        }
        if (hipStreamSynchronize(e->stream) != hipSuccess) { rc = FWA_E_DEVICE; break; }
    } while (0);
    if (rc) { fwa_destroy(e); return rc; }
    *out = e;
    return FWA_OK;
}

static int stage_inputs(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* cols,
                        const uint8_t* const* nulls, const int32_t* kh, int64_t n, IngestArgs& a) {
    size_t need = (size_t)n * 24 + (kh ? (size_t)n * 4 : 0) + 4096;   // + a session gap column
    for (int j = 0; j < e->cfg.num_aggs; ++j) need += (size_t)n * 8 + 256;
    for (int c = 0; c < FWA_MAX_COLS; ++c)
        if (nulls && ((e->cfg.nullable_cols >> c) & 1) && nulls[c]) need += (size_t)n + 256;
    if (need > e->d_in_bytes) {
        if (e->d_in) HIPCHK(e, hipFree(e->d_in));
        HIPCHK(e, hipMalloc(&e->d_in, need));
        e->d_in_bytes = need;
    }
    char* p = (char*)e->d_in;
    hipError_t err = hipSuccess;
    auto put = [&](const void* src, size_t bytes) -> const void* {
        void* dst = p;
        hipError_t r = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream);
        if (r != hipSuccess) err = r;
        p += (bytes + 255) / 256 * 256;
        return dst;
    };
    a.keys = (const int64_t*)put(keys, (size_t)n * 8);
    a.ts = (const int64_t*)put(ts, (size_t)n * 8);
    a.key_hash = kh ? (const int32_t*)put(kh, (size_t)n * 4) : nullptr;
    for (int c = 0; c < FWA_MAX_COLS; ++c) a.cols[c] = nullptr;
    for (int j = 0; j < e->cfg.num_aggs; ++j) {
        const fwa_agg_spec& s = e->cfg.aggs[j];
        if (s.kind == FWA_COUNT || s.kind == FWA_COUNT_COL || a.cols[s.col]) continue;
        if (e->dev_override[s.col]) { a.cols[s.col] = e->dev_override[s.col]; continue; }   // DECIMAL pieces
        if (!cols || !cols[s.col]) return fail(e, FWA_E_ARG, "missing value column");
        a.cols[s.col] = put(cols[s.col], (size_t)n * type_size(s.kind));
    }
    for (int c = 0; c < FWA_MAX_COLS; ++c)
        a.nulls[c] = (nulls && ((e->cfg.nullable_cols >> c) & 1) && nulls[c]) ? (const uint8_t*)put(nulls[c], (size_t)n) : nullptr;
    if ((e->cfg.flags & FWA_CFG_DYNAMIC_GAP) && !a.cols[e->cfg.gap_col]) {
        if (!cols || !cols[e->cfg.gap_col]) return fail(e, FWA_E_ARG, "missing session gap column");
        a.cols[e->cfg.gap_col] = put(cols[e->cfg.gap_col], (size_t)n * 8);
    }
    HIPCHK(e, err);
    return FWA_OK;
}

// Device inputs are produced on the caller's stream (e.g. torch's current stream): the engine's stream
// waits for everything enqueued there so far before its kernels read them.
static int wait_input_stream(fwa_engine* e) {
    if (!e->in_stream) return FWA_OK;
    HIPCHK(e, hipEventRecord(e->ev_in, e->in_stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_in, 0));
    return FWA_OK;
}

// red_iota: the record index column, written only when a reader of the column runs this push (the v1 ingest -- a whole
// push or its miss replays -- or partition3 under variant bit 16); the two-phase ingest derives the index itself.
static int ensure_iota(fwa_engine* e) {
    if (!e->iota_pending) return FWA_OK;
    e->iota_pending = false;
    e->iota_ran = true;
    HIPCHK(e, hipEventRecord(e->ev[8], e->stream));      // (ev[8] / ev[9]: record lists only otherwise)
    iota_kernel<<<grid_for(e->iota_n, 256 * 32), kBlock, 0, e->stream>>>(e->d_iota, e->iota_n);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[9], e->stream));
    return FWA_OK;
}

static int launch_ingest(fwa_engine* e, IngestArgs& a, bool replay) {
    if (e->dir_dirty) { int rc = publish_dir(e); if (rc) return rc; }
    if (e->iota_pending) { int rc = ensure_iota(e); if (rc) return rc; }
    a.spill_cap = e->spill_cap;
    a.key_table = e->d_keys;
    a.key_mask = (uint64_t)e->capacity - 1;
    a.seg_log = e->seg_log;
    a.part_bits = e->part_bits;
    a.dir = e->d_dir;
    a.dir_mask = e->dir_cap - 1;
    a.want = e->d_want;
    a.spill = e->d_spill;
    a.late = e->d_late;
    a.touched = e->d_touched;
    a.epoch = std::max<int32_t>(1, e->push_epoch);
    a.slot_base = e->d_slot_base;
    a.stride = e->stride;
    a.st = e->d_st;
    const int grid = grid_for(a.n, 256 * 32);
    HIPCHK(e, hipEventRecord(e->ev[0], e->stream));
    if (replay) ingest_kernel<true><<<grid, kBlock, 0, e->stream>>>(a, e->d_ec);
    else ingest_kernel<false><<<grid, kBlock, 0, e->stream>>>(a, e->d_ec);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[1], e->stream));
    e->ingest_launches++;
    if (!replay) e->ingest_records += a.n;   // a replay re-visits records the first launch already counted
    else e->replay_records += a.n;
    return FWA_OK;
}

static int account_ingest(fwa_engine* e) {  // after the stream was synchronised
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
    e->ingest_ms += ms;
    return FWA_OK;
}

static int ensure_v2_buffers(fwa_engine* e, int64_t n, bool need_bn) {
    const int64_t per = n / ((int64_t)e->np * kSub);                 // expected records per sub-bucket
    const int64_t capb = per + per / 4 + 2048;
    if (capb > e->capb) {
        for (void* p : {(void*)e->d_bkey, (void*)e->d_brel, (void*)e->d_bn, (void*)e->d_bval[0], (void*)e->d_bval[1]}) if (p) HIPCHK(e, hipFree(p));
        e->d_bkey = nullptr;
        e->d_brel = nullptr;
        e->d_bn = nullptr;
        e->d_bval[0] = e->d_bval[1] = nullptr;
        const int64_t ent = capb * e->np * kSub + 8 * kMaxPart;  // + a trash area (partition3's masked stores)
        HIPCHK(e, hipMalloc(&e->d_bkey, (e->nv == 1 ? 12 : 8) * ent));   // 12: narrow {key, value, slice} entries
        HIPCHK(e, hipMalloc(&e->d_brel, 2 * ent));
        for (int v = 0; v < e->nv; ++v) HIPCHK(e, hipMalloc(&e->d_bval[v], 8 * ent));
        e->capb = capb;
    }
    if (need_bn && !e->d_bn) HIPCHK(e, hipMalloc(&e->d_bn, 2 * (e->capb * e->np * kSub + 8 * kMaxPart)));
    if (!e->d_bcnt) {
        HIPCHK(e, hipMalloc(&e->d_bcnt, sizeof(uint32_t) * kMaxPart * kSub));
        HIPCHK(e, hipMalloc(&e->d_rel2slot, (sizeof(int32_t) + 2) * kRelCap));   // rel2slot | relcode | relfresh
    }
    return FWA_OK;
}

// FWA_OPT_PROFILE: wait for a profiled kernel (events a, b) and print its per-block phase cycle counters (average
// over the nb blocks and the slowest block): Phase P marks 6 phases, Phase A 8.
static int print_phase_profile(fwa_engine* e, const char* tag, hipEvent_t a, hipEvent_t b, int nb, int nph) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, a, b));
    std::vector<long long> hp(8 * (size_t)nb);
    HIPCHK(e, hipMemcpy(hp.data(), e->d_prof, sizeof(long long) * 8 * nb, hipMemcpyDeviceToHost));
    double tot[8] = {0};
    int bmax = 0;
    long long bsum_max = -1;
    for (int blk = 0; blk < nb; ++blk) {
        long long bs = 0;
        for (int k = 0; k < nph; ++k) { tot[k] += (double)hp[blk * 8 + k] / nb; bs += hp[blk * 8 + k]; }
        if (bs > bsum_max) { bsum_max = bs; bmax = blk; }
    }
    fprintf(stderr, "[%s] kernel %.3f ms; per-block avg cycles:", tag, ms);
    for (int k = 0; k < nph; ++k) fprintf(stderr, " %.0f", tot[k]);
    fprintf(stderr, " | slowest block %d:", bmax);
    for (int k = 0; k < nph; ++k) fprintf(stderr, " %lld", hp[bmax * 8 + k]);
    fprintf(stderr, "\n");
    return FWA_OK;
}

// Two-phase ingest. Sets *ran = false (and leaves no state change besides key insertions) when the
// batch must take the v1 path instead (bucket overflow on skewed keys).
static int ensure_sort_tmp(fwa_engine* e, size_t bytes);
static int push_v2(fwa_engine* e, IngestArgs& a, bool* ran) {
    *ran = false;
    // combiner accumulator layout (compile-time in combine3) and the skew mode (PRE, partition3)
    int layout = 0;
    if (e->nacc_comb == 1) layout = 2;
    else if (e->nacc_comb == 2 && e->ec.acc_kind[1] == ACC_ADD_I64) {
        for (int j = 0; j < e->cfg.num_aggs; ++j)
            if (e->ec.agg[j].acc == 1 && e->ec.agg[j].vslot == 0) layout = 1;
    }
    const bool pre_ok = (layout == 2 && e->nv == 0) || (layout == 1 && e->nv == 1 && e->vsize[0] == 8);
    // partial accumulators (fwa_push_partials): the PRE buckets carry each row's record count, the value
    // column is the partial BIGINT sum; other aggregate lists keep the v1 path
    if (a.pcount && (!pre_ok || e->cfg.nullable_cols || e->opt_partials_v1)) return FWA_OK;
    const bool pre = a.pcount || (pre_ok && e->opt_pre != 0 && (e->opt_pre == 1 || e->pre));
    int rc = ensure_v2_buffers(e, a.n, pre);
    if (rc) return rc;
    const int64_t q_base = e->live.empty() ? 0 : e->live.begin()->first;
    // rel2slot (combine) and relcode (partition): the directory restricted to [q_base, q_base + kRelCap)
    // with each slice's acceptance under the current watermark (WindowOperator.isWindowLate /
    // SlicingWindowOperator lateness, as in ingest_kernel)
    std::vector<int32_t> r2s(kRelCap + kRelCap / 2, -1);
    uint8_t* code = (uint8_t*)(r2s.data() + kRelCap);
    memset(code, kCodeSlow, kRelCap);
    // slots no record reached yet hold their identities: the combiner's merge of such a slice stores without reading
    uint8_t* fresh = code + kRelCap;
    memset(fresh, 0, kRelCap);
    for (auto& kv : e->live) {
        const int64_t rel = kv.first - q_base;
        if (rel < 0 || rel >= kRelCap) continue;
        r2s[rel] = kv.second;
        fresh[rel] = (e->touched[kv.second] || (e->opt_variant & 1)) ? 0 : 1;   // variant bit 0: A/B without
        int64_t thr;
        bool always;
        accept_threshold(e, kv.first, &thr, &always);
        if (!always && !(a.wm < thr)) code[rel] = kCodeDrop;
        else if (e->lateness > 0 && a.wm >= trig(e, jm::wsub(first_window_end(e, kv.first), 1))) code[rel] = kCodeSlow;
        else code[rel] = kCodeAccept;
    }
    rc = upload(e, e->d_rel2slot, r2s.data(), (sizeof(int32_t) + 2) * kRelCap);
    if (rc) return rc;
    rc = reset_push_status(e, true);
    if (rc) return rc;
    PartArgs pa;
    memset(&pa, 0, sizeof(pa));
    pa.keys = a.keys;
    pa.ts = a.ts;
    for (int c = 0; c < FWA_MAX_COLS; ++c) pa.cols[c] = a.cols[c];
    if (a.pcount) {                   // partial rows: cols[] is indexed by aggregate; the carried value is the
        pa.pcount = a.pcount;         // accumulator column of the BIGINT sum (layout 1)
        for (int j = 0; j < e->cfg.num_aggs; ++j)
            if (e->ec.agg[j].acc == 1 && layout == 1) pa.cols[e->vcol[0]] = a.cols[j];
    }
    pa.key_hash = a.key_hash;
    pa.n = a.n;
    pa.wm = a.wm;
    pa.relcode = (const uint8_t*)(e->d_rel2slot + kRelCap);
    pa.rel2slot = e->d_rel2slot;
    pa.touched = e->d_touched;
    pa.epoch = std::max<int32_t>(1, e->push_epoch);
    pa.spill = e->d_spill;
    pa.q_base = q_base;
    pa.fast_m = 0;
    pa.fast_lim = 0;
    pa.base_ts = 0;
    pa.fast_sh = 0;
    if (!e->cfg.tz_n && e->g > 0 && (uint64_t)e->g * kRelCap < (1ull << 32) && q_base > -(1ll << 40) && q_base < (1ll << 40)) {
        // floor(n / g) = (n * ceil(2^(32+L) / g)) >> (32+L) for every n < 2^32, L = ceil(log2 g) (round-up method;
        // the magic has at most 33 bits, so n * m fits 64 bits)
        int L = 0;
        while ((1ull << L) < (uint64_t)e->g) ++L;
        const __int128 b = (__int128)e->off + (__int128)q_base * e->g;
        if (b > (__int128)INT64_MIN / 2 && b < (__int128)INT64_MAX / 2) {
            pa.fast_sh = 32 + L;
            pa.fast_m = ((1ull << (32 + L)) + (uint64_t)e->g - 1) / (uint64_t)e->g;
            pa.fast_lim = (uint64_t)e->g * kRelCap;
            pa.base_ts = (int64_t)b;
        }
    }
    pa.b_key = e->d_bkey;
    pa.b_rel = e->d_brel;
    pa.b_n = pre ? e->d_bn : nullptr;
    pa.key_table = e->d_keys;
    pa.key_mask = (uint64_t)e->capacity - 1;
    pa.seg_log = e->seg_log;
    pa.slot_base = e->d_slot_base;
    pa.stride = e->stride;
    pa.b_val0 = e->d_bval[0];
    pa.b_val1 = e->d_bval[1];
    pa.b_cnt = e->d_bcnt;
    pa.capb = e->capb;
    pa.trash = (uint64_t)e->capb * e->np * kSub;
    pa.spill_cap = e->spill_cap;
    pa.part_bits = e->part_bits;
    pa.np = e->np;
    pa.sub_major = (e->opt_variant & 4) ? 0 : 1;   // variant bit 2: partition-major buckets (A/B)
    pa.iota1 = e->ec.red_iota && e->nv == 2 && e->vcol[1] == kIotaCol && e->vsize[1] == 4 && !(e->opt_variant & 16);
    if (e->iota_pending && !pa.iota1) { int rc = ensure_iota(e); if (rc) return rc; }
    for (int v = 0; v < 2; ++v) { pa.vcol[v] = e->vcol[v]; pa.vsize[v] = e->vsize[v]; }
    pa.dropidx = a.pcount ? nullptr : a.dropidx;   // partial rows: no record indices (as in v1)
    for (int c = 0; c < FWA_MAX_COLS; ++c) { pa.nulls[c] = a.nulls[c]; pa.any_null |= a.nulls[c] != nullptr; }
    pa.st = e->d_st;
    if (e->opt_profile && !e->d_prof) HIPCHK(e, hipMalloc(&e->d_prof, sizeof(long long) * 8 * kMaxPart));
    pa.prof = e->opt_profile ? e->d_prof : nullptr;
    HIPCHK(e, hipEventRecord(e->ev[4], e->stream));
    const int threads = 1024;
    const int items = e->nv == 2 ? 4 : (e->nv == 1 ? 6 : 8);
    const int64_t tile = (int64_t)items * threads;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((a.n + tile - 1) / tile, 256));
    const int vw = (e->vsize[0] == 8 ? 1 : 0) | (e->vsize[1] == 8 ? 2 : 0);
    // ownership is checked per record unless the handle owns every key group; dictionary ids always (their key group
    // may be past max_parallelism: key group -1, rejected with FWA_E_KEYGROUP)
    const bool kg_all = e->cfg.kg_start == 0 && e->cfg.kg_end == e->cfg.max_parallelism - 1 &&
                        e->cfg.key_kind != FWA_KEY_GROUP_PREFIXED;
    const int kgm = kg_all ? 0 : (e->cfg.key_kind == FWA_KEY_PREHASHED ? 2 : 1);
    auto al16 = [](const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; };
    const bool w16 = kgm == 0 && al16(pa.keys) && al16(pa.ts) &&
                     (e->nv == 0 || ((uintptr_t)pa.cols[pa.vcol[0]] & ((e->vsize[0] == 8) ? 15 : 7)) == 0);
    // narrow bucket entries (partition3 / combine3 NW): COUNT + one BIGINT SUM over an 8-byte column, the paired-load
    // kernel; on by default until a push finds more than 1/64 of its records needing 64-bit keys or values
    const bool narrow = e->opt_narrow != 0 && (e->opt_narrow == 1 || e->narrow) && layout == 1 && e->nv == 1 &&
                        (vw & 1) && w16 && !pre && !a.pcount;
    // ... and for an 8-byte value column beside a 4-byte one (C5: DOUBLE and FLOAT): key and FLOAT bits share a word
    const bool narrow2 = e->opt_narrow != 0 && (e->opt_narrow == 1 || e->narrow) && layout == 0 && e->nv == 2 && vw == 1 &&
                         kgm == 0 && !pre && !a.pcount;
    e->narrow_used = narrow || narrow2;
    const bool mp = e->opt_mp == 1 || (e->opt_mp != 0 && e->mp);   // combiner window passes (slices smaller than chunks)
#define P3LAUNCH(NV, IT, VW) do { \
        if (kgm == 0) partition3_kernel<NV, IT, 1024, VW, 0><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec); \
        else if (kgm == 1) partition3_kernel<NV, IT, 1024, VW, 1><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec); \
        else partition3_kernel<NV, IT - 2, 1024, VW, 2><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec); } while (0)
    // (supplied key hashes: one column more per tile, two items fewer per lane keep the kernel free of VGPR spills)
#define PRELAUNCH(NV) do { const int gp = (int)std::max<int64_t>(1, std::min<int64_t>((a.n + 4095) / 4096, 256)); \
        if (kgm == 0) partition3_kernel<NV, 4, 1024, 3, 0, 1><<<gp, 1024, 0, e->stream>>>(pa, e->d_ec); \
        else if (kgm == 1) partition3_kernel<NV, 4, 1024, 3, 1, 1><<<gp, 1024, 0, e->stream>>>(pa, e->d_ec); \
        else partition3_kernel<NV, 4, 1024, 3, 2, 1><<<gp, 1024, 0, e->stream>>>(pa, e->d_ec); } while (0)
    if (pre) { if (e->nv == 0) PRELAUNCH(0); else PRELAUNCH(1); }
    else if (e->nv == 0) P3LAUNCH(0, 8, 3);
    else if (narrow) partition3_kernel<1, 6, 1024, 3, 0, 0, 1, 1><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec);
    else if (narrow2) partition3_kernel<2, 4, 1024, 1, 0, 0, 0, 2><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec);
    else if (e->nv == 1 && w16 && (vw & 1)) partition3_kernel<1, 6, 1024, 3, 0, 0, 1><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec);
    else if (e->nv == 1 && w16) partition3_kernel<1, 6, 1024, 2, 0, 0, 1><<<grid, 1024, 0, e->stream>>>(pa, e->d_ec);
    else if (e->nv == 1) { if (vw & 1) P3LAUNCH(1, 6, 3); else P3LAUNCH(1, 6, 2); }
    else if (vw == 3) P3LAUNCH(2, 4, 3); else if (vw == 2) P3LAUNCH(2, 4, 2);
    else if (vw == 1) P3LAUNCH(2, 4, 1); else P3LAUNCH(2, 4, 0);
#undef P3LAUNCH
#undef PRELAUNCH
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[5], e->stream));
    if (e->opt_profile) {
        int rc2 = print_phase_profile(e, "pprof", e->ev[4], e->ev[5], grid, 6);
        if (rc2) return rc2;
    }
    // no host round trip between the phases: Phase P marks touched slots itself, spills bucket
    // overflow to the v1 replay list, and the combiner applies stragglers in place
    CombineArgs ca;
    memset(&ca, 0, sizeof(ca));
    ca.b_key = e->d_bkey;
    ca.b_rel = e->d_brel;
    ca.b_n = pre ? e->d_bn : nullptr;
    ca.key_table = e->d_keys;
    ca.b_val0 = e->d_bval[0];
    ca.b_val1 = e->d_bval[1];
    ca.b_cnt = e->d_bcnt;
    ca.capb = e->capb;
    ca.seg_log = e->seg_log;
    ca.np = e->np;
    ca.sl = e->sl;
    ca.sub_major = pa.sub_major;
    ca.rel2slot = e->d_rel2slot;
    // (not with PRE buckets: Phase P applies merged entries past a full sub-bucket to the slots with device atomics
    // before this merge -- tests/test_skew_gpu.py::test_pre_entries_past_bucket_end_applied_with_atomics)
    ca.relfresh = pre ? nullptr : (const uint8_t*)(e->d_rel2slot + kRelCap) + kRelCap;
    ca.slot_base = e->d_slot_base;
    ca.stride = e->stride;
    ca.st = e->d_st;
    ca.prof = pa.prof;
    HIPCHK(e, hipEventRecord(e->ev[6], e->stream));
    const size_t seg3 = (size_t)1 << e->seg_log;
    const size_t lds3 = seg3 * 8 + 2 * seg3 * 4 + (size_t)(e->nacc_comb - 1) * 2 * seg3 * 8 + 4 * 4 * kSub + 16;
    // entries per lane and chunk: the largest counts whose kernels keep every value in registers at 1024 threads (a VGPR
    // spill is not harmless here, DESIGN.md section 4 "Skewed keys"; tests/test_abi.py checks the code object): 4, 3 with
    // two carried value columns, 6 for narrow entries, 2 with window passes. 512-thread blocks with twice the entries are
    // spill-free too but slower (r05 A/B, profiles/r05_combine_geometry_ab.txt). -D switches for A/B builds only.
#ifndef FWA_C3_TH
#define FWA_C3_TH 1024
#endif
#ifndef FWA_C3_IT0
#define FWA_C3_IT0 4
#endif
#ifndef FWA_C3_IT1
#define FWA_C3_IT1 4
#endif
#ifndef FWA_C3_IT2
#define FWA_C3_IT2 3
#endif
#ifndef FWA_C3_NIT
#define FWA_C3_NIT 6
#endif
#ifndef FWA_MP_IT
#define FWA_MP_IT 2
#endif
    constexpr int TH3 = FWA_C3_TH;
#define C3M(IT, NV, LY, PR) do { if (mp) combine3_kernel<FWA_MP_IT, 2, NV, TH3, LY, PR, 1><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec); \
        else combine3_kernel<IT, 2, NV, TH3, LY, PR, 0><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec); } while (0)
#define C3L(IT, NV) do { \
        if (pre && layout == 1) C3M(IT, 1, 1, 1); \
        else if (pre) C3M(IT, 0, 2, 1); \
        else if (layout == 1) C3M(IT, NV, 1, 0); \
        else if (layout == 2) C3M(IT, NV, 2, 0); \
        else C3M(IT, NV, 0, 0); } while (0)
    if (narrow) {   // packed entries free the prefetch registers: more entries per lane and chunk
        if (mp) combine3_kernel<FWA_MP_IT, 2, 1, TH3, 1, 0, 1, 1><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec);
        else combine3_kernel<FWA_C3_NIT, 2, 1, TH3, 1, 0, 0, 1><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec);
    } else if (narrow2) {
        if (mp) combine3_kernel<FWA_MP_IT, 2, 2, TH3, 0, 0, 1, 2><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec);
        else combine3_kernel<4, 2, 2, TH3, 0, 0, 0, 2><<<e->np, TH3, lds3, e->stream>>>(ca, e->d_ec);
    } else if (e->nv == 0) C3L(FWA_C3_IT0, 0);
    else if (e->nv == 1) C3L(FWA_C3_IT1, 1);
    else C3L(FWA_C3_IT2, 2);
#undef C3L
#undef C3M
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[7], e->stream));
    e->v2_timing_pending = true;
    if (e->opt_profile) {
        int rc2 = print_phase_profile(e, "aprof", e->ev[6], e->ev[7], e->np, 8);
        if (rc2) return rc2;
    }
    e->ingest_launches++;
    e->ingest_records += a.n;
    *ran = true;
    return FWA_OK;
}

// Sessions: classify -> route -> bulk gap-scan (sort by (kid, start), segmented max-scan,
// cluster ids, wave-segmented reduction) and the arrival-order walk for keys with order-sensitive records.
struct KidEq {                       // equal kid part of a (kid << tb | start - base) sort key
    int tb;
    __host__ __device__ bool operator()(unsigned long long x, unsigned long long y) const { return (x >> tb) == (y >> tb); }
};
struct MaxI64 {
    __host__ __device__ int64_t operator()(int64_t x, int64_t y) const { return x > y ? x : y; }
};

static int ensure_sort_tmp(fwa_engine* e, size_t bytes) {
    if (bytes <= e->sort_tmp_bytes) return FWA_OK;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->d_sort_tmp) HIPCHK(e, hipFree(e->d_sort_tmp));
    e->d_sort_tmp = nullptr;
    HIPCHK(e, hipMalloc(&e->d_sort_tmp, bytes + bytes / 4));
    e->sort_tmp_bytes = bytes + bytes / 4;
    return FWA_OK;
}

static int ensure_sess_lists(fwa_engine* e, int64_t need) {
    if (need <= e->ss_cap) return FWA_OK;
    const int64_t cap = std::max<int64_t>(need + need / 4, 1 << 12);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (int q = 0; q < 2; ++q) {
        SessList nl;
        nl.stride = cap;
        HIPCHK(e, hipMalloc(&nl.kid, 4 * (size_t)cap));
        HIPCHK(e, hipMalloc(&nl.start, 8 * (size_t)cap));
        HIPCHK(e, hipMalloc(&nl.end, 8 * (size_t)cap));
        HIPCHK(e, hipMalloc(&nl.acc, 8 * (size_t)cap * e->nacc));
        SessList& ol = e->ss[q];
        if (q == e->ss_cur && e->n_ss > 0) {             // keep the live sessions
            const size_t n = (size_t)e->n_ss;
            HIPCHK(e, hipMemcpy(nl.kid, ol.kid, 4 * n, hipMemcpyDeviceToDevice));
            HIPCHK(e, hipMemcpy(nl.start, ol.start, 8 * n, hipMemcpyDeviceToDevice));
            HIPCHK(e, hipMemcpy(nl.end, ol.end, 8 * n, hipMemcpyDeviceToDevice));
            for (int cc = 0; cc < e->nacc; ++cc)
                HIPCHK(e, hipMemcpy(nl.acc + (size_t)cc * cap, ol.acc + (size_t)cc * ol.stride, 8 * n, hipMemcpyDeviceToDevice));
        }
        for (void* p : {(void*)ol.kid, (void*)ol.start, (void*)ol.end, (void*)ol.acc}) if (p) HIPCHK(e, hipFree(p));
        ol = nl;
    }
    e->ss_cap = cap;
    return FWA_OK;
}

static int ensure_late_rows(fwa_engine* e, int64_t need);
static int emit_late_rows(fwa_engine* e);

static int read_sess_ctr(fwa_engine* e) {
    HIPCHK(e, hipMemcpyAsync(e->h_sctr, e->d_sctr, sizeof(SessCtr), hipMemcpyDeviceToHost, e->stream));
    return sync_status(e);
}

// Staging buffers, the segment walk (sess2_segment_kernel, or sess3_segment_kernel over cell keys), the scan of the
// per-wave counts and the compaction into s.out.
static int launch_segments(fwa_engine* e, Sess2Args& s, int64_t nb, bool cells) {
    const int64_t nw = (nb + 63) / 64;
    if (nb > e->sg_cap || nw + 1 > e->sgw_cap) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (e->d_sg) HIPCHK(e, hipFree(e->d_sg));
        e->d_sg = nullptr;
        e->sg_cap = std::max<int64_t>(nb + nb / 4, 1 << 14);
        e->sgw_cap = (e->sg_cap + 63) / 64 + 1;
        const size_t bytes = (size_t)e->sg_cap * (4 + 8 + 8 + 8 * (size_t)e->nacc) + (size_t)e->sgw_cap * (4 + 4 + 8) + 1024;
        HIPCHK(e, hipMalloc(&e->d_sg, bytes));
    }
    char* sp = (char*)e->d_sg;
    s.sg_start = (int64_t*)sp; sp += 8 * (size_t)e->sg_cap;
    s.sg_end = (int64_t*)sp; sp += 8 * (size_t)e->sg_cap;
    s.sg_acc = (unsigned long long*)sp; sp += 8 * (size_t)e->sg_cap * e->nacc;
    s.sg_h0 = (int64_t*)sp; sp += 8 * (size_t)e->sgw_cap;
    s.sg_kid = (uint32_t*)sp; sp += 4 * (size_t)e->sg_cap;
    s.sg_cnt = (uint32_t*)sp; sp += 4 * (size_t)e->sgw_cap;
    s.sg_off = (uint32_t*)sp;
    s.sg_cap = e->sg_cap;
    const unsigned sg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nb + 255) / 256, 1 << 16));
    switch (e->nacc) {
        case 1: if (cells) sess3_segment_kernel<1><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); else sess2_segment_kernel<1><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); break;
        case 2: if (cells) sess3_segment_kernel<2><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); else sess2_segment_kernel<2><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); break;
        case 3: if (cells) sess3_segment_kernel<3><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); else sess2_segment_kernel<3><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); break;
        case 4: if (cells) sess3_segment_kernel<4><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); else sess2_segment_kernel<4><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); break;
        default: if (cells) sess3_segment_kernel<5><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); else sess2_segment_kernel<5><<<sg, kBlock, 0, e->stream>>>(s, e->d_ec); break;
    }
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipMemsetAsync(s.sg_cnt + nw, 0, 4, e->stream));
    size_t bytes = 0;
    HIPCHK(e, hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s.sg_cnt, s.sg_off, (int)(nw + 1), e->stream));
    int rc = ensure_sort_tmp(e, bytes);
    if (rc) return rc;
    bytes = e->sort_tmp_bytes;
    HIPCHK(e, hipcub::DeviceScan::ExclusiveSum(e->d_sort_tmp, bytes, s.sg_cnt, s.sg_off, (int)(nw + 1), e->stream));
    sess2_compact_kernel<<<1024, kBlock, 0, e->stream>>>(s, nw, e->nacc);
    HIPCHK(e, hipGetLastError());
    return FWA_OK;
}

#include "sessions4_host.inc"

static int push_session(fwa_engine* e, IngestArgs& a, int64_t* dropped_out) {
    const int64_t n = a.n;
    const int64_t n_in = e->n_ss;
    int rc = FWA_OK;
    if (n + n_in > e->sb_cap) {                           // sort / scan buffers for every element of the push
        HIPCHK(e, hipStreamSynchronize(e->stream));
        const int64_t cap = std::max<int64_t>((n + n_in) + (n + n_in) / 4, 1 << 14);
        auto re = [&](void** p, size_t elem) -> int {
            if (*p) HIPCHK(e, hipFree(*p));
            *p = nullptr;
            HIPCHK(e, hipMalloc(p, elem * (size_t)cap));
            return FWA_OK;
        };
        for (int q = 0; q < 4; ++q) {
            if ((rc = re((void**)&e->d_skey[q], 8))) return rc;
            if ((rc = re((void**)&e->d_sval[q], 4))) return rc;
        }
        if ((rc = re((void**)&e->d_send2, 8)) || (rc = re((void**)&e->d_smax, 8)) || (rc = re((void**)&e->d_scid, 4)) ||
            (rc = re((void**)&e->d_rkid, 4)) || (rc = re((void**)&e->d_spk, 8 * (size_t)e->nacc)) || (rc = re((void**)&e->d_spe, 8)))
            return rc;
        e->sb_cap = cap;
    }
    if ((rc = ensure_sess_lists(e, n_in + n))) return rc;
    SessCtr z;
    memset(&z, 0, sizeof(z));
    z.ts_min = ~0ull;
    if ((rc = upload(e, e->d_sctr, &z, sizeof(z)))) return rc;
    HIPCHK(e, hipMemsetAsync(e->d_kflag, 0, (size_t)e->capacity + 1, e->stream));
    if ((rc = reset_push_status(e))) return rc;

    Sess2Args s;
    memset(&s, 0, sizeof(s));
    s.keys = a.keys;
    s.ts = a.ts;
    if (!e->tz.empty() && n > 0) {                        // Table GROUP BY SESSION over a TIMESTAMP_LTZ rowtime:
        if (n > e->lts_cap) {                             // sessions are formed on local wall-clock time
            if (e->d_lts) HIPCHK(e, hipFree(e->d_lts));
            e->d_lts = nullptr;
            HIPCHK(e, hipMalloc(&e->d_lts, 8 * (size_t)n));
            e->lts_cap = n;
        }
        to_local_kernel<<<grid_for(n), kBlock, 0, e->stream>>>(a.ts, e->d_lts, n, e->d_ec);
        HIPCHK(e, hipGetLastError());
        s.ts = e->d_lts;
    }
    for (int c = 0; c < FWA_MAX_COLS; ++c) s.cols[c] = a.cols[c];
    s.key_hash = a.key_hash;
    s.gapc = (e->cfg.flags & FWA_CFG_DYNAMIC_GAP) ? (const int64_t*)a.cols[e->cfg.gap_col] : nullptr;
    s.n = n;
    s.wm = local_wm(e, e->wm);
    s.gap = e->cfg.gap_ms;
    s.lateness = e->lateness;
    s.key_table = e->d_keys;
    s.key_mask = (uint64_t)e->capacity - 1;
    s.seg_log = e->seg_log;
    s.part_bits = e->part_bits;
    s.capacity = e->capacity;
    s.rkid = e->d_rkid;
    s.kflag = e->d_kflag;
    s.in = e->ss[e->ss_cur];
    s.n_in = n_in;
    s.out = e->ss[e->ss_cur ^ 1];
    for (int cc = 0; cc <= kMaxAggsInt; ++cc) s.col_owner[cc] = -1;
    for (int j = 0; j < e->ec.naggs; ++j)
        if (e->ec.agg[j].acc > 0 && !e->ec.agg[j].alias) s.col_owner[e->ec.agg[j].acc] = j;
    for (int col = 0; col < FWA_MAX_COLS; ++col) s.nulls[col] = a.nulls[col];
    s.ctr = e->d_sctr;
    s.dropidx = a.dropidx;
    s.st = e->d_st;
    // cell path (sess3_*): fixed gap, 32-bit cell keys; redone on the general path below when a record is not
    // order-free or a start falls outside the cell range (then not tried again for 8 pushes)
    const int cb = 32 - e->kid_bits;
    // cell pre-aggregation (sessions4.inc) first; cells or sessions out of its range: the sort-based cell path
    bool s4_general = false;
    if (e->opt_cells != 0 && !s.gapc && e->nacc <= 5 && n > 0 && e->cell_skip <= 0 && n + n_in < ((int64_t)1 << 31) &&
        e->cfg.gap_ms > 0 && e->cfg.gap_ms <= ((int64_t)1 << 27) && e->capacity < ((int64_t)1 << 27) &&
        (e->capacity + 1 + kS4Kids - 1) / kS4Kids <= 24576) {
        int verdict = 1;
        if ((rc = push_session_s4(e, s, n, n_in, dropped_out, &verdict))) return rc;
        if (verdict == 0) { e->sess_path = 2; return FWA_OK; }
        s4_general = verdict == 2;
        memset(&z, 0, sizeof(z));
        z.ts_min = ~0ull;
        if ((rc = upload(e, e->d_sctr, &z, sizeof(z)))) return rc;
        if ((rc = reset_push_status(e))) return rc;
    }
    bool tried3 = false;
    if (e->opt_cells != 0 && !s4_general && !s.gapc && cb >= 1 && e->nacc <= 5 && n > 0 && e->cell_skip <= 0 &&
        n + n_in < ((int64_t)1 << 31)) {
        tried3 = true;
        Sess2Args t = s;
        t.tb = cb;
        t.gap_div = jm::udiv64_make((uint64_t)e->cfg.gap_ms);
        t.nb = n + n_in;
        t.bkey = e->d_skey[0];
        t.bval = e->d_sval[0];
        t.pk = e->d_spk;
        t.pkw = e->nacc;
        t.seg_out = 1;
        HIPCHK(e, hipEventRecord(e->ev[0], e->stream));
        sess3_min_kernel<<<grid_for(n + n_in, 1024), kBlock, 0, e->stream>>>(t);
        const int G = (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 2047) / 2048));   // >= 32 waves per CU (latency-bound probes)
        const int64_t chunk = ((n + G - 1) / G + 255) / 256 * 256;
        sess3_route_kernel<2><<<G, kBlock, 0, e->stream>>>(t, e->d_ec, chunk);
        if (n_in > 0) sess3_route_sessions_kernel<<<grid_for(n_in, 256 * 16), kBlock, 0, e->stream>>>(t);
        HIPCHK(e, hipGetLastError());
        size_t bytes = 0;
        const uint32_t* k0 = (const uint32_t*)e->d_skey[0];
        uint32_t* k1 = (uint32_t*)e->d_skey[1];
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k0, k1, (const uint32_t*)e->d_sval[0], e->d_sval[1],
                                                     (int)t.nb, 0, 32, e->stream));
        if ((rc = ensure_sort_tmp(e, bytes))) return rc;
        bytes = e->sort_tmp_bytes;
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(e->d_sort_tmp, bytes, k0, k1, (const uint32_t*)e->d_sval[0], e->d_sval[1],
                                                     (int)t.nb, 0, 32, e->stream));
        t.bkey = e->d_skey[1];
        t.bval = e->d_sval[1];
        if ((rc = launch_segments(e, t, t.nb, true))) return rc;
        HIPCHK(e, hipEventRecord(e->ev[1], e->stream));
        if ((rc = read_sess_ctr(e))) return rc;
        if (e->h_st->error) return FWA_OK;                // reported by the caller
        if (e->h_sctr->n_special == 0 && e->h_sctr->n_redo == 0) {
            if ((rc = account_ingest(e))) return rc;
            e->ingest_launches++;
            e->ingest_records += n;
            e->n_ss = (int64_t)e->h_sctr->n_out_sp;
            e->ss_cur ^= 1;
            *dropped_out = (int64_t)e->h_st->dropped;
            e->sess_path = 1;
            return FWA_OK;
        }
        e->cell_skip = 8;                                 // the general path redoes the push (key inserts are idempotent)
        e->replay_records += n;
        memset(&z, 0, sizeof(z));
        z.ts_min = ~0ull;
        if ((rc = upload(e, e->d_sctr, &z, sizeof(z)))) return rc;
        HIPCHK(e, hipMemsetAsync(e->d_kflag, 0, (size_t)e->capacity + 1, e->stream));
        if ((rc = reset_push_status(e))) return rc;
    }
    e->sess_path = 0;
    if (s4_general) {
        e->cell_skip = 8;                                 // as the cell path: not tried again for 8 pushes
        e->replay_records += n;
    } else if (!tried3 && e->cell_skip > 0) {
        --e->cell_skip;
    }
    HIPCHK(e, hipEventRecord(e->ev[0], e->stream));
    if (n > 0) sess2_classify_kernel<<<grid_for(n, 256 * 32), kBlock, 0, e->stream>>>(s, e->d_ec);
    if (n_in > 0) sess2_range_kernel<<<grid_for(n_in, 256 * 32), kBlock, 0, e->stream>>>(s);
    HIPCHK(e, hipGetLastError());
    if ((rc = read_sess_ctr(e))) return rc;
    if (e->h_st->error) return FWA_OK;                    // reported by the caller
    const SessCtr c1 = *e->h_sctr;
    if (n + n_in == 0 || c1.ts_min > c1.ts_max) {         // nothing to do (empty push, no sessions)
        *dropped_out = 0;
        return FWA_OK;
    }
    const int64_t lo = jm::unord_i64(c1.ts_min), hi = jm::unord_i64(c1.ts_max);
    const uint64_t span = (uint64_t)hi - (uint64_t)lo;
    int tb = 0;
    while (tb < 64 && (span >> tb) != 0) ++tb;
    s.base = lo;
    s.tb = tb;
    s.all_sp = e->kid_bits + tb > 64 ? 1 : 0;                // start range too wide for one sort key
    if (s.all_sp) s.tb = 0;
    s.bkey = e->d_skey[0];
    s.bval = e->d_sval[0];
    s.pk = e->d_spk;
    s.pe = e->d_spe;
    s.pkw = e->nacc;
    s.skey = e->d_skey[2];
    s.sval = e->d_sval[2];
    sess2_route_kernel<<<(unsigned)((n + n_in + (int64_t)kBlock * kRouteItems - 1) / ((int64_t)kBlock * kRouteItems)), kBlock, 0,
                         e->stream>>>(s, e->d_ec);
    HIPCHK(e, hipGetLastError());
    if ((rc = read_sess_ctr(e))) return rc;
    const int64_t nb = (int64_t)e->h_sctr->n_bulk, nsp = (int64_t)e->h_sctr->n_sp;
    s.nb = nb;
    s.nsp = nsp;
    s.bend = e->d_send2;
    s.bmax = e->d_smax;
    s.bcid = e->d_scid;
    if (nb > 0) {
        size_t bytes = 0;
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned long long*)e->d_skey[0], e->d_skey[1],
                                                     (const uint32_t*)e->d_sval[0], e->d_sval[1], (int)nb, 0, e->kid_bits + tb, e->stream));
        if ((rc = ensure_sort_tmp(e, bytes))) return rc;
        bytes = e->sort_tmp_bytes;
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(e->d_sort_tmp, bytes, (const unsigned long long*)e->d_skey[0], e->d_skey[1],
                                                     (const uint32_t*)e->d_sval[0], e->d_sval[1], (int)nb, 0, e->kid_bits + tb, e->stream));
        s.bkey = e->d_skey[1];
        s.bval = e->d_sval[1];
    }
    s.seg_out = e->nacc <= 5 ? 1 : 0;
    if (nb > 0 && s.seg_out) {
        if ((rc = launch_segments(e, s, nb, false))) return rc;
    } else if (nb > 0) {
        size_t bytes = 0;
        sess2_ends_kernel<<<grid_for(nb, 256 * 32), kBlock, 0, e->stream>>>(s);
        HIPCHK(e, hipGetLastError());
        KidEq eq{tb};
        bytes = 0;
        HIPCHK(e, hipcub::DeviceScan::InclusiveScanByKey(nullptr, bytes, (const unsigned long long*)s.bkey, (const int64_t*)s.bend,
                                                         s.bmax, MaxI64(), (int)nb, eq, e->stream));
        if ((rc = ensure_sort_tmp(e, bytes))) return rc;
        bytes = e->sort_tmp_bytes;
        HIPCHK(e, hipcub::DeviceScan::InclusiveScanByKey(e->d_sort_tmp, bytes, (const unsigned long long*)s.bkey, (const int64_t*)s.bend,
                                                         s.bmax, MaxI64(), (int)nb, eq, e->stream));
        Sess2Args h = s;
        h.bcid = e->d_sval[0];                               // head flags (the unsorted payload is dead)
        sess2_heads_kernel<<<grid_for(nb, 256 * 32), kBlock, 0, e->stream>>>(h);
        HIPCHK(e, hipGetLastError());
        bytes = 0;
        HIPCHK(e, hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const uint32_t*)h.bcid, s.bcid, (int)nb, e->stream));
        if ((rc = ensure_sort_tmp(e, bytes))) return rc;
        bytes = e->sort_tmp_bytes;
        HIPCHK(e, hipcub::DeviceScan::InclusiveSum(e->d_sort_tmp, bytes, (const uint32_t*)h.bcid, s.bcid, (int)nb, e->stream));
        sess2_init_kernel<<<grid_for(nb, 256 * 32), kBlock, 0, e->stream>>>(s, e->d_ec);
        sess2_reduce_kernel<<<grid_for(nb, 256 * 32), kBlock, 0, e->stream>>>(s, e->d_ec);
        HIPCHK(e, hipGetLastError());
    }
    if (nsp > 0) {
        if (nsp > e->sc_cap) {
            HIPCHK(e, hipStreamSynchronize(e->stream));
            if (e->d_sc) HIPCHK(e, hipFree(e->d_sc));
            e->d_sc = nullptr;
            e->sc_cap = nsp + nsp / 4 + 1024;
            HIPCHK(e, hipMalloc(&e->d_sc, 8 * (size_t)e->sc_cap * (2 + e->nacc)));
        }
        size_t bytes = 0;
        const int eb = std::min(64, 32 + e->kid_bits);
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned long long*)e->d_skey[2], e->d_skey[3],
                                                     (const uint32_t*)e->d_sval[2], e->d_sval[3], (int)nsp, 0, eb, e->stream));
        if ((rc = ensure_sort_tmp(e, bytes))) return rc;
        bytes = e->sort_tmp_bytes;
        HIPCHK(e, hipcub::DeviceRadixSort::SortPairs(e->d_sort_tmp, bytes, (const unsigned long long*)e->d_skey[2], e->d_skey[3],
                                                     (const uint32_t*)e->d_sval[2], e->d_sval[3], (int)nsp, 0, eb, e->stream));
        s.skey = e->d_skey[3];
        s.sval = e->d_sval[3];
        s.sc_start = e->d_sc;
        s.sc_end = e->d_sc + nsp;
        s.sc_acc = (unsigned long long*)(e->d_sc + 2 * nsp);
        if ((rc = ensure_late_rows(e, e->late_rows + nsp))) return rc;
        if (!e->d_lr_n) HIPCHK(e, hipMalloc(&e->d_lr_n, 8));
        if ((rc = upload(e, e->d_lr_n, &e->late_rows, 8))) return rc;
        s.lr_key = e->lr_col[0];
        s.lr_start = e->lr_col[1];
        s.lr_end = e->lr_col[2];
        for (int j = 0; j < e->cfg.num_aggs; ++j) s.lr_agg[j] = e->lr_col[3 + j];
        s.lr_n = e->d_lr_n;
        s.lr_cap = e->lr_cap;
        sess2_ordered_kernel<<<grid_for(nsp, 256 * 32), kBlock, 0, e->stream>>>(s, e->d_ec);
        HIPCHK(e, hipGetLastError());
    }
    HIPCHK(e, hipEventRecord(e->ev[1], e->stream));
    uint32_t ncl = 0;
    unsigned long long lrn = (unsigned long long)e->late_rows;
    if (nb > 0 && !s.seg_out) HIPCHK(e, hipMemcpyAsync(&ncl, e->d_scid + nb - 1, 4, hipMemcpyDeviceToHost, e->stream));
    if (nsp > 0) HIPCHK(e, hipMemcpyAsync(&lrn, e->d_lr_n, 8, hipMemcpyDeviceToHost, e->stream));
    if ((rc = read_sess_ctr(e))) return rc;
    if ((rc = account_ingest(e))) return rc;
    e->ingest_launches++;
    e->ingest_records += n;
    if (e->h_st->error) return FWA_OK;
    e->late_rows = (int64_t)lrn;
    e->n_ss = (int64_t)ncl + (int64_t)e->h_sctr->n_out_sp;
    e->ss_cur ^= 1;
    *dropped_out = (int64_t)e->h_st->dropped;
    return FWA_OK;
}

// Watermark advance for sessions: late-firing rows of the pushes since the last call first, then every
// session with prev < end - 1 <= wm; sessions past cleanup are dropped from the list.
static int fire_sessions(fwa_engine* e, int64_t wm, int64_t* nrows) {
    const int64_t n_in = e->n_ss;
    int rc = ensure_out(e, e->late_rows + n_in);
    if (rc) return rc;
    if (e->late_rows > 0 && (rc = emit_late_rows(e))) return rc;
    if ((rc = upload(e, &e->d_st->rows, &e->late_rows, 8))) return rc;
    SessCtr z;
    memset(&z, 0, sizeof(z));
    if ((rc = upload(e, e->d_sctr, &z, sizeof(z)))) return rc;
    if ((rc = ensure_sess_lists(e, n_in))) return rc;
    Sess2FireArgs f;
    memset(&f, 0, sizeof(f));
    f.in = e->ss[e->ss_cur];
    f.out = e->ss[e->ss_cur ^ 1];
    f.n_in = n_in;
    f.prev_wm = local_wm(e, e->wm);
    f.wm = local_wm(e, wm);
    f.lateness = e->lateness;
    f.key_table = e->d_keys;
    f.capacity = e->capacity;
    f.o_key = e->o_key;
    f.o_start = e->o_start;
    f.o_end = e->o_end;
    for (int j = 0; j < e->cfg.num_aggs; ++j) { f.o_agg[j] = e->o_agg[j]; f.o_null[j] = e->o_null[j]; }
    f.out_cap = e->out_cap;
    f.ctr = e->d_sctr;
    f.st = e->d_st;
    HIPCHK(e, hipEventRecord(e->ev[2], e->stream));
    if (n_in > 0)
        sess2_fire_kernel<<<(unsigned)((n_in + (int64_t)kBlock * kSessFireItems - 1) / ((int64_t)kBlock * kSessFireItems)), kBlock, 0,
                            e->stream>>>(f, e->d_ec);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[3], e->stream));
    if ((rc = read_sess_ctr(e))) return rc;
    if (e->h_st->error) return fail(e, e->h_st->error, "session fire failed");
    *nrows = (int64_t)e->h_st->rows;
    e->n_ss = (int64_t)e->h_sctr->n_keep;
    e->ss_cur ^= 1;
    e->late_rows = 0;
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->fire_ms += ms;
    e->fire_launches++;
    e->fire_rows += *nrows;
    return FWA_OK;
}

// Fire kernel over a list of windows (each a union of slots). raw = 1 emits the accumulators and
// COUNT(*) instead of the final aggregate values (fwa_drain_partials).
static int emit_late_rows(fwa_engine* e);
// Enqueue the fire of windows hw (slot lists hs) into the output columns (rows from row0 on; no host wait).
static int enqueue_fire(fwa_engine* e, const std::vector<FireWindow>& hw, const std::vector<int32_t>& hs, int raw) {
    FireArgs f;
    memset(&f, 0, sizeof(f));
    f.key_table = e->d_keys;
    f.capacity = e->capacity;
    f.stride = e->stride;
    f.slot_base = e->d_slot_base;
    f.win = e->d_win;
    f.win_slots = e->d_win_slots;
    f.nwin = (int32_t)hw.size();
    f.blocks_per_win = (int32_t)((e->capacity + 1 + (int64_t)kBlock * kFireJ - 1) / ((int64_t)kBlock * kFireJ));
    f.o_key = e->o_key;
    f.o_start = e->o_start;
    f.o_end = e->o_end;
    for (int j = 0; j < e->cfg.num_aggs; ++j) { f.o_agg[j] = e->o_agg[j]; f.o_null[j] = e->o_null[j]; }
    f.o_count = raw ? e->o_count : nullptr;
    for (int h = 0; h < e->ec.naggs - e->ec.nout; ++h) f.o_hid[h] = e->o_hid[h];
    f.raw = raw;
    f.out_cap = e->out_cap;
    f.st = e->d_st;
    const int64_t grid = (int64_t)f.blocks_per_win * (int64_t)hw.size();
    HIPCHK(e, hipEventRecord(e->ev[2], e->stream));
    // one stateful accumulator column, every window one slot (a raw export of a nullable handle also
    // writes the hidden counters: the generic path)
    bool single = e->nacc == 2 && !(raw && e->ec.naggs > e->ec.nout);
    for (const FireWindow& w : hw) single = single && w.nslots == 1;
    const bool multi = !raw && e->nacc >= 3 && e->nacc <= 5 && !(e->opt_variant & 32) &&   // variant bit 5: A/B
                       std::all_of(hw.begin(), hw.end(), [](const FireWindow& w) { return w.nslots == 1; });
    if (e->red) red_fire_kernel<<<(unsigned)grid, kBlock, 0, e->stream>>>(f, e->d_ec);
    else if (multi) {
        f.blocks_per_win = (int32_t)((e->capacity + 1 + (int64_t)kBlock * 4 - 1) / ((int64_t)kBlock * 4));
        const unsigned g2 = (unsigned)((int64_t)f.blocks_per_win * (int64_t)hw.size());
        if (e->nacc == 3) fire_multi_kernel<3><<<g2, kBlock, 0, e->stream>>>(f, e->d_ec);
        else if (e->nacc == 4) fire_multi_kernel<4><<<g2, kBlock, 0, e->stream>>>(f, e->d_ec);
        else fire_multi_kernel<5><<<g2, kBlock, 0, e->stream>>>(f, e->d_ec);
    } else if (single) fire_kernel<1><<<(unsigned)grid, kBlock, 0, e->stream>>>(f, e->d_ec);
    else fire_kernel<0><<<(unsigned)grid, kBlock, 0, e->stream>>>(f, e->d_ec);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[3], e->stream));
    return FWA_OK;
}

// Windows and their slot list to the device (one upload through the arena).
static int upload_windows(fwa_engine* e, const std::vector<FireWindow>& hw, const std::vector<int32_t>& hs) {
    if ((int32_t)hw.size() > e->win_cap || (int32_t)hs.size() > e->win_slots_cap) {
        if (e->d_win) HIPCHK(e, hipFree(e->d_win));
        e->d_win = nullptr;
        e->win_cap = std::max<int32_t>(e->win_cap, (int32_t)hw.size() * 2);
        e->win_slots_cap = std::max<int32_t>(e->win_slots_cap, (int32_t)hs.size() * 2);
        HIPCHK(e, hipMalloc(&e->d_win, sizeof(FireWindow) * e->win_cap + sizeof(int32_t) * e->win_slots_cap));
        e->d_win_slots = (int32_t*)(e->d_win + e->win_cap);
    }
    std::vector<char> wbuf(sizeof(FireWindow) * e->win_cap + sizeof(int32_t) * hs.size());
    memcpy(wbuf.data(), hw.data(), sizeof(FireWindow) * hw.size());
    memcpy(wbuf.data() + sizeof(FireWindow) * e->win_cap, hs.data(), sizeof(int32_t) * hs.size());
    return upload(e, e->d_win, wbuf.data(), wbuf.size());
}

static int launch_fire(fwa_engine* e, const std::vector<FireWindow>& hw, const std::vector<int32_t>& hs, int raw,
                       int64_t* nrows, int64_t row0 = 0) {
    int rc = upload_windows(e, hw, hs);
    if (rc) return rc;
    // rows <= windows x distinct keys; n_keys is current: every push ends with a status sync
    const int64_t nkeys = std::max<int64_t>((int64_t)e->h_st->n_keys, 1);
    // Output sizing: rows <= windows x live keys, which is tens of GB for 1e8 keys (C4) although a
    // window holds far fewer rows. Start from min(bound, max(current capacity, 4M rows)); the kernel
    // counts rows past the capacity without writing them, and the host grows once and relaunches.
    const int64_t bound = (int64_t)hw.size() * nkeys + row0;
    const int64_t floor_rows = e->opt_out_min > 0 ? e->opt_out_min : ((int64_t)1 << 22);   // tests force the relaunch
    rc = ensure_out(e, std::min<int64_t>(bound, std::max<int64_t>(e->out_cap, floor_rows + row0)));
    if (rc) return rc;
  relaunch:
    if (row0 > 0) {   // late-firing rows of the pushes since the last watermark go first
        rc = emit_late_rows(e);
        if (rc) return rc;
        rc = upload(e, &e->d_st->rows, &row0, 8);
        if (rc) return rc;
    } else {
        HIPCHK(e, hipMemsetAsync(&e->d_st->rows, 0, 8, e->stream));
    }
    rc = enqueue_fire(e, hw, hs, raw);
    if (rc) return rc;
    rc = sync_status(e);
    if (rc) return rc;
    *nrows = (int64_t)e->h_st->rows;
    if (*nrows > e->out_cap) {   // more rows than the first sizing: grow (2x headroom for the following
        rc = ensure_out(e, std::max<int64_t>(*nrows, std::min<int64_t>(bound, 2 * *nrows)));   // fires), fire again
        if (rc) return rc;
        goto relaunch;
    }
    if (row0 > 0) e->late_rows = 0;   // consumed (emit_late_rows copied them to the head of the output);
                                      // a snapshot / drain fire (row0 == 0) leaves them for the next watermark
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->fire_ms += ms;
    e->fire_launches++;
    e->fire_rows += *nrows - row0;
    return FWA_OK;
}

// Capacity of the late-firing row buffer (rows returned by the next fwa_advance_watermark); keeps its rows.
static int ensure_late_rows(fwa_engine* e, int64_t need) {
    if (need <= e->lr_cap) return FWA_OK;
    const int64_t cap = std::max<int64_t>(need * 2, 1024);
    for (int c = 0; c < 3 + e->cfg.num_aggs; ++c) {
        int64_t* p = nullptr;
        HIPCHK(e, hipMalloc(&p, 8 * (size_t)cap));
        if (e->lr_col[c]) {
            if (e->late_rows) HIPCHK(e, hipMemcpyAsync(p, e->lr_col[c], 8 * (size_t)e->late_rows, hipMemcpyDeviceToDevice, e->stream));
            HIPCHK(e, hipStreamSynchronize(e->stream));
            HIPCHK(e, hipFree(e->lr_col[c]));
        }
        e->lr_col[c] = p;
    }
    e->lr_cap = cap;
    return FWA_OK;
}

// Late firings of one push (DataStream, allowed lateness > 0): apply the deferred records in arrival order
// and emit the fired windows' contents into the late-row buffer (late_fire_kernel). The rows are returned
// by the next fwa_advance_watermark, ahead of the windows that watermark fires.
static int process_late(fwa_engine* e, const IngestArgs& a0, std::vector<int32_t>& idx) {
    std::sort(idx.begin(), idx.end());
    const int64_t n = (int64_t)idx.size();
    if (n > e->spill_cap) return fail(e, FWA_E_STATE, "late list overflow");
    HIPCHK(e, hipMemcpyAsync(e->d_late, idx.data(), 4 * (size_t)n, hipMemcpyHostToDevice, e->stream));
    const int64_t per = e->kind == FWA_SLIDE ? (e->size + e->slide - 1) / e->slide : 1;
    int rc0 = ensure_late_rows(e, e->late_rows + n * per);
    if (rc0) return rc0;
    if (!e->d_lr_n) HIPCHK(e, hipMalloc(&e->d_lr_n, 8));
    HIPCHK(e, hipMemcpyAsync(e->d_lr_n, &e->late_rows, 8, hipMemcpyHostToDevice, e->stream));
    if (e->dir_dirty) { int rc = publish_dir(e); if (rc) return rc; }
    LateArgs L;
    memset(&L, 0, sizeof(L));
    L.in = a0;
    L.in.key_table = e->d_keys;
    L.in.key_mask = (uint64_t)e->capacity - 1;
    L.in.seg_log = e->seg_log;
    L.in.part_bits = e->part_bits;
    L.in.dir = e->d_dir;
    L.in.dir_mask = e->dir_cap - 1;
    L.in.touched = e->d_touched;
    L.in.slot_base = e->d_slot_base;
    L.in.stride = e->stride;
    L.in.st = e->d_st;
    L.in.wm = e->wm;
    L.order = e->d_late;
    L.n = n;
    L.kind = e->kind;
    L.size = e->size;
    L.slide = e->kind == FWA_SLIDE ? e->slide : e->size;
    L.slide_div = e->kind == FWA_SLIDE ? e->slide_div : e->size_div;
    L.lateness = e->lateness;
    L.o_key = e->lr_col[0];
    L.o_start = e->lr_col[1];
    L.o_end = e->lr_col[2];
    for (int j = 0; j < e->cfg.num_aggs; ++j) L.o_agg[j] = e->lr_col[3 + j];
    L.rows = e->d_lr_n;
    if (e->red) red_late_fire_kernel<<<1, 64, 0, e->stream>>>(L, e->d_ec, e->red_seq_base + e->records_in);
    else late_fire_kernel<<<1, 64, 0, e->stream>>>(L, e->d_ec);
    HIPCHK(e, hipGetLastError());
    unsigned long long rows = 0;
    HIPCHK(e, hipMemcpyAsync(&rows, e->d_lr_n, 8, hipMemcpyDeviceToHost, e->stream));
    int rc = sync_status(e);   // also mirrors the touched flags the kernel set
    if (rc) return rc;
    if (e->h_st->error) return fail(e, e->h_st->error, "late firing failed");
    e->late_rows = (int64_t)rows;
    return FWA_OK;
}

// Copy the pending late-firing rows to the front of the output columns (rows [0, late_rows)).
static int emit_late_rows(fwa_engine* e) {
    for (int c = 0; c < 3 + e->cfg.num_aggs; ++c) {
        void* dst = c == 0 ? (void*)e->o_key : c == 1 ? (void*)e->o_start : c == 2 ? (void*)e->o_end : e->o_agg[c - 3];
        const size_t w = c < 3 ? 8 : type_size(e->cfg.aggs[c - 3].kind);
        HIPCHK(e, hipMemcpyAsync(dst, e->lr_col[c], w * (size_t)e->late_rows, hipMemcpyDeviceToDevice, e->stream));
    }
    return FWA_OK;   // the caller clears late_rows once the output is final
}

// FWA_CFG_LATE_INDICES: fetch the dropped-record indices of the push just settled (ascending).
static int collect_late_indices(fwa_engine* e) {
    unsigned long long m = 0;
    HIPCHK(e, hipMemcpy(&m, &e->d_st->drop_n, 8, hipMemcpyDeviceToHost));
    e->late_idx.resize((size_t)m);
    if (m) HIPCHK(e, hipMemcpy(e->late_idx.data(), e->d_dropidx, 4 * (size_t)m, hipMemcpyDeviceToHost));
    std::sort(e->late_idx.begin(), e->late_idx.end());
    return FWA_OK;
}

// FWA_KEY_PREHASHED: read-only probe of the key table (the key's kid, or -1), in key_slot's probe order.
__device__ __forceinline__ int64_t key_find(const unsigned long long* table, uint64_t mask, int seg_log, int part_bits,
                                            int64_t key) {
    if ((uint64_t)key == kEmptyKey) return table[mask + 1] == 1ull ? (int64_t)(mask + 1) : -1;
    const uint64_t h = jm::mix64((uint64_t)key);
    const uint64_t base = seg_base(h, seg_log, part_bits);
    const uint64_t smask = ((uint64_t)1 << seg_log) - 1;
    const uint64_t home = h & smask & ~(uint64_t)(kBucket - 1);
    for (uint64_t probe = 0; probe <= smask; ++probe) {
        const uint64_t i = base | ((home + probe) & smask);
        const unsigned long long cur = table[i];
        if (cur == (unsigned long long)key) return (int64_t)i;
        if (cur == kEmptyKey) return -1;
    }
    return -1;
}

// Keep each key's caller-supplied key.hashCode() by kid (after a push inserted its keys): snapshots place the keys in
// their key groups with it (KeyGroupRangeAssignment.assignToKeyGroup(key.hashCode())).
__global__ void __launch_bounds__(kBlock) khash_fill_kernel(const int64_t* keys, const int32_t* kh, int64_t n,
                                                            const unsigned long long* table, uint64_t mask, int seg_log,
                                                            int part_bits, int32_t* khash) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kid = key_find(table, mask, seg_log, part_bits, keys[i]);
        if (kid >= 0) khash[kid] = kh[i];
    }
}

// The kept hash of each of n keys (0 for a key the table does not hold).
__global__ void __launch_bounds__(kBlock) khash_rows_kernel(const int64_t* keys, int64_t n, const unsigned long long* table,
                                                            uint64_t mask, int seg_log, int part_bits,
                                                            const int32_t* khash, int32_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kid = key_find(table, mask, seg_log, part_bits, keys[i]);
        out[i] = kid >= 0 ? khash[kid] : 0;
    }
}

// After a push on a PREHASHED handle that inserted keys: record their hashes (the push's own key / hash columns, still
// valid here; the stream is waited for, since the caller may release them when the call returns).
static int khash_fill(fwa_engine* e, const int64_t* keys, const int32_t* kh, int64_t n) {
    if (!e->d_khash || n <= 0 || !keys || !kh || e->h_st->n_keys == e->khash_nkeys) return FWA_OK;
    khash_fill_kernel<<<grid_for(n), kBlock, 0, e->stream>>>(keys, kh, n, e->d_keys, (uint64_t)e->capacity - 1,
                                                             e->seg_log, e->part_bits, e->d_khash);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->khash_nkeys = e->h_st->n_keys;
    return FWA_OK;
}

// Shared ingest driver: two-phase path when allowed, else the v1 kernel; slice-miss replays;
// lookahead slice allocation; stats.
static int push_settle(fwa_engine* e, IngestArgs& a, int64_t n, bool ran_v2, bool status_enqueued,
                       int64_t* late_dropped_out);

static int finish_afire(fwa_engine* e);

// Settle an FWA_PUSH_ASYNC push (the pushes do this first: an asynchronous watermark's fire may keep running).
static int settle_push(fwa_engine* e) {
    if (!e->pend) return FWA_OK;
    e->pend = false;
    IngestArgs a = e->pend_a;
    return push_settle(e, a, e->pend_n, e->pend_v2, true, nullptr);
}

// ... and every other stateful entry point: also account a completed fwa_advance_watermark_async fire.
static int settle_pending(fwa_engine* e) {
    if (int rc = finish_afire(e)) return rc;
    return settle_push(e);
}

static int push_common(fwa_engine* e, IngestArgs& a, int64_t n, bool allow_v2, bool async, int64_t* late_dropped_out) {
    if (e->sparse) return sp_push(e, a, n, async ? nullptr : late_dropped_out);   // settled at once; async: count via stats
    if (++e->push_epoch == INT32_MAX) { e->push_epoch = 1; e->rs_valid = false; }   // (epochs wrap: carried sums dropped)
    int rc = FWA_OK;
    bool ran_v2 = false;
    if (e->v2 && allow_v2) {
        rc = push_v2(e, a, &ran_v2);
        if (rc) return rc;
    }
    if (!ran_v2) {
        rc = reset_push_status(e);
        if (rc) return rc;
        rc = launch_ingest(e, a, false);
        if (rc) return rc;
    }
    if (async) {   // settled by the next call on the handle (settle_pending)
        rc = enqueue_status(e);
        if (rc) return rc;
        e->pend = true;
        e->pend_a = a;
        e->pend_n = n;
        e->pend_v2 = ran_v2;
        return FWA_OK;
    }
    return push_settle(e, a, n, ran_v2, false, late_dropped_out);
}

// Second half of a push: read the device status, replay missed records (allocating their slices),
// extend the lookahead, account. status_enqueued: the first status copy is already in the stream.
static int push_settle(fwa_engine* e, IngestArgs& a, int64_t n, bool ran_v2, bool status_enqueued,
                       int64_t* late_dropped_out) {
    int rc = FWA_OK;
    int64_t dropped = 0;
    int64_t qmin = LONG_MAX_J, qmax = LONG_MIN_J;
    bool republish = false;
    std::vector<int32_t> late_idx;
    for (int round = 0;; ++round) {
        if (round == 0 && status_enqueued && e->st_ready) rc = FWA_OK;   // waited by wait_status_event
        else rc = (round == 0 && status_enqueued) ? wait_status(e) : sync_status(e);
        e->st_ready = false;
        if (rc) return rc;
        if (e->v2_timing_pending) {
            float ms = 0.f;
            HIPCHK(e, hipEventElapsedTime(&ms, e->ev[4], e->ev[5]));
            e->partition_ms += ms;
            e->ingest_ms += ms;
            HIPCHK(e, hipEventElapsedTime(&ms, e->ev[6], e->ev[7]));
            e->combine_ms += ms;
            e->ingest_ms += ms;
            e->v2_timing_pending = false;
        }
        if (!ran_v2 || round > 0) { rc = account_ingest(e); if (rc) return rc; }
        const DevStatus st = *e->h_st;
        if (ran_v2 && round == 0 && (int64_t)st.ovf_n * 64 > n) e->pre = true;   // skewed keys: PRE from the next push
        if (ran_v2 && round == 0 && (int64_t)st.strag_n * 64 > n) e->mp = true;  // wide chunks: window passes
        if (ran_v2 && round == 0 && e->narrow_used && (int64_t)st.wide_n * 64 > n) e->narrow = false;   // 64-bit keys / values
        if (st.error) {
            const char* m = st.error == FWA_E_KEYGROUP ? "Key group is not in the owned KeyGroupRange (StateTable.getMapForKeyGroup)"
                          : st.error == FWA_E_TS_MIN ? "Record has Long.MIN_VALUE timestamp (= no timestamp marker)."
                          : st.error == FWA_E_OOM ? (st.key_full ? "key table full: raise fwa_config.key_capacity" : "slice want-set overflow")
                                                  : "device error";
            return fail(e, st.error, m);
        }
        if (st.late_fire) {   // deferred late-firing records of this round (the next round resets the list)
            const size_t o = late_idx.size();
            late_idx.resize(o + st.late_fire);
            HIPCHK(e, hipMemcpy(late_idx.data() + o, e->d_late, 4 * (size_t)st.late_fire, hipMemcpyDeviceToHost));
        }
        dropped += (int64_t)st.dropped;
        if (st.max_q) qmax = std::max<int64_t>(qmax, jm::unord_i64(st.max_q));
        if (st.min_q != ~0ull) qmin = std::min<int64_t>(qmin, jm::unord_i64(st.min_q));
        if (st.spill_n == 0) break;
        if (round > 64) return fail(e, FWA_E_STATE, "miss replay did not converge");
        // allocate the wanted slices, republish, replay the missed records
        std::vector<unsigned long long> want(kWantCap);
        HIPCHK(e, hipMemcpy(want.data(), e->d_want, sizeof(unsigned long long) * kWantCap, hipMemcpyDeviceToHost));
        for (unsigned long long w : want) {
            if (!w) continue;
            const int64_t q = jm::unord_i64(w - 1ull);
            int64_t thr;
            bool always;
            accept_threshold(e, q, &thr, &always);
            if (always || e->wm < thr) { rc = alloc_slice(e, q); if (rc) return rc; }
            else e->negative.insert(q);  // late slice: the replay drops its records
        }
        rc = publish_dir(e);
        if (rc) return rc;
        HIPCHK(e, hipMemcpyAsync(e->d_replay, e->d_spill, sizeof(int32_t) * st.spill_n, hipMemcpyDeviceToDevice, e->stream));
        rc = reset_push_status(e);
        if (rc) return rc;
        IngestArgs b = a;
        b.idx = e->d_replay;
        b.n = st.spill_n;
        rc = launch_ingest(e, b, true);
        if (rc) return rc;
    }
    if (!late_idx.empty()) { rc = process_late(e, a, late_idx); if (rc) return rc; }
    if (!e->negative.empty()) { e->negative.clear(); republish = true; }
    // (touched flags were mirrored by the last sync) extend the lookahead so ordered streams rarely miss
    if (qmax != LONG_MIN_J) {
        const int64_t span = qmax - qmin + 1;
        e->lookahead = std::min<int64_t>(std::max<int64_t>(e->lookahead, 2 * span), 256);
        if (!e->have_q || qmax > e->max_q) e->max_q = qmax;
        e->have_q = true;
        const size_t slot_bytes = (size_t)e->stride * 8 * e->nacc;
        int64_t budget_slots = (int64_t)(e->mem_budget / std::max<size_t>(slot_bytes, 1));
        int64_t la = std::min<int64_t>(e->lookahead, std::max<int64_t>(0, budget_slots - (int64_t)e->live.size()));
        for (int64_t q = e->max_q + 1; q <= e->max_q + la; ++q)
            if (!e->live.count(q)) { rc = alloc_slice(e, q); if (rc) return rc; republish = true; }
    }
    if (republish) e->dir_dirty = true;
    if (a.dropidx) { rc = collect_late_indices(e); if (rc) return rc; }
    if (e->d_khash) { rc = khash_fill(e, a.keys, a.key_hash, n); if (rc) return rc; }
    e->records_in += n;
    e->late_dropped += dropped;
    if (late_dropped_out) *late_dropped_out = dropped;
    return FWA_OK;
}

int fwa_push(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
             const int32_t* key_hash, int64_t n, int32_t flags, int64_t* late_dropped_out) {
    return fwa_push_nullable(e, keys, ts, val_cols, nullptr, key_hash, n, flags, late_dropped_out);
}

static int push_body(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
                     const uint8_t* const* null_cols, const int32_t* key_hash, int64_t n, int32_t flags,
                     int64_t* late_dropped_out);

int fwa_push_nullable(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
                      const uint8_t* const* null_cols, const int32_t* key_hash, int64_t n, int32_t flags,
                      int64_t* late_dropped_out) {
    if (!e) return FWA_E_STATE;
    if (!e->dec || n <= 0 || n > INT32_MAX || !keys || !ts)
        return push_body(e, keys, ts, val_cols, null_cols, key_hash, n, flags, late_dropped_out);
    // DECIMAL columns -> piece columns on the GPU, then the ordinary push over the internal configuration
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_push(e)) return rc0;    // a pending push may still replay from the piece columns
    const bool device = (flags & FWA_PUSH_DEVICE_PTRS) != 0;
    if (device) { if (int rc1 = wait_input_stream(e)) return rc1; }
    const void* vals[FWA_MAX_COLS];
    int rc = dec_split(e, val_cols, null_cols, n, device, vals);
    if (!rc) rc = push_body(e, keys, ts, vals, null_cols, key_hash, n, flags, late_dropped_out);
    for (int c = 0; c < FWA_MAX_COLS; ++c) e->dev_override[c] = nullptr;
    return rc;
}

static int push_body(fwa_engine* e, const int64_t* keys, const int64_t* ts, const void* const* val_cols,
                     const uint8_t* const* null_cols, const int32_t* key_hash, int64_t n, int32_t flags,
                     int64_t* late_dropped_out) {
    if (!e) return FWA_E_STATE;
    if (n < 0 || (n > 0 && (!keys || !ts))) return fail(e, FWA_E_ARG, "null input column");
    if (e->cfg.key_kind == FWA_KEY_PREHASHED && n > 0 && !key_hash) return fail(e, FWA_E_ARG, "PREHASHED keys need key_hash");
    if (n > INT32_MAX) return fail(e, FWA_E_ARG, "batch too large (max 2^31-1 records)");
    if (late_dropped_out) *late_dropped_out = 0;
    if (n == 0) { e->late_idx.clear(); return FWA_OK; }
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_push(e)) return rc0;
    IngestArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    e->late_idx.clear();
    if (e->cfg.flags & FWA_CFG_LATE_INDICES) {        // one index per dropped record at most
        if (n > e->dropidx_cap) {
            if (e->d_dropidx) HIPCHK(e, hipFree(e->d_dropidx));
            e->d_dropidx = nullptr;
            HIPCHK(e, hipMalloc(&e->d_dropidx, sizeof(int32_t) * (size_t)n));
            e->dropidx_cap = n;
        }
        HIPCHK(e, hipMemsetAsync(&e->d_st->drop_n, 0, 8, e->stream));
        a.dropidx = e->d_dropidx;
    }
    a.wm = e->wm;
    if (flags & FWA_PUSH_DEVICE_PTRS) {
        if (int rc1 = wait_input_stream(e)) return rc1;
        a.keys = keys;
        a.ts = ts;
        a.key_hash = key_hash;
        for (int j = 0; j < e->cfg.num_aggs; ++j) {
            const fwa_agg_spec& s = e->cfg.aggs[j];
            if (s.kind == FWA_COUNT || s.kind == FWA_COUNT_COL) continue;   // COUNT(col) reads NULL flags only
            if (!val_cols || !val_cols[s.col]) return fail(e, FWA_E_ARG, "missing value column");
            a.cols[s.col] = val_cols[s.col];
        }
        if (e->cfg.flags & FWA_CFG_DYNAMIC_GAP) {
            if (!val_cols || !val_cols[e->cfg.gap_col]) return fail(e, FWA_E_ARG, "missing session gap column");
            a.cols[e->cfg.gap_col] = val_cols[e->cfg.gap_col];
        }
        for (int c = 0; c < FWA_MAX_COLS; ++c)       // only entries of declared nullable columns are read
            a.nulls[c] = (null_cols && ((e->cfg.nullable_cols >> c) & 1)) ? null_cols[c] : nullptr;
    } else {
        int rc = stage_inputs(e, keys, ts, val_cols, null_cols, key_hash, n, a);
        if (rc) return rc;
    }
    if (n > e->spill_cap) {
        if (e->d_spill) HIPCHK(e, hipFree(e->d_spill));
        if (e->d_replay) HIPCHK(e, hipFree(e->d_replay));
        e->spill_cap = std::max<int64_t>(n, 1 << 16);
        HIPCHK(e, hipMalloc(&e->d_spill, sizeof(int32_t) * e->spill_cap));
        HIPCHK(e, hipMalloc(&e->d_replay, sizeof(int32_t) * e->spill_cap));
        if (e->d_late) HIPCHK(e, hipFree(e->d_late));
        HIPCHK(e, hipMalloc(&e->d_late, sizeof(int32_t) * e->spill_cap));
    }
    if (e->kind == FWA_SESSION) {
        int64_t dropped = 0;
        int rc = push_session(e, a, &dropped);
        if (rc) return rc;
        if (e->h_st->error) {
            const int err = e->h_st->error;
            return fail(e, err, err == FWA_E_KEYGROUP ? "Key group is not in the owned KeyGroupRange (StateTable.getMapForKeyGroup)"
                              : err == FWA_E_TS_MIN ? "Record has Long.MIN_VALUE timestamp (= no timestamp marker)."
                              : err == FWA_E_MERGE_LATE ? "The end timestamp of an event-time window cannot become earlier than the current watermark by merging."
                              : err == FWA_E_STATE ? "session state inconsistency"
                              : err == FWA_E_ARG ? "Dynamic session time gap must satisfy 0 < gap"
                                                   : "key table full: raise fwa_config.key_capacity");
        }
        if (a.dropidx) { int rc2 = collect_late_indices(e); if (rc2) return rc2; }
        if (e->d_khash) { int rc2 = khash_fill(e, a.keys, a.key_hash, n); if (rc2) return rc2; }
        e->records_in += n;
        e->late_dropped += dropped;
        if (late_dropped_out) *late_dropped_out = dropped;
        return FWA_OK;
    }
    if (e->red) {   // DataStream reduction: the accumulators (two-phase when eligible), then the selection passes
        const int64_t seq0 = e->red_seq_base + e->records_in;
        if (e->ec.red_iota) {   // the arrival sequence column the SELQ accumulator reads
            if (n > e->iota_cap) {
                if (e->d_iota) HIPCHK(e, hipFree(e->d_iota));
                e->d_iota = nullptr;
                HIPCHK(e, hipMalloc(&e->d_iota, 4 * (size_t)n));
                e->iota_cap = n;
            }
            e->iota_n = n;
            e->iota_pending = true;                              // written on first use (ensure_iota)
            e->iota_ran = false;
            a.cols[kIotaCol] = e->d_iota;
        }
        int rc = push_common(e, a, n, true, false, late_dropped_out);
        e->iota_pending = false;
        if (!rc && e->iota_ran) {                                  // the index column counts as ingest time
            float ms = 0.f;
            HIPCHK(e, hipEventElapsedTime(&ms, e->ev[8], e->ev[9]));
            e->ingest_ms += ms;
        }
        return rc ? rc : red_select(e, a, n, seq0);
    }
    return push_common(e, a, n, true, (flags & FWA_PUSH_ASYNC) != 0, late_dropped_out);
}

int fwa_push_partials(fwa_engine* e, const int64_t* keys, const int64_t* slice_ts, const int64_t* count,
                      const void* const* acc, int64_t n, int32_t flags, int64_t* late_dropped_out) {
    if (!e) return FWA_E_STATE;
    if (e->dec && !e->restoring) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators of DECIMAL aggregates");
    if (e->red) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators of a DataStream reduction");
    if (e->kind == FWA_SESSION) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators need a slicing window");
    if (n < 0 || (n > 0 && (!keys || !slice_ts || !count))) return fail(e, FWA_E_ARG, "null input column");
    // (PREHASHED keys: only a restore, which brings the snapshot's hash column)
    if (e->cfg.key_kind == FWA_KEY_PREHASHED && !(e->restoring && e->rs_hash))
        return fail(e, FWA_E_UNSUPPORTED, "partials need a computable key hash");
    if (n > INT32_MAX) return fail(e, FWA_E_ARG, "batch too large (max 2^31-1 records)");
    if (late_dropped_out) *late_dropped_out = 0;
    if (n == 0) { e->late_idx.clear(); return FWA_OK; }
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_push(e)) return rc0;
    IngestArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    e->late_idx.clear();
    if (e->cfg.flags & FWA_CFG_LATE_INDICES) {        // one index per dropped record at most
        if (n > e->dropidx_cap) {
            if (e->d_dropidx) HIPCHK(e, hipFree(e->d_dropidx));
            e->d_dropidx = nullptr;
            HIPCHK(e, hipMalloc(&e->d_dropidx, sizeof(int32_t) * (size_t)n));
            e->dropidx_cap = n;
        }
        HIPCHK(e, hipMemsetAsync(&e->d_st->drop_n, 0, 8, e->stream));
        a.dropidx = e->d_dropidx;
    }
    a.wm = e->wm;
    const void* src[3 + FWA_MAX_AGGS + FWA_MAX_COLS] = {keys, slice_ts, count};
    int nsrc = 3;
    for (int j = 0; j < e->ec.naggs; ++j) {   // user aggregates, then the hidden non-NULL counters
        if (e->ec.agg[j].acc == 0) continue;
        if (!acc || !acc[j]) return fail(e, FWA_E_ARG, j < e->ec.nout ? "missing accumulator column"
                                                                       : "missing hidden non-NULL counter column");
        src[nsrc++] = acc[j];
    }
    const void* dev[3 + FWA_MAX_AGGS + FWA_MAX_COLS];
    if (flags & FWA_PUSH_DEVICE_PTRS) {
        if (int rc1 = wait_input_stream(e)) return rc1;
        for (int c = 0; c < nsrc; ++c) dev[c] = src[c];
    } else {                                   // stage host columns (8 bytes each) into the input buffer
        const size_t colb = ((size_t)n * 8 + 255) / 256 * 256;
        if (colb * nsrc > e->d_in_bytes) {
            if (e->d_in) HIPCHK(e, hipFree(e->d_in));
            e->d_in = nullptr;
            HIPCHK(e, hipMalloc(&e->d_in, colb * nsrc));
            e->d_in_bytes = colb * nsrc;
        }
        for (int c = 0; c < nsrc; ++c) {
            dev[c] = (char*)e->d_in + colb * c;
            HIPCHK(e, hipMemcpyAsync((void*)dev[c], src[c], (size_t)n * 8, hipMemcpyHostToDevice, e->stream));
        }
    }
    a.keys = (const int64_t*)dev[0];
    a.ts = (const int64_t*)dev[1];
    a.pcount = (const unsigned long long*)dev[2];
    if (e->cfg.key_kind == FWA_KEY_PREHASHED) {      // restore: the snapshot's key.hashCode() column
        if (n > e->rs_hash_cap) {
            if (e->d_rs_hash) HIPCHK(e, hipFree(e->d_rs_hash));
            e->d_rs_hash = nullptr;
            HIPCHK(e, hipMalloc(&e->d_rs_hash, sizeof(int32_t) * (size_t)n));
            e->rs_hash_cap = n;
        }
        HIPCHK(e, hipMemcpyAsync(e->d_rs_hash, e->rs_hash, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, e->stream));
        a.key_hash = e->d_rs_hash;
    }
    for (int j = 0, c = 3; j < e->ec.naggs; ++j)
        if (e->ec.agg[j].acc > 0) a.cols[j] = dev[c++];
    if (n > e->spill_cap) {
        if (e->d_spill) HIPCHK(e, hipFree(e->d_spill));
        if (e->d_replay) HIPCHK(e, hipFree(e->d_replay));
        e->spill_cap = std::max<int64_t>(n, 1 << 16);
        HIPCHK(e, hipMalloc(&e->d_spill, sizeof(int32_t) * e->spill_cap));
        HIPCHK(e, hipMalloc(&e->d_replay, sizeof(int32_t) * e->spill_cap));
        if (e->d_late) HIPCHK(e, hipFree(e->d_late));
        HIPCHK(e, hipMalloc(&e->d_late, sizeof(int32_t) * e->spill_cap));
    }
    if (e->red) {                                 // DataStream reduction: v1 ingest, then the selection passes
        const int64_t seq0 = e->red_seq_base + e->records_in;
        int rc = push_common(e, a, n, false, false, late_dropped_out);
        return rc ? rc : red_select(e, a, n, seq0);
    }
    return push_common(e, a, n, true, (flags & FWA_PUSH_ASYNC) != 0, late_dropped_out);
}

static int retire_slices(fwa_engine* e, int64_t wm);
static int fill_out(fwa_engine* e, int64_t nrows, fwa_out* out);
// fwa_drain_route's launch: the drained slices straight into per-destination send regions; a region past its
// capacity is counted, the host grows the regions and launches again (the drain is idempotent until the reset).
static int launch_drain_route(fwa_engine* e, const std::vector<FireWindow>& hw, const std::vector<int32_t>& hs, int32_t par,
                              int32_t m, const int32_t* cell_acc, std::vector<unsigned long long>& counts) {
    int rc = upload_windows(e, hw, hs);
    if (rc) return rc;
    DrainRouteArgs r;
    memset(&r, 0, sizeof(r));
    r.f.key_table = e->d_keys;
    r.f.capacity = e->capacity;
    r.f.stride = e->stride;
    r.f.slot_base = e->d_slot_base;
    r.f.win = e->d_win;
    r.f.win_slots = e->d_win_slots;
    r.f.nwin = (int32_t)hw.size();
    r.f.blocks_per_win = (int32_t)((e->capacity + 1 + (int64_t)kBlock * kDrJ - 1) / ((int64_t)kBlock * kDrJ));   // chunks
    r.par = par;
    r.m = m;
    r.ncell = m - 3;
    for (int i = 0; i < m - 3; ++i) r.cell_acc[i] = cell_acc[i];
    if (!e->d_dr_cnt) HIPCHK(e, hipMalloc(&e->d_dr_cnt, sizeof(unsigned long long) * kMaxDest));
    // first sizing: the last drain's largest region x 1.25 (at least 2^16 rows, at most every key of every slice)
    const int64_t nkeys = std::max<int64_t>((int64_t)e->h_st->n_keys, 1);
    const int64_t bound = (int64_t)hw.size() * nkeys;
    int64_t cap = std::min<int64_t>(bound, std::max<int64_t>((int64_t)1 << 16, e->dr_cap));
    counts.assign(par, 0);
    for (int round = 0; round < 3; ++round) {
        const size_t need = (size_t)par * cap * m * 8;
        if (need > e->dr_bytes) {
            if (e->d_dr) HIPCHK(e, hipFree(e->d_dr));
            e->d_dr = nullptr;
            e->dr_bytes = 0;
            HIPCHK(e, hipMalloc(&e->d_dr, need));
            e->dr_bytes = need;
        }
        r.cap = cap;
        r.rows = e->d_dr;
        r.dcnt = e->d_dr_cnt;
        HIPCHK(e, hipMemsetAsync(e->d_dr_cnt, 0, sizeof(unsigned long long) * par, e->stream));
        HIPCHK(e, hipEventRecord(e->ev[2], e->stream));
        drain_route_kernel<<<(unsigned)r.f.blocks_per_win, kBlock, 0, e->stream>>>(r, e->d_ec);   // one block per chunk
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipEventRecord(e->ev[3], e->stream));
        HIPCHK(e, hipMemcpyAsync(counts.data(), e->d_dr_cnt, sizeof(unsigned long long) * par, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        int64_t mx = 0;
        for (unsigned long long v : counts) mx = std::max<int64_t>(mx, (int64_t)v);
        e->dr_cap = std::max<int64_t>(e->dr_cap, mx + mx / 4);
        if (mx <= cap) {
            e->dr_cap_used = cap;
            float ms = 0.f;
            HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
            e->fire_ms += ms;
            e->fire_launches++;
            int64_t tot = 0;
            for (unsigned long long v : counts) tot += (int64_t)v;
            e->fire_rows += tot;
            return FWA_OK;
        }
        cap = mx + mx / 4;                         // grow to the exact need (+25 % for the next drains), again
    }
    return fail(e, FWA_E_STATE, "fwa_drain_route: regions did not converge");
}

int fwa_drain_route(fwa_engine* e, int64_t wm, int32_t parallelism, fwa_routed* out) {
    if (!e || !out) return FWA_E_ARG;
    memset(out, 0, sizeof(*out));
    if (parallelism < 1 || parallelism > FWA_MAX_DEST) return fail(e, FWA_E_ARG, "fwa_drain_route: parallelism");
    if (e->red || e->dec || e->kind == FWA_SESSION || e->sparse || !e->cfg.output_on_device ||
        e->cfg.key_kind == FWA_KEY_PREHASHED)
        return fail(e, FWA_E_UNSUPPORTED, "fwa_drain_route: a dense slicing-window handle with output_on_device");
    e->rs_valid = false;
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_pending(e)) return rc0;
    // the previous call's blocks may still be read on the input stream (the exchange's all-to-all): the drain
    // rewrites them only after everything enqueued there
    if (int rc0 = wait_input_stream(e)) return rc0;
    // cells: key, slice start, COUNT(*), one per user aggregate other than COUNT(*), one per hidden counter
    int32_t cell_acc[kMaxAggsInt];
    int32_t m = 3;
    for (int j = 0; j < e->ec.nout; ++j)
        if (e->ec.agg[j].kind != FWA_COUNT) cell_acc[m++ - 3] = e->ec.agg[j].acc;
    for (int h = e->ec.nout; h < e->ec.naggs; ++h) cell_acc[m++ - 3] = e->ec.agg[h].acc;
    std::vector<FireWindow> hw;
    std::vector<int32_t> hs;
    for (auto& kv : e->live) {
        if (!e->touched[kv.second]) continue;
        FireWindow f;
        f.start = slice_start(e, kv.first);
        f.end = jm::wadd(f.start, e->g);
        if (wm != LONG_MAX_J && !(trig(e, jm::wsub(f.end, 1)) <= wm)) continue;   // slice not complete at wm
        f.slot_off = (int32_t)hs.size();
        f.nslots = 1;
        hs.push_back(kv.second);
        hw.push_back(f);
    }
    std::vector<unsigned long long> counts(parallelism, 0);
    if (!hw.empty()) {
        int rc = launch_drain_route(e, hw, hs, parallelism, m, cell_acc, counts);
        if (rc) return rc;
        for (int32_t slot : hs) {
            rc = reset_slot(e, slot);
            if (rc) return rc;
        }
        rc = flush_resets(e);
        if (rc) return rc;
    }
    if (wm > e->wm) {   // forward the watermark, as fwa_drain_partials
        int rc = retire_slices(e, wm);
        if (rc) return rc;
        e->wm = wm;
    }
    out->parallelism = parallelism;
    out->cells = m;
    out->on_device = 1;
    for (int d = 0; d < parallelism; ++d) {
        out->rows[d] = e->d_dr ? e->d_dr + (size_t)d * e->dr_cap_used * m : nullptr;
        out->count[d] = (int64_t)counts[d];
        out->n += (int64_t)counts[d];
    }
    return FWA_OK;
}



// fwa_fire_partials through its two defining calls: the rows' cells as columns, fwa_push_partials, then
// fwa_advance_watermark (every case the merge-fire path does not take, and its redo).
static int fire_partials_generic(fwa_engine* e, const int64_t* rows, int64_t n, int32_t m, const int32_t* cell,
                                 int64_t wm, int32_t flags, fwa_out* out, int64_t* late_dropped_out) {
    const int na = e->ec.naggs;
    int64_t late = 0;
    if (n > 0) {
        const void* acc[FWA_MAX_AGGS + FWA_MAX_COLS] = {};
        int rc = FWA_OK;
        if (flags & FWA_PUSH_DEVICE_PTRS) {
            int64_t* cols = nullptr;
            HIPCHK(e, hipMalloc(&cols, (size_t)8 * n * m));
            int64_t* colp[3 + kMaxAggsInt];
            for (int c = 0; c < m; ++c) colp[c] = cols + (size_t)c * n;
            if (int rc0 = wait_input_stream(e)) { (void)hipFree(cols); return rc0; }
            rc = fwa_unpack_rows(rows, n, m, colp, e->cfg.device, e->stream);
            if (rc == FWA_OK) {
                for (int j = 0; j < na; ++j) if (e->ec.agg[j].acc > 0) acc[j] = colp[cell[j]];
                hipStream_t in_saved = e->in_stream;
                e->in_stream = nullptr;                       // the columns are ordered on the engine's own stream
                rc = fwa_push_partials(e, colp[0], colp[1], colp[2], acc, n, FWA_PUSH_DEVICE_PTRS, &late);
                e->in_stream = in_saved;
            } else {
                rc = fail(e, rc, "fwa_fire_partials: unpacking the rows failed");
            }
            if (hipStreamSynchronize(e->stream) != hipSuccess && rc == FWA_OK) rc = fail(e, FWA_E_DEVICE, "stream");
            (void)hipFree(cols);
        } else {
            std::vector<int64_t> cols((size_t)n * m);
            for (int64_t i = 0; i < n; ++i)
                for (int c = 0; c < m; ++c) cols[(size_t)c * n + i] = rows[(size_t)i * m + c];
            for (int j = 0; j < na; ++j) if (e->ec.agg[j].acc > 0) acc[j] = cols.data() + (size_t)cell[j] * n;
            rc = fwa_push_partials(e, cols.data(), cols.data() + n, cols.data() + 2 * (size_t)n, acc, n, 0, &late);
        }
        if (rc) return rc;
    }
    if (late_dropped_out) *late_dropped_out = late;
    return fwa_advance_watermark(e, wm, out);
}

int fwa_fire_partials(fwa_engine* e, const int64_t* rows, int64_t n, int32_t m, const int32_t* acc_cell, int64_t wm,
                      int32_t flags, fwa_out* out, int64_t* late_dropped_out) {
    if (!e) return FWA_E_STATE;
    if (out) memset(out, 0, sizeof(*out));
    if (late_dropped_out) *late_dropped_out = 0;
    const int na = e->ec.naggs;
    if (n < 0 || m < 3 || m > 3 + kMaxAggsInt || (n > 0 && !rows) || !acc_cell)
        return fail(e, FWA_E_ARG, "fwa_fire_partials: rows / cells");
    for (int j = 0; j < na; ++j)
        if (e->ec.agg[j].acc > 0 && (acc_cell[j] < 3 || acc_cell[j] >= m))
            return fail(e, FWA_E_ARG, "fwa_fire_partials: accumulator cell out of the row");
    if (n > INT32_MAX) return fail(e, FWA_E_ARG, "batch too large (max 2^31-1 rows)");
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rcf = finish_afire(e)) return rcf;
    e->af_pend = false;
    if (int rc0 = settle_pending(e)) return rc0;
    // the merge-fire path: every window merged here fires at wm and nothing else is held (TUMBLE, no lateness,
    // no live slice with data); the redo through the defining calls covers every row it cannot place
    bool fast = e->opt_fire_partials != 0 && n > 0 && (flags & FWA_PUSH_DEVICE_PTRS) && !e->sparse && !e->red &&
                !e->dec && e->kind == FWA_TUMBLE && e->lateness == 0 && e->tz.empty() && e->late_rows == 0 &&
                wm > e->wm && e->cfg.key_kind != FWA_KEY_PREHASHED;
    if (fast) for (auto& kv : e->live) if (e->touched[kv.second]) { fast = false; break; }
    MfArgs a;
    memset(&a, 0, sizeof(a));
    const int nacc = e->nacc;
    if (fast) {
        for (int cc = 0; cc <= kMaxAggsInt; ++cc) a.cell[cc] = -1;
        for (int j = 0; j < na; ++j) {
            const AggDesc& d = e->ec.agg[j];
            if (d.acc > 0 && !d.alias) a.cell[d.acc] = acc_cell[j];
        }
        for (int cc = 1; cc < nacc; ++cc) fast = fast && a.cell[cc] >= 3 && e->ec.acc_kind[cc] != ACC_PAYLOAD;
        fast = fast && nacc - 1 <= kMfAcc;
    }
    if (!fast) return fire_partials_generic(e, rows, n, m, acc_cell, wm, flags, out, late_dropped_out);
    e->mf_calls++;
    constexpr size_t kLds = 150 * 1024;
    const size_t ebytes = 20 + 8 * (size_t)nacc;
    int hlog = 14;
    while (hlog > 8 && ((size_t)1 << hlog) * ebytes + 64 > kLds) --hlog;
    const int64_t H = (int64_t)1 << hlog;
    // buckets: the groups expected (rows x 1.25 x the groups per row of the last call, at most one per row) at a table
    // load <= 0.7 (C2 at N = 8: 512 buckets of ~1700 groups, load ~0.42 -- fewer, longer bucket runs for mf_part than
    // at <= 0.5 x 2: 1.33x vs 1.36x of N = 1 per rank, profiles/r05_partials_cost.txt); a full table redoes the call
    // and resets the estimate to one group per row
    const double exp_groups = std::max(1.0, (double)n * std::min(1.0, 1.25 * e->mf_groups_per_row));
    int nb_log = 0;
    while (nb_log < 12 && (double)H * 0.7 * (double)((int64_t)1 << nb_log) < exp_groups) ++nb_log;
    const int64_t NB = (int64_t)1 << nb_log;
    const int64_t capb = (int64_t)((double)(n / NB) * e->mf_capx) + 512;
    int64_t tile = (int64_t)((150 * 1024 - 12 * (size_t)NB - 16) / (8 + 8 * (size_t)m));
    tile = std::min<int64_t>(8 * kMfThreads, tile / 64 * 64);
    if (tile < 256) {                           // (the row is too wide for an LDS tile: counted as a fallback)
        e->mf_fallbacks++;
        return fire_partials_generic(e, rows, n, m, acc_cell, wm, flags, out, late_dropped_out);
    }
    const size_t hdr = 256 + ((4 * (size_t)NB + 255) & ~(size_t)255);
    const size_t need = hdr + (size_t)NB * capb * m * 8;
    if (need > e->mf_bytes) {
        if (e->d_mf) HIPCHK(e, hipFree(e->d_mf));
        e->d_mf = nullptr;
        e->mf_bytes = 0;
        HIPCHK(e, hipMalloc(&e->d_mf, need));
        e->mf_bytes = need;
    }
    if (int rc = ensure_out(e, n)) return rc;
    a.rows = rows;
    a.n = n;
    a.m = m;
    a.nb_log = nb_log;
    a.tile = (int32_t)tile;
    a.hlog = hlog;
    a.nacc = nacc;
    a.capb = capb;
    a.mf = (unsigned long long*)e->d_mf;
    a.b_cnt = (uint32_t*)((char*)e->d_mf + 256);
    a.b_rows = (int64_t*)((char*)e->d_mf + hdr);
    a.prev_wm = e->wm;
    a.wm = wm;
    a.o_key = e->o_key;
    a.o_start = e->o_start;
    a.o_end = e->o_end;
    for (int j = 0; j < e->cfg.num_aggs; ++j) { a.o_agg[j] = e->o_agg[j]; a.o_null[j] = e->o_null[j]; }
    a.out_cap = e->out_cap;
    a.st = e->d_st;
    if (int rc1 = wait_input_stream(e)) return rc1;
    HIPCHK(e, hipMemsetAsync(e->d_mf, 0, hdr, e->stream));
    HIPCHK(e, hipMemsetAsync(&e->d_st->rows, 0, 8, e->stream));
    HIPCHK(e, hipMemsetAsync(&e->d_st->error, 0, 4, e->stream));
    const size_t lds_p = (((size_t)12 * NB + 15) & ~(size_t)15) + (size_t)tile * (8 + 8 * (size_t)m);
    const size_t lds_m = (((size_t)4 * H + 15) & ~(size_t)15) + (size_t)H * (16 + 8 * (size_t)nacc);
    HIPCHK(e, hipEventRecord(e->ev[2], e->stream));
    mf_part_kernel<<<(unsigned)((n + tile - 1) / tile), kMfThreads, lds_p, e->stream>>>(a);
    mf_merge_kernel<<<(unsigned)NB, kMfThreads, lds_m, e->stream>>>(a, e->d_ec);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[3], e->stream));
    unsigned long long hm[3] = {0, 0, 0};
    HIPCHK(e, hipMemcpyAsync(hm, e->d_mf, sizeof(hm), hipMemcpyDeviceToHost, e->stream));
    if (int rc2 = sync_status(e)) return rc2;
    const DevStatus st = *e->h_st;
    if (st.error) {
        const char* msg = st.error == FWA_E_KEYGROUP ? "Key group is not in the owned KeyGroupRange (StateTable.getMapForKeyGroup)"
                                                     : "device error";
        return fail(e, st.error, msg);
    }
    if (hm[2]) {   // a row this path cannot place: redo through the defining calls (no state was touched)
        e->mf_fallbacks++;
        // a region past its end: the rows of a key (all its windows, from every source) share one bucket, so the
        // spread is wider than the row count suggests -- larger regions from now on, buckets sized from the groups
        // the truncated pass still saw; a full table: buckets sized for one group per row again
        if (hm[2] & kMfOverflow) {
            e->mf_capx = std::min(6.0, e->mf_capx * 1.5);
            e->mf_groups_per_row = std::max(e->mf_groups_per_row, std::min(1.0, (double)hm[1] / (double)n));
        }
        if (hm[2] & kMfFull) e->mf_groups_per_row = 1.0;
        return fire_partials_generic(e, rows, n, m, acc_cell, wm, flags, out, late_dropped_out);
    }
    const int64_t nrows = (int64_t)st.rows;
    if (nrows > e->out_cap) return fail(e, FWA_E_STATE, "fwa_fire_partials: rows past the output bound");
    e->mf_groups_per_row = std::max(1.0 / 65536.0, (double)hm[1] / (double)n);
    const int64_t dropped = (int64_t)hm[0];
    e->records_in += n;
    e->late_dropped += dropped;
    if (late_dropped_out) *late_dropped_out = dropped;
    if (int rc3 = retire_slices(e, wm)) return rc3;   // lookahead slices past cleanup (they hold no data)
    e->wm = wm;
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->fire_ms += ms;
    e->fire_launches++;
    e->fire_rows += nrows;
    e->rows_out += nrows;
    e->af_rows = nrows;
    if (out) return fill_out(e, nrows, out);
    return FWA_OK;
}

// Export every (key, slice) accumulator that received records since the last drain and reset those
// slices (the local half of LocalSlicingWindowAggOperator -> GlobalAggCombiner).
// Free slices whose every window is past cleanup at wm (last window: cleanupTime <= wm).
static int retire_slices(fwa_engine* e, int64_t wm) {
    std::vector<int64_t> dead;
    for (auto& kv : e->live) {
        int64_t thr;
        bool always;
        accept_threshold(e, kv.first, &thr, &always);
        if (!always && wm >= thr) dead.push_back(kv.first);
    }
    for (int64_t q : dead) {
        int rc = release_slot(e, e->live[q]);
        if (rc) return rc;
        e->live.erase(q);
    }
    if (int rc = flush_resets(e)) return rc;
    if (!dead.empty()) e->dir_dirty = true;           // published lazily, before a kernel that reads it
    return FWA_OK;
}

// Local half of LocalSlicingWindowAggOperator -> GlobalAggCombiner: export the (key, slice)
// accumulators of every touched slice complete at wm, reset them, forward the watermark.
int fwa_drain_partials(fwa_engine* e, int64_t wm, fwa_partials* out) {
    if (!e || !out) return FWA_E_ARG;
    e->rs_valid = false;                              // the drained slices leave the carried sums behind
    if (e->red) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators of a DataStream reduction");
    if (e->dec) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators of DECIMAL aggregates");
    if (e->kind == FWA_SESSION) return fail(e, FWA_E_UNSUPPORTED, "partial accumulators need a slicing window");
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_pending(e)) return rc0;
    if (int rc0 = wait_input_stream(e)) return rc0;   // device columns of the last drain may still be read there
    memset(out, 0, sizeof(*out));
    std::vector<FireWindow> hw;
    std::vector<int32_t> hs;
    int64_t nrows = 0;
    if (e->sparse) {
        int rc = sp_fire(e, sp_due(e, wm), 1, true, &nrows);
        if (rc) return rc;
        if (wm > e->wm) e->wm = wm;
    }
    if (!e->sparse) for (auto& kv : e->live) {
        if (!e->touched[kv.second]) continue;
        FireWindow f;
        f.start = slice_start(e, kv.first);
        f.end = jm::wadd(f.start, e->g);
        if (wm != LONG_MAX_J && !(trig(e, jm::wsub(f.end, 1)) <= wm)) continue;   // slice not complete at wm
        f.slot_off = (int32_t)hs.size();
        f.nslots = 1;
        hs.push_back(kv.second);
        hw.push_back(f);
    }
    if (!hw.empty()) {
        int rc = launch_fire(e, hw, hs, 1, &nrows);
        if (rc) return rc;
        for (int32_t slot : hs) {
            rc = reset_slot(e, slot);
            if (rc) return rc;
        }
        rc = flush_resets(e);
        if (rc) return rc;
    }
    if (wm > e->wm && !e->sparse) {   // forward the watermark: lateness from now on, release slices past cleanup
        int rc = retire_slices(e, wm);
        if (rc) return rc;
        e->wm = wm;
    }
    out->n = nrows;
    out->num_aggs = e->cfg.num_aggs;
    out->num_hidden = e->ec.naggs - e->ec.nout;
    out->on_device = e->cfg.output_on_device ? 1 : 0;
    const int64_t* cols[3] = {e->o_key, e->o_start, e->o_count};
    const void* accs[FWA_MAX_AGGS] = {};
    for (int j = 0; j < e->cfg.num_aggs; ++j) accs[j] = e->o_agg[j];
    if (e->cfg.output_on_device) {
        out->key = cols[0];
        out->slice_start = cols[1];
        out->count = cols[2];
        for (int j = 0; j < e->cfg.num_aggs; ++j) out->acc[j] = accs[j];
        for (int h = 0; h < out->num_hidden; ++h) out->hidden[h] = e->o_hid[h];
        return FWA_OK;
    }
    e->h_out.resize(std::max<size_t>((size_t)nrows * 8 * (3 + e->cfg.num_aggs + out->num_hidden), 8));
    char* p = e->h_out.data();
    auto get = [&](const void* d) -> const void* {
        if (nrows) { hipError_t r = hipMemcpy(p, d, 8 * nrows, hipMemcpyDeviceToHost); if (r != hipSuccess) return nullptr; }
        const void* r = p;
        p += 8 * nrows;
        return r;
    };
    out->key = (const int64_t*)get(cols[0]);
    out->slice_start = (const int64_t*)get(cols[1]);
    out->count = (const int64_t*)get(cols[2]);
    for (int j = 0; j < e->cfg.num_aggs; ++j) out->acc[j] = get(accs[j]);
    for (int h = 0; h < out->num_hidden; ++h) out->hidden[h] = (const int64_t*)get(e->o_hid[h]);
    if (!out->key || !out->slice_start || !out->count) return fail(e, FWA_E_DEVICE, "partials copy failed");
    return FWA_OK;
}

// ---- snapshot / restore (include/flink_amd.h) ----
// header word layout: 0 magic, 1 version, 2 window kind, 3 semantics, 4 size, 5 slide, 6 offset, 7 gap,
// 8 allowed lateness, 9 max parallelism, 10 key kind, 11 num aggs, 12..19 agg kinds, 20 watermark,
// 21 entries, 22 kg_start, 23 kg_end of the snapshotting handle, 24 nullable_cols, 25 hidden non-NULL
// counters (columns after the acc_j columns), 26 aggregate input columns (4 bits each), 27..31 reserved (0)

static void snap_header(const fwa_engine* e, int64_t* h, int64_t n) {
    memset(h, 0, sizeof(int64_t) * kSnapHdr);
    h[0] = (int64_t)kSnapMagic;
    h[1] = 1;
    h[2] = e->cfg.window_kind;
    h[3] = e->cfg.semantics;
    h[4] = e->cfg.size_ms;
    h[5] = e->cfg.slide_ms;
    h[6] = e->cfg.offset_ms;
    h[7] = e->cfg.gap_ms;
    h[8] = e->cfg.allowed_lateness_ms;
    h[9] = e->cfg.max_parallelism;
    h[10] = e->cfg.key_kind;
    h[11] = e->cfg.num_aggs;
    for (int j = 0; j < e->cfg.num_aggs; ++j) h[12 + j] = e->cfg.aggs[j].kind;
    h[20] = e->wm;
    h[21] = n;
    h[22] = e->cfg.kg_start;
    h[23] = e->cfg.kg_end;
    h[24] = e->cfg.nullable_cols;
    h[25] = e->ec.naggs - e->ec.nout;
    for (int j = 0; j < e->cfg.num_aggs; ++j) h[26] |= (int64_t)(e->cfg.aggs[j].col & 15) << (4 * j);
}

// Sessions: the blob's entries are the in-flight sessions (key, start, count, acc_j..., end) bucketed by
// key group -- the per-key MergingWindowSet mapping plus the window state of WindowOperator
// (WindowOperator.java:224-238 mergingSetsState / windowState), with the session end as a last column.
static int snapshot_sessions(fwa_engine* e, fwa_blob* out) {
    const int64_t n = e->n_ss;
    const int na = e->cfg.num_aggs, maxp = e->cfg.max_parallelism, nh = e->ec.naggs - e->ec.nout;
    const bool ph = e->cfg.key_kind == FWA_KEY_PREHASHED;   // + one column: each entry's key.hashCode()
    const int ncols = 4 + na + nh + (ph ? 1 : 0);
    const SessList& L = e->ss[e->ss_cur];
    std::vector<int32_t> khash(ph ? (size_t)e->capacity + 1 : 0);
    if (ph && n > 0) HIPCHK(e, hipMemcpy(khash.data(), e->d_khash, 4 * ((size_t)e->capacity + 1), hipMemcpyDeviceToHost));
    std::vector<uint32_t> kid((size_t)n);
    std::vector<int64_t> st((size_t)n), en((size_t)n), acc((size_t)n * e->nacc);
    std::vector<unsigned long long> table((size_t)e->capacity + 1);
    if (n > 0) {
        HIPCHK(e, hipMemcpy(kid.data(), L.kid, 4 * (size_t)n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(st.data(), L.start, 8 * (size_t)n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(en.data(), L.end, 8 * (size_t)n, hipMemcpyDeviceToHost));
        for (int cc = 0; cc < e->nacc; ++cc)
            HIPCHK(e, hipMemcpy(acc.data() + (size_t)cc * n, L.acc + (size_t)cc * L.stride, 8 * (size_t)n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(table.data(), e->d_keys, 8 * (size_t)e->capacity, hipMemcpyDeviceToHost));
    }
    std::vector<int32_t> kg((size_t)n);
    std::vector<int64_t> off((size_t)maxp + 1, 0), key((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        key[i] = (int64_t)kid[i] < e->capacity ? (int64_t)table[kid[i]] : LONG_MIN_J;
        kg[i] = jm::key_group_of(key[i], e->cfg.key_kind, ph ? khash[kid[i]] : 0, maxp);
        if (kg[i] < 0) return fail(e, FWA_E_STATE, "state holds a key outside every key group");
        off[kg[i] + 1]++;
    }
    for (int g = 0; g < maxp; ++g) off[g + 1] += off[g];
    const size_t words = kSnapHdr + (size_t)maxp + 1 + (size_t)n * ncols;
    int64_t* b = (int64_t*)malloc(words * 8);
    if (!b) return fail(e, FWA_E_OOM, "snapshot blob allocation failed");
    snap_header(e, b, n);
    memcpy(b + kSnapHdr, off.data(), 8 * ((size_t)maxp + 1));
    int64_t* body = b + kSnapHdr + maxp + 1;
    std::vector<int64_t> cur(off.begin(), off.end() - 1);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t d = cur[kg[i]]++;
        body[d] = key[i];
        body[(size_t)n + d] = st[i];
        body[(size_t)2 * n + d] = acc[i];                                  // COUNT(*)
        for (int j = 0; j < na; ++j) {
            const AggDesc& ad = e->ec.agg[j];
            body[(size_t)(3 + j) * n + d] = ad.acc > 0 ? acc[(size_t)ad.acc * n + i] : acc[i];
        }
        for (int h = 0; h < nh; ++h) body[(size_t)(3 + na + h) * n + d] = acc[(size_t)e->ec.agg[e->ec.nout + h].acc * n + i];
        body[(size_t)(3 + na + nh) * n + d] = en[i];
        if (ph) body[(size_t)(4 + na + nh) * n + d] = khash[kid[i]];
    }
    out->data = b;
    out->size = (int64_t)(words * 8);
    return FWA_OK;
}

__global__ void __launch_bounds__(kBlock) sess2_restore_kernel(Sess2Args a, const int64_t* keys, const int64_t* start,
                                                               const int64_t* end, const int64_t* const* accs, int64_t m,
                                                               int64_t at, const EngineConst* __restrict__ cp) {
    const EngineConst& c = *cp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kid = key_slot(a.key_table, a.key_mask, a.seg_log, a.part_bits, keys[i], a.st);
        if (kid < 0) { a.st->key_full = 1; raise_error(a.st, FWA_E_OOM); continue; }
        const int64_t o = at + i;
        a.out.kid[o] = (uint32_t)kid;
        a.out.start[o] = start[i];
        a.out.end[o] = end[i];
        for (int cc = 0; cc < c.nacc; ++cc) a.out.acc[(int64_t)cc * a.out.stride + o] = (unsigned long long)accs[cc][i];
    }
}

// Restore sessions: the owned key groups' entries of every blob are appended to the in-flight list
// (a key lives in one subtask's snapshot, so the lists never overlap); watermark = MIN over the blobs.
static int restore_sessions(fwa_engine* e, const void* const* blobs, int32_t n_blobs) {
    const int na = e->cfg.num_aggs, maxp = e->cfg.max_parallelism, nh = e->ec.naggs - e->ec.nout;
    int64_t wm = LONG_MAX_J;
    for (int32_t b = 0; b < n_blobs; ++b) {
        const int64_t* h = (const int64_t*)blobs[b];
        const int64_t n = h[21];
        wm = std::min<int64_t>(wm, h[20]);
        const int64_t* off = h + kSnapHdr;
        const int64_t lo = off[e->cfg.kg_start], hi = off[e->cfg.kg_end + 1];
        if (lo < 0 || hi < lo || hi > n) return fail(e, FWA_E_ARG, "corrupt key-group offsets");
        const int64_t m = hi - lo;
        if (m == 0) continue;
        const int64_t* body = off + maxp + 1;
        int rc = ensure_sess_lists(e, e->n_ss + m);
        if (rc) return rc;
        // device copies: key, start, end, one column per accumulator (COUNT, then each owner aggregate's)
        const int nc = 3 + e->nacc;
        int64_t* d = nullptr;
        HIPCHK(e, hipMalloc(&d, 8 * (size_t)m * nc));
        std::vector<const int64_t*> src(nc);
        src[0] = body + lo;
        src[1] = body + (size_t)n + lo;
        src[2] = body + (size_t)(3 + na + nh) * n + lo;
        src[3] = body + (size_t)2 * n + lo;
        for (int cc = 1; cc < e->nacc; ++cc) {
            for (int j = 0; j < na; ++j)
                if (e->ec.agg[j].acc == cc && !e->ec.agg[j].alias) src[3 + cc] = body + (size_t)(3 + j) * n + lo;
            for (int h = 0; h < nh; ++h)   // hidden non-NULL counters
                if (e->ec.agg[e->ec.nout + h].acc == cc) src[3 + cc] = body + (size_t)(3 + na + h) * n + lo;
        }
        std::vector<const int64_t*> hacc(e->nacc);
        for (int c = 0; c < nc; ++c) HIPCHK(e, hipMemcpy(d + (size_t)c * m, src[c], 8 * (size_t)m, hipMemcpyHostToDevice));
        for (int cc = 0; cc < e->nacc; ++cc) hacc[cc] = d + (size_t)(3 + cc) * m;
        const int64_t** dacc = nullptr;
        HIPCHK(e, hipMalloc(&dacc, sizeof(int64_t*) * e->nacc));
        HIPCHK(e, hipMemcpy(dacc, hacc.data(), sizeof(int64_t*) * e->nacc, hipMemcpyHostToDevice));
        Sess2Args s;
        memset(&s, 0, sizeof(s));
        s.key_table = e->d_keys;
        s.key_mask = (uint64_t)e->capacity - 1;
        s.seg_log = e->seg_log;
        s.part_bits = e->part_bits;
        s.out = e->ss[e->ss_cur];
        s.st = e->d_st;
        sess2_restore_kernel<<<grid_for(m), kBlock, 0, e->stream>>>(s, d, d + m, d + 2 * m, dacc, m, e->n_ss, e->d_ec);
        HIPCHK(e, hipGetLastError());
        if (e->d_khash) {                         // PREHASHED: the entries' key.hashCode() (last column) by kid
            std::vector<int32_t> hv((size_t)m);
            for (int64_t i = 0; i < m; ++i) hv[i] = (int32_t)body[(size_t)(4 + na + nh) * n + lo + i];
            int32_t* dh = nullptr;
            HIPCHK(e, hipMalloc(&dh, sizeof(int32_t) * (size_t)m));
            HIPCHK(e, hipMemcpyAsync(dh, hv.data(), sizeof(int32_t) * (size_t)m, hipMemcpyHostToDevice, e->stream));
            khash_fill_kernel<<<grid_for(m), kBlock, 0, e->stream>>>(d, dh, m, e->d_keys, (uint64_t)e->capacity - 1,
                                                                     e->seg_log, e->part_bits, e->d_khash);
            HIPCHK(e, hipGetLastError());
            HIPCHK(e, hipStreamSynchronize(e->stream));
            (void)hipFree(dh);
        }
        rc = sync_status(e);
        (void)hipFree(d);
        (void)hipFree(dacc);
        if (rc) return rc;
        if (e->h_st->error) return fail(e, e->h_st->error, "key table full: raise fwa_config.key_capacity");
        e->n_ss += m;
    }
    if (n_blobs > 0) e->wm = wm;
    return FWA_OK;
}

// Export every (key, slice) accumulator of every live slice (non-destructive raw fire), then bucket
// the rows by key group on the host (counting sort) into the blob.
int fwa_snapshot(fwa_engine* e, fwa_blob* out) {
    if (!e || !out) return FWA_E_ARG;
    memset(out, 0, sizeof(*out));
    // PREHASHED keys: their key groups come from the hashes the engine kept (d_khash); record lists keep no key table
    if (e->cfg.key_kind == FWA_KEY_PREHASHED && !e->d_khash)
        return fail(e, FWA_E_UNSUPPORTED, "snapshot of PREHASHED keys in record lists");
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rc0 = settle_pending(e)) return rc0;
    if (e->kind == FWA_SESSION) return snapshot_sessions(e, out);
    std::vector<FireWindow> hw;
    std::vector<int32_t> hs;
    int64_t n = 0;
    if (e->sparse) {   // every live window's (key, window) accumulators, lists kept
        std::vector<int64_t> all;
        for (auto& kv : e->sp->wins) all.push_back(kv.first);
        const int64_t rows0 = e->fire_rows, launches0 = e->fire_launches;
        const double ms0 = e->fire_ms;
        int rc = sp_fire(e, all, 1, false, &n);
        if (rc) return rc;
        e->fire_rows = rows0;
        e->fire_launches = launches0;
        e->fire_ms = ms0;
    }
    if (!e->sparse) for (auto& kv : e->live) {
        if (!e->touched[kv.second]) continue;
        FireWindow f;
        f.start = slice_start(e, kv.first);
        f.end = jm::wadd(f.start, e->g);
        f.slot_off = (int32_t)hs.size();
        f.nslots = 1;
        hs.push_back(kv.second);
        hw.push_back(f);
    }
    if (!hw.empty()) {
        const int64_t rows0 = e->fire_rows, launches0 = e->fire_launches;
        const double ms0 = e->fire_ms;
        int rc = launch_fire(e, hw, hs, 1, &n);
        if (rc) return rc;
        e->fire_rows = rows0;            // a snapshot is not a fire: keep the fire counters clean
        e->fire_launches = launches0;
        e->fire_ms = ms0;
    }
    const int na = e->cfg.num_aggs, maxp = e->cfg.max_parallelism, nh = e->ec.naggs - e->ec.nout, ncols = 3 + na + nh;
    const bool ph = e->cfg.key_kind == FWA_KEY_PREHASHED;   // + one column: each entry's key.hashCode()
    const int ncb = ncols + (ph ? 1 : 0);
    std::vector<int64_t> cols((size_t)n * ncb);
    const void* src[3 + FWA_MAX_AGGS + FWA_MAX_COLS] = {e->o_key, e->o_start, e->o_count};
    for (int j = 0; j < na; ++j) src[3 + j] = e->o_agg[j];
    for (int h = 0; h < nh; ++h) src[3 + na + h] = e->o_hid[h];
    for (int c = 0; c < ncols && n > 0; ++c)
        HIPCHK(e, hipMemcpy(cols.data() + (size_t)c * n, src[c], 8 * (size_t)n, hipMemcpyDeviceToHost));
    std::vector<int32_t> hash(ph ? (size_t)n : 0);
    if (ph && n > 0) {
        int32_t* dh = nullptr;
        HIPCHK(e, hipMalloc(&dh, sizeof(int32_t) * (size_t)n));
        khash_rows_kernel<<<grid_for(n), kBlock, 0, e->stream>>>(e->o_key, n, e->d_keys, (uint64_t)e->capacity - 1,
                                                                 e->seg_log, e->part_bits, e->d_khash, dh);
        const hipError_t er = hipMemcpyAsync(hash.data(), dh, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, e->stream);
        const hipError_t es = hipStreamSynchronize(e->stream);
        (void)hipFree(dh);
        if (er != hipSuccess || es != hipSuccess) return fail(e, FWA_E_DEVICE, "key hash export failed");
        for (int64_t i = 0; i < n; ++i) cols[(size_t)ncols * n + i] = hash[i];
    }
    std::vector<int32_t> kg((size_t)n);
    std::vector<int64_t> off((size_t)maxp + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        kg[i] = jm::key_group_of(cols[i], e->cfg.key_kind, ph ? hash[i] : 0, maxp);
        if (kg[i] < 0) return fail(e, FWA_E_STATE, "state holds a key outside every key group");
        off[kg[i] + 1]++;
    }
    for (int g = 0; g < maxp; ++g) off[g + 1] += off[g];
    const size_t words = kSnapHdr + (size_t)maxp + 1 + (size_t)n * ncb;
    int64_t* b = (int64_t*)malloc(words * 8);
    if (!b) return fail(e, FWA_E_OOM, "snapshot blob allocation failed");
    snap_header(e, b, n);
    memcpy(b + kSnapHdr, off.data(), 8 * ((size_t)maxp + 1));
    int64_t* body = b + kSnapHdr + maxp + 1;
    std::vector<int64_t> cur(off.begin(), off.end() - 1);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t d = cur[kg[i]]++;
        for (int c = 0; c < ncb; ++c) body[(size_t)c * n + d] = cols[(size_t)c * n + i];
    }
    out->data = b;
    out->size = (int64_t)(words * 8);
    return FWA_OK;
}

void fwa_blob_free(fwa_blob* b) {
    if (!b) return;
    free(b->data);
    b->data = nullptr;
    b->size = 0;
}

int fwa_restore(fwa_engine* e, const void* const* blobs, const int64_t* sizes, int32_t n_blobs) {
    if (e) e->rs_valid = false;
    if (!e) return FWA_E_STATE;
    if (n_blobs < 0 || (n_blobs > 0 && (!blobs || !sizes))) return fail(e, FWA_E_ARG, "null snapshot list");
    if (int rc0 = settle_pending(e)) return rc0;
    if (e->records_in != 0 || e->wm != LONG_MIN_J || !e->live.empty() || e->n_ss != 0 || sp_live_windows(e) != 0)
        return fail(e, FWA_E_STATE, "restore needs a fresh handle");
    const int na = e->cfg.num_aggs, maxp = e->cfg.max_parallelism, nh = e->ec.naggs - e->ec.nout;
    const bool ph = e->cfg.key_kind == FWA_KEY_PREHASHED;   // a last column holds each entry's key.hashCode()
    const int ncols = (e->kind == FWA_SESSION ? 4 : 3) + na + nh + (ph ? 1 : 0);
    if (ph && !e->d_khash) return fail(e, FWA_E_UNSUPPORTED, "restore of PREHASHED keys into record lists");
    int64_t ref[kSnapHdr];
    snap_header(e, ref, 0);
    // validate every blob before touching state
    for (int32_t b = 0; b < n_blobs; ++b) {
        const int64_t* h = (const int64_t*)blobs[b];
        if (!h || sizes[b] < (int64_t)(8 * (kSnapHdr + maxp + 1)) || (uint64_t)h[0] != kSnapMagic || h[1] != 1)
            return fail(e, FWA_E_ARG, "not a flink_amd snapshot (bad magic/version/size)");
        for (int w = 2; w < 20; ++w)
            if (h[w] != ref[w]) return fail(e, FWA_E_ARG, "snapshot window/aggregate configuration differs");
        for (int w = 24; w < 27; ++w)
            if (h[w] != ref[w]) return fail(e, FWA_E_ARG, "snapshot nullable-column configuration differs");
        const int64_t n = h[21];
        if (n < 0 || sizes[b] != (int64_t)(8 * (kSnapHdr + maxp + 1 + (size_t)n * ncols)))
            return fail(e, FWA_E_ARG, "snapshot size does not match its entry count");
    }
    if (e->kind == FWA_SESSION) return restore_sessions(e, blobs, n_blobs);
    if (e->red) return red_restore(e, blobs, n_blobs);
    int64_t wm = LONG_MAX_J;
    bool any = false;
    for (int32_t b = 0; b < n_blobs; ++b) {
        const int64_t* h = (const int64_t*)blobs[b];
        const int64_t n = h[21];
        wm = std::min<int64_t>(wm, h[20]);
        any = true;
        const int64_t* off = h + kSnapHdr;
        const int64_t lo = off[e->cfg.kg_start], hi = off[e->cfg.kg_end + 1];
        if (lo < 0 || hi < lo || hi > n) return fail(e, FWA_E_ARG, "corrupt key-group offsets");
        if (hi == lo) continue;
        const int64_t* body = off + maxp + 1;
        const void* acc[FWA_MAX_AGGS + FWA_MAX_COLS] = {};
        for (int j = 0; j < na; ++j) acc[j] = body + (size_t)(3 + j) * n + lo;
        for (int h = 0; h < nh; ++h) acc[na + h] = body + (size_t)(3 + na + h) * n + lo;
        int64_t late = 0;
        std::vector<int32_t> hv(ph ? (size_t)(hi - lo) : 0);
        for (int64_t i = lo; ph && i < hi; ++i) hv[i - lo] = (int32_t)body[(size_t)(3 + na + nh) * n + i];
        e->restoring = true;
        e->rs_hash = ph ? hv.data() : nullptr;
        int rc = fwa_push_partials(e, body + lo, body + (size_t)n + lo, body + (size_t)2 * n + lo, acc, hi - lo, 0, &late);
        e->restoring = false;
        e->rs_hash = nullptr;
        if (rc) return rc;
        if (late) return fail(e, FWA_E_STATE, "restored partials were dropped as late");
    }
    if (int rc = settle_pending(e)) return rc;
    e->records_in = 0;   // metrics are not part of the snapshot
    e->late_dropped = 0;
    if (any && wm > e->wm) {   // windows with maxTs <= wm fired before the snapshot: no re-fire
        if (e->sparse) sp_retire(e, wm);
        else if (int rc = retire_slices(e, wm)) return rc;
        e->wm = wm;
    }
    return FWA_OK;
}

// A run of consecutive hop windows with invertible accumulators: fire_slide_kernel. *done = false
// leaves the run to the generic fire.
// The run's slices that retire at wm (their last window is in the run; the same test retire_slices applies next) are
// cleared by the kernel itself and released without reset_slots_kernel's dense column writes.
static int fire_slide(fwa_engine* e, const std::set<std::pair<int64_t, int64_t>>& wins, int64_t wm, int64_t* nrows,
                      bool* done) {
    *done = false;
    if (e->nacc > kSlideAcc || e->cfg.nullable_cols) return FWA_OK;
    for (int c = 1; c < e->nacc; ++c) if (e->ec.acc_kind[c] != ACC_ADD_I64) return FWA_OK;
    if (e->size % e->g || e->slide % e->g) return FWA_OK;
    const int64_t L = e->size / e->g, r = e->slide / e->g;
    const int64_t start0 = wins.begin()->second;
    int64_t nw = 0;
    for (auto& w : wins) {   // consecutive hop windows: start_w = start0 + w * slide
        if (w.second != jm::wadd(start0, (int64_t)((uint64_t)nw * (uint64_t)e->slide)) || w.first != jm::wadd(w.second, e->size))
            return FWA_OK;
        ++nw;
    }
    const int64_t m = (nw - 1) * r + L;
    if (m > kSlideMaxU) return FWA_OK;
    const int64_t q0 = slice_q(e, start0);
    // slices without records read a zero slice (the kernel's loads are unconditional)
    const size_t zbytes = 8 * (size_t)e->nacc * (size_t)e->stride;
    if (zbytes > e->zslice_bytes) {
        if (e->d_zslice) HIPCHK(e, hipFree(e->d_zslice));
        e->d_zslice = nullptr;
        e->zslice_bytes = 0;
        HIPCHK(e, hipMalloc(&e->d_zslice, zbytes));
        HIPCHK(e, hipMemsetAsync(e->d_zslice, 0, zbytes, e->stream));
        e->zslice_bytes = zbytes;
    }
    std::vector<const unsigned long long*> up(m, (const unsigned long long*)e->d_zslice);
    std::vector<int32_t> cleared;
    bool any = false;
    for (int64_t i = 0; i < m; ++i) {
        auto it = e->live.find(q0 + i);
        if (it == e->live.end() || !e->touched[it->second]) continue;
        up[i] = e->slot_ptr[it->second];
        any = true;
        int64_t thr;
        bool always;
        accept_threshold(e, q0 + i, &thr, &always);
        if (i < nw * r && !always && wm >= thr) {   // retires right after this fire: the kernel clears it
            up[i] = (const unsigned long long*)((uintptr_t)up[i] | 1);
            cleared.push_back(it->second);
        }
    }
    *done = true;
    if (!any) return FWA_OK;
    if (!e->d_upos) HIPCHK(e, hipMalloc(&e->d_upos, sizeof(void*) * kSlideMaxU));
    int rc = upload(e, e->d_upos, up.data(), sizeof(void*) * m);
    if (rc) return rc;
    // every present key emits at most one row per window. A launch that clears retiring slices as it reads them must
    // run exactly once, so its bound comes from the device's own key count (every key inserted so far), not from the
    // host copy of the last status sync
    if (!cleared.empty()) {
        HIPCHK(e, hipMemcpyAsync(&e->h_st->n_keys, &e->d_st->n_keys, sizeof(e->h_st->n_keys), hipMemcpyDeviceToHost,
                                 e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
    }
    const int64_t nkeys = std::max<int64_t>((int64_t)e->h_st->n_keys, 1);
    rc = ensure_out(e, nw * nkeys);
    if (rc) return rc;
    // Carried window sums (no allowed lateness: a slice changes only through pushes, which stamp its touched epoch).
    // The previous run stored, per key, the sum over the slices its successor window shares with its last window except
    // the last rs_k of them; this run's window 0 reuses it when it is that successor and no push touched those slices
    // since. Otherwise (first run, a gap, a push into them: the tail rs_k doubles, up to L - r) window 0 sums all L.
    int32_t r_u0 = 0, r_k = 0;
    if (e->lateness == 0 && L - r >= 2 && e->rs_on) {
        if (!e->d_rsum) HIPCHK(e, hipMalloc(&e->d_rsum, sizeof(unsigned long long) * (size_t)e->nacc * (size_t)e->stride));
        bool use = e->rs_valid && q0 == e->rs_q0 && e->rs_u0 > 0 && e->rs_u0 <= L;
        bool dirty = false;
        for (int64_t q = q0; use && q < q0 + e->rs_u0; ++q) {
            auto it = e->live.find(q);
            if (it != e->live.end() && e->touched[it->second] > e->rs_epoch) { use = false; dirty = true; }
        }
        if (dirty) e->rs_k = (int32_t)std::min<int64_t>(L - r, 2 * (int64_t)e->rs_k);
        r_u0 = use ? e->rs_u0 : 0;
        e->rs_used += use ? 1 : 0;
        r_k = (int32_t)std::min<int64_t>(e->rs_k, L - r - 1);
    }
    e->rs_valid = false;
  relaunch:
    HIPCHK(e, hipMemsetAsync(&e->d_st->rows, 0, 8, e->stream));
    FireSlideArgs f;
    memset(&f, 0, sizeof(f));
    f.key_table = e->d_keys;
    f.capacity = e->capacity;
    f.stride = e->stride;
    f.upos = (const unsigned long long* const*)e->d_upos;
    f.m = (int32_t)m;
    f.nw = (int32_t)nw;
    f.L = (int32_t)L;
    f.r = (int32_t)r;
    f.start0 = start0;
    f.slide = e->slide;
    f.size = e->size;
    f.o_key = e->o_key;
    f.o_start = e->o_start;
    f.o_end = e->o_end;
    for (int j = 0; j < e->cfg.num_aggs; ++j) f.o_agg[j] = e->o_agg[j];
    f.out_cap = e->out_cap;
    f.st = e->d_st;
    f.rsum = e->d_rsum;
    f.r_u0 = r_u0;
    f.r_k = r_k;
    const int64_t grid = (e->capacity + 1 + (int64_t)kSlideBlock * kSlideJ - 1) / ((int64_t)kSlideBlock * kSlideJ);
    HIPCHK(e, hipEventRecord(e->ev[2], e->stream));
    switch (e->nacc) {
        case 1: fire_slide_kernel<1><<<(unsigned)grid, kSlideBlock, 0, e->stream>>>(f, e->d_ec); break;
        case 2: fire_slide_kernel<2><<<(unsigned)grid, kSlideBlock, 0, e->stream>>>(f, e->d_ec); break;
        case 3: fire_slide_kernel<3><<<(unsigned)grid, kSlideBlock, 0, e->stream>>>(f, e->d_ec); break;
        default:   // 512 threads: the 4-accumulator running sums do not fit the 128 VGPRs of a 1024-thread block
            fire_slide_kernel<4, kSlideJ, 512><<<(unsigned)((e->capacity + 1 + 512 * kSlideJ - 1) / (512 * kSlideJ)), 512, 0,
                                                 e->stream>>>(f, e->d_ec);
            break;
    }
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev[3], e->stream));
    rc = sync_status(e);
    if (rc) return rc;
    *nrows = (int64_t)e->h_st->rows;
    if (*nrows > e->out_cap) {   // n_keys was stale: grow to the exact count and fire again (idempotent)
        if (!cleared.empty()) return fail(e, FWA_E_STATE, "sliding fire exceeded its output bound");
        rc = ensure_out(e, *nrows);
        if (rc) return rc;
        r_u0 = 0;                                        // the first launch already replaced the carried sums
        goto relaunch;
    }
    for (int32_t s : cleared) e->slot_clean[s] = 1;   // retire_slices releases them without a reset
    if (r_k > 0) {                                    // what the next run's window 0 may reuse
        e->rs_valid = true;
        e->rs_q0 = q0 + nw * r;
        e->rs_u0 = (int32_t)(L - r - r_k);
        e->rs_epoch = e->push_epoch;
    }
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->fire_ms += ms;
    e->fire_launches++;
    e->fire_rows += *nrows;
    return FWA_OK;
}

// Speculative fire (TUMBLE, an FWA_PUSH_ASYNC push still pending): enqueue the fire of every live slice
// whose window is due right behind the pushed kernels, then settle the push. One host synchronisation
// instead of two, and the fire starts without the host round trip in between. The result stands only
// when the push needed no miss replay and had no late firings (then state was final when the fire ran);
// otherwise *ok = false and the caller fires again after the settle.
static int speculative_fire(fwa_engine* e, int64_t wm, int64_t* nrows, bool* ok) {
    *ok = false;
    std::vector<FireWindow> hw;
    std::vector<int32_t> hs;
    for (auto& kv : e->live) {   // touched flags are not settled yet: untouched slots only emit nothing
        FireWindow f;
        f.start = slice_start(e, kv.first);
        f.end = jm::wadd(f.start, e->g);
        const int64_t mt = trig(e, jm::wsub(f.end, 1));
        if (!(mt > e->wm && mt <= wm)) continue;
        f.slot_off = (int32_t)hs.size();
        f.nslots = 1;
        hs.push_back(kv.second);
        hw.push_back(f);
    }
    int rc = FWA_OK;
    if (!hw.empty()) {
        rc = launch_fire(e, hw, hs, 0, nrows, 0);   // synchronises: the push's status is in h_st too
        if (rc) return rc;
    }
    const DevStatus st = *e->h_st;
    *ok = hw.empty() ? false : (st.spill_n == 0 && st.late_fire == 0 && st.error == 0 && e->late_rows == 0);
    // the speculation held: the fired slices retire now, so their resets run on the GPU while the host settles the push
    // (fwa_advance_watermark's own retire_slices then finds nothing left)
    if (*ok && (rc = retire_slices(e, wm))) return rc;
    rc = settle_pending(e);
    if (rc) return rc;
    return FWA_OK;
}

// The output columns of the last fire (nrows rows) as an fwa_out (device pointers, or host copies in h_out).
static int fill_out(fwa_engine* e, int64_t nrows, fwa_out* out) {
    memset(out, 0, sizeof(*out));
    out->n_rows = nrows;
    // the caller's aggregates: DECIMAL ones finished from their piece sums (decimal.inc), the others as fired
    const int na = e->dec ? e->dec->ucfg.num_aggs : e->cfg.num_aggs;
    const void* col[FWA_MAX_AGGS];
    const uint8_t* nul[FWA_MAX_AGGS];
    size_t width[FWA_MAX_AGGS];
    if (e->dec) {
        if (int rc = dec_finish(e, nrows)) return rc;
        for (int j = 0; j < na; ++j) {
            if (e->dec->d[j].kind) { col[j] = e->dec->d_out[j]; nul[j] = e->dec->d_null[j]; width[j] = 16; continue; }
            const int i = e->dec->umap[j];
            col[j] = e->o_agg[i];
            nul[j] = e->o_null[i];
            width[j] = type_size(e->cfg.aggs[i].kind);
        }
    } else {
        for (int j = 0; j < na; ++j) { col[j] = e->o_agg[j]; nul[j] = e->o_null[j]; width[j] = type_size(e->cfg.aggs[j].kind); }
    }
    out->num_aggs = na;
    if (e->cfg.output_on_device) {
        out->on_device = 1;
        out->key = e->o_key;
        out->win_start = e->o_start;
        out->win_end = e->o_end;
        for (int j = 0; j < na; ++j) { out->agg[j] = col[j]; out->agg_null[j] = nul[j]; }
        return FWA_OK;
    }
    out->on_device = 0;
    e->h_out.resize(std::max<size_t>((size_t)nrows * (25 + 17 * (size_t)na), 8));
    char* p = e->h_out.data();
    hipError_t err = hipSuccess;
    auto get = [&](const void* src, size_t bytes) -> const void* {
        if (bytes) { hipError_t r = hipMemcpy(p, src, bytes, hipMemcpyDeviceToHost); if (r != hipSuccess) err = r; }
        const void* r = p;
        p += bytes;
        return r;
    };
    out->key = (const int64_t*)get(e->o_key, 8 * nrows);
    out->win_start = (const int64_t*)get(e->o_start, 8 * nrows);
    out->win_end = (const int64_t*)get(e->o_end, 8 * nrows);
    for (int j = 0; j < na; ++j) out->agg[j] = get(col[j], width[j] * nrows);
    for (int j = 0; j < na; ++j)
        if (nul[j]) out->agg_null[j] = (const uint8_t*)get(nul[j], (size_t)nrows);
    HIPCHK(e, err);
    return FWA_OK;
}

// Account an in-flight fwa_advance_watermark_async fire once it completed (its rows stay in the output columns).
static int finish_afire(fwa_engine* e) {
    if (!e->af_gpu) return FWA_OK;
    HIPCHK(e, hipEventSynchronize(e->ev_af));
    e->af_gpu = false;
    const int64_t rows = *e->h_af_rows;
    if (rows > e->out_cap) return fail(e, FWA_E_STATE, "asynchronous fire exceeded its output bound");
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
    e->fire_ms += ms;
    e->fire_launches++;
    e->fire_rows += rows;
    e->rows_out += rows;
    e->af_rows = rows;
    return FWA_OK;
}

int fwa_advance_watermark(fwa_engine* e, int64_t wm, fwa_out* out) {
    if (!e) return FWA_E_STATE;
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rcf = finish_afire(e)) return rcf;
    e->af_pend = false;                          // an untaken asynchronous output is overwritten
    int64_t nrows = 0;
    bool spec_done = false;
    if (e->pend && e->kind == FWA_TUMBLE && wm > e->wm && e->late_rows == 0) {
        int rc = speculative_fire(e, wm, &nrows, &spec_done);
        if (rc) return rc;
        if (!spec_done) nrows = 0;
    }
    if (int rc0 = settle_pending(e)) return rc0;
    if (out) memset(out, 0, sizeof(*out));
    if (wm > e->wm && e->kind == FWA_SESSION) {
        int rc = fire_sessions(e, wm, &nrows);
        if (rc) return rc;
        e->wm = wm;
    } else if (wm > e->wm && e->sparse) {   // windows with prev < maxTimestamp <= wm (every live one is > prev)
        int rc = sp_fire(e, sp_due(e, wm), 0, true, &nrows);
        if (rc) return rc;
        e->wm = wm;
    } else if (wm > e->wm) {
        const int64_t prev = e->wm;
        // windows of touched slices that fire now: prev < end-1 <= wm  (EventTimeTrigger / isWindowFired)
        std::set<std::pair<int64_t, int64_t>> wins;  // (end, start)
        std::vector<std::pair<int64_t, int64_t>> tmp;
        for (auto& kv : e->live) {
            if (!e->touched[kv.second]) continue;
            tmp.clear();
            windows_of_slice(e, kv.first, tmp);
            for (auto& w : tmp) {
                const int64_t mt = trig(e, jm::wsub(w.second, 1));
                if (mt > prev && mt <= wm) wins.insert({w.second, w.first});
            }
        }
        bool slid = false;
        if (e->kind == FWA_SLIDE && wins.size() >= 2 && e->late_rows == 0 && !e->red) {
            int rc = fire_slide(e, wins, wm, &nrows, &slid);
            if (rc) return rc;
        }
        std::vector<FireWindow> hw;
        std::vector<int32_t> hs;
        if (!slid && !spec_done) for (auto& w : wins) {
            FireWindow f;
            f.end = w.first;
            f.start = w.second;
            f.slot_off = (int32_t)hs.size();
            const int64_t q0 = slice_q(e, f.start);
            const int64_t q1 = slice_q(e, jm::wsub(f.end, 1));
            for (int64_t q = q0; q <= q1; ++q) {
                auto it = e->live.find(q);
                if (it != e->live.end() && e->touched[it->second]) hs.push_back(it->second);
            }
            f.nslots = (int32_t)hs.size() - f.slot_off;
            if (f.nslots > 0) hw.push_back(f);
        }
        if (!hw.empty()) {
            int rc = launch_fire(e, hw, hs, 0, &nrows, e->late_rows);
            if (rc) return rc;
        }
        int rc = retire_slices(e, wm);
        if (rc) return rc;
        e->wm = wm;
    }
    if (e->late_rows > 0) {   // late firings pushed since the last call and no window fired now
        int rc = ensure_out(e, e->late_rows);
        if (rc) return rc;
        nrows = e->late_rows;
        rc = emit_late_rows(e);
        if (rc) return rc;
        rc = stream_sync(e);
        if (rc) return rc;
        e->late_rows = 0;
    }
    e->rows_out += nrows;
    e->af_rows = nrows;
    if (out) return fill_out(e, nrows, out);
    return FWA_OK;
}

// Watermark advance that returns before the fire completes (include/flink_amd.h): a TUMBLE fire after an
// FWA_PUSH_ASYNC push is enqueued speculatively, the host waits only for the push's status (the fire runs meanwhile)
// and, when the push needed nothing replayed, retires the fired slices and returns; the next push can then be
// enqueued while the fire runs. Anything else takes the synchronous path. The rows: fwa_fired_output.
int fwa_advance_watermark_async(fwa_engine* e, int64_t wm) {
    if (!e) return FWA_E_STATE;
    HIPCHK(e, hipSetDevice(e->cfg.device));
    if (int rcf = finish_afire(e)) return rcf;
    e->af_pend = false;
    if (e->pend && e->pend_v2 && e->kind == FWA_TUMBLE && wm > e->wm && e->late_rows == 0 && !e->sparse) {
        std::vector<FireWindow> hw;
        std::vector<int32_t> hs;
        for (auto& kv : e->live) {   // as speculative_fire: untouched slots emit nothing
            FireWindow f;
            f.start = slice_start(e, kv.first);
            f.end = jm::wadd(f.start, e->g);
            const int64_t mt = trig(e, jm::wsub(f.end, 1));
            if (!(mt > e->wm && mt <= wm)) continue;
            f.slot_off = (int32_t)hs.size();
            f.nslots = 1;
            hs.push_back(kv.second);
            hw.push_back(f);
        }
        // every row of the fire must fit: windows x keys (keys known at the last status + the pending push's). The
        // end-of-input watermark (Long.MAX_VALUE) lists every live slice, the lookahead's included, and would grow the
        // output columns far past the rows it fires (hipFree synchronises the device): the synchronous path counts
        // its rows and sizes them instead.
        const int64_t nk = std::min<int64_t>(e->capacity + 1, (int64_t)e->h_st->n_keys + e->pend_n);
        const int64_t need = (int64_t)hw.size() * std::max<int64_t>(nk, 1);
        if (!hw.empty() && (need <= e->out_cap || wm != LONG_MAX_J)) {
            int rc = ensure_out(e, need);
            if (rc) return rc;
            if ((rc = upload_windows(e, hw, hs))) return rc;
            HIPCHK(e, hipMemsetAsync(&e->d_st->rows, 0, 8, e->stream));
            if ((rc = enqueue_fire(e, hw, hs, 0))) return rc;
            HIPCHK(e, hipMemcpyAsync(e->h_af_rows, &e->d_st->rows, 8, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(e, hipEventRecord(e->ev_af, e->stream));
            if ((rc = wait_status_event(e))) return rc;   // the push's status; the fire keeps running
            const DevStatus st = *e->h_st;
            if (st.spill_n == 0 && st.late_fire == 0 && st.error == 0) {
                e->af_gpu = true;
                e->af_pend = true;
                if ((rc = retire_slices(e, wm))) return rc;   // resets enqueued behind the fire
                if ((rc = settle_push(e))) return rc;      // no wait (st_ready)
                e->wm = wm;
                return FWA_OK;
            }
            HIPCHK(e, hipEventSynchronize(e->ev_af));         // the speculation failed: the synchronous path
        }
    }
    int rc = fwa_advance_watermark(e, wm, nullptr);
    if (rc) return rc;
    e->af_pend = true;
    return FWA_OK;
}

int fwa_fired_output(fwa_engine* e, fwa_out* out) {
    if (!e || !out) return FWA_E_ARG;
    if (!e->af_pend) return fail(e, FWA_E_STATE, "no fwa_advance_watermark_async output to take");
    if (int rc = finish_afire(e)) return rc;
    e->af_pend = false;
    return fill_out(e, e->af_rows, out);
}

int fwa_flush(fwa_engine* e) {
    if (!e) return FWA_E_STATE;
    if (int rc0 = settle_pending(e)) return rc0;
    int rc = stream_sync(e);
    if (rc) return rc;
    return FWA_OK;
}

int64_t fwa_stats_size(void) { return (int64_t)sizeof(fwa_stats); }

int fwa_get_stats(fwa_engine* e, fwa_stats* s) {
    if (!e || !s) return FWA_E_ARG;
    if (int rc0 = settle_pending(e)) return rc0;
    int rc = sync_status(e);
    if (rc) return rc;
    s->records_in = e->records_in;
    s->late_dropped = e->late_dropped;
    s->rows_out = e->rows_out;
    s->live_keys = (int64_t)e->h_st->n_keys;
    s->live_slices = e->kind == FWA_SESSION ? e->n_ss : e->sparse ? sp_live_windows(e) : (int64_t)e->live.size();
    s->current_watermark = e->wm;
    s->ingest_launches = e->ingest_launches;
    s->ingest_ms = e->ingest_ms;
    s->ingest_records = e->ingest_records;
    s->replay_records = e->replay_records;
    s->dec_inexact = e->dec ? e->dec->inexact : 0;
    s->fire_launches = e->fire_launches;
    s->fire_ms = e->fire_ms;
    s->fire_rows = e->fire_rows;
    s->partition_ms = e->partition_ms;
    s->combine_ms = e->combine_ms;
    return FWA_OK;
}

int fwa_late_records(fwa_engine* e, const int32_t** idx, int64_t* n) {
    if (!e || !idx || !n) return FWA_E_ARG;
    if (!(e->cfg.flags & FWA_CFG_LATE_INDICES)) return fail(e, FWA_E_STATE, "configure FWA_CFG_LATE_INDICES");
    if (int rc0 = settle_pending(e)) return rc0;
    *idx = e->late_idx.empty() ? nullptr : e->late_idx.data();
    *n = (int64_t)e->late_idx.size();
    return FWA_OK;
}

int fwa_reset_timers(fwa_engine* e) {
    if (!e) return FWA_E_ARG;
    if (int rc0 = settle_pending(e)) return rc0;
    e->ingest_launches = e->ingest_records = e->replay_records = e->fire_launches = e->fire_rows = 0;
    e->ingest_ms = e->fire_ms = e->partition_ms = e->combine_ms = 0;
    return FWA_OK;
}

int fwa_set_option(fwa_engine* e, int32_t option, int64_t value) {
    if (!e) return FWA_E_ARG;
    if (int rc0 = settle_pending(e)) return rc0;
    const int32_t tri = value < 0 ? -1 : (value > 0 ? 1 : 0);
    switch (option) {
        case FWA_OPT_SKEW_MERGE: e->opt_pre = tri; return FWA_OK;
        case FWA_OPT_WINDOW_PASSES: e->opt_mp = tri; return FWA_OK;
        case FWA_OPT_NARROW_ENTRIES: e->opt_narrow = tri; return FWA_OK;
        case FWA_OPT_SESSION_CELLS: e->opt_cells = tri; return FWA_OK;
        case FWA_OPT_OUT_MIN_ROWS: e->opt_out_min = std::max<int64_t>(0, value); return FWA_OK;
        case FWA_OPT_PARTIALS_ONE_PASS: e->opt_partials_v1 = value > 0; return FWA_OK;
        case FWA_OPT_SP_TABLE: case FWA_OPT_SP_FMAX: case FWA_OPT_SP_BUDGET: return sp_set_option(e, option, value);
        case FWA_OPT_PROFILE: e->opt_profile = value > 0 ? 1 : 0; return FWA_OK;
        case FWA_OPT_INGEST_VARIANT: e->opt_variant = (int32_t)std::max<int64_t>(0, value); return FWA_OK;
        case FWA_OPT_SLIDE_CARRIED: e->rs_on = value != 0; e->rs_valid = false; return FWA_OK;
        case FWA_OPT_FIRE_PARTIALS: e->opt_fire_partials = value != 0 ? 1 : 0; return FWA_OK;
        case FWA_OPT_DEC_WRAP_NULL: e->opt_dec_wrap_null = value != 0 ? 1 : 0; return FWA_OK;
        default: return fail(e, FWA_E_ARG, "unknown option");
    }
}

int fwa_get_option(const fwa_engine* e, int32_t option, int64_t* value) {
    if (!e || !value) return FWA_E_ARG;
    auto eff = [](int32_t opt, bool adaptive_on) -> int64_t { return opt == 1 || (opt != 0 && adaptive_on) ? 1 : 0; };
    switch (option) {
        case FWA_OPT_SKEW_MERGE: *value = eff(e->opt_pre, e->pre); return FWA_OK;
        case FWA_OPT_WINDOW_PASSES: *value = eff(e->opt_mp, e->mp); return FWA_OK;
        case FWA_OPT_NARROW_ENTRIES: *value = eff(e->opt_narrow, e->narrow); return FWA_OK;
        case FWA_OPT_SESSION_CELLS: *value = eff(e->opt_cells, e->cell_skip <= 0); return FWA_OK;
        case FWA_OPT_OUT_MIN_ROWS: *value = e->opt_out_min > 0 ? e->opt_out_min : ((int64_t)1 << 22); return FWA_OK;
        case FWA_OPT_PARTIALS_ONE_PASS: *value = e->opt_partials_v1 ? 1 : 0; return FWA_OK;
        case FWA_OPT_SP_TABLE: case FWA_OPT_SP_FMAX: case FWA_OPT_SP_BUDGET:
            if (!e->sp) return FWA_E_UNSUPPORTED;
            *value = option == FWA_OPT_SP_TABLE ? e->sp->T : option == FWA_OPT_SP_FMAX ? (e->sp->fmax ? e->sp->fmax : kSpMaxF)
                                                                                    : (int64_t)e->sp->budget;
            return FWA_OK;
        case FWA_OPT_PROFILE: *value = e->opt_profile; return FWA_OK;
        case FWA_OPT_SESSION_PATH: *value = e->sess_path; return FWA_OK;
        case FWA_OPT_INGEST_VARIANT: *value = e->opt_variant; return FWA_OK;
        case FWA_OPT_SLIDE_CARRIED: *value = e->rs_used; return FWA_OK;
        case FWA_OPT_FIRE_PARTIALS: *value = e->mf_calls - e->mf_fallbacks; return FWA_OK;
        case FWA_OPT_DEC_WRAP_NULL: *value = e->opt_dec_wrap_null; return FWA_OK;
        default: return FWA_E_ARG;
    }
}

int fwa_set_input_stream(fwa_engine* e, void* stream) {
    if (!e) return FWA_E_STATE;
    e->in_stream = (hipStream_t)stream;
    return FWA_OK;
}

int fwa_key_groups(const int64_t* keys, const int32_t* key_hash, int64_t n, int32_t key_kind, int32_t max_par,
                   int32_t par, int32_t* kg_out, int32_t* op_out, int32_t flags, int32_t device) {
    if (n < 0 || max_par <= 0 || par <= 0 || par > max_par || key_kind < 0 || key_kind > 3) return FWA_E_ARG;
    if (key_kind == FWA_KEY_PREHASHED && n > 0 && !key_hash) return FWA_E_ARG;
    if (n == 0) return FWA_OK;
    if (hipSetDevice(device) != hipSuccess) return FWA_E_DEVICE;
    if (flags & FWA_PUSH_DEVICE_PTRS) {
        key_groups_kernel<<<grid_for(n), kBlock>>>(keys, key_hash, n, key_kind, max_par, par, kg_out, op_out);
        return hipDeviceSynchronize() == hipSuccess ? FWA_OK : FWA_E_DEVICE;
    }
    int64_t* dk = nullptr;
    int32_t *dh = nullptr, *dkg = nullptr, *dop = nullptr;
    int rc = FWA_OK;
    do {
        if (hipMalloc(&dk, 8 * n) != hipSuccess || hipMalloc(&dkg, 4 * n) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (key_hash && hipMalloc(&dh, 4 * n) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (op_out && hipMalloc(&dop, 4 * n) != hipSuccess) { rc = FWA_E_OOM; break; }
        if (hipMemcpy(dk, keys, 8 * n, hipMemcpyHostToDevice) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        if (dh && hipMemcpy(dh, key_hash, 4 * n, hipMemcpyHostToDevice) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        key_groups_kernel<<<grid_for(n), kBlock>>>(dk, dh, n, key_kind, max_par, par, dkg, dop);
        if (hipMemcpy(kg_out, dkg, 4 * n, hipMemcpyDeviceToHost) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        if (op_out && hipMemcpy(op_out, dop, 4 * n, hipMemcpyDeviceToHost) != hipSuccess) { rc = FWA_E_DEVICE; break; }
    } while (0);
    for (void* p : {(void*)dk, (void*)dh, (void*)dkg, (void*)dop}) if (p) (void)hipFree(p);
    return rc;
}

int fwa_generate(const fwa_gen_params* p, int64_t n, int64_t* keys, int64_t* ts, int64_t* v_i64, float* v_f32,
                 double* v_f64, int32_t device, void* stream) {
    if (!p || n < 0 || p->total_records <= 0 || p->num_keys <= 0 || p->max_delay_ms < 0) return FWA_E_ARG;
    if (p->key_dist == 1 && !p->zipf_cdf) return FWA_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FWA_E_DEVICE;
    if (n == 0) return FWA_OK;
    generate_kernel<<<grid_for(n, 256 * 64), kBlock, 0, (hipStream_t)stream>>>(*p, n, keys, ts, v_i64, v_f32, v_f64);
    return hipGetLastError() == hipSuccess ? FWA_OK : FWA_E_DEVICE;
}

}  // extern "C"
