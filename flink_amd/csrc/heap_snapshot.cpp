// heap_snapshot.cpp -- keyed window state in the byte layout of Flink's heap keyed-state backend (SURVEY §8(f)
// rank 3), converted on the host from / into the engine's own FWASNAP1 blob (fwa_snapshot / fwa_restore).
//
// What the reference writes per key group (HeapSnapshotStrategy.java:154-175, all java.io.DataOutput, big-endian):
//   int   keyGroupId
//   per registered state (ids: key/value states first, then priority queues, HeapSnapshotResources.java:100-139):
//     short stateId
//     int   n; n x (namespace, key, state)      CopyOnWriteStateMapSnapshot.writeState :138-148
//   (timers) int n; n x (long flipSignBit(ts), key, namespace)   KeyGroupPartitioner + TimerSerializer.serialize :147-152
// KeyGroupRangeOffsets holds each key group's section start. The KeyedBackendSerializationProxy header in front of
// the sections (state names, serializer snapshots) is JVM metadata the Java shim writes itself.
//
// The states per key group (registration order):
//   DATASTREAM TUMBLE  WindowOperator: 0 window contents -- namespace TimeWindow (TimeWindow.Serializer: long start,
//                      long end), key Long; 1 timers at window.maxTimestamp() (EventTimeTrigger.onElement) and at the
//                      cleanup time maxTimestamp + allowedLateness (WindowOperator.registerCleanupTimer :608-620),
//                      deduplicated like HeapPriorityQueueSet.
//   DATASTREAM SESSION 0 window contents under each session's state window; 1 merging-window-set (ListState of
//                      Tuple2<actual, state> TimeWindows under VoidNamespace, MergingWindowSet.persist :100-105);
//                      2 timers as for TUMBLE, per session.
//   TABLE TUMBLE / HOP / CUMULATE  SlicingWindowOperator: 0 namespace Long slice end, key BinaryRowData(BIGINT)
//                      (BinaryRowDataSerializer: int size + row); 1 timers at the first unfired window end - 1 of each
//                      live slice (WindowTimerServiceImpl / TimeWindowUtil, UTC). CUMULATE folds fired slices into the
//                      window's first slice.
// The accumulator is the engine's built-in aggregate state: a Tuple (DataStream, TupleSerializer: big-endian fields)
// or a BinaryRowData (Table) of COUNT(*) followed by one field per aggregate -- BIGINT for COUNT / integer SUM, AVG,
// MIN, MAX, DOUBLE for floating SUM / AVG / MIN / MAX (the AggregateFunction's ACC type in the shim).
// Table rows carry SQL NULLs as BinaryRowData null bits (an aggregate whose column held only NULLs) and one more
// BIGINT field per hidden non-NULL counter; Table timers under a shift time zone are toEpochMillsForTimer(end - 1).
//   DATASTREAM SLIDE   WindowOperator per-window state (window = merge of the engine's slices inside it); the restore
//                      rebuilds slices whose merges equal every restored window (slide_windows_to_slices).
//   TABLE SESSION      legacy Table WindowOperator: 0 session-window-mapping (MapSerializer of TimeWindow pairs under
//                      VoidNamespace), 1 window-aggs (TimeWindow namespace, BinaryRowData key and accumulator), timers
//                      at toEpochMillsForTimer(maxTimestamp) per in-flight session.
// DECIMAL SUM / AVG (Table): the accumulator field is the DECIMAL(38, s) running sum (findSumAggType), rebuilt from the
// engine's 32-bit piece sums (decimal.inc) and written as a non-compact DecimalData; AVG's count is COUNT(*) or the
// column's hidden non-NULL counter, already in the row.
// PREHASHED keys (their Java serialization is the caller's) and DataStream reductions: FWA_E_UNSUPPORTED; the engine
// format (fwa_snapshot, FWASNAP1) carries both, PREHASHED keys with the hash column of their key groups.
#include <algorithm>
#include <cstdint>
#include <map>
#include <set>
#include <tuple>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flink_amd.h"
#include "java_math.h"
#include "dec_view.h"

namespace {

constexpr uint64_t kMagic = 0x3150414E53415746ull;   // "FWASNAP1" (engine.hip snap_header)
constexpr int kHdr = 32;

struct Snap {                                        // parsed FWASNAP1 blob
    int64_t kind, sem, size, slide, off, gap, late, maxp, key_kind, naggs, wm, n, kg_lo, kg_hi, nh;
    int64_t agg[FWA_MAX_AGGS];
    const int64_t* koff;                             // [maxp + 1]
    const int64_t* col;                              // SoA [3 + naggs][n]
};

bool parse(const void* p, int64_t bytes, Snap* s) {
    const int64_t* w = (const int64_t*)p;
    if (bytes < kHdr * 8 || (uint64_t)w[0] != kMagic || w[1] != 1) return false;
    s->kind = w[2]; s->sem = w[3]; s->size = w[4]; s->slide = w[5]; s->off = w[6]; s->gap = w[7]; s->late = w[8];
    s->maxp = w[9]; s->key_kind = w[10]; s->naggs = w[11]; s->wm = w[20]; s->n = w[21]; s->kg_lo = w[22]; s->kg_hi = w[23];
    s->nh = w[25];
    if (s->naggs < 0 || s->naggs > FWA_MAX_AGGS || s->maxp <= 0 || s->nh < 0 || s->nh > FWA_MAX_COLS) return false;
    for (int j = 0; j < s->naggs; ++j) s->agg[j] = w[12 + j];
    const int64_t ncols = (s->kind == FWA_SESSION ? 4 : 3) + s->naggs + s->nh;
    if (bytes != (kHdr + s->maxp + 1 + s->n * ncols) * 8) return false;
    s->koff = w + kHdr;
    s->col = w + kHdr + s->maxp + 1;
    return true;
}

bool is_ord(int64_t kind) { return kind >= FWA_MIN_I64 && kind <= FWA_MAX_F64; }

// engine accumulator word <-> the ACC field value (64 bits: long, or double bits)
uint64_t acc_to_field(int64_t kind, uint64_t a) {
    if (!is_ord(kind)) return a;                                        // counts, i64 sums, f64 sum bits
    if (kind == FWA_MIN_I64 || kind == FWA_MAX_I64) return a ^ 0x8000000000000000ull;
    return (a & 0x8000000000000000ull) ? (a & 0x7fffffffffffffffull) : ~a;   // order-preserving double key
}
uint64_t field_to_acc(int64_t kind, uint64_t f) {
    if (!is_ord(kind)) return f;
    if (kind == FWA_MIN_I64 || kind == FWA_MAX_I64) return f ^ 0x8000000000000000ull;
    return (f & 0x8000000000000000ull) ? ~f : (f | 0x8000000000000000ull);
}

struct Out {
    std::vector<uint8_t> b;
    void u8(uint8_t v) { b.push_back(v); }
    void i16(int v) { u8((uint8_t)(v >> 8)); u8((uint8_t)v); }
    void i32(int64_t v) { for (int s = 24; s >= 0; s -= 8) u8((uint8_t)((uint64_t)v >> s)); }
    void i64(uint64_t v) { for (int s = 56; s >= 0; s -= 8) u8((uint8_t)(v >> s)); }
    void le64(uint64_t v) { for (int s = 0; s < 64; s += 8) u8((uint8_t)(v >> s)); }
    // BinaryRowData with `arity` 8-byte fixed-length fields, RowKind INSERT (BinaryRowDataSerializer; BinaryRowData
    // layout: header byte then one null bit per field from bit 8 on, 8-byte aligned, BinaryRowData.java:68-123)
    void row(const uint64_t* f, int arity, const bool* isnull = nullptr) {
        const int nb = ((arity + 63 + 8) / 64) * 8;
        i32(nb + 8 * arity);
        std::vector<uint8_t> hdr((size_t)nb, 0);
        for (int i = 0; i < arity; ++i) if (isnull && isnull[i]) hdr[(size_t)(i + 8) / 8] |= (uint8_t)(1u << ((i + 8) % 8));
        for (int i = 0; i < nb; ++i) u8(hdr[(size_t)i]);
        for (int i = 0; i < arity; ++i) le64(isnull && isnull[i] ? 0 : f[i]);
    }
    void raw_row(const std::vector<uint8_t>& r) { i32((int64_t)r.size()); b.insert(b.end(), r.begin(), r.end()); }
    // an accumulator row whose fields with isdec[i] are DECIMAL(38, s) -- non-compact (DecimalData.isCompact: precision
    // > 18), so RowDataSerializer.toBinaryRow (:196-212) writes them with AbstractBinaryWriter.writeDecimal (:164-196):
    // 16 zeroed bytes reserved in the variable-length part, toUnscaledBytes at their start, slot = offset << 32 |
    // length; a NULL field goes through setNullAt instead (null bit, slot 0, nothing reserved)
    void acc_row(const uint64_t* f, int arity, const bool* isnull, const bool* isdec, const std::vector<uint8_t>* decb) {
        const int nb = ((arity + 63 + 8) / 64) * 8;
        std::vector<uint8_t> r((size_t)nb + 8 * (size_t)arity, 0);
        for (int i = 0; i < arity; ++i) {
            uint64_t v = f[i];
            if (isnull[i]) {
                r[(size_t)(i + 8) / 8] |= (uint8_t)(1u << ((i + 8) % 8));
                v = 0;
            } else if (isdec[i]) {
                v = ((uint64_t)r.size() << 32) | (uint64_t)decb[i].size();
                r.insert(r.end(), decb[i].begin(), decb[i].end());
                r.resize(r.size() + 16 - decb[i].size(), 0);
            }
            for (int k = 0; k < 8; ++k) r[(size_t)nb + 8 * i + k] = (uint8_t)(v >> (8 * k));
        }
        raw_row(r);
    }
};

typedef __int128 i128;
typedef unsigned __int128 u128;

i128 dec_bound() { i128 r = 1; for (int i = 0; i < 38; ++i) r *= 10; return r; }   // 10^38

// A DECIMAL aggregate's window total T = sum_k S_k * 2^(32k) from the engine's piece sums (decimal.inc: the pieces below
// the top one unsigned, the top one signed), in 192-bit two's complement. false: |T| has more than 38 digits
// (DecimalData.fromBigDecimal returns NULL, DecimalData.java:184-195).
bool dec_total(const uint64_t* S, int npc, i128* out) {
    uint64_t t[3] = {0, 0, 0};
    for (int k = 0; k < npc; ++k) {
        const uint64_t ext = (k == npc - 1 && (int64_t)S[k] < 0) ? ~0ull : 0ull;
        const uint64_t src[4] = {S[k], ext, ext, ext};
        const int li = (32 * k) / 64, bs = (32 * k) % 64;
        u128 carry = 0;
        for (int m = 0; m < 3; ++m) {
            const int i = m - li;
            const uint64_t lo = i >= 0 ? src[i] : 0, prev = i >= 1 ? src[i - 1] : 0;
            const uint64_t w = bs == 0 ? lo : (lo << bs) | (prev >> (64 - bs));
            const u128 a = (u128)t[m] + w + carry;
            t[m] = (uint64_t)a;
            carry = a >> 64;
        }
    }
    if (t[2] != (((int64_t)t[1] < 0) ? ~0ull : 0ull)) return false;
    const i128 v = (i128)(((u128)t[1] << 64) | t[0]);
    if (v >= dec_bound() || v <= -dec_bound()) return false;
    *out = v;
    return true;
}

// The inverse for a restore: piece sums totalling T. Two pieces (int64 input) hold |T| < 2^95 only.
bool dec_split(i128 T, int npc, uint64_t* S) {
    const u128 u = (u128)T;
    if (npc == 2) {
        const i128 hi = T >> 32;
        if (hi > (i128)INT64_MAX || hi < (i128)INT64_MIN) return false;
        S[0] = (uint64_t)(u & 0xffffffffu);
        S[1] = (uint64_t)(int64_t)hi;
        return true;
    }
    S[0] = (uint64_t)(u & 0xffffffffu);
    S[1] = (uint64_t)((u >> 32) & 0xffffffffu);
    S[2] = (uint64_t)((u >> 64) & 0xffffffffu);
    S[3] = (uint64_t)(int64_t)(T >> 96);
    return true;
}

// DecimalData.toUnscaledBytes (BigInteger.toByteArray): minimal big-endian two's complement, and back
std::vector<uint8_t> dec_bytes(i128 v) {
    uint8_t b[16];
    const u128 u = (u128)v;
    for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(u >> (8 * (15 - i)));
    int st = 0;
    while (st < 15 && ((b[st] == 0x00 && !(b[st + 1] & 0x80)) || (b[st] == 0xff && (b[st + 1] & 0x80)))) ++st;
    return std::vector<uint8_t>(b + st, b + 16);
}
bool dec_of_bytes(const uint8_t* p, uint64_t len, i128* v) {
    if (len < 1 || len > 16) return false;
    u128 u = (p[0] & 0x80) ? ~(u128)0 : 0;
    for (uint64_t i = 0; i < len; ++i) u = (u << 8) | p[i];
    *v = (i128)u;
    return true;
}

struct In {
    const uint8_t* p;
    int64_t n, at = 0;
    bool ok = true;
    uint64_t get(int k, bool le = false) {
        if (at + k > n) { ok = false; return 0; }
        uint64_t v = 0;
        for (int i = 0; i < k; ++i) v = le ? v | ((uint64_t)p[at + i] << (8 * i)) : (v << 8) | p[at + i];
        at += k;
        return v;
    }
    int64_t i32() { return (int32_t)get(4); }
    int64_t i64() { return (int64_t)get(8); }
    void row(uint64_t* f, int arity, bool* isnull = nullptr) {
        const int nb = ((arity + 63 + 8) / 64) * 8;
        if (i32() != nb + 8 * arity) { ok = false; return; }
        std::vector<uint8_t> hdr((size_t)nb);
        for (int i = 0; i < nb; ++i) hdr[(size_t)i] = (uint8_t)get(1);
        if (hdr[0] != 0) ok = false;                                  // RowKind INSERT
        for (int i = 0; i < arity; ++i) {
            const bool nl = (hdr[(size_t)(i + 8) / 8] >> ((i + 8) % 8)) & 1;
            if (isnull) isnull[i] = nl;
            else if (nl) ok = false;                                  // a NULL where the layout has none
        }
        for (int i = 0; i < arity; ++i) f[i] = get(8, true);
    }
    // an accumulator row (Out::acc_row): DECIMAL fields (isdec) read from the variable-length part into decv
    void acc_row(uint64_t* f, int arity, bool* isnull, const bool* isdec, i128* decv) {
        const int nb = ((arity + 63 + 8) / 64) * 8;
        bool anydec = false;
        for (int i = 0; i < arity; ++i) anydec |= isdec[i];
        const int64_t size = i32();
        if (!ok || size < nb + 8 * arity || (!anydec && size != nb + 8 * arity) || at + size > n) { ok = false; return; }
        const uint8_t* r = p + at;
        at += size;
        if (r[0] != 0) ok = false;                                    // RowKind INSERT
        for (int i = 0; i < arity; ++i) {
            isnull[i] = (r[(i + 8) / 8] >> ((i + 8) % 8)) & 1;
            uint64_t v = 0;
            for (int k = 0; k < 8; ++k) v |= (uint64_t)r[nb + 8 * i + k] << (8 * k);
            f[i] = isnull[i] ? 0 : v;
            if (!isdec[i] || isnull[i]) continue;
            const uint64_t off = v >> 32, len = v & 0xffffffffull;
            if (off < (uint64_t)(nb + 8 * arity) || off + len > (uint64_t)size || !dec_of_bytes(r + off, len, &decv[i])) ok = false;
        }
    }
    // a key row with STRING fields (the inverse of str_row_bytes): slots of the other fields, null bits, values;
    // *raw = the row's bytes (BinaryRowData equality is byte equality)
    void str_row(int arity, const int32_t* types, uint64_t* f, uint64_t* nulls, std::string* strs, std::string* raw) {
        const int nb = ((arity + 63 + 8) / 64) * 8;
        const int64_t size = i32();
        if (!ok || size < nb + 8 * arity || at + size > n) { ok = false; return; }
        const uint8_t* r = p + at;
        raw->assign((const char*)r, (size_t)size);
        at += size;
        if (r[0] != 0) { ok = false; return; }                      // RowKind INSERT
        *nulls = 0;
        for (int c = 0; c < arity; ++c) {
            const bool nl = (r[(c + 8) / 8] >> ((c + 8) % 8)) & 1;
            uint64_t v = 0;
            for (int k = 0; k < 8; ++k) v |= (uint64_t)r[nb + 8 * c + k] << (8 * k);
            f[c] = v;
            strs[c].clear();
            if (nl) { *nulls |= 1ull << c; continue; }
            if (types[c] != FWA_KEY_FIELD_STRING) continue;
            if (v >> 63) {
                const int len = (int)((v >> 56) & 0x7f);
                if (len > 7) { ok = false; return; }
                for (int k = 0; k < len; ++k) strs[c].push_back((char)(uint8_t)(v >> (8 * k)));
            } else {
                const uint64_t off = v >> 32, len = v & 0xffffffffull;
                if (off < (uint64_t)(nb + 8 * arity) || off + len > (uint64_t)size) { ok = false; return; }
                strs[c].assign((const char*)r + off, (size_t)len);
            }
        }
    }
};

// Layouts this file writes: DataStream TUMBLE and SESSION (WindowOperator), Table TUMBLE / HOP / CUMULATE
// (SlicingWindowOperator: per-slice state, so the engine's slices map 1:1), Table shift time zones and SQL NULLs.
bool supported(const fwa_config& c, bool dict = false) {
    if (c.key_kind == FWA_KEY_PREHASHED) return false;
    if (c.flags & FWA_CFG_REDUCE) return false;                        // a reduction keeps the reduced element
    for (int j = 0; j < c.num_aggs; ++j)                               // reduce kinds: the reduced element, no ACC
        if (c.aggs[j].kind >= FWA_SUM_I32) return false;
    if ((c.key_kind == FWA_KEY_GROUP_PREFIXED) != dict) return false;   // dictionary ids <=> a key dictionary
    if (dict && c.semantics != FWA_SEM_TABLE) return false;            // BinaryRowData keys: Table only
    if (c.semantics == FWA_SEM_DATASTREAM)
        return c.window_kind == FWA_TUMBLE || c.window_kind == FWA_SESSION || c.window_kind == FWA_SLIDE;
    return c.window_kind == FWA_TUMBLE || c.window_kind == FWA_SLIDE || c.window_kind == FWA_CUMULATE ||
           c.window_kind == FWA_SESSION;
}
const char* kUnsupported = "heap layout: DataStream TUMBLE / SLIDE / SESSION aggregates and Table TUMBLE / HOP / CUMULATE / "
                           "SESSION with a computable key hash";

int64_t gcd64(int64_t a, int64_t b) { while (b) { const int64_t t = a % b; a = b; b = t; } return a; }

// Table slice width (SliceAssigners: tumble = size, hop = gcd(size, slide), cumulate = step)
int64_t slice_width(const fwa_config& c) {
    if (c.window_kind == FWA_SLIDE) return gcd64(c.size_ms, c.slide_ms);
    if (c.window_kind == FWA_CUMULATE) return c.slide_ms;
    return c.size_ms;
}

int64_t floor_div(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) --q; return q; }

// End of the first window containing the slice that ends at se (SliceAssigner.nextTriggerWindow chain start):
// hop windows end at offset + k * slide, cumulative and tumbling windows at every slice end.
int64_t first_window_end(const fwa_config& c, int64_t se) {
    if (c.window_kind != FWA_SLIDE) return se;
    const int64_t k = -floor_div(-(se - c.offset_ms), c.slide_ms);   // ceil((se - off) / slide)
    return c.offset_ms + k * c.slide_ms;
}

// AggregateFunction.merge on one engine accumulator word (engine.hip acc_combine: counts and BIGINT sums add,
// floating sums add as double, MIN / MAX compare the order-preserving words)
uint64_t merge_word(int64_t kind, uint64_t x, uint64_t y) {
    switch (kind) {
        case FWA_SUM_F32: case FWA_SUM_F64: case FWA_AVG_F32: case FWA_AVG_F64: {
            double a, b;
            memcpy(&a, &x, 8); memcpy(&b, &y, 8);
            a += b;
            memcpy(&x, &a, 8);
            return x;
        }
        case FWA_MIN_I64: case FWA_MIN_F32: case FWA_MIN_F64: return y < x ? y : x;
        case FWA_MAX_I64: case FWA_MAX_F32: case FWA_MAX_F64: return y > x ? y : x;
        default: return x + y;
    }
}

// the accumulator word of an aggregate that saw no (non-NULL) input (engine.hip ident_of)
uint64_t identity_word(int64_t kind) { return (kind == FWA_MIN_I64 || kind == FWA_MIN_F32 || kind == FWA_MIN_F64) ? ~0ull : 0ull; }

// SQL NULLs: the engine keeps one hidden non-NULL counter per nullable input column an aggregate reads, in first-use
// order (engine.hip fwa_create); hid[j] = that counter's index for aggregate j, -1 for none. Returns their number.
int hidden_map(const fwa_config& c, int* hid) {
    int of_col[FWA_MAX_COLS], nh = 0;
    for (int k = 0; k < FWA_MAX_COLS; ++k) of_col[k] = -1;
    for (int j = 0; j < c.num_aggs; ++j) {
        hid[j] = -1;
        const int col = c.aggs[j].col;
        if (c.aggs[j].kind == FWA_COUNT || col < 0 || col >= FWA_MAX_COLS || !((c.nullable_cols >> col) & 1)) continue;
        if (of_col[col] < 0) of_col[col] = nh++;
        hid[j] = of_col[col];
    }
    return nh;
}

// The heap row of an accumulator against the engine's FWASNAP1 words. The heap row (the shim's ACC type) follows the
// caller's configuration: COUNT(*), one field per aggregate, one BIGINT per hidden non-NULL counter (hidden_map). A
// handle with DECIMAL aggregates runs an internal configuration (decimal.inc dec_plan) and its FWASNAP1 words follow
// that one: COUNT(*), the internal aggregates (the caller's others in order, the 32-bit piece sums, the counts) and the
// internal hidden counters; a DECIMAL field is the window total of its piece sums. Without DECIMAL both coincide.
enum { W_COUNT = 0, W_FIELD = 1, W_PIECE = 2, W_HIDDEN = 3 };
struct AccMap {
    fwa_config ic;                          // the configuration of the FWASNAP1 words
    int na = 0, nh = 0, ina = 0, inh = 0;   // caller / internal aggregates and hidden counters
    int hid[FWA_MAX_AGGS];                  // caller aggregate -> its hidden counter (-1: none)
    int uw[FWA_MAX_AGGS];                   // caller non-DECIMAL aggregate -> its word (-1: DECIMAL)
    int npc[FWA_MAX_AGGS];                  // caller DECIMAL aggregate: 2 / 4 piece sums (0: not DECIMAL) ...
    int pw[FWA_MAX_AGGS][4];                // ... and their words
    int hw[FWA_MAX_COLS];                   // caller hidden counter -> its word
    // restore: the source of each word (W_*), with the caller aggregate / hidden counter (sa) and piece (sk)
    int src[1 + FWA_MAX_AGGS + FWA_MAX_COLS], sa[1 + FWA_MAX_AGGS + FWA_MAX_COLS], sk[1 + FWA_MAX_AGGS + FWA_MAX_COLS];
    bool any_dec = false;
};
bool acc_map(const fwa_config& c, const FwaDecView& v, AccMap* m) {
    m->ic = v.active ? v.icfg : c;
    m->na = c.num_aggs;
    m->nh = hidden_map(c, m->hid);
    int ihid[FWA_MAX_AGGS];
    m->ina = m->ic.num_aggs;
    m->inh = hidden_map(m->ic, ihid);
    int ih_of_col[FWA_MAX_COLS], uh_of_col[FWA_MAX_COLS], col_of_ih[FWA_MAX_COLS], col_of_uh[FWA_MAX_COLS];
    for (int k = 0; k < FWA_MAX_COLS; ++k) ih_of_col[k] = uh_of_col[k] = col_of_ih[k] = col_of_uh[k] = -1;
    for (int i = 0; i < m->ina; ++i)
        if (ihid[i] >= 0) { ih_of_col[m->ic.aggs[i].col] = ihid[i]; col_of_ih[ihid[i]] = m->ic.aggs[i].col; }
    for (int j = 0; j < m->na; ++j)
        if (m->hid[j] >= 0) { uh_of_col[c.aggs[j].col] = m->hid[j]; col_of_uh[m->hid[j]] = c.aggs[j].col; }
    for (int h = 0; h < m->nh; ++h) {
        const int ih = ih_of_col[col_of_uh[h]];
        if (ih < 0) return false;
        m->hw[h] = 1 + m->ina + ih;
    }
    const int nw = 1 + m->ina + m->inh;
    for (int w = 0; w < nw; ++w) m->src[w] = m->sa[w] = m->sk[w] = -1;
    m->src[0] = W_COUNT;
    for (int j = 0; j < m->na; ++j) {
        m->npc[j] = (v.active && v.umap[j] < 0) ? v.npc[j] : 0;
        if (m->npc[j]) {
            m->any_dec = true;
            m->uw[j] = -1;
            for (int k = 0; k < m->npc[j]; ++k) m->pw[j][k] = 1 + v.pc[j][k];
        } else {
            m->uw[j] = 1 + (v.active ? v.umap[j] : j);
            m->src[m->uw[j]] = W_FIELD;
            m->sa[m->uw[j]] = j;
        }
    }
    for (int j = 0; j < m->na; ++j)                      // piece sums shared by a SUM and an AVG of one column: the same
        for (int k = 0; k < m->npc[j]; ++k) {            // total, any of them
            const int w = m->pw[j][k];
            if (m->src[w] < 0) { m->src[w] = W_PIECE; m->sa[w] = j; m->sk[w] = k; }
        }
    for (int i = 0; i < m->ina; ++i) {                   // the counts DECIMAL aggregates added
        const int w = 1 + i;
        if (m->src[w] >= 0) continue;
        if (m->ic.aggs[i].kind == FWA_COUNT) m->src[w] = W_COUNT;
        else if (m->ic.aggs[i].kind == FWA_COUNT_COL && uh_of_col[m->ic.aggs[i].col] >= 0) {
            m->src[w] = W_HIDDEN;
            m->sa[w] = uh_of_col[m->ic.aggs[i].col];
        } else {
            return false;
        }
    }
    for (int ih = 0; ih < m->inh; ++ih) {
        const int w = 1 + m->ina + ih, uh = uh_of_col[col_of_ih[ih]];
        if (uh < 0) return false;
        m->src[w] = W_HIDDEN;
        m->sa[w] = uh;
    }
    return true;
}

// Key rows of a key dictionary (fwa_keydict, multi-column Table keys): the slots and null bits of every row so far,
// read back from the device (keydict.hip fwa_keydict_host_rows); id bits 0-47 index them.
struct DictRows {
    int arity = 0;
    int32_t types[FWA_KEYDICT_MAX_ARITY] = {};
    std::vector<uint64_t> slots;     // [row][arity]
    std::vector<uint64_t> nulls;     // [row]
    std::vector<std::string> strs;   // [row][arity]: STRING values
    bool has_str = false;
};

// The bytes of a key row with STRING fields as BinaryRowWriter writes it (AbstractBinaryWriter.java:80-105,279-334):
// the header (null bits from bit 8), one 8-byte slot per field, a STRING of <= 7 bytes inline in its slot (first byte
// 0x80 | length, the bytes in the low 7, writeBytesToFixLenPart), a longer one appended to the variable-length part
// rounded up to 8 bytes with zero padding and slot = offset << 32 | length (writeBytesToVarLenPart, setOffsetAndSize).
std::vector<uint8_t> str_row_bytes(int arity, const int32_t* types, const uint64_t* slots, uint64_t nulls,
                                   const std::string* strs) {
    const int nb = ((arity + 63 + 8) / 64) * 8;
    std::vector<uint8_t> b((size_t)nb + 8 * (size_t)arity, 0);
    for (int i = 0; i < arity; ++i) if ((nulls >> i) & 1) b[(size_t)(i + 8) / 8] |= (uint8_t)(1u << ((i + 8) % 8));
    for (int c = 0; c < arity; ++c) {
        uint64_t v = 0;
        if ((nulls >> c) & 1) {
            v = 0;
        } else if (types[c] == FWA_KEY_FIELD_STRING) {
            const std::string& t = strs[c];
            if (t.size() <= 7) {
                v = (uint64_t)(0x80u | (uint32_t)t.size()) << 56;
                for (size_t k = 0; k < t.size(); ++k) v |= (uint64_t)(uint8_t)t[k] << (8 * k);
            } else {
                v = ((uint64_t)b.size() << 32) | (uint64_t)t.size();
                b.insert(b.end(), t.begin(), t.end());
                b.resize((b.size() + 7) & ~(size_t)7, 0);
            }
        } else {
            v = slots[c];
        }
        for (int k = 0; k < 8; ++k) b[(size_t)nb + 8 * c + k] = (uint8_t)(v >> (8 * k));
    }
    return b;
}

// Event-time timer of a window end under the shift time zone (TimeWindowUtil.toEpochMillsForTimer :67-100; UTC:
// the end - 1 itself)
int64_t timer_of(const fwa_config& c, int64_t max_ts) { return c.tz_n ? jm::tz_timer(c.tz, c.tz_n, max_ts) : max_ts; }

// State ids of the registered states, as a heap backend numbers them (HeapSnapshotResources.java:100-139: key/value
// states first, then the timer queues, each group in java.util.HashMap order of the state names -- pinned by the
// reference's own snapshots in tests/test_heap_reference_cpu.py):
//   DataStream TUMBLE  (WindowOperator):        0 window-contents, 1 processing timers, 2 event timers
//   DataStream SESSION (WindowOperator):        0 window-contents, 1 merging-window-set, 2 processing, 3 event timers
//   Table (SlicingWindowOperator, window-aggs): 0 window-aggs, 1 processing timers, 2 event timers
//   Table SESSION (TR WindowOperator :254-286):  0 session-window-mapping, 1 window-aggs, 2 processing, 3 event timers
//     (String.hashCode buckets of a 16-slot HashMap: "session-window-mapping" 6 < "window-aggs" 8)
struct Ids { int contents, mset, proc, event, n; };
Ids ids_of(const fwa_config& c) {
    if (c.window_kind == FWA_SESSION) return c.semantics == FWA_SEM_DATASTREAM ? Ids{0, 1, 2, 3, 4} : Ids{1, 0, 2, 3, 4};
    return Ids{0, -1, 1, 2, 3};
}

bool is_min(int64_t kind) { return kind == FWA_MIN_I64 || kind == FWA_MIN_F32 || kind == FWA_MIN_F64; }
bool is_max(int64_t kind) { return kind == FWA_MAX_I64 || kind == FWA_MAX_F32 || kind == FWA_MAX_F64; }
bool is_fsum(int64_t kind) { return kind == FWA_SUM_F32 || kind == FWA_SUM_F64 || kind == FWA_AVG_F32 || kind == FWA_AVG_F64; }

// WindowOperator.cleanupTime (:647-654): maxTimestamp + allowedLateness, Long.MAX_VALUE on overflow
int64_t cleanup_of(int64_t max_ts, int64_t late) { return max_ts > INT64_MAX - late ? INT64_MAX : max_ts + late; }

// TimeWindow.getWindowStartWithOffset (:264-272)
int64_t wstart(int64_t ts, int64_t off, int64_t size) {
    const int64_t r = (ts - off) % size;
    return r < 0 ? ts - (r + size) : ts - r;
}

// DataStream SLIDE restore: WindowOperator holds one accumulator per (key, window) and windows overlap, the engine one
// per (key, slice of width g = gcd(size, slide)). Slices whose window merges equal every restored window are built per
// key: a window k covers slices q_k .. q_k + m - 1 (m = size / g), the next window starts r = slide / g slices later.
//  * additive words (COUNT(*), integer / floating sums, hidden counters): windows from the highest restored one down
//    to the lowest uncleaned one that overlaps them, each setting its first slice to its value minus the slices above
//    it (already set; none above the highest window) -- every such window then sums to its value, an uncleaned window
//    without state to 0 (no record reached it, so none can be in its slices);
//  * MIN (MAX): each slice takes the largest (smallest) value of the uncleaned windows containing it, the identity for
//    one without state -- every window's MIN (MAX) is then reached at the slice where its true minimum lies.
// Future fires of the uncleaned windows (the only ones that can still fire) equal the reference's; floating sums are
// reassociated (within the DataStream tolerance).
using Words = std::vector<uint64_t>;
void slide_windows_to_slices(const fwa_config& c, int64_t wm, const std::map<int64_t, Words>& win, int nw,
                             std::vector<std::pair<int64_t, Words>>& out) {
    out.clear();
    if (win.empty()) return;
    const int64_t g = gcd64(c.size_ms, c.slide_ms), m = c.size_ms / g, r = c.slide_ms / g;
    const int na = c.num_aggs;
    const int64_t kmin = win.begin()->first, kmax = win.rbegin()->first;
    int64_t lo = kmin;                                          // lowest uncleaned window overlapping the restored ones
    while (lo - c.slide_ms > kmin - c.size_ms &&
           (wm == INT64_MIN || cleanup_of(lo - c.slide_ms + c.size_ms - 1, c.allowed_lateness_ms) > wm))
        lo -= c.slide_ms;
    auto qof = [&](int64_t t) { return floor_div(t - c.offset_ms, g); };
    const int64_t q0 = qof(lo), q1 = qof(kmax) + m - 1;
    const size_t ns = (size_t)(q1 - q0 + 1);
    std::vector<Words> x(ns, Words((size_t)nw, 0));
    auto kind_of = [&](int w) -> int64_t { return (w >= 1 && w <= na) ? c.aggs[w - 1].kind : FWA_COUNT; };
    for (int w = 0; w < nw; ++w) {
        const int64_t k = kind_of(w);
        if (is_min(k) || is_max(k)) {
            for (size_t i = 0; i < ns; ++i) {
                const int64_t q = q0 + (int64_t)i;
                uint64_t y = is_min(k) ? 0ull : ~0ull;
                // windows containing slice q: starts on the slide grid in (t - size, t], t = the slice start
                const int64_t t = c.offset_ms + q * g;
                for (int64_t st = wstart(t, c.offset_ms, c.slide_ms); st > t - c.size_ms; st -= c.slide_ms) {
                    if (st < lo) break;
                    auto it = win.find(st);
                    const uint64_t v = it == win.end() ? identity_word(k) : it->second[(size_t)w];
                    y = is_min(k) ? std::max(y, v) : std::min(y, v);
                }
                x[i][(size_t)w] = y;
            }
            continue;
        }
        const bool fl = is_fsum(k);
        for (int64_t st = kmax; st >= lo; st -= c.slide_ms) {
            const int64_t qa = qof(st) - q0;
            auto it = win.find(st);
            const uint64_t sv = it == win.end() ? 0ull : it->second[(size_t)w];
            if (fl) {
                double a, hsum = 0;
                memcpy(&a, &sv, 8);
                for (int64_t q = qa + r; q <= qa + m - 1; ++q) { double h; memcpy(&h, &x[(size_t)q][(size_t)w], 8); hsum += h; }
                a -= hsum;
                memcpy(&x[(size_t)qa][(size_t)w], &a, 8);
            } else {
                uint64_t hsum = 0;
                for (int64_t q = qa + r; q <= qa + m - 1; ++q) hsum += x[(size_t)q][(size_t)w];
                x[(size_t)qa][(size_t)w] = sv - hsum;
            }
        }
    }
    for (size_t i = 0; i < ns; ++i) {
        bool any = false;
        for (int w = 0; w < nw; ++w) any = any || x[i][(size_t)w] != (w >= 1 && w <= na ? identity_word(kind_of(w)) : 0ull);
        if (any) out.push_back({c.offset_ms + (q0 + (int64_t)i) * g, x[i]});
    }
}

}  // namespace

// keydict.hip (internal, C++): STRING values of the dictionary's rows, and an encode of host rows with STRING values
int fwa_keydict_host_strings(fwa_keydict* d, std::vector<std::string>* strs);
int fwa_keydict_encode_host_str(fwa_keydict* d, const uint64_t* slots, const uint64_t* nulls,
                                const std::vector<std::string>& strs, int64_t n, int64_t* ids);

extern "C" {

// engine-side accessors (engine.hip)
int fwa_get_config(const fwa_engine* e, fwa_config* out);
int fwa_set_error(fwa_engine* e, int code, const char* msg);
// keydict.hip (internal): the dictionary's rows on the host, and an encode of host rows
int fwa_keydict_host_rows(fwa_keydict* d, int32_t* arity, int32_t* types, std::vector<uint64_t>* slots,
                          std::vector<uint64_t>* nulls);
int fwa_keydict_encode_host(fwa_keydict* d, const uint64_t* slots, const uint64_t* nulls, int64_t n, int64_t* ids);

static int snapshot_heap_impl(fwa_engine* e, fwa_keydict* dict, fwa_blob* out, int64_t* kg_offsets, int64_t* watermark) {
    if (!e) return FWA_E_ARG;
    if (!out || !kg_offsets || !watermark) return fwa_set_error(e, FWA_E_ARG, "fwa_snapshot_heap: null output pointer");
    fwa_config c;
    int rc = fwa_get_config(e, &c);
    if (rc) return rc;
    if (!supported(c, dict != nullptr)) return fwa_set_error(e, FWA_E_UNSUPPORTED, kUnsupported);
    DictRows dr;
    if (dict && (rc = fwa_keydict_host_rows(dict, &dr.arity, dr.types, &dr.slots, &dr.nulls)))
        return fwa_set_error(e, rc, "key dictionary rows");
    for (int i = 0; i < dr.arity; ++i) dr.has_str |= dr.types[i] == FWA_KEY_FIELD_STRING;
    if (dr.has_str && (rc = fwa_keydict_host_strings(dict, &dr.strs))) return fwa_set_error(e, rc, "key dictionary strings");
    // the key as a BinaryRowData: one BIGINT field, or the dictionary row of an id
    auto key_row = [&](Out& o, int64_t key) -> bool {
        if (!dict) { const uint64_t kf = (uint64_t)key; o.row(&kf, 1); return true; }
        const uint64_t seq = (uint64_t)key & ((1ull << 48) - 1);
        if (seq >= dr.nulls.size()) return false;
        if (dr.has_str) {
            o.raw_row(str_row_bytes(dr.arity, dr.types, &dr.slots[seq * (size_t)dr.arity], dr.nulls[seq],
                                    &dr.strs[seq * (size_t)dr.arity]));
            return true;
        }
        bool nl[FWA_KEYDICT_MAX_ARITY];
        for (int i = 0; i < dr.arity; ++i) nl[i] = (dr.nulls[seq] >> i) & 1;
        o.row(&dr.slots[seq * (size_t)dr.arity], dr.arity, nl);
        return true;
    };
    bool keys_ok = true;
    fwa_blob snap{nullptr, 0};
    if ((rc = fwa_snapshot(e, &snap))) return rc;
    Snap s;
    if (!parse(snap.data, snap.size, &s)) { fwa_blob_free(&snap); return fwa_set_error(e, FWA_E_STATE, "bad FWASNAP1 blob"); }
    const bool ds = c.semantics == FWA_SEM_DATASTREAM;
    const bool sess = c.window_kind == FWA_SESSION;
    const bool ds_slide = ds && c.window_kind == FWA_SLIDE;
    const Ids id = ids_of(c);
    FwaDecView dv;
    AccMap am;
    if ((rc = fwa_dec_view(e, &dv)) || !acc_map(c, dv, &am) || am.ina != (int)s.naggs || am.inh != (int)s.nh) {
        fwa_blob_free(&snap);
        return fwa_set_error(e, FWA_E_STATE, "heap layout: accumulator words do not match the configuration");
    }
    const int na = am.na, nh = am.nh, ina = am.ina, inh = am.inh, arity = 1 + na + nh;
    const int* hid = am.hid;
    const int64_t n = s.n, g = ds ? (ds_slide ? gcd64(c.size_ms, c.slide_ms) : s.size) : slice_width(c);
    auto end_of = [&](int64_t i) { return sess ? s.col[(3 + ina + inh) * n + i] : s.col[n + i] + g; };
    const bool fired_any = s.wm != INT64_MIN;
    Out o;
    std::vector<uint64_t> f((size_t)arity);
    std::vector<uint8_t> fnull((size_t)arity);
    bool isdec[1 + FWA_MAX_AGGS + FWA_MAX_COLS] = {};
    std::vector<uint8_t> decb[1 + FWA_MAX_AGGS + FWA_MAX_COLS];
    struct Row { int64_t key, start, end; uint64_t w[1 + FWA_MAX_AGGS + FWA_MAX_COLS]; };
    std::vector<Row> rows;
    auto merge_into = [&](Row& a, const Row& b) {                  // on the FWASNAP1 words
        a.w[0] += b.w[0];
        for (int j = 0; j < ina; ++j) a.w[1 + j] = merge_word(s.agg[j], a.w[1 + j], b.w[1 + j]);
        for (int h = 0; h < inh; ++h) a.w[1 + ina + h] += b.w[1 + ina + h];
    };
    for (int64_t kg = c.kg_start; kg <= c.kg_end; ++kg) {
        kg_offsets[kg - c.kg_start] = (int64_t)o.b.size();
        o.i32(kg);
        const int64_t lo = s.koff[kg], hi = s.koff[kg + 1];
        // the state entries: the engine keeps every slice until its last window fires; a CUMULATE window's fired
        // slices are folded into its first slice in ascending order, the shared state SliceSharedWindowAggProcessor
        // merges them into (CumulativeSliceAssigner.mergeSlices / expiredSlices, SliceAssigners.java:335-371)
        rows.clear();
        for (int64_t i = lo; i < hi; ++i) {
            Row r{s.col[i], s.col[n + i], end_of(i), {}};
            r.w[0] = (uint64_t)s.col[2 * n + i];
            for (int j = 0; j < ina + inh; ++j) r.w[1 + j] = (uint64_t)s.col[(3 + j) * n + i];
            rows.push_back(r);
        }
        if (ds_slide) {
            // WindowOperator keeps one state per (key, window) (SlidingEventTimeWindows.assignWindows :70-82): a window's
            // contents are the merge of the engine's slices inside it; windows past cleanup (isWindowLate) are gone and a
            // window holds state iff a record reached it
            std::map<std::pair<int64_t, int64_t>, Row> win;
            for (const Row& r : rows)
                for (int64_t st = wstart(r.start, c.offset_ms, c.slide_ms); st > r.start - c.size_ms; st -= c.slide_ms) {
                    if (fired_any && cleanup_of(st + c.size_ms - 1, s.late) <= s.wm) continue;
                    auto it = win.find({r.key, st});
                    if (it == win.end()) {
                        Row w = r;
                        w.start = st;
                        w.end = st + c.size_ms;
                        win.emplace(std::make_pair(r.key, st), w);
                    } else {
                        merge_into(it->second, r);
                    }
                }
            rows.clear();
            for (auto& kv : win) if ((int64_t)kv.second.w[0] > 0) rows.push_back(kv.second);
        }
        if (!ds && c.window_kind == FWA_CUMULATE && fired_any) {
            std::map<std::pair<int64_t, int64_t>, Row> first;          // (key, window start) -> folded first slice
            std::vector<Row> keep;
            std::sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) {
                return a.key != b.key ? a.key < b.key : a.start < b.start; });
            for (const Row& r : rows) {
                if (timer_of(c, r.end - 1) > s.wm) { keep.push_back(r); continue; }
                const int64_t ws = c.offset_ms + floor_div(r.end - 1 - c.offset_ms, c.size_ms) * c.size_ms;
                auto it = first.find({r.key, ws});
                if (it == first.end()) {
                    Row m = r;
                    m.start = ws;
                    m.end = ws + g;
                    first.emplace(std::make_pair(r.key, ws), m);
                } else {
                    merge_into(it->second, r);
                }
            }
            rows.clear();
            for (auto& kv : first) rows.push_back(kv.second);
            rows.insert(rows.end(), keep.begin(), keep.end());
        }
        auto contents = [&]() {                                        // window contents / window-aggs
            o.i16(id.contents);
            o.i32((int64_t)rows.size());
            for (const Row& r : rows) {
                const int64_t key = r.key, start = r.start, end = r.end;
                f[0] = r.w[0];
                fnull[0] = 0;
                for (int j = 0; j < na; ++j) {
                    const int64_t kind = c.aggs[j].kind;
                    // SQL: an aggregate whose input column held only NULLs has a NULL buffer (Sum/Min/MaxAggFunction,
                    // DecimalSum/AvgAggFunction); COUNT(col) is the counter itself
                    fnull[1 + j] = hid[j] >= 0 && kind != FWA_COUNT_COL && r.w[am.hw[hid[j]]] == 0;
                    isdec[1 + j] = am.npc[j] != 0;
                    if (!am.npc[j]) { f[1 + j] = acc_to_field(kind, r.w[am.uw[j]]); continue; }
                    // DECIMAL: the running sum DECIMAL(38, s); NULL past 38 digits (the engine decides on the exact
                    // total, include/flink_amd.h)
                    uint64_t S[4];
                    i128 T = 0;
                    for (int k = 0; k < am.npc[j]; ++k) S[k] = r.w[am.pw[j][k]];
                    if (!dec_total(S, am.npc[j], &T)) fnull[1 + j] = 1;
                    f[1 + j] = 0;
                    decb[1 + j] = dec_bytes(T);
                }
                for (int h = 0; h < nh; ++h) { f[1 + na + h] = r.w[am.hw[h]]; fnull[1 + na + h] = 0; }
                if (ds) {
                    o.i64((uint64_t)start); o.i64((uint64_t)end);          // TimeWindow.Serializer
                    o.i64((uint64_t)key);                                  // LongSerializer
                    for (int k = 0; k < arity; ++k) o.i64(f[k]);           // TupleSerializer of the ACC fields
                } else {
                    if (sess) { o.i64((uint64_t)start); o.i64((uint64_t)end); }   // TR TimeWindow.Serializer :169-172
                    else o.i64((uint64_t)end);                              // slice end (LongSerializer)
                    keys_ok = key_row(o, key) && keys_ok;                  // key row
                    bool nl[1 + FWA_MAX_AGGS + FWA_MAX_COLS];
                    for (int k = 0; k < arity; ++k) nl[k] = fnull[k] != 0;
                    o.acc_row(f.data(), arity, nl, isdec, decb);           // accumulator row
                }
            }
        };
        auto mset = [&]() {                                            // merging-window-set / session-window-mapping:
            std::map<int64_t, std::vector<int64_t>> by_key;            // each in-flight session maps to itself as its
            for (int64_t i = lo; i < hi; ++i) by_key[s.col[i]].push_back(i);   // state window
            o.i16(id.mset);
            o.i32((int64_t)by_key.size());
            for (auto& kv : by_key) {
                o.u8(0);                                               // VoidNamespaceSerializer: one byte
                if (ds) o.i64((uint64_t)kv.first);
                else keys_ok = key_row(o, kv.first) && keys_ok;
                o.i32((int64_t)kv.second.size());                      // ListSerializer / MapSerializer: size, then
                for (int64_t i : kv.second) {                          // (actual, state) TimeWindow pairs
                    const int64_t st = s.col[n + i], en = end_of(i);
                    o.i64((uint64_t)st); o.i64((uint64_t)en);
                    if (!ds) o.u8(0);                                  // MapSerializer: value not null
                    o.i64((uint64_t)st); o.i64((uint64_t)en);
                }
            }
        };
        if (sess && id.mset < id.contents) { mset(); contents(); }     // sections in state-id order
        else { contents(); if (sess) mset(); }
        o.i16(id.proc);                                                // processing-time timers: none on this path
        o.i32(0);
        // event-time timers. DataStream (per (key, window) of the state written above): window.maxTimestamp() while
        // the window has not fired (EventTimeTrigger.onElement / onEventTime: a fired window keeps no trigger timer, a
        // late element within allowed lateness FIREs at once) and always the cleanup timer maxTimestamp +
        // allowedLateness (WindowOperator.registerCleanupTimer :608-620, cleanupTime :647-654; the same timer when the
        // lateness is 0). Table sessions: toEpochMillsForTimer(maxTimestamp) per in-flight session (the trigger and the
        // cleanup timer coincide, TR WindowOperator :421-446). Table slices: toEpochMillsForTimer(end - 1) of the first
        // unfired window containing each slice, one per (key, window) (AbstractWindowAggProcessor.processElement
        // :160-164, SliceSharedWindowAggProcessor.fireWindow :76-84).
        std::set<std::tuple<int64_t, int64_t, int64_t, int64_t>> timers;   // (ts, key, ns start, ns end)
        if (ds) {
            for (const Row& r : rows) {
                if (!fired_any || r.end - 1 > s.wm) timers.insert({r.end - 1, r.key, r.start, r.end});
                timers.insert({cleanup_of(r.end - 1, s.late), r.key, r.start, r.end});
            }
        } else if (sess) {
            for (const Row& r : rows) timers.insert({timer_of(c, r.end - 1), r.key, r.start, r.end});
        } else {
            for (int64_t i = lo; i < hi; ++i) {
                const int64_t key = s.col[i], end = end_of(i);
                int64_t we = first_window_end(c, end);
                while (fired_any && timer_of(c, we - 1) <= s.wm) we += (c.window_kind == FWA_SLIDE ? c.slide_ms : g);
                timers.insert({timer_of(c, we - 1), key, 0, we});
            }
        }
        o.i16(id.event);
        o.i32((int64_t)timers.size());
        for (const auto& t : timers) {
            o.i64((uint64_t)std::get<0>(t) ^ 0x8000000000000000ull);   // MathUtils.flipSignBit
            const int64_t key = std::get<1>(t);
            if (ds) { o.i64((uint64_t)key); o.i64((uint64_t)std::get<2>(t)); o.i64((uint64_t)std::get<3>(t)); }
            else {
                keys_ok = key_row(o, key) && keys_ok;
                if (sess) o.i64((uint64_t)std::get<2>(t));             // TimeWindow namespace
                o.i64((uint64_t)std::get<3>(t));
            }
        }
    }
    *watermark = s.wm;
    fwa_blob_free(&snap);
    if (!keys_ok) return fwa_set_error(e, FWA_E_ARG, "a key id is not in the key dictionary");
    out->size = (int64_t)o.b.size();
    out->data = malloc(o.b.size() ? o.b.size() : 1);
    if (!out->data) return fwa_set_error(e, FWA_E_OOM, "heap snapshot allocation failed");
    if (!o.b.empty()) memcpy(out->data, o.b.data(), o.b.size());
    return FWA_OK;
}

static int restore_heap_impl(fwa_engine* e, fwa_keydict* dict, const void* const* bodies, const int64_t* sizes,
                             const int64_t* watermarks, int32_t n_bodies) {
    if (!e || n_bodies <= 0 || !bodies || !sizes || !watermarks) return FWA_E_ARG;
    fwa_config c;
    int rc = fwa_get_config(e, &c);
    if (rc) return rc;
    if (!supported(c, dict != nullptr)) return fwa_set_error(e, FWA_E_UNSUPPORTED, kUnsupported);
    int32_t darity = 1;
    int32_t dtypes[FWA_KEYDICT_MAX_ARITY] = {};
    bool dstr = false;
    if (dict) {
        std::vector<uint64_t> tmp_s, tmp_n;
        if ((rc = fwa_keydict_host_rows(dict, &darity, dtypes, &tmp_s, &tmp_n))) return fwa_set_error(e, rc, "key dictionary");
        for (int i = 0; i < darity; ++i) dstr |= dtypes[i] == FWA_KEY_FIELD_STRING;
    }
    const bool ds = c.semantics == FWA_SEM_DATASTREAM;
    const bool sess = c.window_kind == FWA_SESSION;
    const bool ds_slide = ds && c.window_kind == FWA_SLIDE;
    const Ids id = ids_of(c);
    FwaDecView dv;
    AccMap am;
    if ((rc = fwa_dec_view(e, &dv)) || !acc_map(c, dv, &am))
        return fwa_set_error(e, FWA_E_STATE, "heap layout: accumulator words do not match the configuration");
    const int na = am.na, nh = am.nh, ina = am.ina, inh = am.inh, arity = 1 + na + nh, maxp = c.max_parallelism;
    const fwa_config& ic = am.ic;
    bool isdec[1 + FWA_MAX_AGGS + FWA_MAX_COLS] = {};
    for (int j = 0; j < na; ++j) isdec[1 + j] = am.npc[j] != 0;
    const int64_t g = ds ? c.size_ms : slice_width(c);
    const int64_t ncols = (sess ? 4 : 3) + ina + inh;
    bool dec_range = true;
    std::vector<std::vector<int64_t>> blobs((size_t)n_bodies);
    std::vector<const void*> ptrs;
    std::vector<int64_t> bsz;
    for (int b = 0; b < n_bodies; ++b) {
        std::vector<std::vector<int64_t>> per((size_t)maxp);   // flattened (key, start, count, acc_j..., hid_h... [, end]) rows
        In in{(const uint8_t*)bodies[b], sizes[b]};
        int64_t lo = maxp, hi = -1, total = 0;
        std::vector<uint64_t> f((size_t)arity);
        bool fnull[1 + FWA_MAX_AGGS + FWA_MAX_COLS];
        i128 decv[1 + FWA_MAX_AGGS + FWA_MAX_COLS] = {};
        struct Pending { int64_t kg, key, start, end; std::vector<int64_t> w; };
        std::vector<Pending> pend;
        std::map<std::tuple<int64_t, int64_t, int64_t>, std::pair<int64_t, int64_t>> actual;
        // the engine's words of one accumulator tuple / row (AccMap): COUNT(*), each aggregate (NULL: its identity),
        // the piece sums of a DECIMAL total (NULL: 0 -- the reference's next value restarts a NULL sum,
        // DecimalSumAggFunction), the counts, the hidden counters
        auto words = [&](std::vector<int64_t>& v) {
            uint64_t S[FWA_MAX_AGGS][4] = {};
            for (int j = 0; j < na; ++j)
                if (am.npc[j] && !fnull[1 + j] && !dec_split(decv[1 + j], am.npc[j], S[j])) dec_range = false;
            for (int w = 0; w < 1 + ina + inh; ++w) {
                const int j = am.sa[w];
                switch (am.src[w]) {
                    case W_COUNT: v.push_back((int64_t)f[0]); break;
                    case W_FIELD:
                        v.push_back((int64_t)(fnull[1 + j] ? identity_word(c.aggs[j].kind) : field_to_acc(c.aggs[j].kind, f[1 + j])));
                        break;
                    case W_PIECE: v.push_back((int64_t)S[j][am.sk[w]]); break;
                    default: v.push_back((int64_t)f[1 + na + j]); break;
                }
            }
        };
        std::map<int64_t, std::map<int64_t, Words>> slide_win;    // DataStream SLIDE: key -> window start -> words
        std::vector<std::pair<int64_t, Words>> slices;
        // dictionary keys: each distinct key row read gets a placeholder key (its index), encoded to ids at the end
        std::map<std::vector<uint64_t>, int64_t> comp_idx;
        std::map<std::string, int64_t> comp_raw;                     // rows with STRING fields: by their bytes
        std::vector<uint64_t> comp_slots, comp_nulls;
        std::vector<std::string> comp_strs;
        auto read_key = [&](In& in) -> int64_t {
            if (!dict) { uint64_t kf; in.row(&kf, 1); return (int64_t)kf; }
            if (dstr) {
                uint64_t f[FWA_KEYDICT_MAX_ARITY], nb = 0;
                std::string sv[FWA_KEYDICT_MAX_ARITY], raw;
                in.str_row(darity, dtypes, f, &nb, sv, &raw);
                if (!in.ok) return 0;
                auto it = comp_raw.find(raw);
                if (it != comp_raw.end()) return it->second;
                const int64_t idx = (int64_t)comp_nulls.size();
                comp_raw.emplace(raw, idx);
                comp_slots.insert(comp_slots.end(), f, f + darity);
                comp_nulls.push_back(nb);
                for (int i = 0; i < darity; ++i) comp_strs.push_back(sv[i]);
                return idx;
            }
            uint64_t f[FWA_KEYDICT_MAX_ARITY];
            bool nl[FWA_KEYDICT_MAX_ARITY];
            in.row(f, darity, nl);
            std::vector<uint64_t> k(f, f + darity);
            uint64_t nb = 0;
            for (int i = 0; i < darity; ++i) nb |= (uint64_t)nl[i] << i;
            k.push_back(nb);
            auto it = comp_idx.find(k);
            if (it != comp_idx.end()) return it->second;
            const int64_t idx = (int64_t)comp_nulls.size();
            comp_idx.emplace(k, idx);
            comp_slots.insert(comp_slots.end(), f, f + darity);
            comp_nulls.push_back(nb);
            return idx;
        };
        while (in.ok && in.at < in.n) {
            const int64_t kg = in.i32();
            if (!in.ok || kg < 0 || kg >= maxp) return fwa_set_error(e, FWA_E_ARG, "heap body: bad key group id");
            lo = std::min(lo, kg); hi = std::max(hi, kg);
            for (int st = 0; st < id.n; ++st) {
                const int64_t sid = (int16_t)in.get(2), cnt = in.i32();
                if (!in.ok || sid < 0 || sid >= id.n || cnt < 0) return fwa_set_error(e, FWA_E_ARG, "heap body: bad state section");
                for (int64_t i = 0; i < cnt && in.ok; ++i) {
                    if (sid == id.proc || sid == id.event) {           // timers: re-derived from the window state
                        in.i64();
                        if (ds) { in.i64(); in.i64(); in.i64(); }
                        else { read_key(in); in.i64(); if (sess) in.i64(); }
                        continue;
                    }
                    if (sid == id.mset) {                              // merging-window-set: (actual, state) pairs
                        in.get(1);                                     // MergingWindowSet(...) :83-87
                        int64_t key;
                        if (ds) key = in.i64();
                        else key = read_key(in);
                        const int64_t m = in.i32();
                        for (int64_t q = 0; q < m && in.ok; ++q) {
                            const int64_t as = in.i64(), ae = in.i64();
                            if (!ds && in.get(1) != 0) in.ok = false;      // MapSerializer: null value flag
                            const int64_t ss = in.i64(), se = in.i64();
                            actual[std::make_tuple(key, ss, se)] = std::make_pair(as, ae);
                        }
                        continue;
                    }
                    int64_t key, start, end;
                    for (int k = 0; k < arity; ++k) fnull[k] = false;
                    if (ds) { start = in.i64(); end = in.i64(); key = in.i64(); for (int k = 0; k < arity; ++k) f[k] = (uint64_t)in.i64(); }
                    else {
                        start = sess ? in.i64() : 0;                   // Table sessions: TimeWindow namespace
                        end = in.i64();
                        key = read_key(in);
                        in.acc_row(f.data(), arity, fnull, isdec, decv);
                        if (fnull[0]) in.ok = false;                   // COUNT(*) is never NULL
                        if (!sess) start = end - g;
                    }
                    if (ds_slide) {                                    // per-window state: slices built below
                        std::vector<int64_t> v;
                        words(v);
                        slide_win[key][start] = Words(v.begin(), v.end());
                        continue;
                    }
                    if (sess) {                                        // resolved against the mapping below
                        Pending p{kg, key, start, end, {}};
                        words(p.w);
                        pend.push_back(std::move(p));
                        continue;
                    }
                    std::vector<int64_t>& v = per[(size_t)kg];
                    v.push_back(key);
                    v.push_back(start);
                    words(v);
                    ++total;
                }
            }
            // a session's window contents live under its state window; the session itself is the actual window
            // that maps to it (Flink names an older window as the state namespace after merges)
            for (const Pending& p : pend) {
                auto it = actual.find(std::make_tuple(p.key, p.start, p.end));
                const int64_t st = it == actual.end() ? p.start : it->second.first;
                const int64_t en = it == actual.end() ? p.end : it->second.second;
                std::vector<int64_t>& v = per[(size_t)p.kg];
                v.push_back(p.key);
                v.push_back(st);
                v.insert(v.end(), p.w.begin(), p.w.end());
                v.push_back(en);
                ++total;
            }
            pend.clear();
            actual.clear();
            for (auto& kw : slide_win) {
                slide_windows_to_slices(c, watermarks[b], kw.second, 1 + na + nh, slices);
                std::vector<int64_t>& v = per[(size_t)kg];
                for (auto& sl : slices) {
                    v.push_back(kw.first);
                    v.push_back(sl.first);
                    for (uint64_t x : sl.second) v.push_back((int64_t)x);
                    ++total;
                }
            }
            slide_win.clear();
        }
        if (!in.ok) return fwa_set_error(e, FWA_E_ARG, "heap body: truncated or malformed");
        if (!dec_range)
            return fwa_set_error(e, FWA_E_UNSUPPORTED, "heap body: a DECIMAL sum of a DECIMAL(p <= 18) column past 2^95");
        if (dict && !comp_nulls.empty()) {                            // placeholder keys -> dictionary ids
            std::vector<int64_t> ids(comp_nulls.size());
            rc = dstr ? fwa_keydict_encode_host_str(dict, comp_slots.data(), comp_nulls.data(), comp_strs, (int64_t)ids.size(),
                                                    ids.data())
                      : fwa_keydict_encode_host(dict, comp_slots.data(), comp_nulls.data(), (int64_t)ids.size(), ids.data());
            if (rc) return fwa_set_error(e, rc, "key dictionary encode");
            for (int kg = 0; kg < maxp; ++kg) {
                std::vector<int64_t>& v = per[(size_t)kg];
                for (size_t r = 0; r < v.size(); r += (size_t)ncols) {
                    const int64_t id = ids[(size_t)v[r]];
                    if ((int64_t)((uint64_t)id >> 48) != kg)
                        return fwa_set_error(e, FWA_E_ARG, "heap body: a key row outside its key group (maxParallelism?)");
                    v[r] = id;
                }
            }
        }
        // the equivalent FWASNAP1 blob (engine.hip snap_header layout)
        std::vector<int64_t>& w = blobs[(size_t)b];
        w.assign((size_t)(kHdr + maxp + 1 + total * ncols), 0);
        w[0] = (int64_t)kMagic; w[1] = 1; w[2] = c.window_kind; w[3] = c.semantics; w[4] = c.size_ms;
        w[5] = c.slide_ms; w[6] = c.offset_ms; w[7] = c.gap_ms; w[8] = c.allowed_lateness_ms; w[9] = maxp;
        w[10] = c.key_kind; w[11] = ina;                              // the internal configuration's words (AccMap)
        for (int j = 0; j < ina; ++j) w[12 + j] = ic.aggs[j].kind;
        w[20] = watermarks[b]; w[21] = total; w[22] = hi >= 0 ? lo : 0; w[23] = hi >= 0 ? hi : maxp - 1;
        w[24] = ic.nullable_cols; w[25] = inh;
        for (int j = 0; j < ina; ++j) w[26] |= (int64_t)(ic.aggs[j].col & 15) << (4 * j);
        int64_t* koff = w.data() + kHdr;
        int64_t* body = koff + maxp + 1;
        int64_t d = 0;
        for (int kg = 0; kg < maxp; ++kg) {
            koff[kg] = d;
            const std::vector<int64_t>& v = per[(size_t)kg];
            for (size_t r = 0; r < v.size(); r += (size_t)ncols, ++d)
                for (int64_t k = 0; k < ncols; ++k) body[k * total + d] = v[r + (size_t)k];
        }
        koff[maxp] = d;
        ptrs.push_back(w.data());
        bsz.push_back((int64_t)w.size() * 8);
    }
    return fwa_restore(e, ptrs.data(), bsz.data(), n_bodies);
}

int fwa_snapshot_heap(fwa_engine* e, fwa_blob* out, int64_t* kg_offsets, int64_t* watermark) {
    return snapshot_heap_impl(e, nullptr, out, kg_offsets, watermark);
}

int fwa_restore_heap(fwa_engine* e, const void* const* bodies, const int64_t* sizes, const int64_t* watermarks,
                     int32_t n_bodies) {
    return restore_heap_impl(e, nullptr, bodies, sizes, watermarks, n_bodies);
}

int fwa_snapshot_heap_keys(fwa_engine* e, fwa_keydict* dict, fwa_blob* out, int64_t* kg_offsets, int64_t* watermark) {
    if (!dict) return e ? fwa_set_error(e, FWA_E_ARG, "fwa_snapshot_heap_keys: null key dictionary") : FWA_E_ARG;
    return snapshot_heap_impl(e, dict, out, kg_offsets, watermark);
}

int fwa_restore_heap_keys(fwa_engine* e, fwa_keydict* dict, const void* const* bodies, const int64_t* sizes,
                          const int64_t* watermarks, int32_t n_bodies) {
    if (!dict) return e ? fwa_set_error(e, FWA_E_ARG, "fwa_restore_heap_keys: null key dictionary") : FWA_E_ARG;
    return restore_heap_impl(e, dict, bodies, sizes, watermarks, n_bodies);
}

}  // extern "C"
