/*
 * fwa_oracle.c -- TEST INFRASTRUCTURE ONLY (see fwa_oracle.h). A plain-C restatement of the
 * reference's keyed event-time window aggregation, written from the reference sources:
 *
 *   Java arithmetic   MathUtils.java:137-155,194-201 (murmurHash/bitMix), KeyGroupRangeAssignment.java:63-127,
 *                     MurmurHashUtils.java:92-170 + BinaryRowData.java:68-123,452-454 (Table key hash),
 *                     TimeWindow.java:264-272 (getWindowStartWithOffset)
 *   DataStream        WindowOperator.java:278-481,537-654 (processElement/onEventTime/cleanup),
 *                     EventTimeTrigger.java:37-84, MergingWindowSet.java:99-236, TimeWindow.java:116-124,208-254,
 *                     InternalTimerServiceImpl.java:238-314 (dedup timers, advanceWatermark)
 *   Table (slicing)   AbstractWindowAggProcessor.java:142-213, SliceAssigners.java:134-385,
 *                     SliceSharedWindowAggProcessor.java:64-171, SliceUnsharedWindowAggProcessor.java:46-55,
 *                     AggCombiner.java:76-111, TimeWindowUtil.java:175-183, SlicingWindowOperator.java:230-264
 *   Aggregates        SumAggFunction/AvgAggFunction/MaxAggFunction/MinAggFunction/Count1AggFunction (a16),
 *                     SumAggregator/SumFunction (a15)
 *
 * It is deliberately structured like the reference (per-window heap state, a deduplicating timer heap,
 * per-key merging window sets) and NOT like the GPU engine (slices + dense tables), so the two are
 * independent implementations of the same observable semantics.
 */
#include "fwa_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define J_LONG_MIN ((int64_t)0x8000000000000000LL)
#define J_LONG_MAX ((int64_t)0x7fffffffffffffffLL)

/* Java two's-complement wrap-around helpers */
static inline int32_t jimul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t jiadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t jrotl(int32_t x, int r) { uint32_t u = (uint32_t)x; return (int32_t)((u << r) | (u >> (32 - r))); }
static inline int32_t jushr(int32_t x, int r) { return (int32_t)((uint32_t)x >> r); }
static inline int64_t jladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t jlsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t jlmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
/* Java long '%': truncating, sign of dividend; LONG_MIN % -1 == 0 */
static inline int64_t jlrem(int64_t a, int64_t b) { if (b == -1) return 0; return a % b; }

/* ------------------------------------------------------------------ Java arithmetic */

int32_t or_bit_mix(int32_t in) {            /* MathUtils.bitMix :194-201 */
    in ^= jushr(in, 16);
    in = jimul(in, (int32_t)0x85ebca6b);
    in ^= jushr(in, 13);
    in = jimul(in, (int32_t)0xc2b2ae35);
    in ^= jushr(in, 16);
    return in;
}

int32_t or_murmur_hash(int32_t code) {      /* MathUtils.murmurHash :137-155 */
    code = jimul(code, (int32_t)0xcc9e2d51);
    code = jrotl(code, 15);
    code = jimul(code, 0x1b873593);
    code = jrotl(code, 13);
    code = jiadd(jimul(code, 5), (int32_t)0xe6546b64);
    code ^= 4;
    code = or_bit_mix(code);
    if (code >= 0) return code;
    if (code != (int32_t)0x80000000) return -code;
    return 0;
}

int32_t or_long_hash(int64_t v) { return (int32_t)(v ^ (int64_t)((uint64_t)v >> 32)); }

/* MurmurHashUtils.mixK1 :143-148 / mixH1 :150-155 / fmix :158-170 */
static int32_t mh_mix_k1(int32_t k1) { k1 = jimul(k1, (int32_t)0xcc9e2d51); k1 = jrotl(k1, 15); return jimul(k1, 0x1b873593); }
static int32_t mh_mix_h1(int32_t h1, int32_t k1) { h1 ^= k1; h1 = jrotl(h1, 13); return jiadd(jimul(h1, 5), (int32_t)0xe6546b64); }
static int32_t mh_fmix(int32_t h) {
    h ^= jushr(h, 16); h = jimul(h, (int32_t)0x85ebca6b);
    h ^= jushr(h, 13); h = jimul(h, (int32_t)0xc2b2ae35);
    h ^= jushr(h, 16); return h;
}

/* BinaryRowData of arity 1 holding a BIGINT: 8-byte header (RowKind byte 0 = INSERT, null bits
 * zeroed by BinaryRowWriter.reset :50-55) + 8-byte little-endian long. hashByWords reads 4-byte
 * native-order (LE) ints: [0, 0, lo32, hi32]; seed DEFAULT_SEED = 42; fmix(h ^ 16). */
int32_t or_binrow_bigint_hash(int64_t v) {
    int32_t words[4] = {0, 0, (int32_t)(uint32_t)((uint64_t)v & 0xffffffffu), (int32_t)(uint32_t)((uint64_t)v >> 32)};
    int32_t h1 = 42;
    for (int i = 0; i < 4; i++) h1 = mh_mix_h1(h1, mh_mix_k1(words[i]));
    return mh_fmix(h1 ^ 16);
}

/* BinaryRowData.hashCode of a row of `arity` fixed-length fields (BinaryRowData.java:68-123, 452-454;
   MurmurHashUtils.hashBytesByWords :92-170): bytes = 8-byte header (RowKind INSERT 0, null bit of field i at bit
   8 + i, BinaryRowData.setNullAt) + one little-endian 8-byte slot per field (BIGINT / DOUBLE bits; INT in the low 4
   bytes; a NULL field's slot zeroed, BinaryRowWriter.setNullAt); the row's 4-byte words mixed in order from seed 42,
   then fmix(h ^ length). slots[i] = field i's 8 slot bytes as a little-endian integer. */
int32_t or_binrow_hash(const int64_t* slots, int32_t arity, uint64_t nullbits) {
    int32_t h1 = 42;
    const uint64_t hdr = nullbits << 8;
    h1 = mh_mix_h1(h1, mh_mix_k1((int32_t)(uint32_t)(hdr & 0xffffffffu)));
    h1 = mh_mix_h1(h1, mh_mix_k1((int32_t)(uint32_t)(hdr >> 32)));
    for (int32_t i = 0; i < arity; i++) {
        const uint64_t v = ((nullbits >> i) & 1) ? 0 : (uint64_t)slots[i];
        h1 = mh_mix_h1(h1, mh_mix_k1((int32_t)(uint32_t)(v & 0xffffffffu)));
        h1 = mh_mix_h1(h1, mh_mix_k1((int32_t)(uint32_t)(v >> 32)));
    }
    return mh_fmix(h1 ^ (8 + 8 * arity));
}

/* MurmurHashUtils.hashBytesByWords (MurmurHashUtils.java:92-170) over any byte row (numBytes a multiple of 4):
   BinaryRowData.hashCode of a row with variable-length parts (BinarySegmentUtils.hashByWords :374-380) */
int32_t or_hash_bytes_by_words(const uint8_t* p, int32_t n) {
    int32_t h1 = 42;
    for (int32_t i = 0; i + 4 <= n; i += 4) {
        const int32_t w = (int32_t)((uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24));
        h1 = mh_mix_h1(h1, mh_mix_k1(w));
    }
    return mh_fmix(h1 ^ n);
}

int32_t or_key_group(int64_t key, int32_t key_kind, int32_t key_hash, int32_t max_par) {
    int32_t h;
    if (key_kind == 3) return (int32_t)((uint64_t)key >> 48);   /* key-dictionary ids carry their key group */
    if (key_kind == FWA_KEY_JAVA_LONG) h = or_long_hash(key);
    else if (key_kind == FWA_KEY_BINROW_BIGINT) h = or_binrow_bigint_hash(key);
    else h = key_hash;
    return or_murmur_hash(h) % max_par;     /* computeKeyGroupForKeyHash :75-77 */
}

int32_t or_operator_index(int32_t max_par, int32_t par, int32_t kg) { return kg * par / max_par; } /* :124-127 */

void or_key_group_range(int32_t max_par, int32_t par, int32_t idx, int32_t* start, int32_t* end) { /* :93-106 */
    *start = (idx * max_par + par - 1) / par;
    *end = ((idx + 1) * max_par - 1) / par;
}

int64_t or_window_start(int64_t ts, int64_t offset, int64_t size) {   /* TimeWindow.java:264-272 */
    int64_t rem = jlrem(jlsub(ts, offset), size);
    if (rem < 0) return jlsub(ts, jladd(rem, size));
    return jlsub(ts, rem);
}

int32_t or_long_to_int_with_bit_mixing(int64_t in) {
    uint64_t x = (uint64_t)in;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    x = x ^ (x >> 31);
    return (int32_t)x;
}

static int64_t gcd64(int64_t a, int64_t b) { while (b) { int64_t t = a % b; a = b; b = t; } return a < 0 ? -a : a; }

/* ------------------------------------------------------------------ assigners */

int or_assign_windows(const fwa_config* c, int64_t ts, int64_t* starts, int64_t* ends, int cap) {
    if (ts == J_LONG_MIN) return FWA_E_TS_MIN;      /* "Record has Long.MIN_VALUE timestamp" */
    if (c->window_kind == FWA_TUMBLE) {             /* TumblingEventTimeWindows.assignWindows :70-88 */
        int64_t st = or_window_start(ts, c->offset_ms % c->size_ms, c->size_ms);
        if (cap < 1) return FWA_E_ARG;
        starts[0] = st; ends[0] = jladd(st, c->size_ms);
        return 1;
    }
    if (c->window_kind == FWA_SLIDE) {              /* SlidingEventTimeWindows.assignWindows :70-82 */
        int n = 0;
        int64_t last_start = or_window_start(ts, c->offset_ms, c->slide_ms);
        for (int64_t st = last_start; st > jlsub(ts, c->size_ms); st = jlsub(st, c->slide_ms)) {
            if (n >= cap) return FWA_E_ARG;
            starts[n] = st; ends[n] = jladd(st, c->size_ms); n++;
        }
        return n;
    }
    if (c->window_kind == FWA_SESSION) {            /* EventTimeSessionWindows.assignWindows :61-63 */
        if (cap < 1) return FWA_E_ARG;
        starts[0] = ts; ends[0] = jladd(ts, c->gap_ms);
        return 1;
    }
    return FWA_E_UNSUPPORTED;
}

/* ---- shift time zone (TimeWindowUtil.java:52-100), tz = tz_n (instant, offset) pairs ---- */
static int64_t or_tz_offset(const fwa_config* c, int64_t instant) {       /* ZoneRules.getOffset(Instant) */
    int32_t best = 0;
    for (int32_t i = 1; i < c->tz_n; i++) if (c->tz[2 * i] <= instant) best = i;
    return c->tz[2 * best + 1];
}
int64_t or_to_local(const fwa_config* c, int64_t epoch) {                /* toUtcTimestampMills :52-60 */
    if (c->tz_n == 0 || epoch == J_LONG_MAX) return epoch;
    return jladd(epoch, or_tz_offset(c, epoch));
}
static int64_t or_at_zone(const fwa_config* c, int64_t local) {           /* LocalDateTime.atZone(zone) */
    /* valid offsets o: the instant local - o really has offset o; gap (none): local - offset before the
       transition; overlap (two): the earlier offset */
    int64_t found = 0, first = 0;
    int nf = 0;
    for (int32_t i = 0; i < c->tz_n; i++) {
        int64_t o = c->tz[2 * i + 1];
        int64_t e = jlsub(local, o);
        int dup = 0;
        for (int32_t k = 0; k < i; k++) if (c->tz[2 * k + 1] == o) dup = 1;
        if (dup || or_tz_offset(c, e) != o) continue;
        if (nf == 0 || e < first) first = e;           /* earlier offset = smaller instant */
        found = e; nf++;
    }
    (void)found;
    if (nf >= 1) return first;
    /* gap: the transition T with T + before <= local < T + after */
    for (int32_t i = 1; i < c->tz_n; i++) {
        int64_t before = c->tz[2 * (i - 1) + 1], after = c->tz[2 * i + 1], t = c->tz[2 * i];
        if (jladd(t, before) <= local && local < jladd(t, after)) return jlsub(local, before);
    }
    return jlsub(local, c->tz[1]);
}
int64_t or_tz_timer(const fwa_config* c, int64_t local) {                 /* toEpochMillsForTimer :67-100 */
    if (c->tz_n == 0 || local == J_LONG_MAX) return local;
    if (c->tz_n == 1) return jlsub(local, c->tz[1]);
    const int64_t hour = 3600000;                      /* useDaylightTime(): more than one offset */
    int64_t t1 = or_at_zone(c, local), t2 = or_at_zone(c, jladd(local, hour));
    if (t1 == t2) return t1 - t1 % hour;
    if (t2 - t1 > hour) return t1 + hour;
    return t1;
}

int64_t or_assign_slice_end(const fwa_config* c, int64_t ts) {
    ts = or_to_local(c, ts);                           /* AbstractSliceAssigner: rowtime -> local millis */
    if (c->window_kind == FWA_TUMBLE) return jladd(or_window_start(ts, c->offset_ms, c->size_ms), c->size_ms);
    if (c->window_kind == FWA_SLIDE) {
        int64_t g = gcd64(c->size_ms, c->slide_ms);
        return jladd(or_window_start(ts, c->offset_ms, g), g);
    }
    /* CUMULATE: step */
    return jladd(or_window_start(ts, c->offset_ms, c->slide_ms), c->slide_ms);
}

/* ------------------------------------------------------------------ containers */

typedef struct { int64_t k[4]; } k4;

static inline uint64_t k4_hash(const k4* x) {
    uint64_t h = 0x9e3779b97f4a7c15ULL;
    for (int i = 0; i < 4; i++) { h ^= (uint64_t)x->k[i] + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2); h *= 0xff51afd7ed558ccdULL; h ^= h >> 33; }
    return h;
}
static inline int k4_eq(const k4* a, const k4* b) { return a->k[0] == b->k[0] && a->k[1] == b->k[1] && a->k[2] == b->k[2] && a->k[3] == b->k[3]; }

/* open addressing, linear probing, backward-shift deletion; one slot = key, value and used flag together (one cache
   line fetch per probe: the full-size digest oracles probe tables of tens of millions of entries) */
typedef struct { k4 key; int64_t val; int64_t used; } hslot;
typedef struct { hslot* s; int64_t cap, n; } hmap;

static void hm_init(hmap* m, int64_t cap) {
    int64_t c = 16; while (c < cap * 2) c <<= 1;
    m->cap = c; m->n = 0;
    m->s = (hslot*)calloc(c, sizeof(hslot));
}
static void hm_free(hmap* m) { free(m->s); memset(m, 0, sizeof(*m)); }
static int64_t* hm_find(hmap* m, const k4* k) {
    uint64_t i = k4_hash(k) & (m->cap - 1);
    while (m->s[i].used) { if (k4_eq(&m->s[i].key, k)) return &m->s[i].val; i = (i + 1) & (m->cap - 1); }
    return NULL;
}
static void hm_grow(hmap* m);
static int64_t* hm_put(hmap* m, const k4* k, int64_t v, int* inserted) {
    if ((m->n + 1) * 10 > m->cap * 7) hm_grow(m);
    uint64_t i = k4_hash(k) & (m->cap - 1);
    while (m->s[i].used) { if (k4_eq(&m->s[i].key, k)) { if (inserted) *inserted = 0; return &m->s[i].val; } i = (i + 1) & (m->cap - 1); }
    m->s[i].used = 1; m->s[i].key = *k; m->s[i].val = v; m->n++;
    if (inserted) *inserted = 1;
    return &m->s[i].val;
}
static void hm_grow(hmap* m) {
    hmap o = *m; hm_init(m, o.cap);
    for (int64_t i = 0; i < o.cap; i++) if (o.s[i].used) hm_put(m, &o.s[i].key, o.s[i].val, NULL);
    hm_free(&o);
}
static int hm_del(hmap* m, const k4* k) {
    uint64_t mask = m->cap - 1, i = k4_hash(k) & mask;
    while (m->s[i].used && !k4_eq(&m->s[i].key, k)) i = (i + 1) & mask;
    if (!m->s[i].used) return 0;
    uint64_t j = i;
    for (;;) {
        j = (j + 1) & mask;
        if (!m->s[j].used) break;
        uint64_t h = k4_hash(&m->s[j].key) & mask;
        /* move j back to i if h is cyclically outside (i, j] */
        if ((i <= j) ? (h <= i || h > j) : (h <= i && h > j)) { m->s[i].key = m->s[j].key; m->s[i].val = m->s[j].val; i = j; }
    }
    m->s[i].used = 0; m->n--;
    return 1;
}

/* timer heap ordered by timestamp only (TimerHeapInternalTimer.comparePriorityTo :131-133) */
typedef struct { int64_t ts; int64_t key; int64_t a, b; uint64_t seq; } timer_t_;
typedef struct { timer_t_* h; int64_t n, cap; hmap set; uint64_t seq; } theap;

static void th_init(theap* t) { t->cap = 64; t->n = 0; t->h = (timer_t_*)malloc(sizeof(timer_t_) * t->cap); hm_init(&t->set, 64); t->seq = 0; }
static void th_free(theap* t) { free(t->h); hm_free(&t->set); }
static int tless(const timer_t_* x, const timer_t_* y) { return x->ts < y->ts || (x->ts == y->ts && x->seq < y->seq); }
/* registerEventTimeTimer with (ts, key, namespace) dedup (HeapPriorityQueueSet :148-156) */
static void th_add(theap* t, int64_t ts, int64_t key, int64_t a, int64_t b) {
    k4 k = {{ts, key, a, b}}; int ins;
    hm_put(&t->set, &k, 1, &ins);
    if (!ins) return;
    if (t->n == t->cap) { t->cap *= 2; t->h = (timer_t_*)realloc(t->h, sizeof(timer_t_) * t->cap); }
    timer_t_ x = {ts, key, a, b, t->seq++};
    int64_t i = t->n++;
    while (i > 0) { int64_t p = (i - 1) / 2; if (!tless(&x, &t->h[p])) break; t->h[i] = t->h[p]; i = p; }
    t->h[i] = x;
}
/* deleteEventTimeTimer: lazy (the entry is skipped when popped if no longer in the set) */
static void th_del(theap* t, int64_t ts, int64_t key, int64_t a, int64_t b) { k4 k = {{ts, key, a, b}}; hm_del(&t->set, &k); }
static int th_pop_due(theap* t, int64_t wm, timer_t_* out) {
    while (t->n > 0 && t->h[0].ts <= wm) {
        timer_t_ top = t->h[0];
        timer_t_ x = t->h[--t->n];
        int64_t i = 0;
        for (;;) {
            int64_t l = 2 * i + 1, r = l + 1, m = i;
            timer_t_* best = &x;
            if (l < t->n && tless(&t->h[l], best)) { m = l; best = &t->h[l]; }
            if (r < t->n && tless(&t->h[r], best)) { m = r; }
            if (m == i) break;
            t->h[i] = t->h[m]; i = m;
        }
        if (t->n > 0) t->h[i] = x;
        k4 k = {{top.ts, top.key, top.a, top.b}};
        if (hm_del(&t->set, &k)) { *out = top; return 1; }
    }
    return 0;
}

/* ------------------------------------------------------------------ accumulators */

typedef union { int64_t i; double d; float f; __int128 q; } aval;   /* q: DECIMAL unscaled value */

/* ---- DECIMAL (DecimalSumAggFunction / DecimalAvgAggFunction, SumAggFunction.java:150-168, AvgAggFunction.java:213-251):
   DecimalDataUtils.add (:106-121) -> DecimalData.fromBigDecimal (DecimalData.java:184-195): NULL past 38 digits */
static int is_dec(int k) { return k >= FWA_SUM_DEC && k <= FWA_AVG_DEC128; }
static int is_dec_avg(int k) { return k == FWA_AVG_DEC || k == FWA_AVG_DEC128; }

/* ---- DataStream built-in reductions (FWA_CFG_REDUCE): SumAggregator / ComparableAggregator applied in arrival order
   (WindowedStream.java:680-890 -> reduce(); HeapReducingState.add reduces the stored value1 with each new element) */
static int is_byk(int k) { return k >= FWA_MINBY_I64 && k <= FWA_MAXBY_F32; }
static int is_maxby(int k) { return k == FWA_MAXBY_I64 || k == FWA_MAXBY_I32 || k == FWA_MAXBY_F64 || k == FWA_MAXBY_F32; }
/* Double.compare / Float.compare (Double.java compare: doubleToLongBits order, so -0.0 < 0.0 and NaN above +Inf) */
static int64_t jbits_d(double v) { int64_t b; if (v != v) return 0x7ff8000000000000LL; memcpy(&b, &v, 8); return b; }
static int32_t jbits_f(float v) { int32_t b; if (v != v) return 0x7fc00000; memcpy(&b, &v, 4); return b; }
static int jcmp_d(double a, double b) {
    if (a < b) return -1;
    if (a > b) return 1;
    const int64_t x = jbits_d(a), y = jbits_d(b);
    return x == y ? 0 : (x < y ? -1 : 1);
}
static int jcmp_f(float a, float b) {
    if (a < b) return -1;
    if (a > b) return 1;
    const int32_t x = jbits_f(a), y = jbits_f(b);
    return x == y ? 0 : (x < y ? -1 : 1);
}
/* compare(state, v) of the field a by/min/max aggregate reads; 4-byte types sit in the low half of aval */
static int red_cmp(int kind, const aval* x, const void* col, int64_t i) {
    switch (kind) {
    case FWA_MIN_I64: case FWA_MAX_I64: case FWA_MINBY_I64: case FWA_MAXBY_I64: {
        const int64_t v = ((const int64_t*)col)[i]; return x->i < v ? -1 : (x->i > v ? 1 : 0); }
    case FWA_MIN_I32: case FWA_MAX_I32: case FWA_MINBY_I32: case FWA_MAXBY_I32: {
        const int32_t v = ((const int32_t*)col)[i], u = (int32_t)x->i; return u < v ? -1 : (u > v ? 1 : 0); }
    case FWA_MIN_F64: case FWA_MAX_F64: case FWA_MINBY_F64: case FWA_MAXBY_F64: return jcmp_d(x->d, ((const double*)col)[i]);
    default: return jcmp_f(x->f, ((const float*)col)[i]);
    }
}
static void red_set(int kind, aval* x, const void* col, int64_t i) {   /* x := the element's field */
    switch (kind) {
    case FWA_FIRST_32: case FWA_SEL_32: x->i = (int64_t)((const uint32_t*)col)[i]; break;
    case FWA_MIN_I32: case FWA_MAX_I32: case FWA_MINBY_I32: case FWA_MAXBY_I32: case FWA_SUM_I32: x->i = ((const int32_t*)col)[i]; break;
    case FWA_MIN_F32: case FWA_MAX_F32: case FWA_MINBY_F32: case FWA_MAXBY_F32: case FWA_SUM_F32:
        x->i = 0; x->f = ((const float*)col)[i]; break;
    case FWA_MIN_F64: case FWA_MAX_F64: case FWA_MINBY_F64: case FWA_MAXBY_F64: case FWA_SUM_F64: x->d = ((const double*)col)[i]; break;
    default: x->i = ((const int64_t*)col)[i]; break;
    }
}
static const unsigned __int128 DEC_LIM = (unsigned __int128)10000000000000000000ull * 10000000000000000000ull; /* 10^38 */
static int dec_fits(__int128 v) { unsigned __int128 a = v < 0 ? -(unsigned __int128)v : (unsigned __int128)v; return a < DEC_LIM; }
static __int128 dec_input(const void* col, int64_t i, int kind) {
    if (kind == FWA_SUM_DEC || kind == FWA_AVG_DEC) return (__int128)((const int64_t*)col)[i];
    const uint64_t* p = (const uint64_t*)col + 2 * i;            /* 16-byte little-endian two's complement */
    return (__int128)(((unsigned __int128)p[1] << 64) | p[0]);
}
/* AVG's value (AvgAggFunction.getValueExpression :100-106): DecimalDataUtils.divide(sum, count) (:145-148): the exact
   quotient |sum| * 10^-s / cnt rounded HALF_UP to 38 significant digits (MathContext MC_DIVIDE :40), then
   fromBigDecimal at the result type DECIMAL(38, t): setScale(t, HALF_UP), NULL past 38 digits. Written as a decimal
   digit expansion of the quotient. Returns 0 for NULL. */
static int dec_divide(__int128 sum, int64_t cnt, int s, int t, __int128* out) {
    const int neg = sum < 0;
    unsigned __int128 a = neg ? -(unsigned __int128)sum : (unsigned __int128)sum;
    if (a == 0) { *out = 0; return 1; }
    enum { ND = 200 };
    signed char d[ND];                                     /* digits of a / cnt; the point sits after ni digits */
    int ni = 0;
    unsigned __int128 ip = a / (uint64_t)cnt;
    uint64_t r = (uint64_t)(a % (uint64_t)cnt);
    char tmp[48]; int k = 0;
    while (ip) { tmp[k++] = (char)(ip % 10); ip /= 10; }
    for (int i = k - 1; i >= 0; i--) d[ni++] = tmp[i];
    for (int i = ni; i < ND; i++) { unsigned __int128 x = (unsigned __int128)r * 10u; d[i] = (signed char)(x / (uint64_t)cnt); r = (uint64_t)(x % (uint64_t)cnt); }
    int p0 = 0;
    while (d[p0] == 0) p0++;                               /* first significant digit */
    unsigned __int128 q1 = 0;
    for (int i = p0; i < p0 + 38; i++) q1 = q1 * 10u + (unsigned)d[i];
    if (d[p0 + 38] >= 5) q1 += 1u;                         /* HALF_UP at 38 significant digits */
    const int u = s + (p0 + 38 - ni);                      /* scale of q1 */
    unsigned __int128 res;
    if (u > t) {                                           /* setScale(t, HALF_UP) */
        int drop = u - t; unsigned last = 0;
        res = q1;
        for (int i = 0; i < drop; i++) { last = (unsigned)(res % 10u); res /= 10u; }
        if (last >= 5) res += 1u;
    } else {
        res = q1;
        for (int i = 0; i < t - u; i++) { if (res >= DEC_LIM / 10u) return 0; res *= 10u; }
    }
    if (res >= DEC_LIM) return 0;
    *out = neg ? -(__int128)res : (__int128)res;
    return 1;
}

typedef struct or_engine {
    fwa_config c;
    int64_t wm;                 /* currentWatermark / currentProgress, init Long.MIN_VALUE */
    int nacc;                   /* 1 (count) + aggs (values) + aggs (non-NULL input counts) */
    const uint8_t* const* nulls;/* NULL flags of the push being applied (fwa_push_nullable), or NULL */
    aval* pool; int64_t pool_n, pool_cap; int64_t* free_list; int64_t free_n, free_cap;
    hmap state;                 /* (key, nsA, nsB, 0) -> acc id */
    theap timers;
    /* per-key list of in-flight windows for sessions (key,-1,-1,-1) -> head idx in win list */
    int64_t* wl_key; int64_t* wl_start; int64_t* wl_end; int64_t* wl_sws; int64_t* wl_sw_end; int64_t* wl_next; int64_t wl_n, wl_cap;
    hmap wl_head;
    /* output */
    int64_t out_n, out_cap;
    int out_ret;   /* the rows were returned by the last or_advance_watermark: clear at the next call */
    int64_t *o_key, *o_start, *o_end; aval* o_agg[FWA_MAX_AGGS]; uint8_t* o_null[FWA_MAX_AGGS];
    fwa_stats st;
    int32_t* late_idx; int64_t late_n, late_cap;   /* records the last or_push dropped as late */
    char err[256];
} or_engine;

static int64_t acc_new(or_engine* e) {
    int64_t id;
    if (e->free_n) id = e->free_list[--e->free_n];
    else {
        if (e->pool_n == e->pool_cap) { e->pool_cap = e->pool_cap ? e->pool_cap * 2 : 1024; e->pool = (aval*)realloc(e->pool, sizeof(aval) * e->nacc * e->pool_cap); }
        id = e->pool_n++;
    }
    aval* a = &e->pool[id * e->nacc];
    memset(a, 0, sizeof(aval) * e->nacc);
    for (int j = 0; j < e->c.num_aggs; j++) {           /* createAccumulators */
        switch (e->c.aggs[j].kind) {
        case FWA_SUM_F32: a[1 + j].i = 0; a[1 + j].f = 0.0f; break;
        case FWA_SUM_F64: case FWA_AVG_F32: case FWA_AVG_F64: a[1 + j].d = 0.0; break;
        default: a[1 + j].i = 0; break;                   /* MIN/MAX: "null" until count>0 */
        }
    }
    return id;
}
static void acc_free(or_engine* e, int64_t id) {
    if (e->free_n == e->free_cap) { e->free_cap = e->free_cap ? e->free_cap * 2 : 1024; e->free_list = (int64_t*)realloc(e->free_list, 8 * e->free_cap); }
    e->free_list[e->free_n++] = id;
}

/* One element reduced into a reduce handle's window state (value1 = the state, value2 = the element). */
static void red_add(or_engine* e, aval* a, const void* const* cols, int64_t i) {
    const int na = e->c.num_aggs;
    const int64_t before = a[0].i;
    a[0].i = jladd(a[0].i, 1);
    int sel = before == 0;                            /* minBy / maxBy: the element replaces the selected one */
    for (int j = 0; j < na && before > 0; j++) {
        const int k = e->c.aggs[j].kind;
        if (!is_byk(k)) continue;
        const int c = red_cmp(k, &a[1 + j], cols[e->c.aggs[j].col], i);   /* ComparableAggregator.reduce :83-107 */
        sel = c == 0 ? ((e->c.flags & FWA_CFG_BY_LAST) != 0) : (is_maxby(k) ? c < 0 : c > 0);
    }
    for (int j = 0; j < na; j++) {
        const int k = e->c.aggs[j].kind;
        const void* col = k == FWA_COUNT ? NULL : cols[e->c.aggs[j].col];
        aval* x = &a[1 + j];
        switch (k) {
        case FWA_COUNT: break;
        case FWA_FIRST_64: case FWA_FIRST_32: if (before == 0) red_set(k, x, col, i); break;   /* value1's fields */
        case FWA_SEL_64: case FWA_SEL_32: if (sel) red_set(k, x, col, i); break;
        case FWA_SUM_I64: x->i = jladd(x->i, ((const int64_t*)col)[i]); break;              /* SumFunction */
        case FWA_SUM_I32: x->i = (int32_t)((uint32_t)x->i + (uint32_t)((const int32_t*)col)[i]); break;
        case FWA_SUM_F64: x->d += ((const double*)col)[i]; break;
        case FWA_SUM_F32: x->f = x->f + ((const float*)col)[i]; break;
        case FWA_MIN_I64: case FWA_MIN_I32: case FWA_MIN_F64: case FWA_MIN_F32:   /* isExtremal == 0 -> value2's */
            if (before == 0 || !(red_cmp(k, x, col, i) < 0)) red_set(k, x, col, i);
            break;
        case FWA_MAX_I64: case FWA_MAX_I32: case FWA_MAX_F64: case FWA_MAX_F32:
            if (before == 0 || !(red_cmp(k, x, col, i) > 0)) red_set(k, x, col, i);
            break;
        default: if (is_byk(k) && sel) red_set(k, x, col, i); break;
        }
    }
}

/* accumulate one record (AggregateFunction.add / ReduceFunction.reduce / SQL accumulate) */
static void acc_add(or_engine* e, aval* a, const void* const* cols, int64_t i) {
    if (e->c.flags & FWA_CFG_REDUCE) { red_add(e, a, cols, i); return; }
    const int na = e->c.num_aggs;
    a[0].i = jladd(a[0].i, 1);
    for (int j = 0; j < na; j++) {
        const int cj = e->c.aggs[j].col;
        const void* col = cols ? cols[cj] : NULL;
        aval* x = &a[1 + j];
        if (e->c.aggs[j].kind == FWA_COUNT) continue;
        /* SQL NULL input: skipped by SUM/MIN/MAX/AVG/COUNT(col) (their accumulate expressions test isNull) */
        if ((e->c.nullable_cols >> cj & 1) && e->nulls && e->nulls[cj] && e->nulls[cj][i]) continue;
        int first = (a[1 + na + j].i == 0);               /* buffer still NULL */
        a[1 + na + j].i++;
        if (is_dec(e->c.aggs[j].kind)) {
            const __int128 v = dec_input(col, i, e->c.aggs[j].kind);
            int64_t* ovf = &a[1 + 2 * na + j].i;
            if (is_dec_avg(e->c.aggs[j].kind)) {          /* sum starts at 0; plus(NULL, v) stays NULL */
                if (!*ovf) { x->q += v; if (!dec_fits(x->q)) *ovf = 1; }
            } else if (first || *ovf) {                   /* SUM: ifThenElse(isNull(sum), operand, ...) */
                x->q = v; *ovf = 0;
            } else {
                x->q += v;
                if (!dec_fits(x->q)) *ovf = 1;
            }
            continue;
        }
        switch (e->c.aggs[j].kind) {
        case FWA_COUNT: case FWA_COUNT_COL: break;
        case FWA_SUM_I64: case FWA_AVG_I64: x->i = jladd(x->i, ((const int64_t*)col)[i]); break;
        case FWA_SUM_F32: x->f = x->f + ((const float*)col)[i]; break;            /* float32 buffer (a16) */
        case FWA_SUM_F64: x->d += ((const double*)col)[i]; break;
        case FWA_AVG_F32: x->d += (double)((const float*)col)[i]; break;          /* FloatAvg: DOUBLE sum */
        case FWA_AVG_F64: x->d += ((const double*)col)[i]; break;
        case FWA_MIN_I64: { int64_t v = ((const int64_t*)col)[i]; if (first || v < x->i) x->i = v; break; }
        case FWA_MAX_I64: { int64_t v = ((const int64_t*)col)[i]; if (first || v > x->i) x->i = v; break; }
        case FWA_MIN_F32: { float v = ((const float*)col)[i]; if (first || v < x->f) x->f = v; break; }
        case FWA_MAX_F32: { float v = ((const float*)col)[i]; if (first || v > x->f) x->f = v; break; }
        case FWA_MIN_F64: { double v = ((const double*)col)[i]; if (first || v < x->d) x->d = v; break; }
        case FWA_MAX_F64: { double v = ((const double*)col)[i]; if (first || v > x->d) x->d = v; break; }
        }
    }
}

/* merge accumulator b into a (AggregateFunction.merge / SQL mergeExpressions) */
/* HeapReducingState.mergeState(a, b) = reduce(a, b) (AbstractHeapMergingState.mergeNamespaces :65-90): the merged
   session keeps value1's fields and folds field pos -- the only value field of a session reduction (the engine's
   scope), so the merge order MergingWindowSet's HashSet gives does not matter except for float sums' rounding */
static void red_merge(or_engine* e, aval* a, const aval* b) {
    const int64_t before = a[0].i;
    a[0].i = jladd(a[0].i, b[0].i);
    for (int j = 0; j < e->c.num_aggs; j++) {
        const int k = e->c.aggs[j].kind;
        aval* x = &a[1 + j]; const aval* y = &b[1 + j];
        if (before == 0) { *x = *y; continue; }
        switch (k) {
        case FWA_SUM_I64: x->i = jladd(x->i, y->i); break;
        case FWA_SUM_I32: x->i = (int32_t)((uint32_t)x->i + (uint32_t)y->i); break;
        case FWA_SUM_F64: x->d += y->d; break;
        case FWA_SUM_F32: x->f = x->f + y->f; break;
        default: {                                       /* MIN / MAX / MINBY / MAXBY of field pos */
            int c;
            switch (k) {
            case FWA_MIN_I64: case FWA_MAX_I64: case FWA_MINBY_I64: case FWA_MAXBY_I64:
                c = x->i < y->i ? -1 : (x->i > y->i ? 1 : 0); break;
            case FWA_MIN_I32: case FWA_MAX_I32: case FWA_MINBY_I32: case FWA_MAXBY_I32: {
                const int32_t u = (int32_t)x->i, v = (int32_t)y->i; c = u < v ? -1 : (u > v ? 1 : 0); break; }
            case FWA_MIN_F64: case FWA_MAX_F64: case FWA_MINBY_F64: case FWA_MAXBY_F64: c = jcmp_d(x->d, y->d); break;
            default: c = jcmp_f(x->f, y->f); break;
            }
            const int wantmax = k == FWA_MAX_I64 || k == FWA_MAX_I32 || k == FWA_MAX_F64 || k == FWA_MAX_F32 || is_maxby(k);
            if (is_byk(k)) { if (c == 0 ? (e->c.flags & FWA_CFG_BY_LAST) != 0 : (wantmax ? c < 0 : c > 0)) *x = *y; }
            else if (wantmax ? !(c > 0) : !(c < 0)) *x = *y;   /* isExtremal == 0 -> value2's */
        }
        }
    }
}

static void acc_merge(or_engine* e, aval* a, const aval* b) {
    if (b[0].i == 0) return;
    if (e->c.flags & FWA_CFG_REDUCE) { red_merge(e, a, b); return; }
    const int na = e->c.num_aggs;
    a[0].i = jladd(a[0].i, b[0].i);
    for (int j = 0; j < na; j++) {
        aval* x = &a[1 + j]; const aval* y = &b[1 + j];
        if (is_dec(e->c.aggs[j].kind)) {                  /* mergeExpressions */
            const int kind = e->c.aggs[j].kind;
            int64_t* ovf = &a[1 + 2 * na + j].i;
            const int64_t ovb = b[1 + 2 * na + j].i;
            const int anull = a[1 + na + j].i == 0 || *ovf, bnull = b[1 + na + j].i == 0 || ovb;
            a[1 + na + j].i += b[1 + na + j].i;
            if (is_dec_avg(kind)) {                       /* sum + other.sum: NULL if either is */
                if (*ovf || ovb) *ovf = 1;
                else { x->q += y->q; if (!dec_fits(x->q)) *ovf = 1; }
            } else if (bnull) {
            } else if (anull) {
                x->q = y->q; *ovf = 0;
            } else {
                x->q += y->q;
                if (!dec_fits(x->q)) *ovf = 1;
            }
            continue;
        }
        if (b[1 + na + j].i == 0) continue;               /* merging a NULL buffer changes nothing */
        int first = (a[1 + na + j].i == 0);
        a[1 + na + j].i += b[1 + na + j].i;
        switch (e->c.aggs[j].kind) {
        case FWA_COUNT: case FWA_COUNT_COL: break;
        case FWA_SUM_I64: case FWA_AVG_I64: x->i = jladd(x->i, y->i); break;
        case FWA_SUM_F32: x->f = x->f + y->f; break;
        case FWA_SUM_F64: case FWA_AVG_F32: case FWA_AVG_F64: x->d += y->d; break;
        case FWA_MIN_I64: if (first || y->i < x->i) x->i = y->i; break;
        case FWA_MAX_I64: if (first || y->i > x->i) x->i = y->i; break;
        case FWA_MIN_F32: if (first || y->f < x->f) x->f = y->f; break;
        case FWA_MAX_F32: if (first || y->f > x->f) x->f = y->f; break;
        case FWA_MIN_F64: if (first || y->d < x->d) x->d = y->d; break;
        case FWA_MAX_F64: if (first || y->d > x->d) x->d = y->d; break;
        }
    }
}

static void emit(or_engine* e, int64_t key, int64_t ws, int64_t we, const aval* a) {
    if (e->out_n == e->out_cap) {
        e->out_cap = e->out_cap ? e->out_cap * 2 : 1024;
        e->o_key = (int64_t*)realloc(e->o_key, 8 * e->out_cap);
        e->o_start = (int64_t*)realloc(e->o_start, 8 * e->out_cap);
        e->o_end = (int64_t*)realloc(e->o_end, 8 * e->out_cap);
        for (int j = 0; j < e->c.num_aggs; j++) e->o_agg[j] = (aval*)realloc(e->o_agg[j], sizeof(aval) * e->out_cap);
        for (int j = 0; j < e->c.num_aggs; j++) e->o_null[j] = (uint8_t*)realloc(e->o_null[j], e->out_cap);
    }
    int64_t r = e->out_n++;
    e->o_key[r] = key; e->o_start[r] = ws; e->o_end[r] = we;
    int64_t cnt = a[0].i;
    const int na = e->c.num_aggs;
    for (int j = 0; j < na; j++) {                /* getResult / getValueExpression */
        const aval* x = &a[1 + j]; aval* o = &e->o_agg[j][r]; o->i = 0;
        const int64_t nn = a[1 + na + j].i;           /* non-NULL inputs */
        const int kind = e->c.aggs[j].kind;
        if (e->c.flags & FWA_CFG_REDUCE) {            /* the reduced tuple's fields */
            e->o_null[j][r] = 0;
            if (kind == FWA_COUNT) o->i = a[0].i;
            else if (kind == FWA_SUM_F32 || kind == FWA_MIN_F32 || kind == FWA_MAX_F32 || kind == FWA_MINBY_F32 ||
                     kind == FWA_MAXBY_F32) { o->f = x->f; if (o->f != o->f) o->i = 0x7fc00000; }
            else if (kind == FWA_SUM_F64 || kind == FWA_MIN_F64 || kind == FWA_MAX_F64 || kind == FWA_MINBY_F64 ||
                     kind == FWA_MAXBY_F64) { o->d = x->d; if (o->d != o->d) o->i = 0x7ff8000000000000LL; }
            else if (kind == FWA_SUM_I32 || kind == FWA_MIN_I32 || kind == FWA_MAX_I32 || kind == FWA_MINBY_I32 ||
                     kind == FWA_MAXBY_I32 || kind == FWA_FIRST_32 || kind == FWA_SEL_32) o->i = (int64_t)(uint32_t)x->i;
            else o->i = x->i;
            continue;
        }
        e->o_null[j][r] = (kind != FWA_COUNT && kind != FWA_COUNT_COL && nn == 0);   /* SQL NULL result */
        if (e->o_null[j][r]) continue;
        if (is_dec(kind)) {
            o->q = 0;
            if (a[1 + 2 * na + j].i) { e->o_null[j][r] = 1; continue; }   /* the sum overflowed */
            if (!is_dec_avg(kind)) { o->q = x->q; continue; }
            const int s = e->c.dec_scale[j];
            if (!dec_divide(x->q, nn, s, s > 6 ? s : 6, &o->q)) { e->o_null[j][r] = 1; o->q = 0; }
            continue;
        }
        if (kind == FWA_AVG_I64 || kind == FWA_AVG_F32 || kind == FWA_AVG_F64) cnt = nn;   /* AVG: non-NULL count */
        else cnt = a[0].i;
        switch (kind) {
        case FWA_COUNT: o->i = cnt; break;
        case FWA_COUNT_COL: o->i = nn; break;
        case FWA_SUM_I64: case FWA_MIN_I64: case FWA_MAX_I64: o->i = x->i; break;
        case FWA_SUM_F32: case FWA_MIN_F32: case FWA_MAX_F32: o->f = x->f; break;
        case FWA_SUM_F64: case FWA_MIN_F64: case FWA_MAX_F64: o->d = x->d; break;
        case FWA_AVG_I64: o->i = (cnt == 0) ? 0 : ((cnt == -1 && x->i == J_LONG_MIN) ? J_LONG_MIN : x->i / cnt); break;
        case FWA_AVG_F32: o->f = (float)(x->d / (double)cnt); break;
        case FWA_AVG_F64: o->d = x->d / (double)cnt; break;
        }
    }
    e->st.rows_out++;
}

/* ------------------------------------------------------------------ engine */

static int set_err(or_engine* e, int code, const char* msg) { snprintf(e->err, sizeof(e->err), "%s", msg); return code; }

int or_create(const fwa_config* c, or_engine** out) {
    *out = NULL;
    if (c->num_aggs < 0 || c->num_aggs > FWA_MAX_AGGS) return FWA_E_ARG;
    if (c->nullable_cols && c->semantics != FWA_SEM_TABLE) return FWA_E_ARG;   /* SQL NULLs: Table only */
    if (c->window_kind == FWA_TUMBLE && (c->size_ms <= 0 || (c->offset_ms < 0 ? -c->offset_ms : c->offset_ms) >= c->size_ms)) return FWA_E_ARG;
    if (c->window_kind == FWA_SLIDE) {
        if (c->size_ms <= 0 || c->slide_ms <= 0) return FWA_E_ARG;
        if (c->semantics == FWA_SEM_DATASTREAM && (c->offset_ms < 0 ? -c->offset_ms : c->offset_ms) >= c->slide_ms) return FWA_E_ARG;
        if (c->semantics == FWA_SEM_TABLE && c->size_ms % c->slide_ms != 0) return FWA_E_ARG;
    }
    if (c->window_kind == FWA_CUMULATE && (c->semantics != FWA_SEM_TABLE || c->size_ms <= 0 || c->slide_ms <= 0 || c->size_ms % c->slide_ms)) return FWA_E_ARG;
    if (c->window_kind == FWA_SESSION && c->gap_ms <= 0 && !(c->flags & FWA_CFG_DYNAMIC_GAP)) return FWA_E_ARG;
    if (c->semantics == FWA_SEM_TABLE && c->allowed_lateness_ms != 0) return FWA_E_ARG;
    {   /* reduce kinds only in FWA_CFG_REDUCE handles, which are non-merging DataStream windows */
        int nby = 0, nsel = 0, nfirst = 0, nred = 0;
        for (int j = 0; j < c->num_aggs; j++) {
            const int k = c->aggs[j].kind;
            nby += is_byk(k); nsel += (k == FWA_SEL_64 || k == FWA_SEL_32); nfirst += (k == FWA_FIRST_64 || k == FWA_FIRST_32);
            nred += k >= FWA_SUM_I32 && k <= FWA_SEL_32;
            if ((c->flags & FWA_CFG_REDUCE) && (is_dec(k) || k == FWA_AVG_I64 || k == FWA_AVG_F32 || k == FWA_AVG_F64 ||
                                                k == FWA_COUNT_COL || k == FWA_COUNT)) return FWA_E_UNSUPPORTED;
        }
        if (nred && !(c->flags & FWA_CFG_REDUCE)) return FWA_E_ARG;
        if (c->flags & FWA_CFG_REDUCE) {
            if (nby > 1 || (nsel && !nby) || (nfirst && nby)) return FWA_E_ARG;
            /* session windows: a tuple whose one value field is the reduced one (Tuple2<key, f1>) -- the engine's scope */
            const int sess_ok = c->window_kind == FWA_SESSION && c->num_aggs == 1 && !nsel && !nfirst;
            if (c->semantics != FWA_SEM_DATASTREAM || (c->window_kind != FWA_TUMBLE && c->window_kind != FWA_SLIDE && !sess_ok))
                return FWA_E_UNSUPPORTED;
        }
    }
    if (c->tz_n < 0 || (c->tz_n > 0 && (!c->tz || c->semantics != FWA_SEM_TABLE))) return FWA_E_ARG;
    or_engine* e = (or_engine*)calloc(1, sizeof(or_engine));
    e->c = *c;
    if (c->tz_n > 0) {                                 /* own copy of the shift-time-zone table */
        int64_t* t = (int64_t*)malloc(16 * (size_t)c->tz_n);
        memcpy(t, c->tz, 16 * (size_t)c->tz_n);
        e->c.tz = t;
    }
    if (e->c.max_parallelism <= 0) e->c.max_parallelism = 128;
    e->wm = J_LONG_MIN;
    e->nacc = 1 + 3 * c->num_aggs;            /* count, values, non-NULL counts, DECIMAL overflow flags */
    hm_init(&e->state, 1024);
    th_init(&e->timers);
    hm_init(&e->wl_head, 64);
    e->st.current_watermark = J_LONG_MIN;
    *out = e;
    return FWA_OK;
}

void or_destroy(or_engine* e) {
    if (!e) return;
    hm_free(&e->state); th_free(&e->timers); hm_free(&e->wl_head);
    if (e->c.tz_n > 0) free((void*)e->c.tz);
    free(e->late_idx);
    free(e->pool); free(e->free_list);
    free(e->wl_key); free(e->wl_start); free(e->wl_end); free(e->wl_sws); free(e->wl_sw_end); free(e->wl_next);
    free(e->o_key); free(e->o_start); free(e->o_end);
    for (int j = 0; j < FWA_MAX_AGGS; j++) { free(e->o_agg[j]); free(e->o_null[j]); }
    free(e);
}

const char* or_last_error(or_engine* e) { return e ? e->err : "null engine"; }

/* ---------------- DataStream WindowOperator (non-merging) ---------------- */

static int64_t cleanup_time(or_engine* e, int64_t ws, int64_t we) {    /* WindowOperator.cleanupTime :647-654 */
    int64_t max_ts = jlsub(we, 1);
    int64_t ct = jladd(max_ts, e->c.allowed_lateness_ms);
    return ct >= max_ts ? ct : J_LONG_MAX;
}

static aval* ds_state(or_engine* e, int64_t key, int64_t ws, int64_t we, int create) {
    k4 k = {{key, ws, we, 0}};
    int64_t* v = hm_find(&e->state, &k);
    if (v) return &e->pool[*v * e->nacc];
    if (!create) return NULL;
    int64_t id = acc_new(e);
    hm_put(&e->state, &k, id, NULL);
    return &e->pool[id * e->nacc];
}
static void ds_clear_state(or_engine* e, int64_t key, int64_t ws, int64_t we) {
    k4 k = {{key, ws, we, 0}};
    int64_t* v = hm_find(&e->state, &k);
    if (v) { acc_free(e, *v); hm_del(&e->state, &k); }
}

static void ds_process_element_aligned(or_engine* e, int64_t key, int64_t ts, const void* const* cols, int64_t i,
                                       const int64_t* ws, const int64_t* we, int nw, int* skipped) {
    for (int w = 0; w < nw; w++) {
        if (cleanup_time(e, ws[w], we[w]) <= e->wm) continue;      /* isWindowLate :586-589 */
        *skipped = 0;
        aval* a = ds_state(e, key, ws[w], we[w], 1);
        acc_add(e, a, cols, i);
        int64_t max_ts = jlsub(we[w], 1);
        if (max_ts <= e->wm) emit(e, key, ws[w], we[w], a);           /* EventTimeTrigger.onElement -> FIRE */
        else th_add(&e->timers, max_ts, key, ws[w], we[w]);
        int64_t ct = cleanup_time(e, ws[w], we[w]);                   /* registerCleanupTimer :608-620 */
        if (ct != J_LONG_MAX) th_add(&e->timers, ct, key, ws[w], we[w]);
    }
}

/* ---------------- DataStream sessions: MergingWindowSet per key ---------------- */
/* In-flight windows of a key are kept in a singly linked list (wl_*), each with its state window. */

static int64_t wl_alloc(or_engine* e) {
    if (e->wl_n == e->wl_cap) {
        e->wl_cap = e->wl_cap ? e->wl_cap * 2 : 256;
        e->wl_key = (int64_t*)realloc(e->wl_key, 8 * e->wl_cap); e->wl_start = (int64_t*)realloc(e->wl_start, 8 * e->wl_cap);
        e->wl_end = (int64_t*)realloc(e->wl_end, 8 * e->wl_cap); e->wl_sws = (int64_t*)realloc(e->wl_sws, 8 * e->wl_cap);
        e->wl_sw_end = (int64_t*)realloc(e->wl_sw_end, 8 * e->wl_cap); e->wl_next = (int64_t*)realloc(e->wl_next, 8 * e->wl_cap);
    }
    return e->wl_n++;
}
static int64_t* wl_headp(or_engine* e, int64_t key) { k4 k = {{key, -1, -1, -1}}; int ins; int64_t* p = hm_put(&e->wl_head, &k, -1, &ins); return p; }
static int wl_get_state_window(or_engine* e, int64_t key, int64_t ws, int64_t we, int64_t* sws, int64_t* swe) {
    for (int64_t i = *wl_headp(e, key); i >= 0; i = e->wl_next[i])
        if (e->wl_start[i] == ws && e->wl_end[i] == we) { *sws = e->wl_sws[i]; *swe = e->wl_sw_end[i]; return 1; }
    return 0;
}
static int wl_remove(or_engine* e, int64_t key, int64_t ws, int64_t we) {
    int64_t* pp = wl_headp(e, key);
    while (*pp >= 0) { int64_t i = *pp; if (e->wl_start[i] == ws && e->wl_end[i] == we) { *pp = e->wl_next[i]; return 1; } pp = &e->wl_next[i]; }
    return 0;
}
static void wl_put(or_engine* e, int64_t key, int64_t ws, int64_t we, int64_t sws, int64_t swe) {
    int64_t* pp = wl_headp(e, key);
    for (int64_t i = *pp; i >= 0; i = e->wl_next[i]) if (e->wl_start[i] == ws && e->wl_end[i] == we) { e->wl_sws[i] = sws; e->wl_sw_end[i] = swe; return; }
    int64_t n = wl_alloc(e); pp = wl_headp(e, key);
    e->wl_key[n] = key; e->wl_start[n] = ws; e->wl_end[n] = we; e->wl_sws[n] = sws; e->wl_sw_end[n] = swe; e->wl_next[n] = *pp; *pp = n;
}

typedef struct { int64_t s, e; } tw;
static int tw_cmp(const void* a, const void* b) { const tw* x = (const tw*)a; const tw* y = (const tw*)b; return x->s < y->s ? -1 : x->s > y->s; }

/* Table GROUP BY SESSION over a TIMESTAMP_LTZ rowtime: windows are formed on the local wall-clock timestamp
 * (TR WindowOperator.processElement :340 toUtcTimestampMills) and every event-time instant the operator compares with
 * the watermark or registers as a timer is toEpochMillsForTimer of it (InternalWindowProcessFunction.isWindowLate
 * :119-123, MergingWindowProcessFunction :137-141, EventTimeTriggers.AfterEndOfWindow, registerCleanupTimer :422-429).
 * UTC / DataStream: the instant itself. */
static int64_t ev_time(or_engine* e, int64_t local) { return e->c.tz_n ? or_tz_timer(&e->c, local) : local; }

/* MergingWindowSet.addWindow :153-236 + TimeWindow.mergeWindows :208-254 + the MergeFunction of
 * WindowOperator.processElement :292-349, then the per-window body :352-386. */
static int ds_process_element_session(or_engine* e, int64_t key, int64_t ts, const void* const* cols, int64_t i, int* skipped) {
    /* EventTimeSessionWindows.assignWindows :61-63; DynamicEventTimeSessionWindows.assignWindows :57-68 */
    const int64_t gap = (e->c.flags & FWA_CFG_DYNAMIC_GAP) ? ((const int64_t*)cols[e->c.gap_col])[i] : e->c.gap_ms;
    if (gap <= 0) return set_err(e, FWA_E_ARG, "Dynamic session time gap must satisfy 0 < gap");
    if (e->c.tz_n) ts = or_to_local(&e->c, ts);
    const int64_t nws = ts, nwe = jladd(ts, gap);
    int64_t cnt = 0;
    for (int64_t j = *wl_headp(e, key); j >= 0; j = e->wl_next[j]) cnt++;
    tw* ws = (tw*)malloc(sizeof(tw) * (cnt + 1));
    int64_t n = 0;
    for (int64_t j = *wl_headp(e, key); j >= 0; j = e->wl_next[j]) { ws[n].s = e->wl_start[j]; ws[n].e = e->wl_end[j]; n++; }
    ws[n].s = nws; ws[n].e = nwe; n++;
    qsort(ws, n, sizeof(tw), tw_cmp);                           /* sort by start */
    int64_t res_s = nws, res_e = nwe;
    int merged_new = 0, any_merge = 0;
    for (int64_t g0 = 0; g0 < n;) {
        int64_t cs = ws[g0].s, ce = ws[g0].e, g1 = g0 + 1;
        while (g1 < n && cs <= ws[g1].e && ce >= ws[g1].s) {    /* intersects (touching merges) -> cover */
            if (ws[g1].s < cs) cs = ws[g1].s;
            if (ws[g1].e > ce) ce = ws[g1].e;
            g1++;
        }
        /* the merge set is a HashSet: equal windows collapse */
        int64_t distinct = 0;
        for (int64_t q = g0; q < g1; q++) {
            int dup = 0;
            for (int64_t r = g0; r < q; r++) if (ws[r].s == ws[q].s && ws[r].e == ws[q].e) dup = 1;
            if (!dup) distinct++;
        }
        if (distinct > 1) {
            any_merge = 1;
            /* mergedWindows.remove(newWindow) */
            int has_new = 0;
            for (int64_t q = g0; q < g1; q++) if (ws[q].s == nws && ws[q].e == nwe) has_new = 1;
            if (has_new) { merged_new = 1; res_s = cs; res_e = ce; }
            /* remaining merged windows are all in-flight; the first one's state window survives */
            int64_t sws = 0, swe = 0; int have = 0, self_only = 0, nrem = 0;
            for (int64_t q = g0; q < g1; q++) {
                int64_t a, b;
                if (ws[q].s == nws && ws[q].e == nwe && !wl_get_state_window(e, key, ws[q].s, ws[q].e, &a, &b)) continue;
                if (!wl_get_state_window(e, key, ws[q].s, ws[q].e, &a, &b)) continue;
                if (!have) { sws = a; swe = b; have = 1; }
                nrem++;
                if (ws[q].s == cs && ws[q].e == ce) self_only = 1;
            }
            self_only = self_only && nrem == 1;
            if (!self_only) {
                /* MergeFunction.merge: lateness check, onMerge, clear merged triggers, mergeNamespaces */
                if (jladd(ev_time(e, jlsub(ce, 1)), e->c.allowed_lateness_ms) <= e->wm) {
                    free(ws);
                    return set_err(e, FWA_E_MERGE_LATE, "The end timestamp of an event-time window cannot become earlier than the current watermark by merging.");
                }
                if (ev_time(e, jlsub(ce, 1)) > e->wm) th_add(&e->timers, ev_time(e, jlsub(ce, 1)), key, cs, ce);   /* EventTimeTrigger.onMerge */
            }
            for (int64_t q = g0; q < g1; q++) {
                int64_t a, b;
                if (!wl_get_state_window(e, key, ws[q].s, ws[q].e, &a, &b)) continue;       /* the new window */
                if (!self_only) {
                    th_del(&e->timers, ev_time(e, jlsub(ws[q].e, 1)), key, ws[q].s, ws[q].e);   /* trigger.clear */
                    int64_t ct = cleanup_time(e, ws[q].s, ws[q].e);                       /* deleteCleanupTimer */
                    if (ct != J_LONG_MAX) th_del(&e->timers, ev_time(e, ct), key, ws[q].s, ws[q].e);
                    if (!(a == sws && b == swe)) {
                        aval* src = ds_state(e, key, a, b, 0);
                        if (src) { aval* dst = ds_state(e, key, sws, swe, 1); src = ds_state(e, key, a, b, 0); acc_merge(e, dst, src); ds_clear_state(e, key, a, b); }
                    }
                }
                wl_remove(e, key, ws[q].s, ws[q].e);
            }
            wl_put(e, key, cs, ce, sws, swe);
        }
        g0 = g1;
    }
    free(ws);
    if (!any_merge || (res_s == nws && res_e == nwe && !merged_new)) wl_put(e, key, nws, nwe, nws, nwe);
    if (ev_time(e, cleanup_time(e, res_s, res_e)) <= e->wm) { wl_remove(e, key, res_s, res_e); return FWA_OK; }   /* retireWindow */
    *skipped = 0;
    int64_t sws, swe;
    if (!wl_get_state_window(e, key, res_s, res_e, &sws, &swe)) return set_err(e, FWA_E_STATE, "Window is not in in-flight window set.");
    aval* a = ds_state(e, key, sws, swe, 1);
    acc_add(e, a, cols, i);
    int64_t max_ts = ev_time(e, jlsub(res_e, 1));
    if (max_ts <= e->wm) emit(e, key, res_s, res_e, a);           /* EventTimeTrigger.onElement FIRE */
    else th_add(&e->timers, max_ts, key, res_s, res_e);
    int64_t ct = cleanup_time(e, res_s, res_e);
    if (ct != J_LONG_MAX) th_add(&e->timers, ev_time(e, ct), key, res_s, res_e);
    return FWA_OK;
}

static void ds_on_event_time(or_engine* e, const timer_t_* t) {   /* WindowOperator.onEventTime :437-481 */
    int64_t key = t->key, ws = t->a, we = t->b;
    int64_t sws = ws, swe = we;
    if (e->c.window_kind == FWA_SESSION) {
        if (!wl_get_state_window(e, key, ws, we, &sws, &swe)) return;
    }
    aval* a = ds_state(e, key, sws, swe, 0);
    if (t->ts == ev_time(e, jlsub(we, 1)) && a) emit(e, key, ws, we, a);   /* EventTimeTrigger.onEventTime FIRE */
    if (t->ts == ev_time(e, cleanup_time(e, ws, we))) {            /* clearAllState :537-548 */
        ds_clear_state(e, key, sws, swe);
        th_del(&e->timers, ev_time(e, jlsub(we, 1)), key, ws, we);
        if (e->c.window_kind == FWA_SESSION) wl_remove(e, key, ws, we);
    }
}

/* ---------------- Table slicing window aggregation ---------------- */

static int64_t tb_slice_size(const fwa_config* c) {
    if (c->window_kind == FWA_TUMBLE) return c->size_ms;
    if (c->window_kind == FWA_SLIDE) return gcd64(c->size_ms, c->slide_ms);
    return c->slide_ms;
}
static int tb_is_fired_tz(const fwa_config* c, int64_t window_end, int64_t progress) {   /* TimeWindowUtil.isWindowFired :175-183 */
    if (window_end == J_LONG_MAX) return 0;
    return progress >= or_tz_timer(c, jlsub(window_end, 1));
}
#define tb_is_fired(we, pr) tb_is_fired_tz(&e->c, (we), (pr))
static int64_t tb_cum_window_start(const fwa_config* c, int64_t window_end) { return or_window_start(jlsub(window_end, 1), c->offset_ms, c->size_ms); }
static int64_t tb_last_window_end(const fwa_config* c, int64_t slice_end) {
    if (c->window_kind == FWA_TUMBLE) return slice_end;
    if (c->window_kind == FWA_SLIDE) return jladd(jlsub(slice_end, tb_slice_size(c)), c->size_ms);
    return jladd(tb_cum_window_start(c, slice_end), c->size_ms);
}
static int64_t tb_merge_target(const fwa_config* c, int64_t slice_end) {
    if (c->window_kind == FWA_CUMULATE) return jladd(tb_cum_window_start(c, slice_end), c->slide_ms);  /* first slice */
    return slice_end;
}
static aval* tb_state(or_engine* e, int64_t key, int64_t slice, int create) { return ds_state(e, key, slice, 0, create); }
static void tb_clear(or_engine* e, int64_t key, int64_t slice) { ds_clear_state(e, key, slice, 0); }
/* WindowTimerServiceImpl.registerEventTimeWindowTimer: the timer fires at toEpochMillsForTimer(windowEnd - 1) */
static void tb_register(or_engine* e, int64_t key, int64_t window_end) { th_add(&e->timers, or_tz_timer(&e->c, jlsub(window_end, 1)), key, window_end, 0); }

static int tb_process_element(or_engine* e, int64_t key, int64_t ts, const void* const* cols, int64_t i) {
    const fwa_config* c = &e->c;
    int64_t slice_end = or_assign_slice_end(c, ts);
    if (tb_is_fired(slice_end, e->wm)) {
        int64_t last = tb_last_window_end(c, slice_end);
        if (tb_is_fired(last, e->wm)) return 1;                     /* dropped */
        int64_t target = tb_merge_target(c, slice_end);
        acc_add(e, tb_state(e, key, target, 1), cols, i);
        int64_t unfired = slice_end;
        while (tb_is_fired(unfired, e->wm)) unfired = jladd(unfired, tb_slice_size(c));
        tb_register(e, key, unfired);
        return 0;
    }
    acc_add(e, tb_state(e, key, slice_end, 1), cols, i);            /* buffer -> AggCombiner.combine */
    if (!tb_is_fired(slice_end, e->wm)) tb_register(e, key, slice_end);
    return 0;
}

static void tb_fire(or_engine* e, int64_t key, int64_t window_end) {  /* SlicingWindowOperator.onTimer :257-264 */
    const fwa_config* c = &e->c;
    int64_t g = tb_slice_size(c);
    if (c->window_kind == FWA_TUMBLE) {                             /* SliceUnsharedWindowAggProcessor.fireWindow */
        aval* a = tb_state(e, key, window_end, 0);
        if (a) emit(e, key, jlsub(window_end, c->size_ms), window_end, a);
        else { int64_t id = acc_new(e); emit(e, key, jlsub(window_end, c->size_ms), window_end, &e->pool[id * e->nacc]); acc_free(e, id); }
        tb_clear(e, key, window_end);
        return;
    }
    int64_t tmp = acc_new(e);
    aval* acc = &e->pool[tmp * e->nacc];
    if (c->window_kind == FWA_SLIDE) {                              /* HoppingSlicesIterable, lastSliceEnd downwards */
        int64_t nslices = c->size_ms / g, s = window_end;
        for (int64_t q = 0; q < nslices; q++, s = jlsub(s, g)) { aval* sa = tb_state(e, key, s, 0); if (sa) acc_merge(e, acc, sa); }
        int empty = (acc[0].i == 0);
        if (!empty) emit(e, key, jlsub(window_end, c->size_ms), window_end, acc);
        if (!empty) tb_register(e, key, jladd(window_end, g));       /* nextTriggerWindow */
        /* expiredSlices: first slice of the window */
        tb_clear(e, key, jladd(jlsub(window_end, c->size_ms), g));
    } else {                                                        /* CUMULATE */
        int64_t wstart = tb_cum_window_start(c, window_end);
        int64_t first = jladd(wstart, c->slide_ms), last = jladd(wstart, c->size_ms);
        aval* fa = tb_state(e, key, first, 0);
        if (fa) acc_merge(e, acc, fa);
        if (window_end != first) {
            aval* sa = tb_state(e, key, window_end, 0);
            if (sa) acc_merge(e, acc, sa);
            /* the merged acc goes back into the first-slice state */
            aval* f2 = tb_state(e, key, first, 1);
            memcpy(f2, acc, sizeof(aval) * e->nacc);
            acc = &e->pool[tmp * e->nacc];
        }
        if (acc[0].i != 0) emit(e, key, wstart, window_end, acc);
        if (jladd(window_end, c->slide_ms) <= last) tb_register(e, key, jladd(window_end, c->slide_ms));
        if (window_end == first) { /* nothing expires */ }
        else if (window_end == last) { tb_clear(e, key, window_end); tb_clear(e, key, first); }
        else tb_clear(e, key, window_end);
    }
    acc_free(e, tmp);
}

/* ------------------------------------------------------------------ public API */

int or_push(or_engine* e, const int64_t* keys, const int64_t* ts, const void* const* cols,
            const int32_t* key_hash, int64_t n, int64_t* late_dropped_out) {
    return or_push_nullable(e, keys, ts, cols, NULL, key_hash, n, late_dropped_out);
}

int or_push_nullable(or_engine* e, const int64_t* keys, const int64_t* ts, const void* const* cols,
                     const uint8_t* const* nulls, const int32_t* key_hash, int64_t n, int64_t* late_dropped_out) {
    int64_t dropped = 0;
    e->nulls = nulls;
    e->late_n = 0;
    if (n > e->late_cap) { e->late_cap = n; e->late_idx = (int32_t*)realloc(e->late_idx, 4 * (size_t)n); }
    /* rows fired inside processElement (late firings, EventTimeTrigger.onElement :37-45) are kept and
       returned with the next or_advance_watermark, as the engine does */
    if (e->out_ret) { e->out_n = 0; e->out_ret = 0; }
    int64_t wsb[4096], web[4096];
    for (int64_t i = 0; i < n; i++) {
        int32_t kg = or_key_group(keys[i], e->c.key_kind, key_hash ? key_hash[i] : 0, e->c.max_parallelism);
        if (kg < e->c.kg_start || kg > e->c.kg_end) {
            char m[160]; snprintf(m, sizeof m, "Key group %d is not in KeyGroupRange{startKeyGroup=%d, endKeyGroup=%d}.", kg, e->c.kg_start, e->c.kg_end);
            return set_err(e, FWA_E_KEYGROUP, m);
        }
        e->st.records_in++;
        if (e->c.window_kind == FWA_SESSION) {
            /* DataStream EventTimeSessionWindows (no Long.MIN_VALUE check in its assignWindows :61-63) and the
             * Table legacy GROUP BY SESSION (TR WindowOperator.processElement :331-378 over
             * MergingWindowProcessFunction): the same MergingWindowSet walk and trigger */
            int skipped = 1;
            int rc = ds_process_element_session(e, keys[i], ts[i], cols, i, &skipped);
            if (rc) return rc;
            if (skipped && (e->c.semantics == FWA_SEM_TABLE ||                /* TR WindowOperator.java:386-389 */
                            jladd(ts[i], e->c.allowed_lateness_ms) <= e->wm)) {   /* isElementLate :597-601 */
                dropped++;
                e->late_idx[e->late_n++] = (int32_t)i;
            }
            continue;
        }
        if (e->c.semantics == FWA_SEM_TABLE) {
            if (tb_process_element(e, keys[i], ts[i], cols, i)) { dropped++; e->late_idx[e->late_n++] = (int32_t)i; }
            continue;
        }
        if (ts[i] == J_LONG_MIN) return set_err(e, FWA_E_TS_MIN, "Record has Long.MIN_VALUE timestamp (= no timestamp marker).");
        int skipped = 1;
        {
            int nw = or_assign_windows(&e->c, ts[i], wsb, web, 4096);
            if (nw < 0) return set_err(e, nw, "window assignment failed");
            ds_process_element_aligned(e, keys[i], ts[i], cols, i, wsb, web, nw, &skipped);
        }
        if (skipped && jladd(ts[i], e->c.allowed_lateness_ms) <= e->wm) {   /* isElementLate :597-601 */
            dropped++;
            e->late_idx[e->late_n++] = (int32_t)i;
        }
    }
    e->st.late_dropped += dropped;
    if (late_dropped_out) *late_dropped_out = dropped;
    e->nulls = NULL;
    return FWA_OK;
}

/* indices of the records the last or_push dropped as late (sideOutput / processElement() == true) */
int or_late_records(or_engine* e, const int32_t** idx, int64_t* n) { *idx = e->late_idx; *n = e->late_n; return FWA_OK; }

int or_advance_watermark(or_engine* e, int64_t wm, fwa_out* out) {
    if (e->out_ret) { e->out_n = 0; e->out_ret = 0; }
    if (wm > e->wm) {
        e->wm = wm;                                          /* InternalTimerServiceImpl.advanceWatermark :302-314 */
        timer_t_ t;
        while (th_pop_due(&e->timers, wm, &t)) {
            if (e->c.semantics == FWA_SEM_TABLE && e->c.window_kind != FWA_SESSION) tb_fire(e, t.key, t.a);
            else ds_on_event_time(e, &t);
        }
        e->st.current_watermark = wm;
    }
    if (out) {
        memset(out, 0, sizeof(*out));
        out->n_rows = e->out_n; out->on_device = 0; out->num_aggs = e->c.num_aggs;
        out->key = e->o_key; out->win_start = e->o_start; out->win_end = e->o_end;
        for (int j = 0; j < e->c.num_aggs; j++) {
            out->agg[j] = e->o_agg[j];
            const int kind = e->c.aggs[j].kind;
            if (((e->c.nullable_cols >> e->c.aggs[j].col & 1) && kind != FWA_COUNT && kind != FWA_COUNT_COL) || is_dec(kind))
                out->agg_null[j] = e->o_null[j];                 /* DECIMAL: NULL on overflow too */
        }
    }
    e->out_ret = 1;
    return FWA_OK;
}

int or_get_stats(or_engine* e, fwa_stats* st) {
    *st = e->st;
    st->live_slices = e->state.n;
    return FWA_OK;
}

/* ------------------------------------------------------------------ synthetic stream */

uint64_t or_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

void or_generate(const fwa_gen_params* p, int64_t n, int64_t* keys, int64_t* ts, int64_t* v_i64,
                 float* v_f32, double* v_f64, const double* cdf) {
    for (int64_t j = 0; j < n; j++) {
        uint64_t i = (uint64_t)(p->first_index + j);
        uint64_t hk = or_splitmix64(p->seed_k ^ i);
        int64_t key;
        if (p->key_dist == 0) key = (int64_t)(hk % (uint64_t)p->num_keys);
        else {
            double u = (double)(hk >> 11) * (1.0 / 9007199254740992.0);
            int64_t lo = 0, hi = p->num_keys - 1;
            while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (cdf[mid] > u) hi = mid; else lo = mid + 1; }
            key = lo;
        }
        keys[j] = key;
        int64_t ramp = (int64_t)(((__int128)(int64_t)i * p->span_ms) / p->total_records);
        ts[j] = p->t0_ms + ramp - (int64_t)(or_splitmix64(p->seed_t ^ i) % (uint64_t)(p->max_delay_ms + 1));
        uint64_t hv = or_splitmix64(p->seed_v ^ i);
        if (v_i64) v_i64[j] = (int64_t)(hv >> 33);
        if (v_f32) v_f32[j] = (float)(hv >> 40) * (1.0f / 16777216.0f);
        if (v_f64) v_f64[j] = (double)(or_splitmix64(hv) >> 11) * (1.0 / 9007199254740992.0);
    }
}

/* ------------------------------------------------------------------ threaded CPU baseline */

typedef struct {
    const fwa_config* cfg; int idx, nthreads;
    int64_t n; int64_t batch;
    int64_t** bk; int64_t** bt; int64_t** bv; int64_t* bn;   /* per-batch partitions for this thread */
    int64_t nbatches; int64_t* wms;
    int64_t rows; uint64_t checksum;
} bench_arg;

/* Order-free digest of one fired row (key, window, int64 aggregates): a linear mix of the fields with odd constants,
   then a 64-bit finalizer; a watermark's digest is the sum mod 2^64 over its rows, so emission order (unspecified in
   the reference, TimerHeapInternalTimer.comparePriorityTo) does not matter. Restated by tests/digest.py (torch). */
uint64_t or_row_digest(int64_t key, int64_t start, int64_t end, const int64_t* aggs, int naggs) {
    uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull + (uint64_t)start * 0xC2B2AE3D27D4EB4Full +
                 (uint64_t)end * 0x165667B19E3779F9ull;
    for (int j = 0; j < naggs; j++) h += (uint64_t)aggs[j] * (0xD6E8FEB86659FD93ull + 2ull * (uint64_t)j);
    h ^= h >> 33; h *= 0xC4CEB9FE1A85EC53ull; h ^= h >> 29; h *= 0x94D049BB133111EBull; h ^= h >> 32;
    return h;
}

static void* bench_worker(void* vp) {
    bench_arg* a = (bench_arg*)vp;
    fwa_config c = *a->cfg;
    or_key_group_range(c.max_parallelism, a->nthreads, a->idx, &c.kg_start, &c.kg_end);
    or_engine* e; or_create(&c, &e);
    fwa_out o;
    for (int64_t b = 0; b < a->nbatches; b++) {
        const void* cols[1] = {a->bv[b]};
        or_push(e, a->bk[b], a->bt[b], cols, NULL, a->bn[b], NULL);
        or_advance_watermark(e, a->wms[b], &o);
        a->rows += o.n_rows;
        for (int64_t r = 0; r < o.n_rows; r++) a->checksum += (uint64_t)o.key[r] * 31u + (uint64_t)o.win_end[r] + (c.num_aggs ? (uint64_t)((const aval*)o.agg[c.num_aggs - 1])[r].i : 0);
    }
    or_destroy(e);
    return NULL;
}

double or_bench_pipeline(const fwa_config* cfg, const fwa_gen_params* p, int64_t n, int64_t batch,
                         int threads, int64_t* rows_out, uint64_t* checksum_out) {
    int64_t nb = (n + batch - 1) / batch;
    int64_t* keys = (int64_t*)malloc(8 * batch); int64_t* ts = (int64_t*)malloc(8 * batch); int64_t* vv = (int64_t*)malloc(8 * batch);
    bench_arg* args = (bench_arg*)calloc(threads, sizeof(bench_arg));
    int64_t* wms = (int64_t*)malloc(8 * (nb + 1));
    for (int t = 0; t < threads; t++) {
        args[t].cfg = cfg; args[t].idx = t; args[t].nthreads = threads; args[t].nbatches = nb + 1; args[t].wms = wms;
        args[t].bk = (int64_t**)calloc(nb + 1, sizeof(void*)); args[t].bt = (int64_t**)calloc(nb + 1, sizeof(void*));
        args[t].bv = (int64_t**)calloc(nb + 1, sizeof(void*)); args[t].bn = (int64_t*)calloc(nb + 1, 8);
    }
    /* generate + keyBy partition (KeyGroupStreamPartitioner.selectChannel) up front: untimed */
    int64_t max_ts = J_LONG_MIN;
    int maxp = cfg->max_parallelism > 0 ? cfg->max_parallelism : 128;
    int32_t* dest = (int32_t*)malloc(4 * batch);
    for (int64_t b = 0; b < nb; b++) {
        int64_t m = (b == nb - 1) ? n - b * batch : batch;
        fwa_gen_params q = *p; q.first_index = p->first_index + b * batch;
        or_generate(&q, m, keys, ts, vv, NULL, NULL, NULL);
        int64_t* cnt = (int64_t*)calloc(threads, 8);
        for (int64_t i = 0; i < m; i++) {
            int kg = or_key_group(keys[i], cfg->key_kind, 0, maxp);
            dest[i] = or_operator_index(maxp, threads, kg); cnt[dest[i]]++;
            if (ts[i] > max_ts) max_ts = ts[i];
        }
        for (int t = 0; t < threads; t++) {
            args[t].bk[b] = (int64_t*)malloc(8 * (cnt[t] + 1)); args[t].bt[b] = (int64_t*)malloc(8 * (cnt[t] + 1));
            args[t].bv[b] = (int64_t*)malloc(8 * (cnt[t] + 1)); args[t].bn[b] = 0;
        }
        for (int64_t i = 0; i < m; i++) {
            bench_arg* a = &args[dest[i]]; int64_t k = a->bn[b]++;
            a->bk[b][k] = keys[i]; a->bt[b][k] = ts[i]; a->bv[b][k] = vv[i];
        }
        free(cnt);
        wms[b] = max_ts - p->max_delay_ms - 1;                 /* BoundedOutOfOrdernessWatermarks :57-69 */
    }
    for (int t = 0; t < threads; t++) { args[t].bk[nb] = keys; args[t].bt[nb] = ts; args[t].bv[nb] = vv; args[t].bn[nb] = 0; }
    wms[nb] = J_LONG_MAX;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, bench_worker, &args[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    int64_t rows = 0; uint64_t cs = 0;
    for (int t = 0; t < threads; t++) {
        rows += args[t].rows; cs += args[t].checksum;
        for (int64_t b = 0; b < nb; b++) { free(args[t].bk[b]); free(args[t].bt[b]); free(args[t].bv[b]); }
        free(args[t].bk); free(args[t].bt); free(args[t].bv); free(args[t].bn);
    }
    free(th); free(args); free(keys); free(ts); free(vv); free(wms); free(dest);
    if (rows_out) *rows_out = rows;
    if (checksum_out) *checksum_out = cs;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}


typedef struct {
    const fwa_config* cfg; const fwa_gen_params* p; int idx, nthreads;
    int64_t n, batch, nb;
    int64_t* wrows; uint64_t* wdig;     /* [nb + 1] */
    int rc;
} digest_arg;

/* One operator instance (a key-group range) over the generated stream: every worker generates each batch itself and
   keeps its own key groups, so the set-up is parallel and memory stays one batch per thread. */
static void* digest_worker(void* vp) {
    digest_arg* a = (digest_arg*)vp;
    fwa_config c = *a->cfg;
    const int maxp = c.max_parallelism > 0 ? c.max_parallelism : 128;
    c.max_parallelism = maxp;
    or_key_group_range(maxp, a->nthreads, a->idx, &c.kg_start, &c.kg_end);
    or_engine* e;
    a->rc = or_create(&c, &e);
    if (a->rc) return NULL;
    int64_t* keys = (int64_t*)malloc(8 * a->batch); int64_t* ts = (int64_t*)malloc(8 * a->batch);
    int64_t* vv = (int64_t*)malloc(8 * a->batch);
    int64_t max_ts = J_LONG_MIN;
    fwa_out o;
    int64_t av[FWA_MAX_AGGS];
    for (int64_t b = 0; b <= a->nb; b++) {
        int64_t m = 0, wm = J_LONG_MAX;
        if (b < a->nb) {
            const int64_t cnt = (b == a->nb - 1) ? a->n - b * a->batch : a->batch;
            fwa_gen_params q = *a->p; q.first_index = a->p->first_index + b * a->batch;
            or_generate(&q, cnt, keys, ts, vv, NULL, NULL, NULL);
            for (int64_t i = 0; i < cnt; i++) {
                if (ts[i] > max_ts) max_ts = ts[i];
                const int kg = or_key_group(keys[i], c.key_kind, 0, maxp);
                if (kg < c.kg_start || kg > c.kg_end) continue;
                keys[m] = keys[i]; ts[m] = ts[i]; vv[m] = vv[i]; m++;
            }
            wm = max_ts - a->p->max_delay_ms - 1;                   /* BoundedOutOfOrdernessWatermarks :57-69 */
        }
        const void* cols[1] = {vv};
        if ((a->rc = or_push(e, keys, ts, cols, NULL, m, NULL)) != 0) break;
        if ((a->rc = or_advance_watermark(e, wm, &o)) != 0) break;
        uint64_t d = 0;
        for (int64_t r = 0; r < o.n_rows; r++) {
            for (int j = 0; j < c.num_aggs; j++) av[j] = ((const aval*)o.agg[j])[r].i;   /* 16-byte result slots */
            d += or_row_digest(o.key[r], o.win_start[r], o.win_end[r], av, c.num_aggs);
        }
        a->wdig[b] = d; a->wrows[b] = o.n_rows;
    }
    free(keys); free(ts); free(vv);
    or_destroy(e);
    return NULL;
}

/* The generated stream's fired rows per watermark, as (row count, or_row_digest sum) for each of the ceil(n / batch)
   batch watermarks (max_ts - D - 1) and the final Long.MAX_VALUE one (nb + 1 entries), `threads` operator instances
   over key-group ranges: the full-size parity check of the benched configurations (tests/test_full_size_digests_gpu.py).
   Aggregates must be int64 (COUNT / SUM(BIGINT) / MIN / MAX over BIGINT). */
double or_pipeline_digests(const fwa_config* cfg, const fwa_gen_params* p, int64_t n, int64_t batch, int threads,
                           int64_t* wm_rows, uint64_t* wm_dig) {
    const int64_t nb = (n + batch - 1) / batch;
    digest_arg* args = (digest_arg*)calloc(threads, sizeof(digest_arg));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        args[t] = (digest_arg){cfg, p, t, threads, n, batch, nb, (int64_t*)calloc(nb + 1, 8), (uint64_t*)calloc(nb + 1, 8), 0};
        pthread_create(&th[t], NULL, digest_worker, &args[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int64_t b = 0; b <= nb; b++) { wm_rows[b] = 0; wm_dig[b] = 0; }
    for (int t = 0; t < threads; t++) {
        if (args[t].rc && !rc) rc = args[t].rc;
        for (int64_t b = 0; b <= nb; b++) { wm_rows[b] += args[t].wrows[b]; wm_dig[b] += args[t].wdig[b]; }
        free(args[t].wrows); free(args[t].wdig);
    }
    free(args); free(th);
    if (rc) return (double)rc;              /* an FWA_E_* code (negative) */
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------ full-size digests, general form */

/* The benched configurations C3 / C5 / C5s at full size (tests/test_full_size_digests_gpu.py): Zipf keys (the CDF the
   device generator samples), the float value columns (f32 column 0, f64 column 1), any window kind. Per batch the T
   threads first generate a 1/T share of the batch each (with its key groups; the Zipf binary search is the costly
   part, done once), then each thread runs one operator instance over its key-group range of the whole batch
   (KeyGroupStreamPartitioner.selectChannel), as or_pipeline_digests does. Per watermark: the row count, the order-free
   digest of (key, start, end, the aggregates in exact_mask -- their 8-byte result words) and, for the aggregates in
   sum_mask (double results: SUM / AVG over a DOUBLE, whose GPU order of additions differs), per bucket of rows
   (bucket = or_row_digest(key, start, 0) & (nbuckets - 1)) the sum of the values and of their magnitudes. */
typedef struct {
    const fwa_config* cfg; const fwa_gen_params* p; const double* cdf;
    int idx, nthreads, fp;
    int64_t n, batch, nb;
    uint32_t exact_mask, sum_mask; int nbuckets, nsum;
    /* shared batch buffers */
    int64_t* keys; int64_t* ts; int64_t* vi; float* vf; double* vd; int16_t* kg; int64_t* tmax;
    pthread_barrier_t* bar;
    int64_t* wrows; uint64_t* wdig; double* wbsum; double* wbabs;   /* [nb + 1] ([nsum][nbuckets]) */
    int rc;
} digest2_arg;

static void* digest2_worker(void* vp) {
    digest2_arg* a = (digest2_arg*)vp;
    fwa_config c = *a->cfg;
    const int maxp = c.max_parallelism > 0 ? c.max_parallelism : 128;
    c.max_parallelism = maxp;
    or_key_group_range(maxp, a->nthreads, a->idx, &c.kg_start, &c.kg_end);
    or_engine* e = NULL;
    a->rc = or_create(&c, &e);
    int64_t* mk = (int64_t*)malloc(8 * a->batch); int64_t* mt = (int64_t*)malloc(8 * a->batch);
    int64_t* mi = (int64_t*)malloc(8 * a->batch); float* mf = (float*)malloc(4 * a->batch);
    double* md = (double*)malloc(8 * a->batch);
    int64_t max_ts = J_LONG_MIN;
    fwa_out o;
    int64_t av[FWA_MAX_AGGS];
    for (int64_t b = 0; b <= a->nb; b++) {
        int64_t m = 0, wm = J_LONG_MAX;
        if (b < a->nb) {
            const int64_t cnt = (b == a->nb - 1) ? a->n - b * a->batch : a->batch;
            /* phase G: this thread's share of the batch */
            const int64_t lo = cnt * a->idx / a->nthreads, hi = cnt * (a->idx + 1) / a->nthreads;
            fwa_gen_params q = *a->p; q.first_index = a->p->first_index + b * a->batch + lo;
            or_generate(&q, hi - lo, a->keys + lo, a->ts + lo, a->fp ? NULL : a->vi + lo, a->fp ? a->vf + lo : NULL,
                        a->fp ? a->vd + lo : NULL, a->cdf);
            int64_t tm = J_LONG_MIN;
            for (int64_t i = lo; i < hi; i++) {
                a->kg[i] = (int16_t)or_key_group(a->keys[i], c.key_kind, 0, maxp);
                if (a->ts[i] > tm) tm = a->ts[i];
            }
            a->tmax[a->idx] = tm;
            pthread_barrier_wait(a->bar);
            /* phase O: this operator instance's records of the whole batch, in arrival order */
            for (int t = 0; t < a->nthreads; t++) if (a->tmax[t] > max_ts) max_ts = a->tmax[t];
            for (int64_t i = 0; i < cnt; i++) {
                if (a->kg[i] < c.kg_start || a->kg[i] > c.kg_end) continue;
                mk[m] = a->keys[i]; mt[m] = a->ts[i];
                if (a->fp) { mf[m] = a->vf[i]; md[m] = a->vd[i]; } else mi[m] = a->vi[i];
                m++;
            }
            pthread_barrier_wait(a->bar);   /* the shared buffers are free for the next batch */
            wm = max_ts - a->p->max_delay_ms - 1;                   /* BoundedOutOfOrdernessWatermarks :57-69 */
        }
        if (a->rc) continue;                                     /* (keep meeting the barriers) */
        /* integer streams: column 1 is the timestamp (bench.py --config reduce keeps it as the tuple's f2) */
        const void* cols[2] = {a->fp ? (const void*)mf : (const void*)mi, a->fp ? (const void*)md : (const void*)mt};
        if ((a->rc = or_push(e, mk, mt, cols, NULL, m, NULL)) != 0) continue;
        if ((a->rc = or_advance_watermark(e, wm, &o)) != 0) continue;
        uint64_t d = 0;
        double* bs = a->wbsum + (size_t)b * a->nsum * a->nbuckets;
        double* ba = a->wbabs + (size_t)b * a->nsum * a->nbuckets;
        for (int64_t r = 0; r < o.n_rows; r++) {
            int k = 0, s = 0;
            const uint64_t bk = or_row_digest(o.key[r], o.win_start[r], 0, NULL, 0) & (uint64_t)(a->nbuckets - 1);
            for (int j = 0; j < c.num_aggs; j++) {
                const aval* x = &((const aval*)o.agg[j])[r];
                if (a->exact_mask >> j & 1u) av[k++] = x->i;
                if (a->sum_mask >> j & 1u) {
                    bs[(size_t)s * a->nbuckets + bk] += x->d;
                    ba[(size_t)s * a->nbuckets + bk] += fabs(x->d);
                    s++;
                }
            }
            d += or_row_digest(o.key[r], o.win_start[r], o.win_end[r], av, k);
        }
        a->wdig[b] = d; a->wrows[b] = o.n_rows;
    }
    free(mk); free(mt); free(mi); free(mf); free(md);
    if (e) or_destroy(e);
    return NULL;
}

double or_pipeline_digests2(const fwa_config* cfg, const fwa_gen_params* p, const double* cdf, int float_cols,
                            uint32_t exact_mask, uint32_t sum_mask, int nbuckets, int64_t n, int64_t batch, int threads,
                            int64_t* wm_rows, uint64_t* wm_dig, double* wm_bsum, double* wm_babs) {
    const int64_t nb = (n + batch - 1) / batch;
    int nsum = 0;
    for (int j = 0; j < 32; j++) nsum += (sum_mask >> j) & 1u;
    if (nbuckets < 1 || (nbuckets & (nbuckets - 1)) || (p->key_dist && !cdf)) return (double)FWA_E_ARG;
    digest2_arg* args = (digest2_arg*)calloc(threads, sizeof(digest2_arg));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    int64_t* keys = (int64_t*)malloc(8 * batch); int64_t* ts = (int64_t*)malloc(8 * batch);
    int64_t* vi = float_cols ? NULL : (int64_t*)malloc(8 * batch);
    float* vf = float_cols ? (float*)malloc(4 * batch) : NULL;
    double* vd = float_cols ? (double*)malloc(8 * batch) : NULL;
    int16_t* kg = (int16_t*)malloc(2 * batch);
    int64_t* tmax = (int64_t*)calloc(threads, 8);
    const size_t bsz = (size_t)(nb + 1) * nsum * nbuckets;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        args[t] = (digest2_arg){cfg, p, cdf, t, threads, float_cols != 0, n, batch, nb, exact_mask, sum_mask, nbuckets,
                                nsum, keys, ts, vi, vf, vd, kg, tmax, &bar, (int64_t*)calloc(nb + 1, 8),
                                (uint64_t*)calloc(nb + 1, 8), (double*)calloc(bsz + 1, 8), (double*)calloc(bsz + 1, 8), 0};
        pthread_create(&th[t], NULL, digest2_worker, &args[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int64_t b = 0; b <= nb; b++) { wm_rows[b] = 0; wm_dig[b] = 0; }
    for (size_t i = 0; i < bsz; i++) { wm_bsum[i] = 0.0; wm_babs[i] = 0.0; }
    for (int t = 0; t < threads; t++) {
        if (args[t].rc && !rc) rc = args[t].rc;
        for (int64_t b = 0; b <= nb; b++) { wm_rows[b] += args[t].wrows[b]; wm_dig[b] += args[t].wdig[b]; }
        for (size_t i = 0; i < bsz; i++) { wm_bsum[i] += args[t].wbsum[i]; wm_babs[i] += args[t].wbabs[i]; }
        free(args[t].wrows); free(args[t].wdig); free(args[t].wbsum); free(args[t].wbabs);
    }
    pthread_barrier_destroy(&bar);
    free(args); free(th); free(keys); free(ts); free(vi); free(vf); free(vd); free(kg); free(tmax);
    if (rc) return (double)rc;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
