// java_math.h -- bit-exact Java integer semantics for the gfx950 kernels (host+device).
//
//   murmur_hash     MathUtils.murmurHash(int)          flink-core/.../util/MathUtils.java:137-155
//   bit_mix         MathUtils.bitMix(int)              MathUtils.java:194-201
//   long_hash       java.lang.Long.hashCode            (JLS: (int)(v ^ (v >>> 32)))
//   binrow_hash     BinaryRowData.hashCode, 1 BIGINT   BinaryRowData.java:452-454 -> MurmurHashUtils.java:92-170
//   key_group       KeyGroupRangeAssignment.computeKeyGroupForKeyHash  KeyGroupRangeAssignment.java:75-77
//   window_start    TimeWindow.getWindowStartWithOffset TimeWindow.java:264-272 (Java '%' on negatives)
//
// 64-bit '%' by a runtime-constant divisor is done with a precomputed multiply-high "magic"
// (round-up method, 65-bit magic handled with the add-and-shift fix-up), so the per-record window
// assignment costs a few 32-bit MULs instead of a ~100-instruction 64-bit division loop.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define JM_HD __host__ __device__ __forceinline__
#else
#define JM_HD static inline
#endif

namespace jm {

JM_HD int32_t rotl32(int32_t x, int r) {
    uint32_t u = (uint32_t)x;
    return (int32_t)((u << r) | (u >> (32 - r)));
}
JM_HD int32_t imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

JM_HD int32_t bit_mix(int32_t in) {
    uint32_t u = (uint32_t)in;
    u ^= u >> 16;
    u *= 0x85ebca6bu;
    u ^= u >> 13;
    u *= 0xc2b2ae35u;
    u ^= u >> 16;
    return (int32_t)u;
}

JM_HD int32_t murmur_hash(int32_t code) {
    uint32_t c = (uint32_t)code;
    c *= 0xcc9e2d51u;
    c = (c << 15) | (c >> 17);
    c *= 0x1b873593u;
    c = (c << 13) | (c >> 19);
    c = c * 5u + 0xe6546b64u;
    c ^= 4u;
    int32_t r = bit_mix((int32_t)c);
    if (r >= 0) return r;
    if (r != (int32_t)0x80000000) return -r;
    return 0;
}

JM_HD int32_t long_hash(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32)); }

JM_HD uint32_t mh_k1(uint32_t k1) {
    k1 *= 0xcc9e2d51u;
    k1 = (k1 << 15) | (k1 >> 17);
    return k1 * 0x1b873593u;
}
JM_HD uint32_t mh_h1(uint32_t h1, uint32_t k1) {
    h1 ^= k1;
    h1 = (h1 << 13) | (h1 >> 19);
    return h1 * 5u + 0xe6546b64u;
}
// BinaryRowData(arity 1, BIGINT): words [0, 0, lo32, hi32] (LE), seed 42, fmix(h ^ 16)
JM_HD int32_t binrow_bigint_hash(int64_t v) {
    uint32_t h = 42u;
    h = mh_h1(h, mh_k1(0u));
    h = mh_h1(h, mh_k1(0u));
    h = mh_h1(h, mh_k1((uint32_t)((uint64_t)v & 0xffffffffu)));
    h = mh_h1(h, mh_k1((uint32_t)((uint64_t)v >> 32)));
    h ^= 16u;
    return bit_mix((int32_t)h);  // MurmurHashUtils.fmix(int) == MathUtils.bitMix
}

// BinaryRowData of `arity` fixed-length fields (BinaryRowData.java:68-123): an 8-byte header (byte 0 = RowKind
// INSERT = 0, then one null bit per field from bit 8 on) and one 8-byte little-endian slot per field (BIGINT, DOUBLE
// raw bits; INT in the low 4 bytes; a NULL field's slot zeroed, BinaryRowWriter.setNullAt); hashCode() =
// MurmurHashUtils.hashBytesByWords(row, 8 + 8 * arity bytes, seed 42) (:92-170): every 4-byte little-endian word
// mixed in order, then fmix(h ^ length). `slots[i]` is field i's slot, `nullbits` bit i = field i is NULL (arity <= 56).
JM_HD int32_t binrow_hash(const uint64_t* slots, int arity, uint64_t nullbits) {
    uint32_t h = 42u;
    const uint64_t hdr = nullbits << 8;                   // RowKind byte 0, null bits from bit 8
    h = mh_h1(h, mh_k1((uint32_t)hdr));
    h = mh_h1(h, mh_k1((uint32_t)(hdr >> 32)));
    for (int i = 0; i < arity; ++i) {
        const uint64_t v = (nullbits >> i) & 1 ? 0ull : slots[i];
        h = mh_h1(h, mh_k1((uint32_t)v));
        h = mh_h1(h, mh_k1((uint32_t)(v >> 32)));
    }
    h ^= (uint32_t)(8 + 8 * arity);
    return bit_mix((int32_t)h);
}

// key_kind: 0 JAVA_LONG, 1 BINROW_BIGINT, 2 PREHASHED (hash supplied), 3 GROUP_PREFIXED (key ids of a key
// dictionary, fwa_keydict: the key group in the top 16 bits; an id whose key group is >= max_par -- a dictionary
// created with another max parallelism, or not a dictionary id at all -- has key group -1, which no subtask owns)
JM_HD int32_t key_hash(int64_t key, int key_kind, int32_t supplied) {
    return key_kind == 0 ? long_hash(key) : (key_kind == 1 ? binrow_bigint_hash(key) : supplied);
}
JM_HD int32_t key_group(int32_t hash, int32_t max_par) { return murmur_hash(hash) % max_par; }
JM_HD int32_t key_group_of(int64_t key, int key_kind, int32_t supplied, int32_t max_par) {
    if (key_kind == 3) {
        const int32_t kg = (int32_t)((uint64_t)key >> 48);
        return kg < max_par ? kg : -1;
    }
    return key_group(key_hash(key, key_kind, supplied), max_par);
}
JM_HD int32_t operator_index(int32_t max_par, int32_t par, int32_t kg) { return kg < 0 ? -1 : kg * par / max_par; }

// ---- 64-bit unsigned division by a runtime constant -------------------------------------------

JM_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

struct UDiv64 {
    uint64_t d;      // divisor (>0)
    uint64_t magic;  // low 64 bits of the 65-bit magic (when add==1)
    int32_t shift;
    int32_t mode;    // 0: power of two (shift only), 1: q = mulhi >> shift, 2: add fix-up
};

// Host-side precomputation (round-up method, Granlund-Montgomery / libdivide "u64 gen").
static inline UDiv64 udiv64_make(uint64_t d) {
    UDiv64 r;
    r.d = d;
    r.magic = 0;
    r.shift = 0;
    r.mode = 0;
    int lg = 63;
    while (lg > 0 && !((d >> lg) & 1)) lg--;
    if ((d & (d - 1)) == 0) {
        r.shift = lg;
        r.mode = 0;
        return r;
    }
    // 2^(64+lg) / d
    unsigned __int128 num = ((unsigned __int128)1) << (64 + lg);
    uint64_t m = (uint64_t)(num / d);
    uint64_t rem = (uint64_t)(num - (unsigned __int128)m * d);
    uint64_t e = d - rem;
    if (e < ((uint64_t)1 << lg)) {
        r.magic = m + 1;
        r.shift = lg;
        r.mode = 1;
    } else {
        // 65-bit magic: 2*m + (2*rem >= d), add-indicator path
        uint64_t m2 = m + m;
        uint64_t twice_rem = rem + rem;
        if (twice_rem >= d || twice_rem < rem) m2 += 1;
        r.magic = m2 + 1;
        r.shift = lg;
        r.mode = 2;
    }
    return r;
}

JM_HD uint64_t udiv64(uint64_t n, const UDiv64& dv) {
    if (dv.mode == 0) return n >> dv.shift;
    uint64_t q = mulhi64(dv.magic, n);
    if (dv.mode == 1) return q >> dv.shift;
    uint64_t t = ((n - q) >> 1) + q;
    return t >> dv.shift;
}

// Java long '%' by positive d (sign follows the dividend), with d given as a magic divider.
JM_HD int64_t jrem(int64_t a, const UDiv64& dv) {
    uint64_t ua = a < 0 ? (uint64_t)0 - (uint64_t)a : (uint64_t)a;
    uint64_t q = udiv64(ua, dv);
    uint64_t ur = ua - q * dv.d;
    return a < 0 ? -(int64_t)ur : (int64_t)ur;
}

// TimeWindow.getWindowStartWithOffset(ts, offset, size) with Java wrap-around arithmetic.
JM_HD int64_t window_start(int64_t ts, int64_t offset, const UDiv64& size) {
    int64_t rem = jrem((int64_t)((uint64_t)ts - (uint64_t)offset), size);
    if (rem < 0) return (int64_t)((uint64_t)ts - ((uint64_t)rem + size.d));
    return (int64_t)((uint64_t)ts - (uint64_t)rem);
}

JM_HD int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
JM_HD int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

// Order-preserving map of i64 / f64 / f32 to u64, so MIN/MAX can use unsigned atomicMin/Max
// with memset-able identities (0xFF.. for MIN, 0x00.. for MAX).
JM_HD uint64_t ord_i64(int64_t x) { return (uint64_t)x ^ 0x8000000000000000ull; }
JM_HD int64_t unord_i64(uint64_t u) { return (int64_t)(u ^ 0x8000000000000000ull); }
JM_HD uint64_t ord_bits64(uint64_t b) { return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull); }
JM_HD uint64_t unord_bits64(uint64_t u) { return (u & 0x8000000000000000ull) ? (u & 0x7fffffffffffffffull) : ~u; }

// A strong 64-bit mix for the engine's own hash tables (independent of Flink's key-group hash).
JM_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
JM_HD uint64_t splitmix64(uint64_t x) { return mix64(x + 0x9e3779b97f4a7c15ull); }

// ---- shift time zone of a TIMESTAMP_LTZ rowtime (Table), TimeWindowUtil.java:52-100 ----
// tz: n pairs (utc_instant_ms, offset_ms), ascending by instant; pair i's offset applies from its instant
// until the next pair's (pair 0 also before its instant). n == 0: UTC.
JM_HD int64_t tz_offset_at(const int64_t* tz, int n, int64_t instant) {   // ZoneRules.getOffset(Instant)
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tz[2 * mid] <= instant) lo = mid; else hi = mid - 1;
    }
    return tz[2 * lo + 1];
}
// toUtcTimestampMills: the local wall-clock time of an instant, as epoch millis of that time in UTC.
JM_HD int64_t tz_to_local(const int64_t* tz, int n, int64_t epoch) {
    if (n == 0 || epoch == INT64_MAX) return epoch;          // Long.MAX_VALUE: the max-watermark flag
    return wadd(epoch, tz_offset_at(tz, n, epoch));
}
// LocalDateTime.atZone(zone).toInstant() (ZonedDateTime.ofLocal, no preferred offset): a unique offset ->
// local - offset; a gap -> shifted later by the gap (local - offset before); an overlap -> the earlier offset.
JM_HD int64_t tz_at_zone(const int64_t* tz, int n, int64_t local) {
    int j = 0;                                                // last segment whose local range starts <= local
    for (int lo = 1, hi = n - 1; lo <= hi;) {
        const int mid = (lo + hi) >> 1;
        if (wadd(tz[2 * mid], tz[2 * mid + 1]) <= local) { j = mid; lo = mid + 1; } else hi = mid - 1;
    }
    if (j > 0 && local < wadd(tz[2 * j], tz[2 * (j - 1) + 1])) return wsub(local, tz[2 * (j - 1) + 1]);   // overlap
    return wsub(local, tz[2 * j + 1]);
}
// toEpochMillsForTimer: the instant a local window time triggers at; with daylight saving (more than one
// offset in the table) the gap / overlap hours follow TimeWindowUtil.java:74-95.
JM_HD int64_t tz_timer(const int64_t* tz, int n, int64_t local) {
    if (n == 0 || local == INT64_MAX) return local;
    if (n == 1) return wsub(local, tz[1]);
    const int64_t hour = 3600000;
    const int64_t t1 = tz_at_zone(tz, n, local), t2 = tz_at_zone(tz, n, wadd(local, hour));
    if (t1 == t2) return t1 - t1 % hour;                      // no epoch maps to this local time
    if (t2 - t1 > hour) return t1 + hour;                     // two epochs: the later one
    return t1;
}

}  // namespace jm
