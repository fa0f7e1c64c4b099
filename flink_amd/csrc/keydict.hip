// keydict.hip -- the key dictionary of include/flink_amd.h (multi-column Table keys).
//
// A key row of `arity` fixed-length fields becomes the 8-byte slots of its BinaryRowData (BinaryRowData.java:68-123):
// BIGINT as is, INT zero-extended (the low 4 bytes of its slot), DOUBLE as its raw bits, a NULL field as 0 with its
// null bit set. hashCode() is jm::binrow_hash (MurmurHashUtils.hashBytesByWords over those bytes); its key group is
// KeyGroupRangeAssignment.assignToKeyGroup (murmur % maxParallelism). The row's identity is a 64-bit hash of the same
// bytes; an encode runs three passes, each a kernel, so a pass only reads what an earlier launch finished writing:
//   kd_insert_kernel  every row claims or finds its identity in the open-addressing table (one CAS per row);
//   kd_assign_kernel  the rows that claimed a slot take a sequence number (one reservation per wave), store the
//                     row's slots and publish id = key group << 48 | sequence in the table;
//   kd_lookup_kernel  every row reads its id, checks its slots against the stored row (a different row with the
//                     same 64-bit hash raises FWA_E_STATE) and writes its id and hash.
// STRING fields (FWA_KEY_FIELD_STRING): a value of up to 7 bytes is its BinaryRowData slot (0x80 | length in the top
// byte, the bytes below); a longer one is identified by a 63-bit hash of its bytes (top bit clear: never a short
// slot) and stored in the dictionary's byte heap, its slot word then length << 40 | heap offset. hashCode() is
// computed over the row as BinaryRowWriter lays it out (kd_row_hash): the long values' slots are offset << 32 |
// length with the offsets of the row's variable-length part, which holds the bytes zero-padded to 8.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "../../include/flink_amd.h"
#include "java_math.h"

namespace {

constexpr int kBlockKd = 256;
constexpr uint64_t kKdEmpty = 0ull;
constexpr uint64_t kSeqMask = (1ull << 48) - 1;
constexpr int64_t kStrMax = (1 << 23) - 1;        // longest STRING value (its length field in the stored word)
constexpr uint64_t kHeapMask = (1ull << 40) - 1;

struct KdCols {
    const void* col[FWA_KEYDICT_MAX_ARITY];
    const uint8_t* nul[FWA_KEYDICT_MAX_ARITY];
    int32_t type[FWA_KEYDICT_MAX_ARITY];
    int32_t arity, has_str;
    const int32_t* soff[FWA_KEYDICT_MAX_ARITY];    // STRING fields: Arrow offsets / bytes
    const uint8_t* sbytes[FWA_KEYDICT_MAX_ARITY];
};

struct KdDev {
    unsigned long long* ht_key;    // [cap] row identity (0 = empty)
    long long* ht_id;              // [cap] id, published by the assign pass
    uint32_t* ht_rep;              // [cap] the row that claimed the slot (this encode only)
    unsigned long long* fslot;     // [arity][max_rows] stored slots
    unsigned long long* fnull;     // [max_rows] stored null bits
    unsigned long long* nrows;     // distinct rows so far
    uint32_t* pos;                 // [n] per row: table slot | 0x80000000 when the row claimed it
    int32_t* status;               // FWA_E_* of the kernels (0 = ok)
    uint64_t mask;                 // table capacity - 1
    int64_t max_rows;
    int32_t max_par;
    uint8_t* heap;                 // STRING values longer than 7 bytes
    unsigned long long* heap_used;
    uint64_t heap_cap;
};

// ---- STRING values (BinaryRowData layout, AbstractBinaryWriter.java:80-105,279-334) ----
__device__ __forceinline__ uint64_t str_short_slot(const uint8_t* p, int64_t len) {   // writeBytesToFixLenPart
    uint64_t v = (uint64_t)(0x80u | (uint32_t)len) << 56;
    for (int64_t b = 0; b < len; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}
__device__ __forceinline__ uint64_t str_word64(const uint8_t* p, int64_t len, int64_t at) {   // zero past len
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) if (at + b < len) v |= (uint64_t)p[at + b] << (8 * b);
    return v;
}
__device__ __forceinline__ uint64_t str_identity(const uint8_t* p, int64_t len) {   // 63-bit content hash
    uint64_t h = jm::mix64(0x243F6A8885A308D3ull ^ (uint64_t)len);
    for (int64_t at = 0; at < len; at += 8) h = jm::mix64(h ^ str_word64(p, len, at) ^ ((uint64_t)at << 40));
    return h & 0x7fffffffffffffffull;
}
__device__ __forceinline__ int64_t str_len(const KdCols& k, int c, int64_t i) { return (int64_t)k.soff[c][i + 1] - k.soff[c][i]; }
__device__ __forceinline__ const uint8_t* str_ptr(const KdCols& k, int c, int64_t i) { return k.sbytes[c] + k.soff[c][i]; }

__device__ __forceinline__ void row_of(const KdCols& k, int64_t i, uint64_t* slots, uint64_t* nullbits) {
    uint64_t nb = 0;
    for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
        if (c >= k.arity) break;
        const bool isnull = k.nul[c] && k.nul[c][i];
        uint64_t v = 0;
        if (!isnull) {
            if (k.type[c] == FWA_KEY_FIELD_INT) v = (uint64_t)(uint32_t)((const int32_t*)k.col[c])[i];
            else if (k.type[c] == FWA_KEY_FIELD_STRING) {   // short: the slot itself; long: its content identity
                const int64_t len = str_len(k, c, i);
                v = len <= 7 ? str_short_slot(str_ptr(k, c, i), len) : str_identity(str_ptr(k, c, i), len);
            }
            else v = ((const uint64_t*)k.col[c])[i];   // BIGINT, DOUBLE raw bits
        }
        nb |= (uint64_t)isnull << c;
        slots[c] = v;
    }
    *nullbits = nb;
}

__device__ __forceinline__ uint64_t row_identity(const uint64_t* slots, int arity, uint64_t nullbits) {
    uint64_t h = jm::mix64(nullbits ^ 0x9E3779B97F4A7C15ull ^ (uint64_t)arity);
    for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
        if (c >= arity) break;
        h = jm::mix64(h ^ slots[c] ^ ((uint64_t)(c + 1) << 56));
    }
    return h == kKdEmpty ? 1ull : h;
}

// BinaryRowData.hashCode() of row i (MurmurHashUtils.hashBytesByWords over the whole row, seed 42): the header, the
// slots (a long STRING's slot = its offset in the row << 32 | length), the variable-length part, fmix(h ^ size)
__device__ int32_t kd_row_hash(const KdCols& k, int64_t i, const uint64_t* slots, uint64_t nb) {
    if (!k.has_str) return jm::binrow_hash(slots, k.arity, nb);
    uint32_t h = 42u;
    const uint64_t hdr = nb << 8;
    h = jm::mh_h1(h, jm::mh_k1((uint32_t)hdr));
    h = jm::mh_h1(h, jm::mh_k1((uint32_t)(hdr >> 32)));
    uint64_t off = 8 + 8 * (uint64_t)k.arity;
    for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
        if (c >= k.arity) break;
        uint64_t v = (nb >> c) & 1 ? 0ull : slots[c];
        if (k.type[c] == FWA_KEY_FIELD_STRING && !((nb >> c) & 1)) {
            const int64_t len = str_len(k, c, i);
            if (len > 7) { v = (off << 32) | (uint64_t)len; off += ((uint64_t)len + 7) & ~7ull; }
        }
        h = jm::mh_h1(h, jm::mh_k1((uint32_t)v));
        h = jm::mh_h1(h, jm::mh_k1((uint32_t)(v >> 32)));
    }
    for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
        if (c >= k.arity) break;
        if (k.type[c] != FWA_KEY_FIELD_STRING || ((nb >> c) & 1)) continue;
        const int64_t len = str_len(k, c, i);
        if (len <= 7) continue;
        const uint8_t* p = str_ptr(k, c, i);
        for (int64_t at = 0; at < ((len + 7) & ~7ll); at += 8) {
            const uint64_t w = str_word64(p, len, at);
            h = jm::mh_h1(h, jm::mh_k1((uint32_t)w));
            h = jm::mh_h1(h, jm::mh_k1((uint32_t)(w >> 32)));
        }
    }
    h ^= (uint32_t)off;
    return jm::bit_mix((int32_t)h);
}

__global__ void __launch_bounds__(kBlockKd) kd_hash_kernel(KdCols k, int64_t n, int32_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t slots[FWA_KEYDICT_MAX_ARITY], nb;
        row_of(k, i, slots, &nb);
        out[i] = kd_row_hash(k, i, slots, nb);
    }
}

__global__ void __launch_bounds__(kBlockKd) kd_insert_kernel(KdCols k, KdDev d, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t slots[FWA_KEYDICT_MAX_ARITY], nb;
        row_of(k, i, slots, &nb);
        const uint64_t h = row_identity(slots, k.arity, nb);
        uint64_t s = (h * 0x9E3779B97F4A7C15ull) & d.mask;
        uint32_t got = 0xffffffffu;
        for (uint64_t probe = 0; probe <= d.mask; ++probe) {
            const unsigned long long old = atomicCAS(&d.ht_key[s], kKdEmpty, (unsigned long long)h);
            if (old == kKdEmpty) { d.ht_rep[s] = (uint32_t)i; got = (uint32_t)s | 0x80000000u; break; }
            if (old == h) { got = (uint32_t)s; break; }
            s = (s + 1) & d.mask;
        }
        if (got == 0xffffffffu) atomicCAS(d.status, 0, FWA_E_OOM);
        d.pos[i] = got;
    }
}

__global__ void __launch_bounds__(kBlockKd) kd_assign_kernel(KdCols k, KdDev d, int64_t n) {
    const int lane = threadIdx.x & 63;
    for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n; t0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t0 + threadIdx.x;
        const uint32_t ps = i < n ? d.pos[i] : 0xffffffffu;
        const bool win = ps != 0xffffffffu && (ps & 0x80000000u);
        const unsigned long long m = __ballot(win);
        if (!m) continue;
        const int ld = __ffsll((long long)m) - 1;
        unsigned long long base = 0;
        if (lane == ld) base = atomicAdd(d.nrows, (unsigned long long)__popcll(m));
        base = __shfl(base, ld);
        if (!win) continue;
        const unsigned long long seq = base + __popcll(m & ((1ull << lane) - 1ull));
        const uint64_t s = ps & 0x7fffffffu;
        if ((int64_t)seq >= d.max_rows) { atomicCAS(d.status, 0, FWA_E_OOM); continue; }
        uint64_t slots[FWA_KEYDICT_MAX_ARITY], nb;
        row_of(k, i, slots, &nb);
        const int32_t kg = jm::key_group(kd_row_hash(k, i, slots, nb), d.max_par);
        for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
            if (c >= k.arity) break;
            uint64_t v = slots[c];
            if (k.type[c] == FWA_KEY_FIELD_STRING && !((nb >> c) & 1) && str_len(k, c, i) > 7) {   // to the heap
                const int64_t len = str_len(k, c, i);
                const unsigned long long at = atomicAdd(d.heap_used, (unsigned long long)len);
                if (len > kStrMax || at + (uint64_t)len > d.heap_cap) { atomicCAS(d.status, 0, FWA_E_OOM); v = 0; }
                else {
                    const uint8_t* p = str_ptr(k, c, i);
                    for (int64_t b = 0; b < len; ++b) d.heap[at + b] = p[b];
                    v = ((uint64_t)len << 40) | (at & kHeapMask);
                }
            }
            d.fslot[(int64_t)c * d.max_rows + (int64_t)seq] = v;
        }
        d.fnull[seq] = nb;
        d.ht_id[s] = (long long)(((uint64_t)kg << 48) | (seq & kSeqMask));
    }
}

__global__ void __launch_bounds__(kBlockKd) kd_lookup_kernel(KdCols k, KdDev d, int64_t n, int64_t* ids, int32_t* hashes) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t ps = d.pos[i];
        if (ps == 0xffffffffu) continue;
        const int64_t id = d.ht_id[ps & 0x7fffffffu];
        if (id < 0) { atomicCAS(d.status, 0, FWA_E_OOM); ids[i] = -1; continue; }   // claimed when the dictionary was full
        const uint64_t seq = (uint64_t)id & kSeqMask;
        uint64_t slots[FWA_KEYDICT_MAX_ARITY], nb;
        row_of(k, i, slots, &nb);
        bool same = (int64_t)seq < d.max_rows && d.fnull[seq] == nb;
        for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
            if (c >= k.arity || !same) break;
            const uint64_t fs = d.fslot[(int64_t)c * d.max_rows + (int64_t)seq];
            if (k.type[c] == FWA_KEY_FIELD_STRING && !((nb >> c) & 1) && str_len(k, c, i) > 7) {   // bytes vs heap
                const int64_t len = str_len(k, c, i);
                same = (fs >> 63) == 0 && (int64_t)(fs >> 40) == len;
                const uint8_t* p = str_ptr(k, c, i);
                const uint8_t* q = d.heap + (fs & kHeapMask);
                for (int64_t b = 0; b < len && same; ++b) same = p[b] == q[b];
            } else {
                same = fs == slots[c];
            }
        }
        if (!same) atomicCAS(d.status, 0, FWA_E_STATE);    // two rows with one 64-bit identity
        ids[i] = id;
        if (hashes) hashes[i] = kd_row_hash(k, i, slots, nb);
    }
}

__global__ void __launch_bounds__(kBlockKd) kd_decode_kernel(KdDev d, KdCols k, int64_t n, const int64_t* ids,
                                                              void* const* cols, uint8_t* const* nul, int has_nul) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t seq = (uint64_t)ids[i] & kSeqMask;
        if ((int64_t)seq >= d.max_rows) { atomicCAS(d.status, 0, FWA_E_ARG); continue; }
        const uint64_t nb = d.fnull[seq];
        for (int c = 0; c < FWA_KEYDICT_MAX_ARITY; ++c) {
            if (c >= k.arity) break;
            const uint64_t v = d.fslot[(int64_t)c * d.max_rows + (int64_t)seq];
            if (k.type[c] == FWA_KEY_FIELD_INT) ((int32_t*)cols[c])[i] = (int32_t)(uint32_t)v;
            else if (k.type[c] != FWA_KEY_FIELD_STRING) ((uint64_t*)cols[c])[i] = v;   // strings: kd_str_* kernels
            if (has_nul && nul[c]) nul[c][i] = (uint8_t)((nb >> c) & 1);
        }
    }
}

// STRING decode: the length of each id's value into offsets[i + 1] (then scanned), and its bytes
__device__ __forceinline__ int64_t stored_len(uint64_t fs, bool isnull) {
    if (isnull || fs == 0) return 0;
    return (fs >> 63) ? (int64_t)((fs >> 56) & 0x7f) : (int64_t)(fs >> 40);
}
__global__ void __launch_bounds__(kBlockKd) kd_strlen_kernel(KdDev d, int c, int64_t n, const int64_t* ids, int32_t* offs) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t seq = (uint64_t)ids[i] & kSeqMask;
        if ((int64_t)seq >= d.max_rows) { atomicCAS(d.status, 0, FWA_E_ARG); offs[i + 1] = 0; continue; }
        offs[i + 1] = (int32_t)stored_len(d.fslot[(int64_t)c * d.max_rows + (int64_t)seq], (d.fnull[seq] >> c) & 1);
        if (i == 0) offs[0] = 0;
    }
}
__global__ void __launch_bounds__(kBlockKd) kd_strcopy_kernel(KdDev d, int c, int64_t n, const int64_t* ids, const int32_t* offs,
                                                               uint8_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t seq = (uint64_t)ids[i] & kSeqMask;
        if ((int64_t)seq >= d.max_rows) continue;
        const uint64_t fs = d.fslot[(int64_t)c * d.max_rows + (int64_t)seq];
        const int64_t len = stored_len(fs, (d.fnull[seq] >> c) & 1);
        uint8_t* o = out + offs[i];
        if (fs >> 63) for (int64_t b = 0; b < len; ++b) o[b] = (uint8_t)(fs >> (8 * b));
        else for (int64_t b = 0; b < len; ++b) o[b] = d.heap[(fs & kHeapMask) + b];
    }
}

int grid_kd(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlockKd - 1) / kBlockKd, 8192)); }

}  // namespace

struct fwa_keydict {
    int32_t arity = 0, device = 0;
    int32_t types[FWA_KEYDICT_MAX_ARITY] = {};
    KdDev d{};
    int64_t cap = 0;                 // table slots
    int64_t pos_cap = 0;
    hipStream_t stream = nullptr;
    std::string err;
    void** d_colptr = nullptr;       // decode: device copies of the column / null pointer arrays
    bool has_str = false;
    void* d_scan_tmp = nullptr;      // decode: hipcub scan scratch
    size_t scan_tmp_bytes = 0;
};

namespace {
int kd_fail(fwa_keydict* d, int code, const char* msg) { d->err = msg; return code; }
#define KDCHK(d, call) do { hipError_t _e = (call); if (_e != hipSuccess) return kd_fail(d, FWA_E_DEVICE, hipGetErrorString(_e)); } while (0)

// STRING fields: cols[c] is a host fwa_key_strings (the device offsets / bytes)
bool fill_cols(int arity, const int32_t* types, const void* const* cols, const uint8_t* const* nulls, KdCols* k) {
    memset(k, 0, sizeof(*k));
    k->arity = arity;
    for (int c = 0; c < arity; ++c) {
        if (!cols[c]) return false;
        k->col[c] = cols[c];
        k->nul[c] = nulls ? nulls[c] : nullptr;
        k->type[c] = types[c];
        if (types[c] == FWA_KEY_FIELD_STRING) {
            const fwa_key_strings* ks = (const fwa_key_strings*)cols[c];
            if (!ks->offsets || !ks->bytes) return false;
            k->soff[c] = ks->offsets;
            k->sbytes[c] = ks->bytes;
            k->col[c] = ks->offsets;
            k->has_str = 1;
        }
    }
    return true;
}
bool cols_of(const fwa_keydict* d, const void* const* cols, const uint8_t* const* nulls, KdCols* k) {
    return fill_cols(d->arity, d->types, cols, nulls, k);
}

int read_status(fwa_keydict* d) {
    int32_t st = 0;
    KDCHK(d, hipMemcpyAsync(&st, d->d.status, 4, hipMemcpyDeviceToHost, d->stream));
    KDCHK(d, hipStreamSynchronize(d->stream));
    if (st == FWA_E_OOM) return kd_fail(d, st, "key dictionary full (capacity, or a STRING value over 2^23 - 1 bytes)");
    if (st == FWA_E_STATE) return kd_fail(d, st, "two key rows with one 64-bit identity");
    if (st) return kd_fail(d, st, "bad key id");
    return FWA_OK;
}
// Make room in the STRING heap for every long value of a batch before it is encoded (the assign pass cannot grow it):
// at most the batch's string bytes.
int ensure_heap(fwa_keydict* d, const KdCols& k, int64_t n) {
    uint64_t need = 0;
    for (int c = 0; c < d->arity; ++c) {
        if (d->types[c] != FWA_KEY_FIELD_STRING) continue;
        int32_t ends[2] = {0, 0};
        KDCHK(d, hipMemcpyAsync(&ends[0], k.soff[c], 4, hipMemcpyDeviceToHost, d->stream));
        KDCHK(d, hipMemcpyAsync(&ends[1], k.soff[c] + n, 4, hipMemcpyDeviceToHost, d->stream));
        KDCHK(d, hipStreamSynchronize(d->stream));
        if (ends[1] < ends[0]) return kd_fail(d, FWA_E_ARG, "STRING offsets decrease");
        need += (uint64_t)(ends[1] - ends[0]);
    }
    unsigned long long used = 0;
    KDCHK(d, hipMemcpyAsync(&used, d->d.heap_used, 8, hipMemcpyDeviceToHost, d->stream));
    KDCHK(d, hipStreamSynchronize(d->stream));
    if (used + need <= d->d.heap_cap) return FWA_OK;
    uint64_t cap = std::max<uint64_t>(d->d.heap_cap * 2, used + need + (1 << 20));
    if (cap > kHeapMask) return kd_fail(d, FWA_E_OOM, "key dictionary string heap past 2^40 bytes");
    uint8_t* nh = nullptr;
    KDCHK(d, hipMalloc(&nh, cap));
    if (used) KDCHK(d, hipMemcpyAsync(nh, d->d.heap, used, hipMemcpyDeviceToDevice, d->stream));
    KDCHK(d, hipStreamSynchronize(d->stream));
    if (d->d.heap) KDCHK(d, hipFree(d->d.heap));
    d->d.heap = nh;
    d->d.heap_cap = cap;
    return FWA_OK;
}
}  // namespace

extern "C" {

int fwa_keydict_create(int32_t arity, const int32_t* field_types, int32_t max_parallelism, int64_t capacity,
                       int32_t device, fwa_keydict** out) {
    if (!out || arity < 1 || arity > FWA_KEYDICT_MAX_ARITY || !field_types || max_parallelism <= 0 ||
        max_parallelism > 32768 || capacity <= 0 || capacity > ((int64_t)1 << 29))   // slot index: 31 bits < sentinel
        return FWA_E_ARG;
    for (int c = 0; c < arity; ++c)
        if (field_types[c] < FWA_KEY_FIELD_BIGINT || field_types[c] > FWA_KEY_FIELD_STRING) return FWA_E_ARG;
    fwa_keydict* d = new fwa_keydict();
    d->arity = arity;
    d->device = device;
    for (int c = 0; c < arity; ++c) { d->types[c] = field_types[c]; d->has_str |= field_types[c] == FWA_KEY_FIELD_STRING; }
    int64_t cap = 1024;
    while (cap < 2 * capacity) cap <<= 1;
    d->cap = cap;
    d->d.mask = (uint64_t)cap - 1;
    d->d.max_rows = capacity;
    d->d.max_par = max_parallelism;
    int rc = FWA_OK;
    do {
        if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        if (hipMalloc(&d->d.ht_key, 8 * cap) != hipSuccess || hipMalloc(&d->d.ht_id, 8 * cap) != hipSuccess ||
            hipMalloc(&d->d.ht_rep, 4 * cap) != hipSuccess ||
            hipMalloc(&d->d.fslot, 8 * (size_t)arity * (size_t)capacity) != hipSuccess ||
            hipMalloc(&d->d.fnull, 8 * (size_t)capacity) != hipSuccess || hipMalloc(&d->d.nrows, 8) != hipSuccess ||
            hipMalloc(&d->d.status, 4) != hipSuccess || hipMalloc(&d->d_colptr, 2 * sizeof(void*) * FWA_KEYDICT_MAX_ARITY) != hipSuccess ||
            hipMalloc(&d->d.heap_used, 8) != hipSuccess) {
            rc = FWA_E_OOM; break;
        }
        // ht_id -1: a slot whose row was claimed but never given an id (the dictionary filled up) reads as "no id"
        if (hipMemsetAsync(d->d.ht_key, 0, 8 * cap, d->stream) != hipSuccess || hipMemsetAsync(d->d.ht_id, 0xff, 8 * cap, d->stream) != hipSuccess ||
            hipMemsetAsync(d->d.nrows, 0, 8, d->stream) != hipSuccess || hipMemsetAsync(d->d.heap_used, 0, 8, d->stream) != hipSuccess ||
            hipMemsetAsync(d->d.status, 0, 4, d->stream) != hipSuccess || hipStreamSynchronize(d->stream) != hipSuccess) {
            rc = FWA_E_DEVICE; break;
        }
    } while (0);
    if (rc) { fwa_keydict_destroy(d); return rc; }
    *out = d;
    return FWA_OK;
}

void fwa_keydict_destroy(fwa_keydict* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (void* p : {(void*)d->d.ht_key, (void*)d->d.ht_id, (void*)d->d.ht_rep, (void*)d->d.fslot, (void*)d->d.fnull,
                    (void*)d->d.nrows, (void*)d->d.pos, (void*)d->d.status, (void*)d->d_colptr, (void*)d->d.heap,
                    (void*)d->d.heap_used, d->d_scan_tmp})
        if (p) (void)hipFree(p);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

const char* fwa_keydict_last_error(const fwa_keydict* d) { return d ? d->err.c_str() : "null key dictionary"; }

int64_t fwa_keydict_size(const fwa_keydict* d) {
    if (!d) return -1;
    unsigned long long n = 0;
    if (hipSetDevice(d->device) != hipSuccess) return -1;
    if (hipMemcpyAsync(&n, d->d.nrows, 8, hipMemcpyDeviceToHost, d->stream) != hipSuccess) return -1;
    if (hipStreamSynchronize(d->stream) != hipSuccess) return -1;
    return (int64_t)std::min<unsigned long long>(n, (unsigned long long)d->d.max_rows);
}

int fwa_keydict_encode(fwa_keydict* d, const void* const* cols, const uint8_t* const* nulls, int64_t n, int64_t* ids,
                       int32_t* hashes) {
    if (!d) return FWA_E_ARG;
    if (n < 0 || (n > 0 && (!cols || !ids)) || n > INT32_MAX) return kd_fail(d, FWA_E_ARG, "fwa_keydict_encode: bad arguments");
    if (n == 0) return FWA_OK;
    KdCols k;
    if (!cols_of(d, cols, nulls, &k)) return kd_fail(d, FWA_E_ARG, "fwa_keydict_encode: null key column");
    KDCHK(d, hipSetDevice(d->device));
    if (d->has_str) { if (int rc = ensure_heap(d, k, n)) return rc; }
    if (n > d->pos_cap) {
        KDCHK(d, hipStreamSynchronize(d->stream));
        if (d->d.pos) KDCHK(d, hipFree(d->d.pos));
        d->d.pos = nullptr;
        d->pos_cap = std::max<int64_t>(n + n / 4, 1 << 16);
        KDCHK(d, hipMalloc(&d->d.pos, 4 * (size_t)d->pos_cap));
    }
    KDCHK(d, hipMemsetAsync(d->d.status, 0, 4, d->stream));
    kd_insert_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(k, d->d, n);
    kd_assign_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(k, d->d, n);
    kd_lookup_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(k, d->d, n, ids, hashes);
    KDCHK(d, hipGetLastError());
    return read_status(d);
}

int fwa_keydict_decode(fwa_keydict* d, const int64_t* ids, int64_t n, void* const* cols, uint8_t* const* nulls) {
    if (!d) return FWA_E_ARG;
    if (n < 0 || (n > 0 && (!ids || !cols))) return kd_fail(d, FWA_E_ARG, "fwa_keydict_decode: bad arguments");
    if (n == 0) return FWA_OK;
    KDCHK(d, hipSetDevice(d->device));
    void* h[2 * FWA_KEYDICT_MAX_ARITY] = {};
    for (int c = 0; c < d->arity; ++c) {
        if (!cols[c]) return kd_fail(d, FWA_E_ARG, "fwa_keydict_decode: null key column");
        h[c] = d->types[c] == FWA_KEY_FIELD_STRING ? nullptr : cols[c];   // strings: through fwa_key_strings_out
        h[FWA_KEYDICT_MAX_ARITY + c] = nulls ? (void*)nulls[c] : nullptr;
    }
    KDCHK(d, hipMemcpyAsync(d->d_colptr, h, sizeof(h), hipMemcpyHostToDevice, d->stream));
    KDCHK(d, hipMemsetAsync(d->d.status, 0, 4, d->stream));
    KdCols k;
    memset(&k, 0, sizeof(k));
    k.arity = d->arity;
    for (int c = 0; c < d->arity; ++c) k.type[c] = d->types[c];
    kd_decode_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(d->d, k, n, ids, d->d_colptr,
                                                             (uint8_t* const*)(d->d_colptr + FWA_KEYDICT_MAX_ARITY),
                                                             nulls ? 1 : 0);
    KDCHK(d, hipGetLastError());
    bool short_out = false;
    for (int c = 0; c < d->arity; ++c) {        // STRING fields: lengths -> offsets (inclusive scan from [1]) -> bytes
        if (d->types[c] != FWA_KEY_FIELD_STRING) continue;
        fwa_key_strings_out* so = (fwa_key_strings_out*)cols[c];
        if (!so->offsets) return kd_fail(d, FWA_E_ARG, "fwa_keydict_decode: null STRING offsets");
        kd_strlen_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(d->d, c, n, ids, so->offsets);
        size_t tb = 0;
        KDCHK(d, hipcub::DeviceScan::InclusiveSum(nullptr, tb, so->offsets + 1, so->offsets + 1, (int)n, d->stream));
        if (tb > d->scan_tmp_bytes) {
            KDCHK(d, hipStreamSynchronize(d->stream));
            if (d->d_scan_tmp) KDCHK(d, hipFree(d->d_scan_tmp));
            d->d_scan_tmp = nullptr;
            KDCHK(d, hipMalloc(&d->d_scan_tmp, tb));
            d->scan_tmp_bytes = tb;
        }
        tb = d->scan_tmp_bytes;
        KDCHK(d, hipcub::DeviceScan::InclusiveSum(d->d_scan_tmp, tb, so->offsets + 1, so->offsets + 1, (int)n, d->stream));
        int32_t total = 0;
        KDCHK(d, hipMemcpyAsync(&total, so->offsets + n, 4, hipMemcpyDeviceToHost, d->stream));
        KDCHK(d, hipStreamSynchronize(d->stream));
        so->needed = total;
        if (!so->bytes) continue;
        if (so->capacity < total) { short_out = true; continue; }
        kd_strcopy_kernel<<<grid_kd(n), kBlockKd, 0, d->stream>>>(d->d, c, n, ids, so->offsets, so->bytes);
        KDCHK(d, hipGetLastError());
    }
    if (int rc = read_status(d)) return rc;
    if (short_out) return kd_fail(d, FWA_E_ARG, "fwa_keydict_decode: STRING bytes past the output capacity");
    return FWA_OK;
}

// internal (heap_snapshot.cpp): every row of the dictionary on the host -- slots [row][arity] and null bits
int fwa_keydict_host_rows(fwa_keydict* d, int32_t* arity, int32_t* types, std::vector<uint64_t>* slots,
                          std::vector<uint64_t>* nulls) {
    if (!d) return FWA_E_ARG;
    *arity = d->arity;
    for (int c = 0; c < d->arity; ++c) types[c] = d->types[c];
    const int64_t n = fwa_keydict_size(d);
    if (n < 0) return FWA_E_DEVICE;
    std::vector<uint64_t> cols((size_t)n * d->arity);
    nulls->assign((size_t)n, 0);
    KDCHK(d, hipSetDevice(d->device));
    for (int c = 0; c < d->arity && n > 0; ++c)
        KDCHK(d, hipMemcpyAsync(cols.data() + (size_t)c * n, d->d.fslot + (size_t)c * d->d.max_rows, 8 * (size_t)n,
                                hipMemcpyDeviceToHost, d->stream));
    if (n > 0) KDCHK(d, hipMemcpyAsync(nulls->data(), d->d.fnull, 8 * (size_t)n, hipMemcpyDeviceToHost, d->stream));
    KDCHK(d, hipStreamSynchronize(d->stream));
    slots->assign((size_t)n * d->arity, 0);
    for (int64_t r = 0; r < n; ++r)
        for (int c = 0; c < d->arity; ++c) (*slots)[(size_t)r * d->arity + c] = cols[(size_t)c * n + r];
    return FWA_OK;
}

// internal (heap_snapshot.cpp): encode n rows given on the host as slots [row][arity] + null bits; ids to the host
int fwa_keydict_encode_host(fwa_keydict* d, const uint64_t* slots, const uint64_t* nulls, int64_t n, int64_t* ids) {
    if (!d || n < 0) return FWA_E_ARG;
    if (n == 0) return FWA_OK;
    KDCHK(d, hipSetDevice(d->device));
    const int a = d->arity;
    std::vector<uint64_t> cols((size_t)n * a);
    std::vector<uint8_t> nul((size_t)n * a);
    for (int64_t r = 0; r < n; ++r)
        for (int c = 0; c < a; ++c) {
            const uint64_t v = slots[(size_t)r * a + c];
            if (d->types[c] == FWA_KEY_FIELD_INT) reinterpret_cast<int32_t*>(cols.data() + (size_t)c * n)[r] = (int32_t)(uint32_t)v;
            else cols[(size_t)c * n + r] = v;
            nul[(size_t)c * n + r] = (uint8_t)((nulls[r] >> c) & 1);
        }
    char* buf = nullptr;
    const size_t bc = 8 * (size_t)n * a, bn = (size_t)n * a, bi = 8 * (size_t)n;
    KDCHK(d, hipMalloc(&buf, bc + bn + bi + 64));
    int rc = FWA_OK;
    do {
        if (hipMemcpyAsync(buf, cols.data(), bc, hipMemcpyHostToDevice, d->stream) != hipSuccess ||
            hipMemcpyAsync(buf + bc, nul.data(), bn, hipMemcpyHostToDevice, d->stream) != hipSuccess) { rc = FWA_E_DEVICE; break; }
        const void* cp[FWA_KEYDICT_MAX_ARITY];
        const uint8_t* np_[FWA_KEYDICT_MAX_ARITY];
        for (int c = 0; c < a; ++c) { cp[c] = buf + 8 * (size_t)c * n; np_[c] = (const uint8_t*)(buf + bc + (size_t)c * n); }
        int64_t* did = (int64_t*)(buf + ((bc + bn + 7) & ~(size_t)7));
        if ((rc = fwa_keydict_encode(d, cp, np_, n, did, nullptr))) break;
        if (hipMemcpy(ids, did, bi, hipMemcpyDeviceToHost) != hipSuccess) rc = FWA_E_DEVICE;
    } while (0);
    (void)hipFree(buf);
    return rc;
}

int fwa_binrow_hash(int32_t arity, const int32_t* field_types, const void* const* cols, const uint8_t* const* nulls,
                    int64_t n, int32_t* out, int32_t device) {
    if (arity < 1 || arity > FWA_KEYDICT_MAX_ARITY || !field_types || n < 0 || (n > 0 && (!cols || !out))) return FWA_E_ARG;
    if (n == 0) return FWA_OK;
    KdCols k;
    for (int c = 0; c < arity; ++c)
        if (!cols[c] || field_types[c] < FWA_KEY_FIELD_BIGINT || field_types[c] > FWA_KEY_FIELD_STRING) return FWA_E_ARG;
    if (!fill_cols(arity, field_types, cols, nulls, &k)) return FWA_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FWA_E_DEVICE;
    kd_hash_kernel<<<grid_kd(n), kBlockKd>>>(k, n, out);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return FWA_E_DEVICE;
    return FWA_OK;
}

}  // extern "C"

// internal (heap_snapshot.cpp): the STRING values of every dictionary row on the host, strs[row * arity + c] (empty
// for the other fields and for NULLs)
int fwa_keydict_host_strings(fwa_keydict* d, std::vector<std::string>* strs) {
    if (!d) return FWA_E_ARG;
    const int64_t n = fwa_keydict_size(d);
    if (n < 0) return FWA_E_DEVICE;
    strs->assign((size_t)n * d->arity, std::string());
    if (!d->has_str || n == 0) return FWA_OK;
    KDCHK(d, hipSetDevice(d->device));
    std::vector<uint64_t> fs((size_t)n), nb((size_t)n);
    unsigned long long used = 0;
    KDCHK(d, hipMemcpyAsync(&used, d->d.heap_used, 8, hipMemcpyDeviceToHost, d->stream));
    KDCHK(d, hipMemcpyAsync(nb.data(), d->d.fnull, 8 * (size_t)n, hipMemcpyDeviceToHost, d->stream));
    KDCHK(d, hipStreamSynchronize(d->stream));
    std::vector<uint8_t> heap((size_t)used);
    if (used) KDCHK(d, hipMemcpyAsync(heap.data(), d->d.heap, used, hipMemcpyDeviceToHost, d->stream));
    for (int c = 0; c < d->arity; ++c) {
        if (d->types[c] != FWA_KEY_FIELD_STRING) continue;
        KDCHK(d, hipMemcpyAsync(fs.data(), d->d.fslot + (size_t)c * d->d.max_rows, 8 * (size_t)n, hipMemcpyDeviceToHost, d->stream));
        KDCHK(d, hipStreamSynchronize(d->stream));
        for (int64_t r = 0; r < n; ++r) {
            if ((nb[(size_t)r] >> c) & 1) continue;
            const uint64_t w = fs[(size_t)r];
            std::string& s = (*strs)[(size_t)r * d->arity + c];
            if (w >> 63) {
                const int len = (int)((w >> 56) & 0x7f);
                for (int b = 0; b < len; ++b) s.push_back((char)(uint8_t)(w >> (8 * b)));
            } else if (w) {
                const uint64_t len = w >> 40, at = w & kHeapMask;
                if (at + len > used) return kd_fail(d, FWA_E_STATE, "key dictionary string heap inconsistent");
                s.assign((const char*)heap.data() + at, (size_t)len);
            }
        }
    }
    return FWA_OK;
}

// internal (heap_snapshot.cpp): encode n rows given on the host as slots [row][arity] (ignored for STRING fields),
// null bits and STRING values strs[row * arity + c]; ids to the host
int fwa_keydict_encode_host_str(fwa_keydict* d, const uint64_t* slots, const uint64_t* nulls,
                                const std::vector<std::string>& strs, int64_t n, int64_t* ids) {
    if (!d || n < 0) return FWA_E_ARG;
    if (!d->has_str) return fwa_keydict_encode_host(d, slots, nulls, n, ids);
    if (n == 0) return FWA_OK;
    KDCHK(d, hipSetDevice(d->device));
    const int a = d->arity;
    std::vector<uint64_t> cols((size_t)n * a);
    std::vector<uint8_t> nul((size_t)n * a);
    std::vector<std::vector<int32_t>> offs((size_t)a);
    std::vector<std::string> bytes((size_t)a);
    for (int c = 0; c < a; ++c) {
        if (d->types[c] == FWA_KEY_FIELD_STRING) offs[(size_t)c].assign(1, 0);
        for (int64_t r = 0; r < n; ++r) {
            nul[(size_t)c * n + r] = (uint8_t)((nulls[r] >> c) & 1);
            if (d->types[c] == FWA_KEY_FIELD_STRING) {
                bytes[(size_t)c] += strs[(size_t)r * a + c];
                if (bytes[(size_t)c].size() > (size_t)INT32_MAX) return kd_fail(d, FWA_E_ARG, "STRING column past 2^31 bytes");
                offs[(size_t)c].push_back((int32_t)bytes[(size_t)c].size());
            } else if (d->types[c] == FWA_KEY_FIELD_INT) {
                reinterpret_cast<int32_t*>(cols.data() + (size_t)c * n)[r] = (int32_t)(uint32_t)slots[(size_t)r * a + c];
            } else {
                cols[(size_t)c * n + r] = slots[(size_t)r * a + c];
            }
        }
    }
    size_t tot = 8 * (size_t)n * a + (size_t)n * a + 8 * (size_t)n + 64;
    for (int c = 0; c < a; ++c) tot += 4 * offs[(size_t)c].size() + bytes[(size_t)c].size() + 16;
    char* buf = nullptr;
    KDCHK(d, hipMalloc(&buf, tot));
    int rc = FWA_OK;
    do {
        char* p = buf;
        auto put = [&](const void* src, size_t nb) -> char* {
            char* dst = p;
            if (nb && src && hipMemcpyAsync(dst, src, nb, hipMemcpyHostToDevice, d->stream) != hipSuccess) rc = FWA_E_DEVICE;
            p += (nb + 15) & ~(size_t)15;
            return dst;
        };
        const void* cp[FWA_KEYDICT_MAX_ARITY];
        const uint8_t* np_[FWA_KEYDICT_MAX_ARITY];
        fwa_key_strings ks[FWA_KEYDICT_MAX_ARITY];
        for (int c = 0; c < a; ++c) {
            np_[c] = (const uint8_t*)put(nul.data() + (size_t)c * n, (size_t)n);
            if (d->types[c] == FWA_KEY_FIELD_STRING) {
                ks[c].offsets = (const int32_t*)put(offs[(size_t)c].data(), 4 * offs[(size_t)c].size());
                ks[c].bytes = (const uint8_t*)put(bytes[(size_t)c].data(), bytes[(size_t)c].size());
                cp[c] = &ks[c];
            } else {
                cp[c] = put(cols.data() + (size_t)c * n, 8 * (size_t)n);
            }
        }
        int64_t* did = (int64_t*)put(nullptr, 8 * (size_t)n);   // output only: reserved, not copied
        if (rc) break;
        if ((rc = fwa_keydict_encode(d, cp, np_, n, did, nullptr))) break;
        if (hipMemcpy(ids, did, 8 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) rc = FWA_E_DEVICE;
    } while (0);
    (void)hipFree(buf);
    return rc;
}
