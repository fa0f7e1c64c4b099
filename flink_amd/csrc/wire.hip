// wire.hip -- GPU decoder of Flink's network wire format behind include/flink_amd_wire.h.
//
// Input: the data-buffer payloads of one channel, concatenated (an element may span buffers, as in
// SpillingAdaptiveSpanningRecordDeserializer.java:88-131). Each element is a 4-byte big-endian length L
// followed by L bytes: the StreamElementSerializer tag and body (StreamElementSerializer.java:158-211,
// framed by RecordWriter.serializeRecord :145-157). Element boundaries are a sequential chain, so the decoder
// splits the bytes into 4 KiB chunks and runs three steps, all on the GPU:
//
//   scan    : per chunk, for EVERY candidate entry offset e in [0, S) (S = longest element + 4, so the first
//             element starting in a chunk is always one of them) walk the chain through the chunk in LDS and
//             record where it leaves (entry offset into the next chunk), END (stream ends / partial element)
//             or CORRUPT (tag / length mismatch), plus the records and events it passed: a map e -> exit.
//   compose : the maps of 64 consecutive chunks are composed in LDS (function composition is associative),
//             level by level, until one map covers the stream; its value at e = 0 is the whole call's count.
//   resolve : back down the levels, every chunk learns its true entry offset and the global record / event
//             index of its first element; chunks past the END are marked dead.
//   decode  : per chunk, one lane walks the true chain in LDS to list the element starts, then the wave
//             decodes the elements in parallel into SoA columns (key, ts, value columns, NULL flags) and an
//             event list (watermark / status / latency marker / record attributes) with record positions.
//
// HBM traffic: the wire bytes are read twice (scan, decode), the maps are S x 4 B per 4 KiB chunk, the
// columns are written once. Bound: HBM (wire decoder).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flink_amd_wire.h"

namespace {

constexpr int kChunk = 4096;            // bytes per chunk
constexpr int kMaxStep = 253;           // S limit: entry offsets < S must fit a byte next to two status codes
constexpr uint32_t kNxtEnd = 0xFE;      // chain ends inside the chunk (stream end or partial element)
constexpr uint32_t kNxtCorrupt = 0xFF;  // chain hits a malformed element
constexpr uint32_t kDead = 0xFF;        // resolve: chunk lies after the stream's END (nothing to decode)
constexpr int kLdsBudget = 60 * 1024;   // compose / resolve LDS per block
constexpr int64_t kPersistBlocks = 256 * 24;   // scan / decode: persistent single-wave blocks (24 per CU)

// Per-schema constants (kernel argument, copied by value).
struct WireConst {
    int32_t body[6];                   // element body length per tag (the 4-byte length prefix must equal it)
    int32_t step;                      // S
    int32_t format, arity;
    int32_t ftype[FWA_WIRE_MAX_FIELDS];
    int32_t foff[FWA_WIRE_MAX_FIELDS]; // TUPLE: offset of the field in the value; ROWDATA: offset of its slot in the row
    int32_t key_field, ts_field, num_cols;
    int32_t col_field[FWA_MAX_COLS];
    int32_t row_size, nullbits;        // ROWDATA: BinaryRowData size (fixed part only) and null-bit-set width
};

struct WireStatus {
    int32_t error;                     // first fwa_status raised by the decode kernel
    int32_t err_tag;
    int64_t err_pos;                   // byte offset of the offending element
    int64_t consumed;                  // bytes of whole elements (written by the END chunk)
};

// The staged chunk in LDS, read through aligned 32-bit words (two ds_read_b32 + a funnel shift per unaligned
// 4-byte field instead of four byte reads); the buffer carries 8 bytes of padding past the last staged byte.
struct Lds {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t u32le(int p) const {
        const int i = p >> 2, sh = (p & 3) * 8;
        return (uint32_t)((((uint64_t)w[i + 1] << 32) | w[i]) >> sh);
    }
    __device__ __forceinline__ uint32_t byte(int p) const { return (w[p >> 2] >> ((p & 3) * 8)) & 0xFF; }
    __device__ __forceinline__ uint32_t be32(int p) const { return __builtin_bswap32(u32le(p)); }
    __device__ __forceinline__ uint64_t le64(int p) const {
        const int i = p >> 2, sh = (p & 3) * 8;
        const uint32_t a = w[i], b = w[i + 1], c = w[i + 2];
        const uint32_t lo = (uint32_t)((((uint64_t)b << 32) | a) >> sh);
        const uint32_t hi = (uint32_t)((((uint64_t)c << 32) | b) >> sh);
        return ((uint64_t)hi << 32) | lo;
    }
    __device__ __forceinline__ uint64_t be64(int p) const { return __builtin_bswap64(le64(p)); }
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBufWords = (kChunk + kMaxStep + 3 + 8 + 3) / 4;

// Copy bytes [0, lim) of src (a chunk start: 4 KiB-aligned offset into the input) into LDS.
__device__ __forceinline__ void stage_chunk(uint32_t* words, const uint8_t* __restrict__ src, int lim, bool aligned) {
    uint8_t* buf = reinterpret_cast<uint8_t*>(words);
    int done = 0;
    if (aligned) {
        const int n16 = lim >> 4;
        for (int i = threadIdx.x; i < n16; i += blockDim.x)
            reinterpret_cast<u32x4*>(buf)[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
        done = n16 << 4;
    }
    for (int i = done + threadIdx.x; i < lim; i += blockDim.x) buf[i] = src[i];
}

// The chain step shared by scan and decode: classify the element starting at p (rem = bytes left in the stream
// from the chunk start). Returns 0: a whole element of length 4 + *len; 1: END; 2: CORRUPT. The expected body
// lengths are selected from uniform values (no per-lane indexed load of the kernel argument).
__device__ __forceinline__ int element_at(const Lds& b, int p, int rem, const WireConst& w, uint32_t* len,
                                          int* tag) {
    if (p + 5 > rem) return 1;
    const uint32_t l = b.be32(p);
    const int t = (int)b.byte(p + 4);
    *tag = t;
    const int32_t want = t == 0 ? w.body[0] : t == 1 ? w.body[1] : t == 2 ? w.body[2] : t == 3 ? w.body[3]
                       : t == 4 ? w.body[4] : t == 5 ? w.body[5] : -1;
    if (l != (uint32_t)want) return 2;
    if (p + 4 + (int)l > rem) return 1;
    *len = l;
    return 0;
}

// Wave-cooperative walk of the element chain from p through the chunk. Element boundaries are a sequential
// chain, but almost every element has the length of the one before it (a channel carries one record type), so
// the wave SPECULATES: lane i checks the header at p + i * R (R = the last element's size); the longest prefix of
// lanes whose header is a whole element of size R is exactly the next stretch of the chain (each check confirms
// the previous lane's boundary), one ballot per 64 elements. The first lane that fails is resolved by one scalar
// step (another element kind / END / CORRUPT), which also sets the new R. visit(pos, tag, rec_before, evt_rank)
// runs on the lane owning each element. Returns 0 (left the chunk: *stop >= kChunk), 1 END, 2 CORRUPT.
template <class F>
__device__ __forceinline__ int wave_walk(const Lds& b, int p, int remi, const WireConst& w, uint32_t* nrec,
                                         uint32_t* nevt, int* stop, int* badtag, F&& visit) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    uint32_t nr = 0, ne = 0;
    int R = 0;
    for (;;) {
        if (p >= kChunk) { *nrec = nr; *nevt = ne; *stop = p; return 0; }
        if (R > 0) {
            const int pos = p + lane * R;
            uint32_t len = 0;
            int tag = 0;
            const bool ok = pos < kChunk && element_at(b, pos, remi, w, &len, &tag) == 0 && (int)len + 4 == R;
            const uint64_t m = __ballot(ok);
            const int k = ~m == 0 ? 64 : __builtin_ctzll(~m);
            const bool mine = lane < k;
            const uint64_t rm = __ballot(mine && tag <= 1), em = __ballot(mine && tag > 1);
            if (mine) visit(pos, tag, nr + (uint32_t)__popcll(rm & below), ne + (uint32_t)__popcll(em & below));
            nr += (uint32_t)__popcll(rm);
            ne += (uint32_t)__popcll(em);
            p += k * R;
            if (k == 64 || p >= kChunk) continue;
        }
        uint32_t len = 0;                                          // scalar step at p (uniform)
        int tag = 0;
        const int st = element_at(b, p, remi, w, &len, &tag);
        if (st) { *nrec = nr; *nevt = ne; *stop = p; *badtag = tag; return st; }
        if (lane == 0) visit(p, tag, nr, ne);
        if (tag <= 1) ++nr; else ++ne;
        R = 4 + (int)len;
        p += R;
    }
}

// Next-chunk prefetch in registers: while the wave walks chunk c, the 16-byte loads of its next chunk are in
// flight (they land in LDS after the walk). Chunks reaching the stream end and unaligned inputs are staged byte-wise.
struct Prefetch {
    static constexpr int kVec = 5;                     // 16-byte loads per lane: 320 x 16 B >= kChunk + kMaxStep + 3
    u32x4 r[kVec];
    bool ok = false;
    __device__ __forceinline__ void issue(const uint8_t* __restrict__ in, int64_t nbytes, int64_t c, int nvec,
                                          bool aligned) {
        const int64_t cs = c * kChunk;
        ok = aligned && cs + (int64_t)nvec * 16 <= nbytes;
        if (!ok) return;
        const u32x4* src = reinterpret_cast<const u32x4*>(in + cs);
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int i = threadIdx.x + 64 * k;
            if (i < nvec) r[k] = __builtin_nontemporal_load(src + i);
        }
    }
    __device__ __forceinline__ void land(uint32_t* buf, int nvec) const {
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int i = threadIdx.x + 64 * k;
            if (i < nvec) reinterpret_cast<u32x4*>(buf)[i] = r[k];
        }
    }
};
static_assert(Prefetch::kVec * 64 * 16 >= kChunk + kMaxStep + 3, "prefetch covers a chunk and its halo");

// Stage chunk c from the prefetch (or byte-wise), then put chunk `next` in flight. Returns the bytes left.
__device__ __forceinline__ int stage_pf(uint32_t* buf, const uint8_t* __restrict__ in, int64_t nbytes, int64_t nchunks,
                                        int64_t c, int64_t next, const WireConst& w, bool aligned, Prefetch& pf) {
    const int nvec = (kChunk + w.step + 15) / 16;
    const int64_t cs = c * kChunk;
    const int64_t rem = nbytes - cs;
    __syncthreads();                                              // previous chunk fully read
    if (pf.ok) pf.land(buf, nvec);
    else {
        const int lim = (int)std::min<int64_t>(rem, kChunk + w.step);
        if (lim > 0) stage_chunk(buf, in + cs, lim, aligned);
    }
    __syncthreads();
    if (next < nchunks) pf.issue(in, nbytes, next, nvec, aligned);
    else pf.ok = false;
    return (int)std::min<int64_t>(rem, 1 << 30);                  // bytes left, clamped (chains stop within C + S)
}

// ---- scan: persistent 64-lane blocks, one chunk at a time. Candidates whose first header is already invalid
// (nearly all of them on real data) are settled in one lane-parallel check; each surviving candidate is walked
// by the whole wave. ----
__global__ __launch_bounds__(64) void wire_scan_kernel(const uint8_t* __restrict__ in, int64_t nbytes,
                                                        int64_t nchunks, WireConst w, bool aligned,
                                                        uint32_t* __restrict__ map0) {
    __shared__ uint32_t buf[kBufWords];
    const Lds b{buf};
    const int lane = threadIdx.x;
    Prefetch pf;
    if ((int64_t)blockIdx.x < nchunks) pf.issue(in, nbytes, blockIdx.x, (kChunk + w.step + 15) / 16, aligned);
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const int remi = stage_pf(buf, in, nbytes, nchunks, c, c + gridDim.x, w, aligned, pf);
        for (int e0 = 0; e0 < w.step; e0 += 64) {
            const int e = e0 + lane;
            uint32_t len = 0;
            int tag = 0;
            const int first = e < w.step ? element_at(b, e, remi, w, &len, &tag) : 3;
            if (first == 1 || first == 2) map0[c * w.step + e] = first == 1 ? kNxtEnd : kNxtCorrupt;
            uint64_t alive = __ballot(first == 0);
            while (alive) {
                const int j = __builtin_ctzll(alive);
                alive &= alive - 1;
                uint32_t nrec = 0, nevt = 0;
                int stop = 0, bt = 0;
                const int r = wave_walk(b, e0 + j, remi, w, &nrec, &nevt, &stop, &bt, [](int, int, uint32_t, uint32_t) {});
                const uint32_t nx = r == 0 ? (uint32_t)(stop - kChunk) : r == 1 ? kNxtEnd : kNxtCorrupt;
                if (lane == 0) map0[c * w.step + e0 + j] = nx | (nrec << 8) | (nevt << 20);   // <= 683 elements per chunk
            }
        }
    }
}

// Level maps: SoA (next u8, nrec u32, nevt u32) per (item, entry offset). Level 0 is the packed scan map.
struct LevelMap {
    const uint32_t* packed;            // level 0
    const uint8_t* nxt;
    const uint32_t* nrec;
    const uint32_t* nevt;
};

__device__ __forceinline__ void load_children(const LevelMap& m, int64_t first, int nch, int S, uint8_t* s_nxt,
                                              uint32_t* s_nrec, uint32_t* s_nevt) {
    const int64_t base = first * S;
    for (int i = threadIdx.x; i < nch * S; i += blockDim.x) {
        if (m.packed) {
            const uint32_t v = m.packed[base + i];
            s_nxt[i] = (uint8_t)(v & 0xFF);
            s_nrec[i] = (v >> 8) & 0xFFF;
            s_nevt[i] = v >> 20;
        } else {
            s_nxt[i] = m.nxt[base + i];
            s_nrec[i] = m.nrec[base + i];
            s_nevt[i] = m.nevt[base + i];
        }
    }
}

// ---- compose: parent map = composition of its (up to `fan`) children's maps ----
__global__ __launch_bounds__(256) void wire_compose_kernel(LevelMap child, int64_t nitems, int S, int fan,
                                                            uint8_t* __restrict__ p_nxt, uint32_t* __restrict__ p_nrec,
                                                            uint32_t* __restrict__ p_nevt) {
    extern __shared__ uint32_t lds[];
    uint32_t* s_nrec = lds;
    uint32_t* s_nevt = s_nrec + fan * S;
    uint8_t* s_nxt = reinterpret_cast<uint8_t*>(s_nevt + fan * S);
    const int64_t first = (int64_t)blockIdx.x * fan;
    const int nch = (int)std::min<int64_t>(fan, nitems - first);
    load_children(child, first, nch, S, s_nxt, s_nrec, s_nevt);
    __syncthreads();
    for (int e = threadIdx.x; e < S; e += blockDim.x) {
        uint32_t cur = (uint32_t)e, nrec = 0, nevt = 0;
        for (int k = 0; k < nch; ++k) {
            const int i = k * S + (int)cur;
            nrec += s_nrec[i];
            nevt += s_nevt[i];
            cur = s_nxt[i];
            if (cur >= kNxtEnd) break;
        }
        const int64_t o = (int64_t)blockIdx.x * S + e;
        p_nxt[o] = (uint8_t)cur;
        p_nrec[o] = nrec;
        p_nevt[o] = nevt;
    }
}

// ---- resolve: a parent's entry offset and first record / event index -> each child's ----
__global__ __launch_bounds__(256) void wire_resolve_kernel(LevelMap child, int64_t nitems, int S, int fan,
                                                            const uint8_t* __restrict__ p_ent,
                                                            const uint64_t* __restrict__ p_rec,
                                                            const uint64_t* __restrict__ p_evt,
                                                            uint8_t* __restrict__ c_ent, uint64_t* __restrict__ c_rec,
                                                            uint64_t* __restrict__ c_evt) {
    extern __shared__ uint32_t lds[];
    uint32_t* s_nrec = lds;
    uint32_t* s_nevt = s_nrec + fan * S;
    uint8_t* s_nxt = reinterpret_cast<uint8_t*>(s_nevt + fan * S);
    const int64_t first = (int64_t)blockIdx.x * fan;
    const int nch = (int)std::min<int64_t>(fan, nitems - first);
    load_children(child, first, nch, S, s_nxt, s_nrec, s_nevt);
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t cur = p_ent[blockIdx.x];
    uint64_t rb = p_rec[blockIdx.x], eb = p_evt[blockIdx.x];
    for (int k = 0; k < nch; ++k) {
        c_ent[first + k] = (uint8_t)cur;
        c_rec[first + k] = rb;
        c_evt[first + k] = eb;
        if (cur == kDead) continue;
        const int i = k * S + (int)cur;
        rb += s_nrec[i];
        eb += s_nevt[i];
        cur = s_nxt[i] >= kNxtEnd ? kDead : s_nxt[i];
    }
}

struct DecodeOut {
    int64_t* key;
    int64_t* ts;
    void* col[FWA_MAX_COLS];
    uint8_t* col_null[FWA_MAX_COLS];
    uint8_t* key_null;
    int64_t* evt_pos;
    int32_t* evt_tag;
    int64_t* evt_val;
    int64_t evt_cap;
    WireStatus* st;
};

__device__ void raise_err(WireStatus* st, int code, int tag, int64_t pos) {
    if (atomicCAS(&st->error, 0, code) == 0) {
        st->err_tag = tag;
        st->err_pos = pos;
    }
}

// Field f of a record whose value starts at q (TUPLE) / whose row starts at q (ROWDATA), as 64 bits
// (INT sign-extended, FLOAT as its 32 bits in the low word, DOUBLE bits).
__device__ __forceinline__ uint64_t read_field(const Lds& b, int q, int f, const WireConst& w) {
    const int t = w.ftype[f];
    const int at = q + w.foff[f];
    if (w.format == FWA_WIRE_TUPLE) {
        if (t == FWA_FIELD_LONG || t == FWA_FIELD_DOUBLE) return b.be64(at);
        const uint32_t v = b.be32(at);
        return t == FWA_FIELD_INT ? (uint64_t)(int64_t)(int32_t)v : (uint64_t)v;
    }
    if (t == FWA_FIELD_LONG || t == FWA_FIELD_DOUBLE) return b.le64(at);
    const uint32_t v = b.u32le(at);
    return t == FWA_FIELD_INT ? (uint64_t)(int64_t)(int32_t)v : (uint64_t)v;
}

__device__ __forceinline__ bool field_null(const Lds& b, int row, int f) {   // BinarySegmentUtils.bitGet
    const int bit = f + 8;                                                  // (BinaryRowData header: 8 bits)
    return (b.byte(row + (bit >> 3)) >> (bit & 7)) & 1;
}

// ---- decode: persistent 64-lane blocks; the chunk's true chain is walked from its resolved entry and every
// element is decoded by the lane that confirmed it ----
__global__ __launch_bounds__(64) void wire_decode_kernel(const uint8_t* __restrict__ in, int64_t nbytes, int64_t nchunks,
                                                          WireConst w, bool aligned, const uint8_t* __restrict__ c_ent,
                                                          const uint64_t* __restrict__ c_rec,
                                                          const uint64_t* __restrict__ c_evt, DecodeOut o) {
    __shared__ uint32_t buf[kBufWords];
    const Lds b{buf};
    Prefetch pf;
    if ((int64_t)blockIdx.x < nchunks) pf.issue(in, nbytes, blockIdx.x, (kChunk + w.step + 15) / 16, aligned);
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint32_t ent = c_ent[c];
        const int64_t cs = c * kChunk;
        const int remi = stage_pf(buf, in, nbytes, nchunks, c, c + gridDim.x, w, aligned, pf);
        if (ent == kDead) continue;
        const uint64_t rb = c_rec[c], eb = c_evt[c];
        auto visit = [&](int p, int tag, uint32_t rbefore, uint32_t erank) {
            int q = p + 5;
            if (tag <= 1) {
                const int64_t g = (int64_t)(rb + rbefore);
                int64_t ts = (int64_t)0x8000000000000000LL;          // StreamRecord without timestamp
                if (tag == FWA_TAG_REC_WITH_TIMESTAMP) { ts = (int64_t)b.be64(q); q += 8; }
                bool knull = false;
                if (w.format == FWA_WIRE_ROWDATA) {
                    if ((int32_t)b.be32(q) != w.row_size) { raise_err(o.st, FWA_E_UNSUPPORTED, tag, cs + p); return; }
                    q += 4;                                          // row bytes start; byte 0 = RowKind
                    if (b.byte(q) != 0) { raise_err(o.st, FWA_E_UNSUPPORTED, 256 + (int)b.byte(q), cs + p); return; }
                    knull = field_null(b, q, w.key_field);
                    if (w.ts_field >= 0 && field_null(b, q, w.ts_field)) { raise_err(o.st, FWA_E_ARG, tag, cs + p); return; }
                    for (int j = 0; j < w.num_cols; ++j) o.col_null[j][g] = field_null(b, q, w.col_field[j]);
                    o.key_null[g] = knull;
                }
                o.key[g] = knull ? 0 : (int64_t)read_field(b, q, w.key_field, w);
                o.ts[g] = w.ts_field >= 0 ? (int64_t)read_field(b, q, w.ts_field, w) : ts;
                for (int j = 0; j < w.num_cols; ++j) {
                    const int f = w.col_field[j];
                    const uint64_t v = read_field(b, q, f, w);
                    if (w.ftype[f] == FWA_FIELD_FLOAT) reinterpret_cast<uint32_t*>(o.col[j])[g] = (uint32_t)v;
                    else reinterpret_cast<uint64_t*>(o.col[j])[g] = v;
                }
            } else {
                const int64_t g = (int64_t)(eb + erank);
                if (g >= o.evt_cap) return;                          // host grows the list and decodes again
                int64_t v[4] = {0, 0, 0, 0};
                if (tag == FWA_TAG_WATERMARK) v[0] = (int64_t)b.be64(q);
                else if (tag == FWA_TAG_STREAM_STATUS) v[0] = (int32_t)b.be32(q);
                else if (tag == FWA_TAG_LATENCY_MARKER) {
                    v[0] = (int64_t)b.be64(q);
                    v[1] = (int64_t)b.be64(q + 8);
                    v[2] = (int64_t)b.be64(q + 16);
                    v[3] = (int32_t)b.be32(q + 24);
                } else v[0] = b.byte(q) != 0;                        // RECORD_ATTRIBUTES: readBoolean
                o.evt_pos[g] = (int64_t)(rb + rbefore);
                o.evt_tag[g] = tag;
                for (int k = 0; k < 4; ++k) o.evt_val[4 * g + k] = v[k];
            }
        };
        uint32_t nrec = 0, nevt = 0;
        int stop = 0, bt = 0;
        const int r = wave_walk(b, (int)ent, remi, w, &nrec, &nevt, &stop, &bt, visit);
        if (threadIdx.x == 0) {
            if (r == 1) o.st->consumed = cs + stop;
            else if (r == 2) raise_err(o.st, FWA_E_CORRUPT, bt, cs + stop);
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// host side

struct fwa_wire_decoder {
    fwa_wire_schema sc;
    WireConst w;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // input staging (host inputs)
    uint8_t* d_in = nullptr;
    int64_t in_cap = 0;
    // level maps
    uint32_t* map0 = nullptr;
    int64_t map0_cap = 0;                  // entries
    uint8_t* lv_nxt = nullptr;             // all levels >= 1, concatenated
    uint32_t* lv_nrec = nullptr;
    uint32_t* lv_nevt = nullptr;
    int64_t lv_cap = 0;                    // entries
    uint8_t* ent = nullptr;                // per item of every level (concatenated): entry offset / dead
    uint64_t* rec = nullptr;
    uint64_t* evt = nullptr;
    int64_t ent_cap = 0;
    // outputs
    int64_t* key = nullptr;
    int64_t* ts = nullptr;
    void* col[FWA_MAX_COLS] = {};
    uint8_t* col_null[FWA_MAX_COLS] = {};
    uint8_t* key_null = nullptr;
    int64_t out_cap = 0;
    int64_t* d_evt_pos = nullptr;
    int32_t* d_evt_tag = nullptr;
    int64_t* d_evt_val = nullptr;
    int64_t evt_cap = 0;
    std::vector<int64_t> h_evt_pos, h_evt_val;
    std::vector<int32_t> h_evt_tag;
    WireStatus* d_st = nullptr;
    WireStatus* h_st = nullptr;            // pinned
    uint32_t* h_root = nullptr;            // pinned: root nrec / nevt / nxt
    hipEvent_t ev[4] = {};
    fwa_wire_stats stats = {};
};

namespace {

int fail(fwa_wire_decoder* d, int code, const std::string& m) {
    if (d) d->err = m;
    return code;
}

#define WCK(call)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(d, e_ == hipErrorOutOfMemory ? FWA_E_OOM : FWA_E_DEVICE,                  \
                        std::string(#call ": ") + hipGetErrorString(e_));                          \
    } while (0)

template <class T>
int grow(fwa_wire_decoder* d, T** p, int64_t* cap, int64_t need, int64_t elem = sizeof(T)) {
    if (need <= *cap) return 0;
    int64_t n = std::max<int64_t>(need, *cap + *cap / 2);
    if (*p) WCK(hipFree(*p));
    *p = nullptr;
    WCK(hipMalloc((void**)p, std::max<int64_t>(n, 1) * elem));
    *cap = n;
    return 0;
}

int field_bytes(int t) { return (t == FWA_FIELD_LONG || t == FWA_FIELD_DOUBLE) ? 8 : 4; }

int compose_fan(int S) {
    const int per = S * 9;                 // nrec + nevt + nxt per entry
    return std::max(2, std::min(64, kLdsBudget / per));
}

int grow_outputs(fwa_wire_decoder* d, int64_t n) {
    if (n <= d->out_cap) return 0;
    const int64_t cap = std::max<int64_t>(n, d->out_cap + d->out_cap / 2);
    auto re = [&](void** p, int64_t elem) -> int {
        if (*p) WCK(hipFree(*p));
        *p = nullptr;
        WCK(hipMalloc(p, std::max<int64_t>(cap, 1) * elem));
        return 0;
    };
    int rc;
    if ((rc = re((void**)&d->key, 8)) || (rc = re((void**)&d->ts, 8))) return rc;
    for (int j = 0; j < d->w.num_cols; ++j) {
        if ((rc = re(&d->col[j], d->w.ftype[d->w.col_field[j]] == FWA_FIELD_FLOAT ? 4 : 8))) return rc;
        if (d->w.format == FWA_WIRE_ROWDATA && (rc = re((void**)&d->col_null[j], 1))) return rc;
    }
    if (d->w.format == FWA_WIRE_ROWDATA && (rc = re((void**)&d->key_null, 1))) return rc;
    d->out_cap = cap;
    return 0;
}

int grow_events(fwa_wire_decoder* d, int64_t n) {
    if (n <= d->evt_cap) return 0;
    const int64_t cap = std::max<int64_t>(n, 2 * d->evt_cap);
    int64_t c1 = 0, c2 = 0, c3 = 0;
    if (d->d_evt_pos) WCK(hipFree(d->d_evt_pos));
    if (d->d_evt_tag) WCK(hipFree(d->d_evt_tag));
    if (d->d_evt_val) WCK(hipFree(d->d_evt_val));
    d->d_evt_pos = nullptr; d->d_evt_tag = nullptr; d->d_evt_val = nullptr;
    int rc;
    if ((rc = grow(d, &d->d_evt_pos, &c1, cap)) || (rc = grow(d, &d->d_evt_tag, &c2, cap)) ||
        (rc = grow(d, &d->d_evt_val, &c3, 4 * cap)))
        return rc;
    d->evt_cap = cap;
    return 0;
}

}  // namespace

extern "C" {

int fwa_wire_create(const fwa_wire_schema* s, fwa_wire_decoder** out) {
    if (!s || !out) return FWA_E_ARG;
    *out = nullptr;
    fwa_wire_decoder* d = new fwa_wire_decoder();
    d->sc = *s;
    WireConst& w = d->w;
    memset(&w, 0, sizeof(w));
    auto bad = [&](int code, const char* m) { d->err = m; int c = code; fwa_wire_destroy(d); return c; };
    if (s->format != FWA_WIRE_TUPLE && s->format != FWA_WIRE_ROWDATA) return bad(FWA_E_ARG, "unknown wire format");
    if (s->arity < 1 || s->arity > FWA_WIRE_MAX_FIELDS) return bad(FWA_E_ARG, "arity out of range");
    if (s->num_cols < 0 || s->num_cols > FWA_MAX_COLS) return bad(FWA_E_ARG, "num_cols out of range");
    w.format = s->format;
    w.arity = s->arity;
    int off = 0;
    w.nullbits = ((s->arity + 63 + 8) / 64) * 8;                  // BinaryRowData.calculateBitSetWidthInBytes
    for (int f = 0; f < s->arity; ++f) {
        const int t = s->field[f];
        if (t < FWA_FIELD_LONG || t > FWA_FIELD_INT) return bad(FWA_E_UNSUPPORTED, "unsupported field type");
        w.ftype[f] = t;
        if (s->format == FWA_WIRE_TUPLE) { w.foff[f] = off; off += field_bytes(t); }
        else w.foff[f] = w.nullbits + 8 * f;
    }
    auto integral = [&](int f) { return f >= 0 && f < s->arity && (w.ftype[f] == FWA_FIELD_LONG || w.ftype[f] == FWA_FIELD_INT); };
    if (!integral(s->key_field)) return bad(FWA_E_ARG, "key_field must be a LONG or INT field");
    if (s->ts_field != -1 && !integral(s->ts_field)) return bad(FWA_E_ARG, "ts_field must be -1 or a LONG/INT field");
    w.key_field = s->key_field;
    w.ts_field = s->ts_field;
    w.num_cols = s->num_cols;
    for (int j = 0; j < s->num_cols; ++j) {
        if (s->col_field[j] < 0 || s->col_field[j] >= s->arity) return bad(FWA_E_ARG, "col_field out of range");
        w.col_field[j] = s->col_field[j];
    }
    int value_len;
    if (s->format == FWA_WIRE_TUPLE) value_len = off;
    else { w.row_size = w.nullbits + 8 * s->arity; value_len = 4 + w.row_size; }
    w.body[FWA_TAG_REC_WITH_TIMESTAMP] = 1 + 8 + value_len;
    w.body[FWA_TAG_REC_WITHOUT_TIMESTAMP] = 1 + value_len;
    w.body[FWA_TAG_WATERMARK] = 1 + 8;
    w.body[FWA_TAG_LATENCY_MARKER] = 1 + 8 + 8 + 8 + 4;
    w.body[FWA_TAG_STREAM_STATUS] = 1 + 4;
    w.body[FWA_TAG_RECORD_ATTRIBUTES] = 1 + 1;
    int mx = 0;
    for (int t = 0; t < 6; ++t) mx = std::max(mx, w.body[t]);
    w.step = 4 + mx;
    if (w.step > kMaxStep) return bad(FWA_E_UNSUPPORTED, "elements longer than 249 bytes");
    d->device = s->device;
    hipError_t e;
    if ((e = hipSetDevice(d->device)) != hipSuccess || (e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc((void**)&d->d_st, sizeof(WireStatus))) != hipSuccess ||
        (e = hipHostMalloc((void**)&d->h_st, sizeof(WireStatus))) != hipSuccess ||
        (e = hipHostMalloc((void**)&d->h_root, 4 * sizeof(uint32_t))) != hipSuccess)
        return bad(FWA_E_DEVICE, hipGetErrorString(e));
    for (auto& x : d->ev)
        if ((e = hipEventCreate(&x)) != hipSuccess) return bad(FWA_E_DEVICE, hipGetErrorString(e));
    const int64_t hint = s->max_bytes > 0 ? s->max_bytes : (64ll << 20);
    int rc;
    if ((rc = grow_outputs(d, hint / (4 + std::min(w.body[0], w.body[1]))) ) || (rc = grow_events(d, 1 << 14))) {
        int c = rc;
        fwa_wire_destroy(d);
        return c;
    }
    *out = d;
    return FWA_OK;
}

void fwa_wire_destroy(fwa_wire_decoder* d) {
    if (!d) return;
    if (d->device >= 0) (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    void* ps[] = {d->d_in, d->map0, d->lv_nxt, d->lv_nrec, d->lv_nevt, d->ent, d->rec, d->evt, d->key, d->ts,
                  d->key_null, d->d_evt_pos, d->d_evt_tag, d->d_evt_val, d->d_st};
    for (void* p : ps) if (p) (void)hipFree(p);
    for (int j = 0; j < FWA_MAX_COLS; ++j) {
        if (d->col[j]) (void)hipFree(d->col[j]);
        if (d->col_null[j]) (void)hipFree(d->col_null[j]);
    }
    if (d->h_st) (void)hipHostFree(d->h_st);
    if (d->h_root) (void)hipHostFree(d->h_root);
    for (auto& x : d->ev) if (x) (void)hipEventDestroy(x);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

const char* fwa_wire_last_error(const fwa_wire_decoder* d) { return d ? d->err.c_str() : "null decoder"; }

int fwa_wire_get_stats(fwa_wire_decoder* d, fwa_wire_stats* out) {
    if (!d || !out) return FWA_E_ARG;
    *out = d->stats;
    return FWA_OK;
}

int fwa_wire_decode(fwa_wire_decoder* d, const uint8_t* bytes, int64_t nbytes, int32_t flags, fwa_wire_batch* out) {
    if (!d || !out || nbytes < 0 || (nbytes > 0 && !bytes)) return fail(d, FWA_E_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    WCK(hipSetDevice(d->device));
    const WireConst& w = d->w;
    const int S = w.step;
    const uint8_t* in = bytes;
    if (!(flags & FWA_WIRE_DEVICE_BYTES) && nbytes > 0) {
        int rc = grow(d, &d->d_in, &d->in_cap, nbytes);
        if (rc) return rc;
        WCK(hipMemcpyAsync(d->d_in, bytes, nbytes, hipMemcpyHostToDevice, d->stream));
        in = d->d_in;
    }
    const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    const int64_t nchunks = nbytes / kChunk + 1;                  // the last chunk always holds the stream end
    // level sizes
    const int fan = compose_fan(S);
    std::vector<int64_t> n_items{nchunks};
    while (n_items.back() > 1) n_items.push_back((n_items.back() + fan - 1) / fan);
    const int L = (int)n_items.size();                            // levels 0..L-1, level L-1 has 1 item
    std::vector<int64_t> lv_off(L, 0), it_off(L, 0);              // level l >= 1 map offset; item offset (all levels)
    int64_t lv_total = 0, it_total = 0;
    for (int l = 0; l < L; ++l) {
        it_off[l] = it_total;
        it_total += n_items[l] + 1;
        if (l >= 1) { lv_off[l] = lv_total; lv_total += n_items[l] * S; }
    }
    int rc;
    if ((rc = grow(d, &d->map0, &d->map0_cap, nchunks * S))) return rc;
    if (lv_total > d->lv_cap) {                                   // the three level arrays share one capacity
        for (void* p : {(void*)d->lv_nxt, (void*)d->lv_nrec, (void*)d->lv_nevt}) if (p) WCK(hipFree(p));
        d->lv_nxt = nullptr; d->lv_nrec = nullptr; d->lv_nevt = nullptr;
        const int64_t cap = std::max<int64_t>(lv_total, d->lv_cap + d->lv_cap / 2);
        WCK(hipMalloc((void**)&d->lv_nxt, cap));
        WCK(hipMalloc((void**)&d->lv_nrec, cap * 4));
        WCK(hipMalloc((void**)&d->lv_nevt, cap * 4));
        d->lv_cap = cap;
    }
    if (it_total > d->ent_cap) {                                  // per-item entry / bases, all levels
        for (void* p : {(void*)d->ent, (void*)d->rec, (void*)d->evt}) if (p) WCK(hipFree(p));
        d->ent = nullptr; d->rec = nullptr; d->evt = nullptr;
        const int64_t cap = std::max<int64_t>(it_total, d->ent_cap + d->ent_cap / 2);
        WCK(hipMalloc((void**)&d->ent, cap));
        WCK(hipMalloc((void**)&d->rec, cap * 8));
        WCK(hipMalloc((void**)&d->evt, cap * 8));
        d->ent_cap = cap;
    }
    // worst case records: every element a record of the shorter record kind
    if ((rc = grow_outputs(d, nbytes / (4 + std::min(w.body[0], w.body[1])) + 1))) return rc;

    hipStream_t st = d->stream;
    WCK(hipMemsetAsync(d->d_st, 0, sizeof(WireStatus), st));
    WCK(hipEventRecord(d->ev[0], st));
    const unsigned grid = (unsigned)std::min<int64_t>(nchunks, kPersistBlocks);
    hipLaunchKernelGGL(wire_scan_kernel, dim3(grid), dim3(64), 0, st, in, nbytes, nchunks, w, aligned, d->map0);
    WCK(hipGetLastError());
    WCK(hipEventRecord(d->ev[1], st));
    auto level_map = [&](int l) {
        LevelMap m{};
        if (l == 0) m.packed = d->map0;
        else { m.nxt = d->lv_nxt + lv_off[l]; m.nrec = d->lv_nrec + lv_off[l]; m.nevt = d->lv_nevt + lv_off[l]; }
        return m;
    };
    const int tpb = S <= 64 ? 64 : (S <= 128 ? 128 : 256);
    const size_t lds = (size_t)fan * S * 9 + 16;
    for (int l = 0; l + 1 < L; ++l) {
        hipLaunchKernelGGL(wire_compose_kernel, dim3((unsigned)n_items[l + 1]), dim3(tpb), lds, st, level_map(l),
                           n_items[l], S, fan, d->lv_nxt + lv_off[l + 1], d->lv_nrec + lv_off[l + 1],
                           d->lv_nevt + lv_off[l + 1]);
        WCK(hipGetLastError());
    }
    // root: entry 0, first record / event 0
    const int64_t root = it_off[L - 1];
    WCK(hipMemsetAsync(d->ent + root, 0, 1, st));
    WCK(hipMemsetAsync(d->rec + root, 0, 8, st));
    WCK(hipMemsetAsync(d->evt + root, 0, 8, st));
    for (int l = L - 2; l >= 0; --l) {
        hipLaunchKernelGGL(wire_resolve_kernel, dim3((unsigned)n_items[l + 1]), dim3(tpb), lds, st, level_map(l),
                           n_items[l], S, fan, d->ent + it_off[l + 1], d->rec + it_off[l + 1], d->evt + it_off[l + 1],
                           d->ent + it_off[l], d->rec + it_off[l], d->evt + it_off[l]);
        WCK(hipGetLastError());
    }
    // totals of the whole call = the root map at entry 0
    if (L == 1) {
        WCK(hipMemcpyAsync(d->h_root, d->map0, 4, hipMemcpyDeviceToHost, st));
    } else {
        WCK(hipMemcpyAsync(d->h_root + 1, d->lv_nrec + lv_off[L - 1], 4, hipMemcpyDeviceToHost, st));
        WCK(hipMemcpyAsync(d->h_root + 2, d->lv_nevt + lv_off[L - 1], 4, hipMemcpyDeviceToHost, st));
    }
    DecodeOut o{};
    o.key = d->key;
    o.ts = d->ts;
    for (int j = 0; j < FWA_MAX_COLS; ++j) { o.col[j] = d->col[j]; o.col_null[j] = d->col_null[j]; }
    o.key_null = d->key_null;
    o.st = d->d_st;
    for (int pass = 0; pass < 2; ++pass) {
        o.evt_pos = d->d_evt_pos;
        o.evt_tag = d->d_evt_tag;
        o.evt_val = d->d_evt_val;
        o.evt_cap = d->evt_cap;
        hipLaunchKernelGGL(wire_decode_kernel, dim3(grid), dim3(64), 0, st, in, nbytes, nchunks, w, aligned,
                           d->ent, d->rec, d->evt, o);
        WCK(hipGetLastError());
        WCK(hipEventRecord(d->ev[2], st));
        WCK(hipMemcpyAsync(d->h_st, d->d_st, sizeof(WireStatus), hipMemcpyDeviceToHost, st));
        WCK(hipStreamSynchronize(st));
        int64_t nrec, nevt;
        if (L == 1) { nrec = (d->h_root[0] >> 8) & 0xFFF; nevt = d->h_root[0] >> 20; }
        else { nrec = d->h_root[1]; nevt = d->h_root[2]; }
        if (nevt > d->evt_cap && pass == 0) {                     // more events than the list holds: grow, decode again
            if ((rc = grow_events(d, nevt))) return rc;
            WCK(hipMemsetAsync(d->d_st, 0, sizeof(WireStatus), st));
            continue;
        }
        float ms_scan = 0, ms_all = 0;
        (void)hipEventElapsedTime(&ms_scan, d->ev[0], d->ev[1]);
        (void)hipEventElapsedTime(&ms_all, d->ev[0], d->ev[2]);
        d->stats.calls++;
        d->stats.bytes_in += nbytes;
        d->stats.scan_ms += ms_scan;
        d->stats.decode_ms += ms_all;
        const WireStatus& hs = *d->h_st;
        if (hs.error) {
            char m[160];
            if (hs.error == FWA_E_CORRUPT) snprintf(m, sizeof m, "Corrupt stream, found tag: %d (element at byte %lld)", hs.err_tag, (long long)hs.err_pos);
            else if (hs.error == FWA_E_ARG) snprintf(m, sizeof m, "NULL rowtime field in the row at byte %lld", (long long)hs.err_pos);
            else if (hs.err_tag >= 256) snprintf(m, sizeof m, "RowKind %d at byte %lld: window aggregation consumes insert-only rows", hs.err_tag - 256, (long long)hs.err_pos);
            else snprintf(m, sizeof m, "row size differs from the schema's fixed-length row at byte %lld", (long long)hs.err_pos);
            return fail(d, hs.error, m);
        }
        d->stats.records_out += nrec;
        if (nevt > 0) {
            d->h_evt_pos.resize(nevt);
            d->h_evt_tag.resize(nevt);
            d->h_evt_val.resize(4 * nevt);
            WCK(hipMemcpy(d->h_evt_pos.data(), d->d_evt_pos, nevt * 8, hipMemcpyDeviceToHost));
            WCK(hipMemcpy(d->h_evt_tag.data(), d->d_evt_tag, nevt * 4, hipMemcpyDeviceToHost));
            WCK(hipMemcpy(d->h_evt_val.data(), d->d_evt_val, nevt * 32, hipMemcpyDeviceToHost));
        }
        out->n_records = nrec;
        out->n_events = nevt;
        out->consumed = hs.consumed;
        out->key = d->key;
        out->ts = d->ts;
        for (int j = 0; j < w.num_cols; ++j) { out->col[j] = d->col[j]; out->col_null[j] = d->col_null[j]; }
        out->key_null = d->key_null;
        out->evt_pos = nevt ? d->h_evt_pos.data() : nullptr;
        out->evt_tag = nevt ? d->h_evt_tag.data() : nullptr;
        out->evt_val = nevt ? d->h_evt_val.data() : nullptr;
        return FWA_OK;
    }
    return fail(d, FWA_E_STATE, "event list did not settle");
}

}  // extern "C"
