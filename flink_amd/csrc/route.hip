// route.hip -- the keyBy exchange's send side for a columnar batch on the GPU (include/flink_amd.h fwa_route_rows).
//
// Reference: KeyGroupStreamPartitioner.selectChannel (flink-streaming-java/.../partitioner/
// KeyGroupStreamPartitioner.java:55-65) picks each record's channel = computeOperatorIndexForKeyGroup(maxP, P,
// assignToKeyGroup(key)) (KeyGroupRangeAssignment.java:63-127), and the RecordWriter serialises the record into that
// channel's buffer (RecordWriter.java:104-157) in arrival order. Here a batch is counting-sorted by destination in two
// passes, all on the device:
//   count   : per block (a contiguous range of records), the rows per destination (LDS histogram)
//   offsets : one block scans the [destination][block] table into each block's first row per destination
//   scatter : per block, in record order, ranks equal destinations with ballots and writes the packed rows
//             (ncols 8-byte cells, 4-byte columns zero-extended) to their destination's run
// so each destination's rows stay in arrival order (a channel preserves order) and the packed buffer feeds one
// all_to_all_single. Bound: HBM (read the columns twice, write the rows once).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/flink_amd.h"
#include "java_math.h"

namespace {

constexpr int kRouteBlock = 256;
constexpr int kMaxDest = 64;
constexpr int kRouteBlocks = 2048;
constexpr int kMaxRouteCols = 16;

struct UnpackCols {
    int64_t* col[kMaxRouteCols];
};

struct RouteArgs {
    const int64_t* keys;
    const int32_t* key_hash;
    int64_t n, per;                    // records; records per block
    int32_t key_kind, maxp, par, ncols;
    const void* cols[kMaxRouteCols];
    int32_t bytes[kMaxRouteCols];
    uint32_t* hist;                    // [par][nblocks]: counts, then (after the scan) first row
    int64_t* out;                      // [n][ncols]
    int64_t* counts;                   // [par]
};

__device__ __forceinline__ int32_t dest_of(const RouteArgs& a, int64_t i) {
    const int32_t kg = jm::key_group_of(a.keys[i], a.key_kind, a.key_hash ? a.key_hash[i] : 0, a.maxp);
    // an id no subtask owns (key group -1, java_math.h) goes to subtask 0, whose ingest rejects it (FWA_E_KEYGROUP)
    return kg < 0 ? 0 : jm::operator_index(a.maxp, a.par, kg);
}

__global__ void __launch_bounds__(kRouteBlock) route_count_kernel(RouteArgs a) {
    __shared__ uint32_t h[kMaxDest];
    for (int d = threadIdx.x; d < a.par; d += kRouteBlock) h[d] = 0;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * a.per, hi = std::min<int64_t>(lo + a.per, a.n);
    for (int64_t i = lo + threadIdx.x; i < hi; i += kRouteBlock) atomicAdd(&h[dest_of(a, i)], 1u);
    __syncthreads();
    for (int d = threadIdx.x; d < a.par; d += kRouteBlock) a.hist[(int64_t)d * gridDim.x + blockIdx.x] = h[d];
}

// exclusive scan over [dest][block] (destination-major: each destination's rows are one run), one block
__global__ void __launch_bounds__(1024) route_scan_kernel(uint32_t* hist, int64_t total, int32_t par, int32_t nblocks,
                                                          int64_t* counts) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < total; base += 1024) {
        const int64_t i = base + threadIdx.x;
        const uint32_t v = i < total ? hist[i] : 0u;
        uint32_t x = v;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(x, d); if (lane >= d) x += y; }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        if (threadIdx.x == 0) { uint32_t r = 0; for (int k = 0; k < 16; ++k) { const uint32_t t = wsum[k]; wsum[k] = r; r += t; } }
        __syncthreads();
        const uint32_t excl = carry + wsum[w] + x - v;
        if (i < total) hist[i] = excl;
        __syncthreads();
        if (threadIdx.x == 1023) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x < par) {                       // rows per destination
        const int d = threadIdx.x;
        const uint32_t first = hist[(int64_t)d * nblocks];
        const uint32_t next = d + 1 < par ? hist[(int64_t)(d + 1) * nblocks] : carry;
        counts[d] = (int64_t)(next - first);
    }
}

__global__ void __launch_bounds__(kRouteBlock) route_scatter_kernel(RouteArgs a) {
    __shared__ uint32_t run[kMaxDest];             // next row of each destination for this block
    __shared__ uint32_t wcnt[kRouteBlock / 64][kMaxDest];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < a.par; d += kRouteBlock) run[d] = a.hist[(int64_t)d * gridDim.x + blockIdx.x];
    const int64_t lo = (int64_t)blockIdx.x * a.per, hi = std::min<int64_t>(lo + a.per, a.n);
    const uint64_t below = (1ull << lane) - 1;
    for (int64_t base = lo; base < hi; base += kRouteBlock) {
        const int64_t i = base + threadIdx.x;
        const bool ok = i < hi;
        const int32_t d = ok ? dest_of(a, i) : -1;
        uint32_t my_rank = 0;
        __syncthreads();                           // run[] of the previous chunk final
        for (int q = 0; q < a.par; ++q) {
            const uint64_t m = __ballot(d == q);
            if (lane == 0) wcnt[w][q] = (uint32_t)__popcll(m);
            if (d == q) my_rank = (uint32_t)__popcll(m & below);
        }
        __syncthreads();
        if (ok) {
            uint32_t pre = 0;
            for (int v = 0; v < w; ++v) pre += wcnt[v][d];
            const int64_t row = (int64_t)run[d] + pre + my_rank;
            int64_t* dst = a.out + row * a.ncols;
            for (int c = 0; c < a.ncols; ++c)
                dst[c] = a.bytes[c] == 8 ? ((const int64_t*)a.cols[c])[i] : (int64_t)((const uint32_t*)a.cols[c])[i];
        }
        __syncthreads();
        for (int q = threadIdx.x; q < a.par; q += kRouteBlock) {
            uint32_t t = 0;
            for (int v = 0; v < kRouteBlock / 64; ++v) t += wcnt[v][q];
            run[q] += t;
        }
    }
}

// The receive side: packed rows -> one contiguous column per cell (one kernel instead of a strided copy per column)
__global__ void __launch_bounds__(kRouteBlock) unpack_rows_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                                  int32_t ncols, UnpackCols out) {
    for (int64_t i = (int64_t)blockIdx.x * kRouteBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRouteBlock) {
        const int64_t* r = rows + i * ncols;
        for (int c = 0; c < ncols; ++c) out.col[c][i] = r[c];
    }
}

}  // namespace

extern "C" int fwa_unpack_rows(const int64_t* rows, int64_t n, int32_t ncols, int64_t* const* cols, int32_t device,
                               void* stream) {
    if (n < 0 || ncols < 1 || ncols > kMaxRouteCols || (n > 0 && (!rows || !cols))) return FWA_E_ARG;
    if (n == 0) return FWA_OK;
    UnpackCols o{};
    for (int c = 0; c < ncols; ++c) {
        if (!cols[c]) return FWA_E_ARG;
        o.col[c] = cols[c];
    }
    if (hipSetDevice(device) != hipSuccess) return FWA_E_DEVICE;
    hipStream_t st = (hipStream_t)stream;
    const int nb = (int)std::min<int64_t>(4096, (n + kRouteBlock - 1) / kRouteBlock);
    hipLaunchKernelGGL(unpack_rows_kernel, dim3(nb), dim3(kRouteBlock), 0, st, rows, n, ncols, o);
    return hipGetLastError() == hipSuccess ? FWA_OK : FWA_E_DEVICE;   // stream-ordered: no host synchronisation
}

extern "C" int fwa_route_rows(const int64_t* keys, const int32_t* key_hash, int64_t n, int32_t key_kind,
                              int32_t max_parallelism, int32_t parallelism, const void* const* cols,
                              const int32_t* col_bytes, int32_t ncols, int64_t* out, int64_t* counts, int32_t device,
                              void* stream) {
    if (n < 0 || (n > 0 && (!keys || !out)) || !counts || ncols < 1 || ncols > kMaxRouteCols || parallelism < 1 ||
        parallelism > kMaxDest || max_parallelism < parallelism || key_kind < 0 || key_kind > 2 ||
        (n > 0 && key_kind == FWA_KEY_PREHASHED && !key_hash) || n > 0xFFFFFFFFll)
        return FWA_E_ARG;
    for (int c = 0; c < ncols; ++c)
        if ((n > 0 && !cols[c]) || (col_bytes[c] != 4 && col_bytes[c] != 8)) return FWA_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FWA_E_DEVICE;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) return hipMemsetAsync(counts, 0, 8 * parallelism, st) == hipSuccess ? FWA_OK : FWA_E_DEVICE;
    RouteArgs a{};
    a.keys = keys;
    a.key_hash = key_hash;
    a.n = n;
    a.key_kind = key_kind;
    a.maxp = max_parallelism;
    a.par = parallelism;
    a.ncols = ncols;
    for (int c = 0; c < ncols; ++c) { a.cols[c] = cols[c]; a.bytes[c] = col_bytes[c]; }
    const int nb = (int)std::min<int64_t>(kRouteBlocks, (n + kRouteBlock - 1) / kRouteBlock);
    a.per = (n + nb - 1) / nb;
    uint32_t* hist = nullptr;
    if (hipMallocAsync((void**)&hist, (size_t)4 * parallelism * nb, st) != hipSuccess) return FWA_E_OOM;
    a.hist = hist;
    a.out = out;
    a.counts = counts;
    hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(kRouteBlock), 0, st, a);
    hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(1024), 0, st, hist, (int64_t)parallelism * nb, parallelism, nb, counts);
    hipLaunchKernelGGL(route_scatter_kernel, dim3(nb), dim3(kRouteBlock), 0, st, a);
    const hipError_t e1 = hipGetLastError();
    const hipError_t e2 = hipFreeAsync(hist, st);                    // stream-ordered: no host synchronisation
    return (e1 == hipSuccess && e2 == hipSuccess) ? FWA_OK : FWA_E_DEVICE;
}
