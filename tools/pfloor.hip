// Phase P byte floor: what one launch shaped like partition3 can stream on MI355X when it does
// nothing but move Phase P's bytes. Reads the C2 record columns (key, ts, value: 24 B per record, 16-byte loads) and,
// per mode, writes 10 B per record (a packed u64 + a u16) either contiguously (the copy floor) or as runs into 512
// partition regions (the bucket-run shape: ~12 records per partition and 6144-record tile). Geometry as partition3:
// 1024-thread blocks, one per CU (grid 256), 6144-record tiles, the next tile's loads in flight in registers.
//   hipcc -O3 --offload-arch=gfx950 tools/pfloor.hip -o tools/pfloor && tools/pfloor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int IT = 6;

// MODE 0: read only (sum, one store per thread at the end); 1: + contiguous 10 B/record; 2: + 512-partition runs
// into per-block regions; 3: runs appended to partition buckets shared by NSUB groups of blocks (sub = block % NSUB,
// one returning cursor atomic per (tile, partition), as partition3); NT: non-temporal stores
// 4: the unsorted variant of 3 -- each record's partition from its key hash (512 partitions), its rank in the tile's
// run by an LDS counter, the run reserved per (tile, partition), every lane storing its own records (no LDS sort)
// PF: 1 = next tile's loads issued before this tile is consumed (register double buffer), 0 = load then use
template <int MODE, int PF, int NSUB = 16, int NT = 0, int TH = 1024, int NP = 512>
__global__ void __launch_bounds__(TH, 1) pfloor(const ulonglong2* __restrict__ k, const ulonglong2* __restrict__ t,
                                                const ulonglong2* __restrict__ v, int64_t ntiles,
                                                unsigned long long* __restrict__ ok, uint16_t* __restrict__ orel,
                                                unsigned long long* __restrict__ sink, int64_t region) {
    constexpr int TILE = TH * IT;
    const int tid = threadIdx.x;
    unsigned long long acc = 0;
    __shared__ uint32_t s_base[512];
    __shared__ uint32_t s_hist[512];
    if (MODE == 4) for (int q = tid; q < 512; q += TH) s_hist[q] = 0;
    unsigned int* cur = (unsigned int*)sink;   // MODE 3: NSUB x 512 cursors (zeroed by the host)
    const int64_t cap3 = region * 512 * 256 / (512 * NSUB) * 2;
    ulonglong2 rk[IT / 2], rt[IT / 2], rv[IT / 2];
    auto load = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < IT / 2; ++j) {
            const int64_t pi = tile * (TILE / 2) + (int64_t)j * TH + tid;
            rk[j] = k[pi]; rt[j] = t[pi]; rv[j] = v[pi];
        }
    };
    int64_t tile = blockIdx.x;
    if (tile < ntiles) load(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        ulonglong2 ck[IT / 2], ct[IT / 2], cv[IT / 2];
#pragma unroll
        for (int j = 0; j < IT / 2; ++j) { ck[j] = rk[j]; ct[j] = rt[j]; cv[j] = rv[j]; }
        const int64_t nx = tile + gridDim.x;
        if constexpr (MODE == 4) {
            uint32_t rk4[IT];
            unsigned long long pk[IT];
            uint32_t rl[IT];
#pragma unroll
            for (int j = 0; j < IT / 2; ++j) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const unsigned long long key = h ? ck[j].y : ck[j].x;
                    unsigned long long z = key * 0x9E3779B97F4A7C15ull; z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32;
                    const uint32_t p = (uint32_t)(z >> 55);
                    rk4[2 * j + h] = (p << 16) | atomicAdd(&s_hist[p], 1u);
                    pk[2 * j + h] = (key & 0xffffffffull) | ((h ? cv[j].y : cv[j].x) << 32);
                    rl[2 * j + h] = (uint32_t)((h ? ct[j].y : ct[j].x) / 10000) & 0xffff;
                }
            }
            __syncthreads();
            if (tid < 512) { const uint32_t hh = s_hist[tid]; s_hist[tid] = 0;
                             s_base[tid] = atomicAdd(&cur[(blockIdx.x % NSUB) * 512 + tid], hh); }
            if (PF && nx < ntiles) load(nx);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                const uint32_t p = rk4[j] >> 16;
                const int64_t o = ((int64_t)(blockIdx.x % NSUB) * 512 + p) * cap3 + s_base[p] + (rk4[j] & 0xffff);
                if (o < cap3 * 512 * NSUB) { ok[o] = pk[j]; orel[o] = (uint16_t)rl[j]; }
            }
            if (!PF && nx < ntiles) load(nx);
            continue;
        }
        if constexpr (MODE == 3) {
            __syncthreads();
            for (int q = tid; q < NP; q += TH) s_base[q] = atomicAdd(&cur[(blockIdx.x % NSUB) * 512 + q], (unsigned)(TILE / NP));
            __syncthreads();
        }
        if (PF && nx < ntiles) load(nx);
#pragma unroll
        for (int j = 0; j < IT / 2; ++j) {
            const unsigned long long a0 = (ck[j].x & 0xffffffffull) | (cv[j].x << 32);
            const unsigned long long a1 = (ck[j].y & 0xffffffffull) | (cv[j].y << 32);
            const uint16_t r0 = (uint16_t)(ct[j].x / 10000), r1 = (uint16_t)(ct[j].y / 10000);
            if constexpr (MODE == 0) {
                acc += a0 ^ a1 ^ r0 ^ r1;
            } else if constexpr (MODE == 1) {
                const int64_t o = 2 * (tile * (TILE / 2) + (int64_t)j * TH + tid);
                ok[o] = a0; ok[o + 1] = a1; orel[o] = r0; orel[o + 1] = r1;
            } else if constexpr (MODE == 3) {
                const int i0 = 2 * (j * TH + tid);
                const int p = i0 * NP / TILE;
                const int64_t o = ((int64_t)(blockIdx.x % NSUB) * 512 + p) * cap3 * (512 / NP) + s_base[p] + (i0 % (TILE / NP));
                if (o + 1 < cap3 * 512 * NSUB) {
                    if constexpr (NT) {
                        __builtin_nontemporal_store(a0, &ok[o]); __builtin_nontemporal_store(a1, &ok[o + 1]);
                        __builtin_nontemporal_store(r0, &orel[o]); __builtin_nontemporal_store(r1, &orel[o + 1]);
                    } else { ok[o] = a0; ok[o + 1] = a1; orel[o] = r0; orel[o + 1] = r1; }
                }
            } else {
                // runs: record i of the tile goes to partition (i * 512 / TILE) at the block's cursor for it
                const int i0 = 2 * (j * TH + tid);
                const int p = i0 * 512 / TILE;
                const int64_t o = (int64_t)p * region + (tile / gridDim.x) * (TILE / 512) + (i0 % (TILE / 512)) +
                                  (int64_t)blockIdx.x * region * 512;
                ok[o] = a0; ok[o + 1] = a1; orel[o] = r0; orel[o + 1] = r1;
            }
        }
        if (!PF && nx < ntiles) load(nx);
    }
    if (MODE == 0) sink[blockIdx.x * TH + tid] = acc;
}

int main() {
    const int64_t n = (int64_t)1 << 26;
    const int64_t ntiles = n / (1024 * IT);   // 1024-thread tiles (the 512-thread kernels take twice as many)
    int64_t *k, *t, *v;
    unsigned long long *ok, *sink;
    uint16_t* orel;
    CHK(hipMalloc(&k, 8 * n)); CHK(hipMalloc(&t, 8 * n)); CHK(hipMalloc(&v, 8 * n));
    const int64_t region = (ntiles / 256 + 2) * (1024 * IT / 512);  // per (block, partition)
    const int64_t outn = 2 * std::max<int64_t>(n, region * 512 * 256) + 1024 * IT;
    CHK(hipMalloc(&ok, 8 * outn)); CHK(hipMalloc(&orel, 2 * outn)); CHK(hipMalloc(&sink, 8 * 256 * 1024));
    {   // C2-like columns: uniform keys over 1M, timestamps ramping at 1000 records per ms, values
        std::vector<int64_t> h(n);
        for (int64_t i = 0; i < n; ++i) { uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; h[i] = (int64_t)(z % 1000000); }
        CHK(hipMemcpy(k, h.data(), 8 * n, hipMemcpyHostToDevice));
        for (int64_t i = 0; i < n; ++i) h[i] = 1700000000000ll + i / 1000;
        CHK(hipMemcpy(t, h.data(), 8 * n, hipMemcpyHostToDevice));
        for (int64_t i = 0; i < n; ++i) h[i] = i & 0xffff;
        CHK(hipMemcpy(v, h.data(), 8 * n, hipMemcpyHostToDevice));
    }
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    auto run = [&](auto kern, const char* name, double wbytes, int th = 1024) -> int {
        const int64_t nt = n / (th * IT);
        const int grid = th == 1024 ? 256 : 512;
        CHK(hipMemset(sink, 0, 8 * 256 * 1024));
        for (int w = 0; w < 3; ++w) kern<<<grid, th>>>((const ulonglong2*)k, (const ulonglong2*)t, (const ulonglong2*)v, nt, ok, orel, sink, region);
        CHK(hipDeviceSynchronize());
        const int reps = 20;
        CHK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) { CHK(hipMemsetAsync(sink, 0, 4 * 512 * 256)); kern<<<grid, th>>>((const ulonglong2*)k, (const ulonglong2*)t, (const ulonglong2*)v, nt, ok, orel, sink, region); }
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        const double rb = 24.0 * n;
        printf("%-44s %.3f ms per 2^26 records  read %.2f TB/s  read+write %.2f TB/s\n", name, ms, rb / ms / 1e9,
               (rb + wbytes) / ms / 1e9);
        return 0;
    };
    if (run(pfloor<0, 0>, "read only, load then use", 0)) return 1;
    if (run(pfloor<0, 1>, "read only, next tile in flight", 0)) return 1;
    if (run(pfloor<1, 0>, "read + 10 B contiguous, load then use", 10.0 * n)) return 1;
    if (run(pfloor<1, 1>, "read + 10 B contiguous, next tile in flight", 10.0 * n)) return 1;
    if (run(pfloor<2, 1>, "read + 10 B as 512-partition runs, in flight", 10.0 * n)) return 1;
    if (run(pfloor<3, 1, 16>, "runs into shared buckets, 16 subs", 10.0 * n)) return 1;
    if (run(pfloor<3, 1, 8>, "runs into shared buckets, 8 subs (per XCD)", 10.0 * n)) return 1;
    if (run(pfloor<3, 1, 16, 0, 1024, 256>, "runs into shared buckets, 16 subs, 256 parts", 10.0 * n)) return 1;
    if (run(pfloor<3, 1, 16, 0, 1024, 128>, "runs into shared buckets, 16 subs, 128 parts", 10.0 * n)) return 1;
    if (run(pfloor<3, 1, 8, 0, 1024, 256>, "runs into shared buckets, 8 subs, 256 parts", 10.0 * n)) return 1;
    return 0;
}
