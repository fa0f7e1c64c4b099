// Micro-benchmark: LDS operation rates on gfx950 with random addresses (cost model for the combiner).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

template <int OP>
__global__ void __launch_bounds__(1024) k(unsigned long long* out, int iters, int nslots) {
    extern __shared__ unsigned long long lds[];
    for (int i = threadIdx.x; i < nslots; i += blockDim.x) lds[i] = i;
    __syncthreads();
    uint32_t s = hash32(threadIdx.x * 7919 + blockIdx.x * 104729);
    unsigned long long acc = 0;
    const uint32_t mask = nslots - 1;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            s = s * 1664525u + 1013904223u;
            const uint32_t a = (s >> 8) & mask;
            if (OP == 0) acc += lds[a];                                  // ds_read_b64
            if (OP == 1) atomicAdd(&lds[a], 1ull);                       // ds_add_u64
            if (OP == 2) atomicAdd((unsigned*)&lds[0] + a, 1u);          // ds_add_u32
            if (OP == 3) atomicAdd((double*)&lds[a], 1.0);               // ds_add_f64
            if (OP == 4) atomicMax(&lds[a], (unsigned long long)s);      // ds_max_u64
            if (OP == 5) { atomicAdd(&lds[a], 1ull); atomicAdd((unsigned*)&lds[nslots] + a, 1u); }
            if (OP == 6) { const unsigned long long v = lds[a]; if (v == 12345678901ull) acc += atomicAdd(&lds[a], 1ull); else atomicAdd(&lds[(a + 1) & mask], v & 1); }
            if (OP == 7) lds[a] = s;                                     // ds_write_b64
        }
    }
    __syncthreads();
    if (acc == 1) out[0] = acc;
    if (threadIdx.x == 0) out[blockIdx.x + 1] = lds[threadIdx.x];
}

int main() {
    unsigned long long* out;
    hipMalloc(&out, 8 * 4096);
    const int nslots = 8192;   // 64 KB of u64
    const int iters = 256;
    const char* names[] = {"ds_read_b64", "ds_add_u64", "ds_add_u32", "ds_add_f64", "ds_max_u64", "add_u64+add_u32", "read->dep atomic", "ds_write_b64"};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int threads : {256, 1024}) {
        for (int op = 0; op < 8; ++op) {
            const int grid = 256 * (threads == 256 ? 4 : 1);
            const size_t lds = nslots * 8 + nslots * 4 + 64;
            auto launch = [&]() {
                switch (op) {
                    case 0: k<0><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 1: k<1><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 2: k<2><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 3: k<3><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 4: k<4><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 5: k<5><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 6: k<6><<<grid, threads, lds>>>(out, iters, nslots); break;
                    case 7: k<7><<<grid, threads, lds>>>(out, iters, nslots); break;
                }
            };
            launch();
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double ops = (double)grid * threads * iters * 8;
            // per CU: (ops / 256) lane-ops in ms; cycles at 2.4 GHz per wave-instruction
            const double wave_instr_per_cu = ops / 64 / 256;
            printf("%4d thr  %-18s %8.3f ms  %7.1f G lane-ops/s  %6.1f cyc per wave-op per CU\n", threads, names[op], ms,
                   ops / ms / 1e6, ms * 1e-3 * 2.4e9 / wave_instr_per_cu);
        }
    }
    return 0;
}
