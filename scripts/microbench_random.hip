// Microbenchmark: chip-wide rate of random 8-byte loads / CAS / stores into a table of S bytes
// (the visited-set access pattern), to find the transaction ceiling that bounds the expand kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t xs(uint64_t& x) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; }

__global__ void rand_load(const uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) acc += t[xs(x) & mask];
    if (acc == 42) sink[0] = acc;
}
__global__ void rand_load4(const uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; i += 4) {
        uint64_t a = t[xs(x) & mask], b = t[xs(x) & mask], c = t[xs(x) & mask], d = t[xs(x) & mask];
        acc += a + b + c + d;
    }
    if (acc == 42) sink[0] = acc;
}
__global__ void rand_load8(const uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; i += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = t[xs(x) & mask];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j];
    }
    if (acc == 42) sink[0] = acc;
}
__global__ void rand_cas(uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) acc += atomicCAS((unsigned long long*)&t[xs(x) & mask], 0ull, 1ull);
    if (acc == 42) sink[0] = acc;
}
__global__ void rand_store(uint64_t* t, uint64_t mask, int iters) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    for (int i = 0; i < iters; ++i) t[xs(x) & mask] = x;
}

// The visited-set mix: every lane probes random keys; a fraction `claim_pct` of the probes are
// followed by a CAS on the same slot (a claim).
__global__ void rand_mix(uint64_t* t, uint64_t mask, int iters, int claim_pct, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint64_t r = xs(x);
        uint64_t* p = &t[r & mask];
        uint64_t v = *p;
        if ((r >> 40) % 100 < (uint64_t)claim_pct) v += atomicCAS((unsigned long long*)p, v, v + 1);
        acc += v;
    }
    if (acc == 42) sink[0] = acc;
}

// One kernel per (variant, table size), each timed with events; under rocprofv3 --pmc the
// kernel trace gives the EA (beyond-L2) requests of each dispatch (scripts/pmc_ceiling.sh).
int main() {
    const size_t max_bytes = 4ull << 30;
    uint64_t* t; uint64_t* sink;
    hipMalloc(&t, max_bytes); hipMalloc(&sink, 64);
    hipMemset(t, 0, max_bytes);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 256 * 8, threads = 256, iters = 256;
    const double ops = (double)blocks * threads * iters;
    for (size_t bytes : {size_t(8) << 20, size_t(32) << 20, size_t(64) << 20, size_t(128) << 20, size_t(256) << 20,
                         size_t(512) << 20, size_t(1) << 30, size_t(4) << 30}) {
        uint64_t mask = bytes / 8 - 1;
        float ms[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < 5; ++k) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (k == 0) rand_load<<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 1) rand_load4<<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 2) rand_load8<<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 3) rand_cas<<<blocks, threads>>>(t, mask, iters / 4, sink);
                if (k == 4) rand_store<<<blocks, threads>>>(t, mask, iters);
                hipEventRecord(b); hipEventSynchronize(b);
                hipEventElapsedTime(&ms[k], a, b);
            }
            hipMemset(t, 0, bytes);
        }
        printf("table %6zu MiB: load %6.2f G/s  load4 %6.2f G/s  load8 %6.2f G/s  cas %6.2f G/s  store %6.2f G/s\n",
               bytes >> 20, ops / ms[0] / 1e6, ops / ms[1] / 1e6, ops / ms[2] / 1e6, ops / 4 / ms[3] / 1e6, ops / ms[4] / 1e6);
    }
    for (int pct : {0, 10, 20, 35}) {
        uint64_t mask = (size_t(256) << 20) / 8 - 1;
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            rand_mix<<<blocks, threads>>>(t, mask, iters, pct, sink);
            hipEventRecord(b); hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        printf("mix 256 MiB, %d%% CAS: %6.2f G probes/s\n", pct, ops / ms / 1e6);
    }
    return 0;
}
