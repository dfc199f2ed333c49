// Same-address atomic throughput on one MI355X: `waves` waves each add to one of `spread` counters
// (lane 0 only, a wave-aggregated reservation as in expand_fast's stage flush). Reports the kernel
// time from HIP events, against an empty kernel of the same grid.
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_atomics.hip -o scripts/microbench_atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void reserve(unsigned* ctr, unsigned spread, unsigned reps, unsigned stride, unsigned* sink) {
    const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned acc = 0;
    for (unsigned r = 0; r < reps; ++r)
        if ((threadIdx.x & 63) == 0) acc += atomicAdd(&ctr[((wave + r) % spread) * stride], 100u);
    if (acc == 0xffffffffu) sink[0] = acc;
}

__global__ void empty(unsigned* sink) {
    if (threadIdx.x == 1023) sink[0] = 1;
}

int main() {
    unsigned *ctr, *sink;
    CK(hipMalloc(&ctr, 64 * 1024 * 4));
    CK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned grids[] = {3072};
    const unsigned spreads[] = {1, 2, 4, 8};
    for (unsigned g : grids)
        for (unsigned stride : {1u, 32u, 64u, 1024u})  // 4 B, 128 B, 256 B, 4 KB apart
            for (unsigned sp : spreads) {
                const unsigned reps = 1;
                float best = 1e9f, base = 1e9f;
                for (int it = 0; it < 20; ++it) {
                    CK(hipMemset(ctr, 0, 64 * 1024 * 4));
                    CK(hipEventRecord(a));
                    reserve<<<g, 256>>>(ctr, sp, reps, stride, sink);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (ms < best) best = ms;
                    CK(hipEventRecord(a));
                    empty<<<g, 256>>>(sink);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (ms < base) base = ms;
                }
                const double n = (double)g * 4 * reps;
                printf("stride=%4uB blocks=%5u waves=%6u reps=%u spread=%2u: %8.2f us (empty %6.2f us) -> %.2f ns per atomic beyond the empty grid\n",
                       stride * 4, g, g * 4, reps, sp, best * 1e3, base * 1e3, (best - base) * 1e6 / n);
            }
    return 0;
}
