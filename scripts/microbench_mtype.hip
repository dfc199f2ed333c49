// Microbenchmark: does the memory type of the visited set change what a random 8-byte probe costs?
// A 1 GiB table allocated as ordinary device memory (hipMalloc), uncached (hipDeviceMallocUncached)
// and fine-grained (hipDeviceMallocFinegrained), probed with plain, non-temporal and agent-scope
// (sc1) loads, and claimed with random CAS. Each kernel is timed with events; under rocprofv3
// --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum the kernel trace tells the size of the requests the L2 sends
// to memory for each variant (a random probe that moved 64 B instead of a 128-B line would halve
// the visited set's memory traffic).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/microbench_mtype scripts/microbench_mtype.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint64_t xs(uint64_t& x) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; }

template <int POL>
__device__ __forceinline__ uint64_t ld(const uint64_t* p) {
    if constexpr (POL == 1) return __builtin_nontemporal_load(p);
    else if constexpr (POL == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// four independent random loads in flight per lane (the probe batch of the insert kernel)
template <int POL>
__global__ void probe4(const uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; i += 4) {
        const uint64_t a = ld<POL>(&t[xs(x) & mask]), b = ld<POL>(&t[xs(x) & mask]), c = ld<POL>(&t[xs(x) & mask]),
                       d = ld<POL>(&t[xs(x) & mask]);
        acc += a + b + c + d;
    }
    if (acc == 42) sink[0] = acc;
}

__global__ void cas1(uint64_t* t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t x = 0x9E3779B97F4A7C15ull ^ (blockIdx.x * 1024 + threadIdx.x) * 0x632BE59BD9B4E019ull;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) acc += atomicCAS((unsigned long long*)&t[xs(x) & mask], 0ull, 1ull);
    if (acc == 42) sink[0] = acc;
}

int main() {
    const size_t bytes = size_t(1) << 30;
    const uint64_t mask = bytes / 8 - 1;
    const int blocks = 256 * 8, threads = 256, iters = 256;
    const double ops = (double)blocks * threads * iters;
    uint64_t* sink;
    CHECK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const char* names[3] = {"coarse (hipMalloc)", "uncached", "fine-grained"};
    for (int kind = 0; kind < 3; ++kind) {
        uint64_t* t = nullptr;
        if (kind == 0) CHECK(hipMalloc(&t, bytes));
        else CHECK(hipExtMallocWithFlags((void**)&t, bytes, kind == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
        CHECK(hipMemset(t, 0, bytes));
        CHECK(hipDeviceSynchronize());
        float ms[4];
        for (int k = 0; k < 4; ++k) {
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipEventRecord(a));
                if (k == 0) probe4<0><<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 1) probe4<1><<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 2) probe4<2><<<blocks, threads>>>(t, mask, iters, sink);
                if (k == 3) cas1<<<blocks, threads>>>(t, mask, iters / 4, sink);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                CHECK(hipEventElapsedTime(&ms[k], a, b));
            }
            if (k == 3) CHECK(hipMemset(t, 0, bytes));
        }
        std::printf("%-20s probe plain %6.2f G/s  nt %6.2f G/s  sc1 %6.2f G/s  cas %6.2f G/s\n", names[kind], ops / ms[0] / 1e6,
                    ops / ms[1] / 1e6, ops / ms[2] / 1e6, ops / 4 / ms[3] / 1e6);
        CHECK(hipFree(t));
    }
    return 0;
}
