// Per-boundary cost of dependent kernel launches on one stream:
//   plain      : back-to-back launches of a 1024-workgroup kernel that dirties L2 with random stores
//   graph      : the same launches captured once in a hipGraph and replayed
//   pinned     : plain launches whose first thread also stores a sequence number to pinned host
//                memory with a system-scope release (the engine's level publish)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/microbench_gaps scripts/microbench_gaps.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void touch(unsigned long long* t, unsigned long long mask, unsigned it, unsigned* host) {
    if (host && blockIdx.x == 0 && threadIdx.x == 0)  // like the engine's per-level publish to pinned memory
        __hip_atomic_store(host, it, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long i = (blockIdx.x * 256ull + threadIdx.x) * 0x9E3779B97F4A7C15ull + it;
    i ^= i >> 29;
    t[i & mask] = i;  // a random 8-byte store per thread: dirty lines spread over every XCD's L2
}

int main() {
    const unsigned long long slots = 1ull << 25;  // 256 MB table
    unsigned long long* t;
    CK(hipMalloc(&t, slots * 8));
    unsigned* host;
    CK(hipHostMalloc(&host, 64, hipHostMallocCoherent));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int N = 200;
    for (int grid : {4, 1024, 16384}) {
        for (int w = 0; w < 20; ++w) touch<<<grid, 256, 0, s>>>(t, slots - 1, w, nullptr);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        for (int k = 0; k < N; ++k) touch<<<grid, 256, 0, s>>>(t, slots - 1, k, nullptr);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms_plain;
        CK(hipEventElapsedTime(&ms_plain, a, b));
        CK(hipEventRecord(a, s));
        for (int k = 0; k < N; ++k) touch<<<grid, 256, 0, s>>>(t, slots - 1, k, host);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms_pinned;
        CK(hipEventElapsedTime(&ms_pinned, a, b));

        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int k = 0; k < N; ++k) touch<<<grid, 256, 0, s>>>(t, slots - 1, k, nullptr);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms_graph;
        CK(hipEventElapsedTime(&ms_graph, a, b));
        std::printf("grid %6d: plain %.2f us/launch, pinned %.2f us/launch, graph %.2f us/launch\n", grid,
                    ms_plain * 1e3 / N, ms_pinned * 1e3 / N, ms_graph * 1e3 / N);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipFree(t));
    return 0;
}
