// Diagnostic: how long device allocations of arena sizes take (fresh hipMalloc, the first write to
// the block, hipFree), and the same through the virtual memory API (reserve once, create + map +
// set access per chunk), to size the arena growth policy.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 scripts/alloc_bench.hip -o scripts/alloc_bench
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                      \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    for (size_t gb : {1, 4, 16, 43}) {
        const size_t bytes = gb << 30;
        void* p = nullptr;
        auto t = std::chrono::steady_clock::now();
        CK(hipMalloc(&p, bytes));
        const double a = ms_since(t);
        t = std::chrono::steady_clock::now();
        CK(hipMemset(p, 0, bytes));
        CK(hipDeviceSynchronize());
        const double w = ms_since(t);
        t = std::chrono::steady_clock::now();
        CK(hipMemset(p, 1, bytes));
        CK(hipDeviceSynchronize());
        const double w2 = ms_since(t);
        t = std::chrono::steady_clock::now();
        CK(hipFree(p));
        const double f = ms_since(t);
        std::printf("hipMalloc %zu GiB: alloc %.2f ms, first memset %.2f ms, second memset %.2f ms, free %.2f ms\n", gb, a, w, w2, f);
    }
    // virtual memory: reserve 64 GiB, map 4 GiB chunks
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    const size_t chunk = 4ull << 30, total = 64ull << 30;
    void* va = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMemAddressReserve(&va, total, 0, nullptr, 0));
    std::printf("granularity %zu; reserve 64 GiB %.3f ms\n", gran, ms_since(t));
    std::vector<hipMemGenericAllocationHandle_t> hs;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    for (int i = 0; i < 4; ++i) {
        hipMemGenericAllocationHandle_t h;
        t = std::chrono::steady_clock::now();
        CK(hipMemCreate(&h, chunk, &prop, 0));
        const double c = ms_since(t);
        t = std::chrono::steady_clock::now();
        char* at = static_cast<char*>(va) + i * chunk;
        CK(hipMemMap(at, chunk, 0, h, 0));
        CK(hipMemSetAccess(at, chunk, &acc, 1));
        const double m = ms_since(t);
        t = std::chrono::steady_clock::now();
        CK(hipMemset(at, 0, chunk));
        CK(hipDeviceSynchronize());
        std::printf("vmm chunk %d (4 GiB): create %.2f ms, map+access %.2f ms, first memset %.2f ms\n", i, c, m, ms_since(t));
        hs.push_back(h);
    }
    t = std::chrono::steady_clock::now();
    CK(hipMemset(va, 2, 4 * chunk));
    CK(hipDeviceSynchronize());
    std::printf("memset across the 4 mapped chunks (16 GiB): %.2f ms\n", ms_since(t));
    for (int i = 0; i < 4; ++i) {
        CK(hipMemUnmap(static_cast<char*>(va) + i * chunk, chunk));
        CK(hipMemRelease(hs[i]));
    }
    CK(hipMemAddressFree(va, total));
    return 0;
}
