// Clear bandwidth on one MI355X: hipMemsetAsync against store kernels (16-byte stores, grid-stride or
// one tile per workgroup, plain or nontemporal), over a 16 GiB and a 256 MiB buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

template <bool NT>
__global__ void __launch_bounds__(256) clear_stride(uint4* p, size_t n) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store((v4u){0, 0, 0, 0}, reinterpret_cast<v4u*>(p + i));
        else p[i] = z;
    }
}
template <bool NT, int U>
__global__ void __launch_bounds__(256) clear_tile(uint4* p, size_t n) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store((v4u){0, 0, 0, 0}, reinterpret_cast<v4u*>(p + i));
            else p[i] = z;
        }
    }
}

template <class F>
static double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    for (size_t bytes : {(size_t)16 << 30, (size_t)256 << 20}) {
        void* p = nullptr;
        CK(hipMalloc(&p, bytes));
        const size_t n = bytes / 16;
        const int reps = bytes > (1ull << 32) ? 5 : 50;
        auto rep = [&](const char* name, double ms) {
            std::printf("%-28s %8.1f MiB  %9.3f ms  %6.2f TB/s\n", name, bytes / 1048576.0, ms, bytes / ms / 1e9);
        };
        rep("hipMemsetAsync", timeit([&] { CK(hipMemsetAsync(p, 0, bytes)); }, reps));
        for (unsigned g : {2048u, 8192u, 32768u}) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "stride grid %u", g);
            rep(nm, timeit([&] { clear_stride<false><<<g, 256>>>((uint4*)p, n); }, reps));
            std::snprintf(nm, sizeof nm, "stride grid %u nt", g);
            rep(nm, timeit([&] { clear_stride<true><<<g, 256>>>((uint4*)p, n); }, reps));
        }
        const unsigned t4 = (unsigned)((n + 1023) / 1024), t16 = (unsigned)((n + 4095) / 4096);
        rep("tile x4", timeit([&] { clear_tile<false, 4><<<t4, 256>>>((uint4*)p, n); }, reps));
        rep("tile x4 nt", timeit([&] { clear_tile<true, 4><<<t4, 256>>>((uint4*)p, n); }, reps));
        rep("tile x16", timeit([&] { clear_tile<false, 16><<<t16, 256>>>((uint4*)p, n); }, reps));
        rep("tile x16 nt", timeit([&] { clear_tile<true, 16><<<t16, 256>>>((uint4*)p, n); }, reps));
        CK(hipFree(p));
    }
    return 0;
}
