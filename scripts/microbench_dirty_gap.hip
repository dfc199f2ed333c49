// Gap between two dependent kernels in one stream as a function of the data the first one leaves
// dirty in L2: kernel `dirty` stores 8 bytes to each of n random 128-byte lines of a 256 MB buffer
// (like a level's visited-set claims), kernel `empty` follows. Run under
//   rocprofv3 --kernel-trace --output-format csv -d <dir> -o t -- ./scripts/microbench_dirty_gap
// and read End(dirty) -> Start(empty) from the trace (the program prints the plan only).
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_dirty_gap.hip -o scripts/microbench_dirty_gap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void dirty(unsigned long long* buf, unsigned long long lines, unsigned n, unsigned nt) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long h = (i + 1) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    unsigned long long* p = buf + (h % lines) * 16;  // one 8-byte word per 128-byte line
    if (nt) __builtin_nontemporal_store((unsigned long long)i, p);
    else *p = i;
}

__global__ void empty(unsigned* sink) {
    if (threadIdx.x == 1023) sink[0] = 1;
}

int main() {
    const unsigned long long bytes = 256ull << 20, lines = bytes / 128;
    unsigned long long* buf;
    unsigned* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 0, bytes));
    for (unsigned nt = 0; nt < 2; ++nt)
        for (unsigned n : {0u, 1u << 14, 1u << 17, 1u << 20, 1u << 22})
            for (int rep = 0; rep < 5; ++rep) {
                dirty<<<(n + 255) / 256 + 1, 256>>>(buf, lines, n, nt);
                empty<<<4, 256>>>(sink);
                CK(hipDeviceSynchronize());
            }
    printf("plan: nt in {0,1} x n in {0, 16K, 128K, 1M, 4M} x 5 reps, each dirty then empty\n");
    return 0;
}
