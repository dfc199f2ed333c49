// Cost of the publish's system-scope release fence as a function of the dirty data a kernel leaves
// in L2: kernel `work` stores 8 bytes to each of n random 128-byte lines of a 256 MB device buffer,
// then its last workgroup (ticket) stores a word to pinned host memory, with or without a
// system-scope release fence before that store. Event-timed, best of 20.
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_sysfence.hip -o scripts/microbench_sysfence
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void work(unsigned long long* buf, unsigned long long lines, unsigned n, unsigned* ticket,
                     unsigned* host_flag, unsigned fence, unsigned seq) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        unsigned long long h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        buf[(h % lines) * 16] = i;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (atomicAdd(ticket, 1u) != gridDim.x - 1) return;
    *ticket = 0;
    if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    __hip_atomic_store(host_flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    const unsigned long long bytes = 256ull << 20, lines = bytes / 128;
    unsigned long long* buf;
    unsigned *ticket, *flag, *flag_dev;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&ticket, 4));
    CK(hipMemset(ticket, 0, 4));
    CK(hipHostMalloc(&flag, 4, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    unsigned seq = 0;
    for (unsigned n : {0u, 1u << 14, 1u << 17, 1u << 20, 1u << 22})
        for (unsigned fence = 0; fence < 2; ++fence) {
            float best = 1e9f;
            for (int it = 0; it < 20; ++it) {
                CK(hipEventRecord(a));
                work<<<(n + 255) / 256 + 1, 256>>>(buf, lines, n, ticket, flag_dev, fence, ++seq);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
                if (*(volatile unsigned*)flag != seq) { printf("flag not published\n"); return 1; }
            }
            printf("dirty lines %8u  system fence %u: %8.2f us\n", n, fence, best * 1e3);
        }
    return 0;
}
