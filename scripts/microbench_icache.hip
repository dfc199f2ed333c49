// Microbenchmark: what does a workgroup pay to run code its CU has not run before?
// A small level of expand_fast is one short chain per workgroup through ~11 KB of kernel code, and
// its links cost 0.3-1.2 us each even where they are LDS/ALU only (profiles/r03_timeline_*). This
// times one wave running straight-line code (an unrolled chain of dependent adds, BYTES of code)
// from s_memrealtime stamps inside the kernel, against the same dynamic instruction count as a
// loop (a few hundred bytes of code), in three states of the instruction path:
//   cold   after a kernel that streams 2 GiB through L2 (the code must come from HBM),
//   l2     right after a launch of the same kernel on OTHER CUs (the code is in L2),
//   again  the same CU's second launch in a row.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/microbench_icache scripts/microbench_icache.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t now() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memrealtime();
}

// N dependent 8-byte VOP3 adds, unrolled: 8*N bytes of straight-line code
template <int N>
__global__ void straight(uint32_t seed, uint64_t* out, uint32_t* sink) {
    const uint64_t t0 = now();
    uint32_t x = seed + threadIdx.x;
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add3_u32 %0, %0, %1, 1" : "+v"(x) : "v"(x));
    const uint64_t t1 = now();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2] = t0;
        out[blockIdx.x * 2 + 1] = t1;
    }
    if (x == 0x12345) sink[0] = x;
}

// N/4 rounds of 4 INDEPENDENT adds (the issue rate, not the latency) plus the shader clock
// (s_memtime) over the same span, for the clock frequency
template <int N>
__global__ void indep(uint32_t seed, uint64_t* out, uint32_t* sink) {
    uint32_t a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
    const uint64_t t0 = now();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
        asm volatile("v_add3_u32 %0, %0, %0, 1" : "+v"(a));
        asm volatile("v_add3_u32 %0, %0, %0, 1" : "+v"(b));
        asm volatile("v_add3_u32 %0, %0, %0, 1" : "+v"(c));
        asm volatile("v_add3_u32 %0, %0, %0, 1" : "+v"(d));
    }
    const uint64_t t1 = now();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t0;
        out[1] = t1;
        out[2] = c1 - c0;
    }
    if ((a ^ b ^ c ^ d) == 0x12345) sink[0] = a;
}

// the same dependent adds as a loop of 16 per iteration: the code fits in a few lines
__global__ void looped(uint32_t seed, int n, uint64_t* out, uint32_t* sink) {
    const uint64_t t0 = now();
    uint32_t x = seed + threadIdx.x;
    for (int i = 0; i < n; i += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("v_add3_u32 %0, %0, %1, 1" : "+v"(x) : "v"(x));
    }
    const uint64_t t1 = now();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2] = t0;
        out[blockIdx.x * 2 + 1] = t1;
    }
    if (x == 0x12345) sink[0] = x;
}

__global__ void stream(const uint4* in, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= in[i].x ^ in[i].w;
    if (acc == 0x12345) sink[0] = acc;
}

template <int N>
static int run(const uint4* big, size_t nbig, uint64_t* dout, uint32_t* sink) {
    uint64_t h[2 * 512];
    auto us = [&](int b) { return (h[2 * b + 1] - h[2 * b]) / 100.0; };  // 100 MHz clock
    double cold = 0, l2 = 0, again = 0, loop = 0;
    const int reps = 5;
    for (int r = 0; r < reps; ++r) {
        stream<<<2048, 256>>>(big, nbig, sink);
        straight<N><<<1, 64>>>(1, dout, sink);
        CHECK(hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost));
        cold += us(0);
        // a wide launch puts the code in every XCD's L2 (and the I-cache of the CUs it ran on);
        // then one wave on whatever CU the dispatcher picks
        stream<<<2048, 256>>>(big, nbig, sink);
        straight<N><<<512, 64>>>(1, dout, sink);
        straight<N><<<1, 64>>>(1, dout, sink);
        CHECK(hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost));
        l2 += us(0);
        straight<N><<<1, 64>>>(1, dout, sink);
        CHECK(hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost));
        again += us(0);
        stream<<<2048, 256>>>(big, nbig, sink);
        looped<<<1, 64>>>(1, N, dout, sink);
        CHECK(hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost));
        loop += us(0);
    }
    double ind = 0, ghz = 0;
    for (int r = 0; r < reps; ++r) {
        indep<N><<<1, 64>>>(1, dout, sink);
        CHECK(hipMemcpy(h, dout, 24, hipMemcpyDeviceToHost));
        ind += us(0);
        ghz += h[2] / (us(0) * 1e3);
    }
    std::printf("independent: %7.2f us (%.2f ns per add, shader clock %.2f GHz)  ", ind / reps, ind / reps * 1e3 / N, ghz / reps);
    std::printf("code %6d B  straight: cold %7.2f us  after wide launch %7.2f us  again %7.2f us | loop (cold) %7.2f us\n",
                N * 8, cold / reps, l2 / reps, again / reps, loop / reps);
    return 0;
}

int main() {
    const size_t bytes = size_t(2) << 30, nbig = bytes / 16;
    uint4* big;
    uint64_t* dout;
    uint32_t* sink;
    CHECK(hipMalloc(&big, bytes));
    CHECK(hipMemset(big, 1, bytes));
    CHECK(hipMalloc(&dout, 2 * 512 * 8));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipDeviceSynchronize());
    int rc = 0;
    rc |= run<128>(big, nbig, dout, sink);
    rc |= run<512>(big, nbig, dout, sink);
    rc |= run<1024>(big, nbig, dout, sink);
    rc |= run<2048>(big, nbig, dout, sink);
    rc |= run<4096>(big, nbig, dout, sink);
    CHECK(hipDeviceSynchronize());
    return rc;
}
