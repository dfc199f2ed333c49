// Cross-process check of the direct exchange's building blocks on ONE GPU (the multi-GPU runs are
// the driver's): two processes, forked before either touches HIP, each allocate a data buffer and
// a flag array from the engine's DevicePool, exchange IPC blobs (dist.hpp IpcMaps) over a socket
// pair, and then store into the OTHER process's buffer from every workgroup of one kernel whose
// last workgroup raises the other's flag after a system-scope release (expand_route's protocol).
// Each waits for its own flag with peer_wait (bounded) and checks every word it received.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o scripts/ipc_selftest scripts/ipc_selftest.hip -lrccl
//   scripts/ipc_selftest [words]     exit status 0 = both processes saw the other's data
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../stateright_amd/csrc/engine.hpp"  // the engine headers (device pool, kernels, dist.hpp)

using namespace sr;

__global__ void fill_and_signal(u64* dst, u64 n, u64 tag, u32* ticket, u32* flag, u32 seq) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) dst[i] = tag | i;
    __shared__ u32 last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static bool xfer(int fd, void* p, size_t n, bool send) {
    char* c = static_cast<char*>(p);
    while (n) {
        const ssize_t k = send ? write(fd, c, n) : read(fd, c, n);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

static int run(int me, int fd, u64 n) {
    try {
        const int other = 1 - me;
        SR_HIP(hipSetDevice(0));
        hipStream_t s;
        SR_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        DBuf<u64> data;
        data.alloc(0, n);
        DBuf<u32> flags, ticket;
        flags.alloc(0, 2);
        ticket.alloc(0, 1);
        DBuf<u64> lcbuf;
        lcbuf.alloc(0, (sizeof(LevelCounters) + 7) / 8);
        SR_HIP(hipMemsetAsync(data.p, 0, n * 8, s));
        SR_HIP(hipMemsetAsync(flags.p, 0, 8, s));
        SR_HIP(hipMemsetAsync(ticket.p, 0, 4, s));
        SR_HIP(hipMemsetAsync(lcbuf.p, 0, sizeof(LevelCounters), s));
        SR_HIP(hipStreamSynchronize(s));  // cleared before the other process can know the buffers
        PeerBlob mine[2] = {IpcMaps::export_of(0, data.p), IpcMaps::export_of(0, flags.p)}, theirs[2];
        if (!xfer(fd, mine, sizeof(mine), true) || !xfer(fd, theirs, sizeof(theirs), false)) {
            std::fprintf(stderr, "[%d] blob exchange failed\n", me);
            return 2;
        }
        IpcMaps maps;
        u64* pdata = maps.open(0, other, theirs[0]);
        u32* pflags = reinterpret_cast<u32*>(maps.open(0, other, theirs[1]));
        const u64 tag = (u64)(me + 1) << 40;
        fill_and_signal<<<1024, 256, 0, s>>>(pdata, n, tag, ticket.p, pflags + me, 1u);
        auto* lc = reinterpret_cast<LevelCounters*>(lcbuf.p);
        peer_wait<<<1, 64, 0, s>>>(flags.p + other, 1, 1u, lc, 500000000ull);  // 5 s
        SR_HIP(hipGetLastError());
        std::vector<u64> got(n);
        u32 err = 0;
        SR_HIP(hipMemcpyAsync(&err, &lc->err, 4, hipMemcpyDeviceToHost, s));
        SR_HIP(hipMemcpyAsync(got.data(), data.p, n * 8, hipMemcpyDeviceToHost, s));
        SR_HIP(hipStreamSynchronize(s));
        if (err) {
            std::fprintf(stderr, "[%d] peer_wait timed out\n", me);
            return 3;
        }
        const u64 want = (u64)(other + 1) << 40;
        u64 bad = 0;
        for (u64 i = 0; i < n; ++i) bad += got[i] != (want | i);
        // both sides have read what they received before either unmaps or frees
        char c = 1;
        if (!xfer(fd, &c, 1, true) || !xfer(fd, &c, 1, false)) return 2;
        maps.close();
        std::printf("[%d] received %llu words from process %d through IPC: %llu wrong\n", me, (unsigned long long)n, other,
                    (unsigned long long)bad);
        return bad ? 4 : 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "[%d] %s\n", me, e.what());
        return 5;
    }
}

int main(int argc, char** argv) {
    const u64 n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 22);
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
    std::fflush(stdout);
    pid_t pid[2];
    for (int r = 0; r < 2; ++r) {
        pid[r] = fork();  // before any HIP call in this process
        if (pid[r] == 0) {
            close(sv[1 - r]);
            const int rc = run(r, sv[r], n);
            std::fflush(stdout);  // _Exit skips the stdio flush (stdout is a pipe under the test)
            std::fflush(stderr);
            std::_Exit(rc);
        }
    }
    close(sv[0]);
    close(sv[1]);
    int rc = 0;
    for (int r = 0; r < 2; ++r) {
        int st = 0;
        waitpid(pid[r], &st, 0);
        const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
        if (code) rc = code;
    }
    std::printf(rc ? "ipc selftest FAILED (%d)\n" : "ipc selftest ok\n", rc);
    return rc;
}
