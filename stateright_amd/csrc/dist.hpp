// Partitioned breadth-first search over T visited-set partitions.
//
// One partition per GPU, one process per GPU, RCCL over xGMI (`Comm`), or T virtual partitions
// in one process on one GPU (the same level loop with device copies as the exchange: this is how
// the protocol is tested on a single device). FAST order only (the reference's single-threaded
// FIFO order is a single-GPU mode).
//
// Two level loops share the kernels:
//
// PIPELINED (default, `lag_loop`): no host wait inside a level. expand_route writes its row into
// the header of every fixed-capacity send bucket; ONE ncclAllToAll moves buckets and rows;
// insert_recv_lag closes the level on the device and publishes every row to pinned memory. The
// host enqueues level L+1 before reading level L's rows (bucket capacity planned from the rows of
// level L-1, the same on every rank).
//
// SYNCHRONOUS (SR_DIST_SYNC=1, and the restart after a pipelined overflow), one host
// synchronisation per level:
//   1. expand_route: reads its frontier size from the device control block (DistCtl); local
//      successors are inserted directly, the others become records for their owner's send bucket
//      (staged in LDS per chunk, one global reservation per chunk and owner). Its last workgroup
//      writes the partition's row: records per destination, frontier size, successors, local
//      claims, error bits, discovery ranks.
//   2. one all-gather of the rows + a copy to pinned host memory; the host waits for it (every
//      rank then knows the level's global totals and the full T x T record matrix).
//   3. all-to-all of the records (ncclSend/ncclRecv in one group).
//   4. insert_recv: owners insert what they received; its last workgroup closes the level on the
//      device (next frontier size, discoveries among it) so that the NEXT expand_route, enqueued
//      right behind it, needs nothing from the host.
// Capacity planning is optimistic; an overflow on any partition is seen by every rank in the
// rows and all of them restart the check together with larger buffers.
#pragma once
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <set>
#include <tuple>
#include <unordered_map>

#include "kernels_dist.hpp"

namespace sr {

// Element-wise reduction of `rows` vectors of n words (rows x n, row-major) into out.
template <int = 0> __global__ void reduce_rows(const u64* in, u32 rows, u64 n, u32 op, u64* out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u64 v = in[i];
    for (u32 r = 1; r < rows; ++r) {
        const u64 x = in[(u64)r * n + i];
        v = op == 0 ? (x < v ? x : v) : op == 1 ? (x > v ? x : v) : v + x;
    }
    out[i] = v;
}

#define SR_NCCL(expr)                                                                         \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess)                                                                \
            throw ::sr::Error(SR_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// The collectives the partitioned level loop issues, stream-ordered like RCCL's (every rank issues
// the same sequence; a call returns once its work is ENQUEUED on `s`).
//   all_to_all   count words from send[q*count] to rank q's recv[me*count]
//   all_gather   count words from every rank into all[q*count]
//   exchange     grouped point-to-point of per-peer spans (the synchronous mode's exact sizes)
//   broadcast    count words of root's buf to every rank's buf
//   all_reduce   element-wise min / max / sum of count u64 words
enum class RedOp { Min, Max, Sum };

// Internal error code (never returned through the C ABI): the direct exchange failed its check on
// this rank (ERR_EXCHANGE or ERR_PEER_TIMEOUT); DistEngine::run turns it into a fallback.
constexpr int ERR_CODE_EXCHANGE = -101;

// ---- The host side of the level protocol as pure functions: the pipelined engine (lag_loop,
// DistEngine::run) calls these, and so does the GPU-free protocol run over the shared-memory
// transport (dist_host.hpp, tests/test_dist_host_protocol.py), which drives them from two
// processes with rows of its own. ----

// A partition's row of a level: T words of records sent to each partition, then these fields
// (from index T), then one word per property: the rank of its first discovery in the new
// frontier (~0: none). Every rank receives every row.
enum RowField : u32 {
    ROW_N = 0,        // states of the frontier the partition produced (its next level)
    ROW_SUCC = 1,     // successors counted (state_count increments)
    ROW_LOCAL = 2,    // states the partition claimed itself before the exchange
    ROW_ERR = 3,      // ErrBits of the partition's route and insert
    ROW_ENABLED = 4,  // enabled action slots of the expanded parents
    ROW_ROOTS = 5,    // level 0: distinct init states
    ROW_DISC = 6,
};
inline size_t row_words(u32 T, u32 nprops) { return (size_t)T + ROW_DISC + nprops; }

// A level's error bits (OR over every row), acted on by every rank at the same level and in this
// order: an exchange error wins over the capacity errors (a corrupt record can overflow a bucket,
// and a capacity restart would keep the direct exchange).
inline void throw_row_errors(u64 glob_err, u32 level) {
    if (glob_err & ERR_EXCHANGE)
        throw Error(ERR_CODE_EXCHANGE, "direct exchange: a receive slot failed its sequence tag or checksum (level " +
                                           std::to_string(level) + ")");
    if (glob_err & ERR_TABLE_FULL) throw Error(SR_ERR_CAPACITY, "visited set probe limit exceeded");
    if (glob_err & ERR_FRONTIER_OVERFLOW) throw Error(SR_ERR_CAPACITY, "frontier or send bucket overflow");
}

// What the pipelined plan knows, the same on every rank: exact frontier sizes up to the last rows
// read (n_last), an upper bound of the next one (n_hi: local claims + records received), the
// growth of the last exact step, and the largest records per (source, owner) pair per frontier
// state (pair_ratio).
struct LevelPlan {
    std::vector<u64> n_last, n_hi;
    double growth = 1.0, pair_ratio = 0.0;
    bool have_rows = false;
    u64 glob_prev = 0;  // the last level's global frontier (growth is measured against it)
    struct Sums {
        u64 n = 0, succ = 0, err = 0, roots = 0, enabled = 0, maxpair = 0, recs = 0, local = 0;
    };
    // Global totals of a level's rows (T rows of RW words).
    static Sums sums(const u64* all, u32 T, size_t RW) {
        Sums s;
        for (u32 q = 0; q < T; ++q) {
            const u64* row = all + (size_t)q * RW;
            s.n += row[T + ROW_N];
            s.succ += row[T + ROW_SUCC];
            s.local += row[T + ROW_LOCAL];
            s.err |= row[T + ROW_ERR];
            s.enabled += row[T + ROW_ENABLED];
            s.roots += row[T + ROW_ROOTS];
            for (u32 d = 0; d < T; ++d) {
                s.maxpair = std::max<u64>(s.maxpair, row[d]);
                s.recs += row[d];
            }
        }
        return s;
    }
    // The plan after a level's rows (read after throw_row_errors accepted them).
    void absorb(const u64* all, u32 T, size_t RW, const Sums& s) {
        for (u32 q = 0; q < T; ++q) {
            u64 r = 0;
            for (u32 s2 = 0; s2 < T; ++s2) r += all[(size_t)s2 * RW + q];
            n_hi[q] = all[(size_t)q * RW + T + ROW_LOCAL] + r;  // upper bound of partition q's next frontier
            n_last[q] = all[(size_t)q * RW + T + ROW_N];
        }
        if (s.n) {
            pair_ratio = (double)s.maxpair / (double)s.n;
            if (glob_prev) growth = (double)s.n / (double)glob_prev;
            have_rows = true;
        }
        glob_prev = s.n;
    }
    // Bucket capacity (records per pair) of the level `ahead` (1 or 2) levels past the last rows:
    // the growth of the last exact step with a margin, compounded once per level of look-ahead.
    u64 bucket_cap(u32 ahead, u64 cmin) const {
        const double g = growth * 1.1;
        u64 glob_fr = 0;
        for (size_t q = 0; q < n_last.size(); ++q) {
            const u64 c1 = have_rows ? std::min<u64>(n_hi[q], (u64)((double)n_last[q] * g) + 64) : n_last[q];
            glob_fr += ahead == 2 ? (u64)((double)c1 * g) : c1;
        }
        return have_rows ? std::max<u64>(cmin, (u64)(pair_ratio * (double)glob_fr * 1.15) + 256) : cmin;
    }
};

// The outcome of one check attempt on one rank, voted on by every rank (the max and min of the
// codes over the ranks): the direct exchange's failures are seen by one owner only, so no rank may
// decide alone.
enum Outcome : int { OUT_OK = 0, OUT_CAPACITY = 1, OUT_EXCHANGE = 2, OUT_ERROR = 3 };
inline int outcome_of(int error_code) {
    return error_code == SR_ERR_CAPACITY ? OUT_CAPACITY : error_code == ERR_CODE_EXCHANGE ? OUT_EXCHANGE : OUT_ERROR;
}
enum class VoteAction { Done, Fallback, Restart, Fail };
struct VoteDecision {
    VoteAction act = VoteAction::Done;
    bool disagree = false;  // a capacity restart that some rank did not see (it travels in the rows)
    int code = 0;           // Fail: the error code to throw
    std::string why;        // Fallback / Restart / Fail: the reason
};
// Every rank takes the same action (hi and lo are the same everywhere); only the message of a
// failure depends on the rank's own outcome.
inline VoteDecision decide_after_vote(int code, int hi, int lo, int attempt, int ecode, const std::string& what) {
    VoteDecision d;
    if (hi == OUT_ERROR) {
        d.act = VoteAction::Fail;
        d.code = code == OUT_ERROR ? ecode : SR_ERR_HIP;
        d.why = code == OUT_ERROR ? what : std::string("partitioned search: another rank failed");
    } else if (hi == OUT_EXCHANGE) {  // a corrupt exchange somewhere (only this falls back)
        if (attempt >= 3) {
            d.act = VoteAction::Fail;
            d.code = SR_ERR_HIP;
            d.why = "partitioned search: the exchange failed repeatedly: " + what;
        } else {
            d.act = VoteAction::Fallback;
            d.why = code == OUT_EXCHANGE ? what : std::string("another rank's exchange failed");
        }
    } else if (hi == OUT_CAPACITY) {
        // Capacity errors travel in the rows and reach every rank at the same level, so a rank that
        // finished cleanly (lo == 0) means they did not: said, and restarted like the others.
        d.disagree = lo != hi;
        d.why = code ? what : std::string("another rank ran out of capacity");
        if (attempt >= 3) {
            d.act = VoteAction::Fail;
            d.code = code ? ecode : SR_ERR_CAPACITY;
        } else {
            d.act = VoteAction::Restart;
        }
    }
    return d;
}

// A device buffer as another rank can name it (direct exchange): its address in the exporting
// process, the hipMalloc allocation around it, and an IPC handle of that allocation.
struct PeerBlob {
    u64 ptr = 0, base = 0, size = 0;
    u64 epoch = 0;  // the exporter's DevicePool epoch: a re-hipMalloc'd block at the same address differs
    hipIpcMemHandle_t handle{};
};

struct Comm {
    int rank = 0, world = 1, device = 0;
    // process-unique identity (pooled per-device resources remember which communicator they served)
    const u64 uid = next_uid();
    static u64 next_uid() {
        static std::atomic<u64> n{1};
        return n++;
    }
    virtual ~Comm() = default;
    virtual const char* kind() const = 0;
    virtual int nranks() const = 0;  // ranks the transport itself reports (RCCL: ncclCommCount)
    virtual void all_to_all(const u64* send, u64* recv, u64 count, hipStream_t s) = 0;
    virtual void all_gather(const u64* mine, u64* all, u64 count, hipStream_t s) = 0;
    virtual void exchange(const std::vector<const u64*>& send, const std::vector<u64>& scount,
                          const std::vector<u64*>& recv, const std::vector<u64>& rcount, hipStream_t s) = 0;
    virtual void broadcast(u64* buf, u64 count, int root, hipStream_t s) = 0;
    virtual void all_reduce(u64* buf, u64 count, RedOp op, hipStream_t s) = 0;
    // Host barrier (bench timing): every rank's device work issued so far on `s` is finished.
    void barrier(hipStream_t s) {
        DBuf<u64> one;
        one.alloc(device, 1);
        SR_HIP(hipMemsetAsync(one.p, 0, 8, s));
        all_reduce(one.p, 1, RedOp::Sum, s);
        SR_HIP(stream_sync(s));
    }

    // ---- direct exchange (peer pointers) ----
    // Whether this transport can give every rank a pointer to every other rank's buffers
    // (SR_DIRECT=0 turns the direct exchange off; RCCL's all-to-all is then the exchange).
    virtual bool peer_capable() const { return false; }
    // Every rank on its own device (the direct exchange's wait may then run inside the insert grid).
    virtual bool distinct_devices() const { return false; }
    // Collective: every rank's `bytes` bytes of `mine`, rank-major, into `all` (host memory).
    virtual void share(const void* mine, size_t bytes, void* all, hipStream_t s) = 0;
    // This rank's buffer `p` as a blob, and rank q's blob as an address usable by this rank's kernels.
    virtual PeerBlob export_buf(void* p) const {
        PeerBlob b;
        b.ptr = reinterpret_cast<u64>(p);
        return b;
    }
    virtual u64* map(int q, const PeerBlob& b) {
        (void)q;
        return reinterpret_cast<u64*>(b.ptr);
    }
    // Collective: the address of every rank's buffer `mine` as seen by this rank (out[q]).
    void peer_addresses(void* mine, std::vector<u64*>& out, hipStream_t s) {
        const PeerBlob b = export_buf(mine);
        std::vector<PeerBlob> all(world);
        share(&b, sizeof(b), all.data(), s);
        out.resize(world);
        for (int q = 0; q < world; ++q) out[q] = q == rank ? static_cast<u64*>(mine) : map(q, all[q]);
    }
    // Checked once per communicator (collective, on first use): a flag round trip between every
    // pair of ranks through the direct path, with a bounded wait. Every rank gets the same answer.
    int direct_ok = -1;
    bool probe_direct(hipStream_t s);
};

inline bool direct_env_on() {
    const char* e = std::getenv("SR_DIRECT");
    return !(e && std::atoi(e) == 0);
}
// peer_wait's bound in ticks of the 100 MHz real-time counter (SR_PEER_TIMEOUT_MS, default 20 s)
inline u64 peer_timeout_ticks() {
    const char* e = std::getenv("SR_PEER_TIMEOUT_MS");
    const u64 ms = e && std::atoll(e) > 0 ? (u64)std::atoll(e) : 20000;
    return ms * 100000ull;
}

// Flag words of the direct exchange cleared with system-scope stores and a system-scope release: no
// dirty line of them stays in this device's L2 to be written back over a peer's later flag store.
template <int = 0> __global__ void flags_clear(u32* f, u32 n) {
    for (u32 i = threadIdx.x; i < n; i += blockDim.x) __hip_atomic_store(&f[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// The probe's data pattern: word i of the slot that rank `src` stores into rank `dst`'s buffer.
__device__ __host__ __forceinline__ u64 probe_word(u32 src, u32 dst, u64 i, u32 seq) {
    return fmix64(((u64)(src + 1) << 48) ^ ((u64)(dst + 1) << 40) ^ ((u64)seq << 32) ^ i) | 1;
}
// Every word of `buf` set to `v` and read back (the owner's L2 then holds the lines, as it holds
// those of a receive buffer it read two levels earlier); `sink` keeps the reads.
// The stores are written back (system-scope release) before the reads: a dirty line of the owner
// could otherwise be evicted over a peer's later store.
template <int = 0> __global__ void probe_warm(u64* buf, u64 n, u64 v, u64* sink) {
    u64 acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) buf[i] = v;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) acc += buf[i];
    if (acc == 0x5bd1e995ull) sink[0] = acc;
}
// One workgroup of rank `me` stores its pattern into slot `me` of every rank's buffer (btab[q]),
// then releases at system scope and raises its flag in every rank's flags (expand_route's order).
template <int = 0> __global__ void probe_store(u64* const* btab, u32* const* ftab, u32 world, u64 K, u32 me, u32 seq) {
    for (u32 q = 0; q < world; ++q)
        for (u64 i = threadIdx.x; i < K; i += blockDim.x) btab[q][i] = probe_word(me, q, i, seq);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    for (u32 q = threadIdx.x; q < world; q += blockDim.x)
        __hip_atomic_store(ftab[q], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The owner waits for every flag inside the kernel that reads (insert_recv_lag's fused wait: poll,
// system-scope acquire, then plain loads), bounded, and counts the words that differ.
template <int = 0> __global__ void probe_verify(const u64* buf, const u32* flags, u32 world, u64 K, u32 me, u32 seq, u64 timeout,
                             unsigned long long* bad, LevelCounters* lc) {
    __shared__ u32 ok;
    if (threadIdx.x == 0) {
        ok = 1;
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        for (u32 q = 0; q < world; ++q)
            while ((int)(__hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        if (!ok) atomicOr(&lc->err, (u32)ERR_PEER_TIMEOUT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    if (!ok) return;
    u64 nbad = 0;
    for (u32 q = 0; q < world; ++q)
        for (u64 i = threadIdx.x; i < K; i += blockDim.x) nbad += buf[(u64)q * K + i] != probe_word(q, me, i, seq);
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

// Checked once per communicator (collective, on first use), in the exchange's steady state: every
// rank fills and READS its own receive area first (its lines are then cached, as a receive buffer
// read two levels earlier is), then every rank stores a pattern into its slot of every rank's area
// and raises its flag there, and every owner waits for the flags inside the reading kernel and
// checks every word. Same memory kind as the exchange (dx_kind), 1 s bound. Every rank reaches every
// collective whatever failed on it, and all take the same decision.
inline int dx_probe_kind() {
    const char* e = std::getenv("SR_DX_FINE");
    return e && std::atoi(e) == 0 ? 0 : 1;
}
inline bool Comm::probe_direct(hipStream_t s) {
    if (direct_ok >= 0) return direct_ok == 1;
    // Every rank reaches every collective below, whatever failed on it: a local failure becomes
    // a vote, never a skipped collective (which would leave the other ranks waiting in it).
    auto agree = [&](u64 vote) {
        DBuf<u64> v;
        v.alloc(device, 1);
        SR_HIP(hipMemcpyAsync(v.p, &vote, 8, hipMemcpyHostToDevice, s));
        all_reduce(v.p, 1, RedOp::Min, s);
        SR_HIP(hipMemcpyAsync(&vote, v.p, 8, hipMemcpyDeviceToHost, s));
        SR_HIP(stream_sync(s));
        return vote == 1;
    };
    direct_ok = 0;
    if (!agree(peer_capable() ? 1 : 0)) return false;
    constexpr u64 K = 8192;  // words per slot (64 KiB)
    constexpr u32 SEQ = 7;
    const int kind = dx_probe_kind();
    DBuf<u32> flags;
    flags.alloc(device, world, kind);
    DBuf<u64> area;
    area.alloc(device, (u64)world * K, kind);
    DBuf<u32*> ftab;
    ftab.alloc(device, world);
    DBuf<u64*> btab;
    btab.alloc(device, world);
    DBuf<u64> lcbuf;  // a LevelCounters for the wait's error bit, then the mismatch count
    lcbuf.alloc(device, (sizeof(LevelCounters) + 7) / 8 + 2);
    auto* lc = reinterpret_cast<LevelCounters*>(lcbuf.p);
    auto* bad = reinterpret_cast<unsigned long long*>(lcbuf.p + (sizeof(LevelCounters) + 7) / 8);
    flags_clear<<<1, 64, 0, s>>>(flags.p, (u32)world);
    SR_HIP(hipMemsetAsync(lcbuf.p, 0, lcbuf.n * 8, s));
    probe_warm<<<64, 256, 0, s>>>(area.p, (u64)world * K, 0xa5a5a5a5a5a5a5a5ull, reinterpret_cast<u64*>(bad + 1));
    SR_HIP(hipGetLastError());
    SR_HIP(stream_sync(s));
    u64 ok = 1;
    PeerBlob b[2];
    try {
        b[0] = export_buf(flags.p);
        b[1] = export_buf(area.p);
    } catch (const Error&) {
        ok = 0;
        b[0] = b[1] = PeerBlob{};
    }
    std::vector<PeerBlob> all(2 * (size_t)world);
    share(b, sizeof(b), all.data(), s);  // collective: every rank's area is warm and its flags zero from here on
    std::vector<u32*> ft(world);
    std::vector<u64*> bt(world);
    for (int q = 0; q < world && ok; ++q) {
        if (!all[2 * q].ptr || !all[2 * q + 1].ptr) ok = 0;  // that rank could not export
        try {
            if (ok) {
                ft[q] = (q == rank ? flags.p : reinterpret_cast<u32*>(map(q, all[2 * q]))) + rank;
                bt[q] = (q == rank ? area.p : map(q, all[2 * q + 1])) + (u64)rank * K;
            }
        } catch (const Error&) {
            ok = 0;
        }
    }
    if (!agree(ok)) return false;
    SR_HIP(hipMemcpyAsync(ftab.p, ft.data(), world * sizeof(u32*), hipMemcpyHostToDevice, s));
    SR_HIP(hipMemcpyAsync(btab.p, bt.data(), world * sizeof(u64*), hipMemcpyHostToDevice, s));
    probe_store<<<1, 256, 0, s>>>(btab.p, ftab.p, (u32)world, K, (u32)rank, SEQ);
    probe_verify<<<1, 256, 0, s>>>(area.p, flags.p, (u32)world, K, (u32)rank, SEQ, 100000000ull, bad, lc);  // 1 s
    SR_HIP(hipGetLastError());
    u32 err = 0;
    unsigned long long nbad = 0;
    SR_HIP(hipMemcpyAsync(&err, &lc->err, 4, hipMemcpyDeviceToHost, s));
    SR_HIP(hipMemcpyAsync(&nbad, bad, 8, hipMemcpyDeviceToHost, s));
    SR_HIP(stream_sync(s));
    if (err || nbad) {
        // a late peer store may still land: never reuse these blocks
        flags.p = nullptr;
        area.p = nullptr;
        std::fprintf(stderr, "[sr] direct exchange probe failed on rank %d (%s, %llu wrong words): collective exchange\n",
                     rank, err ? "a flag did not arrive" : "stale or lost data", nbad);
    }
    direct_ok = agree(err == 0 && nbad == 0 ? 1 : 0) ? 1 : 0;
    return direct_ok == 1;
}

// IPC export and mapping of pool buffers (the direct exchange across processes; also used by the
// standalone cross-process check scripts/ipc_selftest.hip). A blob names the hipMalloc allocation
// around a buffer; a process opens each (peer, allocation) once and keeps the mapping.
struct IpcMaps {
    static PeerBlob export_of(int device, void* p) {
        PeerBlob b;
        b.ptr = reinterpret_cast<u64>(p);
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        SR_HIP(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(p)));
        b.base = reinterpret_cast<u64>(base);
        b.size = size;
        b.epoch = DevicePool::get().epoch(device);
        SR_HIP(hipIpcGetMemHandle(&b.handle, reinterpret_cast<void*>(base)));
        return b;
    }
    u64* open(int device, int q, const PeerBlob& b) {
        const auto key = std::make_tuple(q, b.base, b.size, b.epoch);
        auto it = opened.find(key);
        if (it == opened.end()) {
            void* m = nullptr;
            SR_HIP(hipSetDevice(device));
            SR_HIP(hipIpcOpenMemHandle(&m, b.handle, hipIpcMemLazyEnablePeerAccess));
            it = opened.emplace(key, m).first;
        }
        return reinterpret_cast<u64*>(static_cast<char*>(it->second) + (b.ptr - b.base));
    }
    void close() {
        for (auto& [k, m] : opened) (void)hipIpcCloseMemHandle(m);
        opened.clear();
    }
    ~IpcMaps() { close(); }
    std::map<std::tuple<int, u64, u64, u64>, void*> opened;
};

// One process per GPU over RCCL (xGMI).
struct RcclComm final : Comm {
    ncclComm_t nccl = nullptr;
    ~RcclComm() override {
        ipc.close();
        if (nccl) (void)ncclCommDestroy(nccl);
    }
    const char* kind() const override { return "rccl"; }
    int nranks() const override {
        int n = 0;
        if (ncclCommCount(nccl, &n) != ncclSuccess) return -1;
        return n;
    }
    void all_to_all(const u64* send, u64* recv, u64 count, hipStream_t s) override {
        SR_NCCL(ncclAllToAll(send, recv, count, ncclUint64, nccl, s));
    }
    void all_gather(const u64* mine, u64* all, u64 count, hipStream_t s) override {
        SR_NCCL(ncclAllGather(mine, all, count, ncclUint64, nccl, s));
    }
    void exchange(const std::vector<const u64*>& send, const std::vector<u64>& scount, const std::vector<u64*>& recv,
                  const std::vector<u64>& rcount, hipStream_t s) override {
        SR_NCCL(ncclGroupStart());
        for (int peer = 0; peer < world; ++peer) {
            if (peer == rank) {
                if (scount[peer]) SR_HIP(hipMemcpyAsync(recv[peer], send[peer], scount[peer] * 8, hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (scount[peer]) SR_NCCL(ncclSend(send[peer], scount[peer], ncclUint64, peer, nccl, s));
            if (rcount[peer]) SR_NCCL(ncclRecv(recv[peer], rcount[peer], ncclUint64, peer, nccl, s));
        }
        SR_NCCL(ncclGroupEnd());
    }
    void broadcast(u64* buf, u64 count, int root, hipStream_t s) override {
        SR_NCCL(ncclBroadcast(buf, buf, count, ncclUint64, root, nccl, s));
    }
    void all_reduce(u64* buf, u64 count, RedOp op, hipStream_t s) override {
        const ncclRedOp_t o = op == RedOp::Min ? ncclMin : op == RedOp::Max ? ncclMax : ncclSum;
        SR_NCCL(ncclAllReduce(buf, buf, count, ncclUint64, o, nccl, s));
    }

    // Direct exchange across processes: buffers travel as IPC handles of their hipMalloc
    // allocation (the DevicePool hands out whole allocations), opened once per (peer, allocation).
    bool peer_capable() const override { return direct_env_on(); }
    bool distinct_devices() const override { return true; }  // RCCL refuses two ranks on one GPU
    void share(const void* mine, size_t bytes, void* all, hipStream_t s) override {
        const u64 words = (bytes + 7) / 8;
        DBuf<u64> d;
        d.alloc(device, words * world);
        SR_HIP(hipMemcpyAsync(d.p + (u64)rank * words, mine, bytes, hipMemcpyHostToDevice, s));
        SR_NCCL(ncclAllGather(d.p + (u64)rank * words, d.p, words, ncclUint64, nccl, s));
        std::vector<u64> h(words * world);
        SR_HIP(hipMemcpyAsync(h.data(), d.p, words * world * 8, hipMemcpyDeviceToHost, s));
        SR_HIP(stream_sync(s));
        for (int q = 0; q < world; ++q)
            std::memcpy(static_cast<char*>(all) + (size_t)q * bytes, h.data() + (u64)q * words, bytes);
    }
    PeerBlob export_buf(void* p) const override { return IpcMaps::export_of(device, p); }
    u64* map(int q, const PeerBlob& b) override { return ipc.open(device, q, b); }
    IpcMaps ipc;  // peers' allocations opened in this process
};

// Ranks that are threads of ONE process (each with its own driver thread, stream and device).
// Collectives keep RCCL's contract: a call is stream-ordered on the caller's stream, every rank
// issues the same sequence, and a call only ENQUEUES work. The ranks meet on a host barrier at
// each call (which also checks that they issue the same collective with the same size: a
// mismatch, which would hang RCCL, raises on every rank), and the data moves by device copies
// ordered with HIP events across the ranks' streams. This runs the partitioned engine's real
// multi-rank code (rank-local partitions, every collective in its order) on one GPU.
struct LocalGroup {
    explicit LocalGroup(int w) : world(w), slots(w), ready(w, nullptr), done(w, nullptr), devices(w, 0) {}
    ~LocalGroup() {
        for (auto e : ready)
            if (e) (void)hipEventDestroy(e);
        for (auto e : done)
            if (e) (void)hipEventDestroy(e);
    }
    struct Slot {
        int op = 0;
        u64 count = 0;
        const u64* send = nullptr;
        const std::vector<const u64*>* sends = nullptr;
        const std::vector<u64>* scount = nullptr;
        int root = 0;
    };
    const int world;
    std::vector<Slot> slots;
    std::vector<hipEvent_t> ready, done;
    std::vector<int> devices;  // each rank's device
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    u64 generation = 0;
    bool failed = false;  // a rank timed out: every later call fails at once (the group is poisoned)
    // How long a rank waits for the others (SR_LOCAL_BARRIER_SEC, default 300 s: a rank may be busy
    // with a long host-side walk or rehash while the others wait).
    const std::chrono::seconds timeout{std::getenv("SR_LOCAL_BARRIER_SEC") ? std::max(1, std::atoi(std::getenv("SR_LOCAL_BARRIER_SEC")))
                                                                          : 300};

    // All ranks arrive; false on timeout (a rank issued a different collective sequence, or failed).
    // A timed-out rank takes its arrival back and marks the group failed, so that no later call can
    // complete with a stale count.
    bool barrier() {
        std::unique_lock<std::mutex> g(mu);
        if (failed) return false;
        const u64 gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        cv.wait_for(g, timeout, [&] { return generation != gen || failed; });
        if (generation != gen) return true;
        if (!failed) {
            --arrived;
            failed = true;
            cv.notify_all();
        }
        return false;
    }
};

struct LocalComm final : Comm {
    std::shared_ptr<LocalGroup> g;
    const char* kind() const override { return "local"; }
    int nranks() const override { return g->world; }

    enum Op { A2A = 1, AGATHER, EXCH, BCAST, RMIN, RMAX, RSUM, SHARE };

    // Phase 1: publish this rank's call and a "ready" event (its inputs are written once the
    // stream reaches it); every rank checks that all ranks issued the same call, then orders its
    // stream after every rank's ready event.
    void arrive(int op, u64 count, const u64* send, hipStream_t s, int root = 0,
                const std::vector<const u64*>* sends = nullptr, const std::vector<u64>* scount = nullptr) {
        SR_HIP(hipSetDevice(device));
        if (!g->ready[rank]) {
            SR_HIP(hipEventCreateWithFlags(&g->ready[rank], hipEventDisableTiming));
            SR_HIP(hipEventCreateWithFlags(&g->done[rank], hipEventDisableTiming));
        }
        auto& sl = g->slots[rank];
        sl.op = op;
        sl.count = count;
        sl.send = send;
        sl.root = root;
        sl.sends = sends;
        sl.scount = scount;
        SR_HIP(hipEventRecord(g->ready[rank], s));
        sync("arrive");
        for (int q = 0; q < world; ++q) {
            const auto& o = g->slots[q];
            if (o.op != op || o.count != count || o.root != root)
                throw Error(SR_ERR_HIP, "local collective mismatch: rank " + std::to_string(q) + " issued op " +
                                            std::to_string(o.op) + " of " + std::to_string(o.count) + " words, rank " +
                                            std::to_string(rank) + " op " + std::to_string(op) + " of " +
                                            std::to_string(count));
        }
        for (int q = 0; q < world; ++q) SR_HIP(hipStreamWaitEvent(s, g->ready[q], 0));
    }
    // Phase 2, after this rank's reads are enqueued: no rank may overwrite an input before every
    // rank has read it, and no slot or event is reused before every rank has waited on it.
    void leave(hipStream_t s) {
        SR_HIP(hipEventRecord(g->done[rank], s));
        sync("reads");
        for (int q = 0; q < world; ++q) SR_HIP(hipStreamWaitEvent(s, g->done[q], 0));
        sync("leave");
    }
    void sync(const char* where) {
        if (!g->barrier())
            throw Error(SR_ERR_HIP, std::string("local collective: ranks did not meet (") + where +
                                        "): a rank issued a different sequence or failed");
    }
    void copy(void* dst, const void* src, u64 bytes, hipStream_t s) {
        if (bytes) SR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    }

    void all_to_all(const u64* send, u64* recv, u64 count, hipStream_t s) override {
        arrive(A2A, count, send, s);
        for (int q = 0; q < world; ++q) copy(recv + (u64)q * count, g->slots[q].send + (u64)rank * count, count * 8, s);
        leave(s);
    }
    void all_gather(const u64* mine, u64* all, u64 count, hipStream_t s) override {
        arrive(AGATHER, count, mine, s);
        for (int q = 0; q < world; ++q) copy(all + (u64)q * count, g->slots[q].send, count * 8, s);
        leave(s);
    }
    void exchange(const std::vector<const u64*>& send, const std::vector<u64>& scount, const std::vector<u64*>& recv,
                  const std::vector<u64>& rcount, hipStream_t s) override {
        arrive(EXCH, 0, nullptr, s, 0, &send, &scount);
        for (int q = 0; q < world; ++q) {
            const u64 c = (*g->slots[q].scount)[rank];
            if (c != rcount[q])
                throw Error(SR_ERR_HIP, "local exchange: rank " + std::to_string(q) + " sends " + std::to_string(c) +
                                            " words, rank " + std::to_string(rank) + " expects " + std::to_string(rcount[q]));
            copy(recv[q], (*g->slots[q].sends)[rank], c * 8, s);
        }
        leave(s);
    }
    void broadcast(u64* buf, u64 count, int root, hipStream_t s) override {
        DBuf<u64> tmp;  // the root's buffer is source and destination: copy through scratch
        tmp.alloc(device, count);
        arrive(BCAST, count, buf, s, root);
        copy(tmp.p, g->slots[root].send, count * 8, s);
        leave(s);
        copy(buf, tmp.p, count * 8, s);
        SR_HIP(stream_sync(s));  // tmp returns to the pool at scope exit
    }
    void all_reduce(u64* buf, u64 count, RedOp op, hipStream_t s) override {
        DBuf<u64> all;  // every rank's vector, reduced locally on the device
        all.alloc(device, count * world);
        arrive(op == RedOp::Min ? RMIN : op == RedOp::Max ? RMAX : RSUM, count, buf, s);
        for (int q = 0; q < world; ++q) copy(all.p + (u64)q * count, g->slots[q].send, count * 8, s);
        leave(s);
        reduce_rows<<<blocks_for(count, 256), 256, 0, s>>>(all.p, (u32)world, count, (u32)op, buf);
        SR_HIP(hipGetLastError());
        SR_HIP(stream_sync(s));  // `all` returns to the pool at scope exit
    }

    // Direct exchange between threads of one process: raw device pointers (peer access enabled
    // when the ranks sit on different devices). share() first finishes this rank's stream, so a
    // rank that shares a buffer it just cleared has cleared it before any peer can write to it.
    // Ranks that share a device wait for each other's flags on that device: each rank's stream
    // needs a hardware queue of its own, or a rank's wait may be queued in front of the expand it
    // waits for. Unless every stream this library created on the device (plus the runtime's own)
    // has one, the ranks take the collective exchange.
    bool peer_capable() const override {
        if (!direct_env_on()) return false;
        int same = 0;
        for (int d : g->devices) same += d == device;
        if (same <= 1) return true;
        return StreamCensus::get().on(device) + 1 <= StreamCensus::hw_queues();
    }
    bool distinct_devices() const override {
        std::set<int> d(g->devices.begin(), g->devices.end());
        return (int)d.size() == world;
    }
    void share(const void* mine, size_t bytes, void* all, hipStream_t s) override {
        SR_HIP(stream_sync(s));
        auto& sl = g->slots[rank];
        sl.op = SHARE;
        sl.count = bytes;
        sl.send = static_cast<const u64*>(mine);
        sl.root = 0;
        sync("share");
        for (int q = 0; q < world; ++q) {
            if (g->slots[q].op != SHARE || g->slots[q].count != bytes)
                throw Error(SR_ERR_HIP, "local collective mismatch in share: rank " + std::to_string(q));
            std::memcpy(static_cast<char*>(all) + (size_t)q * bytes, g->slots[q].send, bytes);
        }
        sync("share done");
    }
    u64* map(int q, const PeerBlob& b) override {
        const int pd = g->devices[q];
        if (pd != device && !peer_enabled.count(pd)) {
            SR_HIP(hipSetDevice(device));
            const hipError_t e = hipDeviceEnablePeerAccess(pd, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) SR_HIP(e);
            (void)hipGetLastError();
            peer_enabled.insert(pd);
        }
        return reinterpret_cast<u64*>(b.ptr);
    }
    std::set<int> peer_enabled;
};

// Ranks that are PROCESSES of one host, with a POSIX shared-memory segment as the host-side
// transport (sr_dist_shm_init): a barrier and one staging slot per rank. Its collectives are
// synchronous host copies (they finish before they return, which the stream-ordered contract
// allows), and buffers travel between the processes as IPC handles, as with RCCL. It exists so that
// the one-process-per-GPU code path, direct exchange included, can run as separate processes on ONE
// GPU, where RCCL refuses two ranks on the same device; `devices_distinct` is set when every rank
// has its own GPU.
struct ShmComm final : Comm {
    static constexpr int MAX_RANKS = 240;
    struct Header {
        std::atomic<u64> arrived;
        std::atomic<u64> generation;
        std::atomic<u32> failed;
        std::atomic<u32> ready;  // READY once rank 0 has initialised this segment
        // attach handshake: rank r > 0 writes a nonce of its own, rank 0 echoes it (ack), rank r
        // confirms (attach |= CONFIRMED). Only a live rank 0 echoes, so a rank that opened a
        // segment a crashed run left (already READY) gets no echo and opens the name again.
        std::atomic<u64> attach[MAX_RANKS];
        std::atomic<u64> ack[MAX_RANKS];
    };
    static_assert(sizeof(Header) <= 4096, "the header fits its page");
    static constexpr u32 READY = 0x53524844u;
    static constexpr u64 CONFIRMED = 1ull << 63;
    static constexpr size_t HDR = 4096;
    std::string name;
    size_t slot_bytes = 0;
    char* base = nullptr;
    size_t bytes = 0;
    bool devices_distinct = false;
    IpcMaps ipc;
    double timeout_s = std::getenv("SR_SHM_TIMEOUT_SEC") ? std::atof(std::getenv("SR_SHM_TIMEOUT_SEC")) : 300.0;

    ShmComm(int r, int w, const std::string& nm, int dev, size_t slot, bool distinct) {
        rank = r;
        world = w;
        device = dev;
        name = nm;
        slot_bytes = slot;
        devices_distinct = distinct;
        bytes = HDR + slot_bytes * (size_t)w;
        if (w > MAX_RANKS) throw Error(SR_ERR_ARG, "shm transport: at most 240 ranks");
        // Rank 0 removes a segment a crashed run may have left under this name and creates a fresh
        // one exclusively, with a zeroed header, marked READY last; the other ranks open it (no
        // create) once it exists at full size, wait for READY and then attach (the handshake in
        // Header): a rank that raced rank 0's unlink and opened the stale segment gets no echo
        // there and opens the name again.
        const auto t0 = Clock::now();
        if (rank == 0) {
            (void)shm_unlink(name.c_str());
            int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0) throw Error(SR_ERR_ARG, "shm_open(" + name + ", O_EXCL) failed");
            if (ftruncate(fd, (off_t)bytes) != 0) {
                ::close(fd);
                throw Error(SR_ERR_ARG, "ftruncate of the shared segment failed");
            }
            map_fd(fd);
            Header* h = hdr();
            h->arrived.store(0);
            h->generation.store(0);
            h->failed.store(0);
            for (int q = 0; q < MAX_RANKS; ++q) h->attach[q].store(0), h->ack[q].store(0);
            h->ready.store(READY, std::memory_order_release);
            // echo every rank's nonce until each has confirmed it
            for (int pending = w - 1; pending > 0;) {
                pending = 0;
                for (int q = 1; q < w; ++q) {
                    const u64 a = h->attach[q].load(std::memory_order_acquire);
                    if (a & CONFIRMED) continue;
                    ++pending;
                    if (a && h->ack[q].load(std::memory_order_relaxed) != a) h->ack[q].store(a, std::memory_order_release);
                }
                if (pending && secs(t0, Clock::now()) > timeout_s) throw Error(SR_ERR_ARG, "shm transport: ranks never attached to " + name);
                if (pending) usleep(100);
            }
            return;
        }
        const u64 nonce = (((u64)::getpid() << 20 ^ (u64)Clock::now().time_since_epoch().count() ^ (u64)r << 8) & ~CONFIRMED) | 1;
        for (;;) {
            int fd = -1;
            for (;;) {
                fd = shm_open(name.c_str(), O_RDWR, 0600);
                if (fd >= 0) {
                    struct stat st;
                    if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
                    ::close(fd);
                    fd = -1;
                }
                if (secs(t0, Clock::now()) > timeout_s) throw Error(SR_ERR_ARG, "shm transport: rank 0 never created " + name);
                usleep(1000);
            }
            map_fd(fd);
            Header* h = hdr();
            const auto t1 = Clock::now();
            bool ok = false;
            while (secs(t1, Clock::now()) < 2.0) {  // READY, then the echo of our nonce
                if (h->ready.load(std::memory_order_acquire) == READY) {
                    h->attach[r].store(nonce, std::memory_order_release);
                    if (h->ack[r].load(std::memory_order_acquire) == nonce) {
                        ok = true;
                        break;
                    }
                }
                usleep(100);
            }
            if (ok) {
                h->attach[r].store(nonce | CONFIRMED, std::memory_order_release);
                return;
            }
            munmap(base, bytes);  // no live rank 0 behind this segment (yet): open the name again
            base = nullptr;
            if (secs(t0, Clock::now()) > timeout_s) throw Error(SR_ERR_ARG, "shm transport: " + name + " never became ready");
        }
    }
    void map_fd(int fd) {
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) throw Error(SR_ERR_ARG, "mmap of the shared segment failed");
        base = static_cast<char*>(m);
    }
    ~ShmComm() override {
        ipc.close();
        if (base) munmap(base, bytes);
        if (rank == 0) shm_unlink(name.c_str());
    }
    const char* kind() const override { return "shm"; }
    int nranks() const override { return world; }
    Header* hdr() { return reinterpret_cast<Header*>(base); }
    char* slot(int q) { return base + HDR + slot_bytes * (size_t)q; }
    void need(size_t b) {
        if (b > slot_bytes) throw Error(SR_ERR_CAPACITY, "shm transport: " + std::to_string(b) + " bytes exceed its staging slot");
    }
    // every rank arrives (sense by generation); bounded
    void sync() {
        Header* h = hdr();
        if (h->failed.load()) throw Error(SR_ERR_HIP, "shm transport: a rank failed");
        const u64 g = h->generation.load();
        if (h->arrived.fetch_add(1) + 1 == (u64)world) {
            h->arrived.store(0);
            h->generation.fetch_add(1);
            return;
        }
        const auto t0 = Clock::now();
        for (u64 spin = 0; h->generation.load() == g; ++spin) {
            if ((spin & 1023) == 0 && secs(t0, Clock::now()) > timeout_s) {
                h->failed.store(1);
                throw Error(SR_ERR_HIP, "shm transport: ranks did not meet within SR_SHM_TIMEOUT_SEC");
            }
            if (spin > 4096) sched_yield();
        }
    }
    // host_only: the GPU-free protocol run (dist_host.hpp) passes host buffers and no stream; the
    // collectives are then plain copies through the segment.
    bool host_only = false;
    void d2h(void* dst, const void* src, size_t b, hipStream_t s) {
        if (b && host_only) std::memcpy(dst, src, b);
        else if (b) SR_HIP(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, s));
    }
    void h2d(void* dst, const void* src, size_t b, hipStream_t s) {
        if (b && host_only) std::memcpy(dst, src, b);
        else if (b) SR_HIP(hipMemcpyAsync(dst, src, b, hipMemcpyHostToDevice, s));
    }
    void drain(hipStream_t s) {
        if (!host_only) SR_HIP(stream_sync(s));
    }
    void all_to_all(const u64* send, u64* recv, u64 count, hipStream_t s) override {
        need(count * 8 * (size_t)world);
        d2h(slot(rank), send, count * 8 * world, s);
        drain(s);
        sync();
        for (int q = 0; q < world; ++q) h2d(recv + (u64)q * count, slot(q) + (size_t)rank * count * 8, count * 8, s);
        drain(s);
        sync();
    }
    void all_gather(const u64* mine, u64* all, u64 count, hipStream_t s) override {
        need(count * 8);
        d2h(slot(rank), mine, count * 8, s);
        drain(s);
        sync();
        for (int q = 0; q < world; ++q) h2d(all + (u64)q * count, slot(q), count * 8, s);
        drain(s);
        sync();
    }
    void exchange(const std::vector<const u64*>& send, const std::vector<u64>& scount, const std::vector<u64*>& recv,
                  const std::vector<u64>& rcount, hipStream_t s) override {
        // my slot: [T offsets][T counts][data]
        size_t off = 16 * (size_t)world, total = off;
        for (int q = 0; q < world; ++q) total += scount[q] * 8;
        need(total);
        u64* meta = reinterpret_cast<u64*>(slot(rank));
        for (int q = 0; q < world; ++q) {
            meta[q] = off;
            meta[world + q] = scount[q];
            d2h(slot(rank) + off, send[q], scount[q] * 8, s);
            off += scount[q] * 8;
        }
        drain(s);
        sync();
        for (int q = 0; q < world; ++q) {
            const u64* m = reinterpret_cast<const u64*>(slot(q));
            if (m[world + rank] != rcount[q])
                throw Error(SR_ERR_HIP, "shm exchange: rank " + std::to_string(q) + " sends " + std::to_string(m[world + rank]) +
                                            " words, rank " + std::to_string(rank) + " expects " + std::to_string(rcount[q]));
            h2d(recv[q], slot(q) + m[rank], rcount[q] * 8, s);
        }
        drain(s);
        sync();
    }
    void broadcast(u64* buf, u64 count, int root, hipStream_t s) override {
        need(count * 8);
        if (rank == root) d2h(slot(root), buf, count * 8, s);
        drain(s);
        sync();
        if (rank != root) h2d(buf, slot(root), count * 8, s);
        drain(s);
        sync();
    }
    void all_reduce(u64* buf, u64 count, RedOp op, hipStream_t s) override {
        need(count * 8);
        d2h(slot(rank), buf, count * 8, s);
        drain(s);
        sync();
        std::vector<u64> v(count);
        std::memcpy(v.data(), slot(0), count * 8);
        for (int q = 1; q < world; ++q) {
            const u64* x = reinterpret_cast<const u64*>(slot(q));
            for (u64 i = 0; i < count; ++i)
                v[i] = op == RedOp::Min ? std::min(v[i], x[i]) : op == RedOp::Max ? std::max(v[i], x[i]) : v[i] + x[i];
        }
        sync();  // every rank has read every slot
        h2d(buf, v.data(), count * 8, s);
        drain(s);
    }
    bool peer_capable() const override { return direct_env_on(); }
    bool distinct_devices() const override { return devices_distinct; }
    void share(const void* mine, size_t b, void* all, hipStream_t s) override {
        need(b);
        drain(s);
        std::memcpy(slot(rank), mine, b);
        sync();
        for (int q = 0; q < world; ++q) std::memcpy(static_cast<char*>(all) + (size_t)q * b, slot(q), b);
        sync();
    }
    PeerBlob export_buf(void* p) const override { return IpcMaps::export_of(device, p); }
    u64* map(int q, const PeerBlob& b) override { return ipc.open(device, q, b); }
};

// Per-device resources of the partitioned engine, pooled across checks like the single-GPU
// engine's DeviceContext (hipHostMalloc and stream creation cost milliseconds; a 2pc N=9 check
// takes ~3 ms): the stream, per-partition device counters / control blocks / pinned mirrors with
// their sequence numbers, the pinned row buffer and the timing events.
struct DistContext {
    struct PartRes {
        LevelCounters* lc = nullptr;
        DistCtl* ctl = nullptr;
        HostCounters* hc = nullptr;
        HostCounters* hc_dev = nullptr;
        u32 seq = 0;
        LagPub* pub[2] = {nullptr, nullptr};      // pipelined mode: pinned, slot = seq & 1
        LagPub* pub_dev[2] = {nullptr, nullptr};
        size_t pub_words = 0;
        // direct exchange: receive buffers by level parity ([T][S] words), and the table of every
        // owner's buffer of that parity (+ DIST_HDR). Kept across checks, like the streams.
        DBuf<u64> drecv[2];
        u64 drecv_words = 0;
        DBuf<u64*> ptab[2];
        DBuf<u64> dsum;  // [NSHARD][MAX_PARTS] record-word sums per owner (exchange check)
    };
    // Direct exchange state kept across the checks of one communicator (or one set of virtual
    // partitions): the flag words of this rank, the table of its word in every owner's flags, and
    // the flag sequence number of the last level (monotonic: flags are never cleared between
    // checks, so a check costs no collective set-up once the addresses are shared).
    struct Direct {
        u64 comm_uid = 0;  // the communicator served (0: virtual partitions)
        u32 T = 0;         // partitions
        bool valid = false;
        u64 gen = 0;       // set-up generation (agreed by the ranks of the communicator)
        u32 fseq = 0;
        u32 fseq_start = 0;  // diagnostics: the sequence number this check started from, and how
        bool reused = false;
        DBuf<u32> flags;
        DBuf<u32*> ftab;
    } dx;
    static constexpr size_t ROW_WORDS = (size_t)MAX_PARTS * (MAX_PARTS + 6 + MAX_PROPS);
    int dev = 0;
    hipStream_t stream = nullptr;
    std::vector<PartRes> parts;
    u64* hrows = nullptr;      // [0] = sequence word, rows from word 8
    u64* hrows_dev = nullptr;
    u32 rows_seq = 0;
    std::vector<hipEvent_t> events;

    void init(int d) {
        dev = d;
        SR_HIP(hipSetDevice(d));
        SR_HIP(create_stream(&stream, d));
        SR_HIP(hipHostMalloc(&hrows, (ROW_WORDS + 8) * 8, hipHostMallocCoherent | hipHostMallocMapped));
        SR_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&hrows_dev), hrows, 0));
        std::memset(hrows, 0, (ROW_WORDS + 8) * 8);
    }
    void ensure_parts(size_t L) {
        while (parts.size() < L) {
            PartRes r;
            SR_HIP(hipMalloc(&r.lc, sizeof(LevelCounters)));
            SR_HIP(hipMalloc(&r.ctl, sizeof(DistCtl)));
            SR_HIP(hipHostMalloc(&r.hc, sizeof(HostCounters), hipHostMallocCoherent | hipHostMallocMapped));
            SR_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.hc_dev), r.hc, 0));
            std::memset(r.hc, 0, sizeof(HostCounters));
            parts.push_back(std::move(r));
        }
    }
    // pinned publish slots of partition i holding `words` row words
    void ensure_pub(size_t i, size_t words) {
        PartRes& r = parts[i];
        if (r.pub_words >= words) return;
        for (int k = 0; k < 2; ++k) {
            if (r.pub[k]) SR_HIP(hipHostFree(r.pub[k]));
            const size_t bytes = sizeof(LagPub) + words * 8;
            SR_HIP(hipHostMalloc(&r.pub[k], bytes, hipHostMallocCoherent | hipHostMallocMapped));
            SR_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.pub_dev[k]), r.pub[k], 0));
            std::memset(r.pub[k], 0, bytes);
            r.pub[k]->seq = ~0u;
        }
        r.pub_words = words;
    }
};

template <class M>
class DistEngine final : public EngineBase {
    static constexpr int W = M::W, REC = W, TREC = W + 1;  // record = state; tree entry = state + parent gid
    static constexpr u64 NONE = ~0ull;

    struct Part {
        u32 id = 0;                      // global partition id
        DBuf<u64> keys;
        u64 cap = 0;
        DBuf<u64> arena;                 // owned states, every level, visit order
        DBuf<u64> apar;                  // parent gid of each arena state
        u64 arena_cap = 0;
        std::vector<u64> lstart{0};      // arena offset of each level
        DBuf<u64> send;                  // [T][bucket_cap][REC]
        DBuf<u64> sent;                  // sent cache (small T): fingerprints this partition routed
        u64 sent_mask = 0;
        u64 bucket_cap = 0;
        DBuf<u32> sendc;                 // [T] records per destination (device)
        DBuf<u64> recv;
        u64 recv_cap = 0;
        LevelCounters* lc = nullptr;
        DistCtl* ctl = nullptr;          // device: frontier size + its discoveries (next level's input)
        HostCounters* hc = nullptr;      // pinned host (root level only)
        HostCounters* hc_dev = nullptr;
        u32 seq = 0;
        u32 res = 0;                     // index of this partition's pooled resources
        u64 send_words = 0, recv_words = 0;  // pipelined mode: allocated bucket words
        HostCounters last{};             // last published snapshot
        u64 n = 0;                       // current frontier size (exact once its row is gathered)
        u64 n_hi = 0, n_est = 0;         // upper bound / estimate of the next frontier size
        u64 local_prev = 0, nrec_prev = 0;
        u64 uniq = 0;                    // states claimed in this partition's visited set
        const M* model = nullptr;
        TableView view() const { return make_table_view(*model, keys.p, nullptr, cap); }
        u64 words() const { return table_words(view(), cap); }  // u64 words of the table
    };

  public:
    DistEngine(M m, const sr_opts& o, Comm* comm, int virtual_parts)
        : m_(m), o_(o), comm_(comm), D_((u32)m.max_out_degree()) {
        disc.resize(M::NPROPS);
        (void)init_states_of(m_);  // a model with more init states than it declares fails at spawn
        if (model_emask(m))
            throw Error(SR_ERR_UNSUPPORTED, "partitioned search: `eventually` properties need a one-GPU check (FIFO or FAST order)");
        T_ = comm_ ? (u32)comm_->world : (u32)std::max(1, virtual_parts);
        // `target_state_count` (bfs.rs:113-135): the reference stops at a 1500-pop block boundary of
        // its worker order; the partitioned levels have no single pop order, so the check stops at
        // the first LEVEL boundary where state_count >= target (the levels synchronous, no head).
        if (o_.target_state_count) {
            lag_ = false;
            head_max_ = 0;
        }
        if (T_ > (u32)MAX_PARTS) throw Error(SR_ERR_ARG, "at most 64 partitions");
        const u32 L = comm_ ? 1 : T_;
        parts_.resize(L);
        for (u32 i = 0; i < L; ++i) {
            parts_[i].id = comm_ ? (u32)comm_->rank : i;
            parts_[i].model = &m_;
        }
        if (!filter_exact(m_)) {
            // exact multi-word quotient-mode tables: the LDS filter and the sent cache compare
            // fingerprints, which are not exact for multi-word states
            filt_log2_ = 0;
            send_cache_max_parts_ = 0;
        }
        // With an owner key most successors stay local and the routed ones are few: the sent cache's
        // lookups (a memory round trip per remote successor, issued with the local probes) cost more
        // than the duplicates it keeps off the link (config 4, 2pc N=11 at T = 2: 45.6 -> 36.9 ms per
        // rank without it, T = 4: 24.5 -> 21.2; profiles/r06_config4_stages.txt).
        if (okey_ && !std::getenv("SR_SEND_CACHE")) send_cache_max_parts_ = 0;
    }
    ~DistEngine() override {
        if (ctx_) {
            (void)stream_sync(stream_);
            for (size_t i = 0; i < parts_.size(); ++i) ctx_->parts[i].seq = parts_[i].seq;
            ContextPool<DistContext>::get().release(ctx_);
        }
    }

    int nprops() const override { return M::NPROPS; }
    const char* prop_name(int p) const override { return m_.prop_name(p); }
    int expectation(int p) const override { return m_.expectation(p); }
    int width() const override { return m_.describe_width(); }
    std::string action_name(i64 id) const override { return m_.action_name(id); }
    i64 action_id_bound() const override { return m_.action_id_bound(); }
    int init_count() const override { return (int)(init_states_of(base_model(m_)).size() / std::decay_t<decltype(base_model(m_))>::W); }
    int replay(int init, const i64* ids, int n, std::vector<i64>& states, std::vector<int>& conds,
               std::vector<int>* all_conds, int* terminal) const override {
        return replay_model(base_model(m_), init, ids, n, states, conds, all_conds, terminal);
    }
    int explore(const u64* fps, int n, std::vector<i64>& action, std::vector<int>& has, std::vector<u64>& fp,
                std::vector<i64>& states) const override {
        return explore_model(base_model(m_), fps, n, action, has, fp, states);
    }
    // The visit record (sr_opts.record_visits: the StateRecorder / PathRecorder / Fn(Path)
    // visitors, src/checker/visitor.rs:19-99, called at every pop by src/checker/bfs.rs:187-189),
    // gathered on every rank at join (gather_visits): the states level by level, a level in
    // partition order and each partition's part in its arena (FAST) order.
    std::vector<i64> visits() const override {
        const int wd = m_.describe_width();
        std::vector<i64> out(vst_.size() / W * wd);
        for (size_t i = 0; i < vst_.size() / W; ++i) m_.describe(&vst_[i * W], &out[i * wd]);
        return out;
    }
    // Each visited state's parent: the FIRST generator of it in the previous level's visit order,
    // by the first action in `actions()` order (a FAST-order BFS tree: any generator is a valid
    // parent, src/checker/path.rs:55-79), found on the host model from the gathered states.
    bool visit_tree(std::vector<i64>& parent, std::vector<i64>& action) const override {
        if (!o_.record_visits) return false;
        parent.clear();
        action.clear();
        std::unordered_map<u64, std::pair<i64, i64>> first;  // fingerprint -> (parent visit index, action id)
        i64 base = 0, prev_base = 0;
        for (size_t d = 0; d < vlev_.size(); ++d) {
            const i64 nv = (i64)vlev_[d];
            if (d > 0) {
                first.clear();
                for (i64 i = prev_base; i < base; ++i) {
                    const u64* ps = &vst_[(size_t)i * W];
                    for_each_successor(m_, ps, [&](int a, const u64* ns) {
                        first.emplace(state_fp<M>(ns), std::make_pair(i, m_.action_id(ps, a)));
                    });
                }
            }
            for (i64 i = 0; i < nv; ++i) {
                if (d == 0) {
                    parent.push_back(-1);
                    action.push_back(-1);
                    continue;
                }
                auto it = first.find(state_fp<M>(&vst_[(size_t)(base + i) * W]));
                if (it == first.end()) throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path` for a visited state");
                parent.push_back(it->second.first);
                action.push_back(it->second.second);
            }
            prev_base = base;
            base += nv;
        }
        return true;
    }
    int partitions() const { return (int)T_; }
    bool early_exit() const { return early_exit_; }

    void run() override {
        SR_HIP(hipSetDevice(o_.device));
        if (!ctx_) {
            ctx_ = ContextPool<DistContext>::get().acquire(o_.device);
            ctx_->ensure_parts(parts_.size());
            stream_ = ctx_->stream;
            for (size_t i = 0; i < parts_.size(); ++i) {
                auto& r = ctx_->parts[i];
                parts_[i].lc = r.lc;
                parts_[i].ctl = r.ctl;
                parts_[i].hc = r.hc;
                parts_[i].hc_dev = r.hc_dev;
                parts_[i].seq = r.seq;
                parts_[i].res = (u32)i;
            }
        }
        for (int attempt = 0;; ++attempt) {
            // With the direct exchange every rank votes on the outcome of the check (one small
            // collective over the communicator's own transport): an exchange that delivered a
            // stale or partial slot is seen by its owner only (ERR_EXCHANGE, ERR_PEER_TIMEOUT), and
            // its rows may not reach the others. Same decision on every rank: `vote` depends only
            // on collectively agreed state.
            const bool vote = comm_ && lag_ && direct_env_on() && comm_->direct_ok != 0 && vote_;
            int code = 0;  // 0 ok, 1 capacity restart, 2 exchange failure, 3 other error
            std::string what;
            int ecode = 0;
            try {
                run_once();
            } catch (const Error& e) {
                code = outcome_of(e.code);
                what = e.what();
                ecode = e.code;
                if (!vote) {
                    if (code == 2 && !comm_ && attempt < 3) {  // virtual partitions: no collective to agree on
                        exchange_fallback(what);
                        continue;
                    }
                    if (code == 2) throw Error(SR_ERR_HIP, what);
                    if (code != 1 || attempt >= 3) throw;
                }
            }
            if (vote) {
                SR_HIP(stream_sync(stream_));  // in-flight levels end (a wait for a stopped peer times out)
                u64 v[2] = {(u64)code, ~(u64)code};  // max and min of the ranks' outcomes
                DBuf<u64> dv;
                dv.alloc(o_.device, 2);
                SR_HIP(hipMemcpyAsync(dv.p, v, sizeof(v), hipMemcpyHostToDevice, stream_));
                comm_->all_reduce(dv.p, 2, RedOp::Max, stream_);
                SR_HIP(hipMemcpyAsync(v, dv.p, sizeof(v), hipMemcpyDeviceToHost, stream_));
                SR_HIP(stream_sync(stream_));
                const VoteDecision d = decide_after_vote(code, (int)v[0], (int)~v[1], attempt, ecode, what);
                if (d.act == VoteAction::Fail) throw Error(d.code, d.why);
                if (d.act == VoteAction::Fallback) {
                    exchange_fallback(d.why);
                    continue;
                }
                if (d.act == VoteAction::Done) {
                    gather_paths();
                    gather_visits();
                    return;
                }
                // a capacity restart on every rank (the direct exchange kept)
                if (d.disagree)
                    std::fprintf(stderr, "[sr] rank %d: the ranks disagree on a capacity restart (this rank: %s); restarting on every rank\n",
                                 comm_->rank, code ? what.c_str() : "finished");
                what = d.why;
            } else if (code == 0) {
                gather_paths();
                gather_visits();
                return;
            }
            // capacity: every rank saw it at the same level (the rows are the same everywhere)
            SR_HIP(stream_sync(stream_));
            stats.restarts++;
            restarts_++;
            if (head_failed_) {  // the head's scratch buffers were too small: no head
                head_ok_ = false;
                head_failed_ = false;
                continue;
            }
            if (lag_) {
                // the pipelined plan under-estimated a level: rerun with one host
                // synchronisation per level (exact bucket sizes)
                if (o_.verbose) std::fprintf(stderr, "[sr] %s; restarting in synchronous mode\n", what.c_str());
                lag_ = false;
                continue;
            }
            if (o_.verbose) std::fprintf(stderr, "[sr] %s; restarting with larger buffers\n", what.c_str());
            pessimistic_ = true;
            grow_factor_ *= 4;
        }
    }

    // The direct exchange failed its check (a slot's sequence tag or checksum, or a source that
    // never raised its flag): the check is redone on the collective exchange, which this
    // communicator (or these virtual partitions) keeps from now on.
    void exchange_fallback(const std::string& why) {
        SR_HIP(stream_sync(stream_));
        if (comm_) comm_->direct_ok = 0;
        direct_off_ = true;
        ctx_->dx.valid = false;  // never reused: a late peer store may still land in it
        exchange_fallbacks_++;
        std::fprintf(stderr, "[sr] direct exchange failed (%s); redoing the check with the collective exchange\n",
                     why.c_str());
    }

    // Every discovery path, gathered on every rank at the end of the run (one collective walk per
    // discovered property, in property order: `disc_at_` is the same on every rank), so that a
    // single rank may ask for a path later. Deferred (sr_opts.defer_paths) paths are walked on
    // demand, collectively.
    void gather_paths() {
        paths_.assign(M::NPROPS, {});
        paths_ready_ = false;
        if (o_.defer_paths || !comm_) return;  // virtual partitions walk on demand, locally
        for (int p = 0; p < M::NPROPS; ++p) {
            if (!disc_at_[p].found) continue;
            tree_path(p, paths_[p]);
            // A walk through the replicated head is local to each rank, whose head arena holds
            // each level in its own (FAST) order: every rank's path is valid, but they may differ.
            // Rank 0's path goes to every rank, so that all report the same one.
            DBuf<u64> buf;
            buf.alloc(o_.device, 1);
            u64 len = paths_[p].size();
            SR_HIP(hipMemcpyAsync(buf.p, &len, 8, hipMemcpyHostToDevice, stream_));
            comm_->broadcast(buf.p, 1, 0, stream_);
            SR_HIP(hipMemcpyAsync(&len, buf.p, 8, hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            buf.alloc(o_.device, std::max<u64>(1, len));
            if (comm_->rank == 0 && len)
                SR_HIP(hipMemcpyAsync(buf.p, paths_[p].data(), len * 8, hipMemcpyHostToDevice, stream_));
            comm_->broadcast(buf.p, std::max<u64>(1, len), 0, stream_);
            paths_[p].resize(len);
            if (len) SR_HIP(hipMemcpyAsync(paths_[p].data(), buf.p, len * 8, hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
        }
        paths_ready_ = true;
    }
    // Every visited state to every rank (record_visits; collective: every rank runs it at join):
    // the replicated head's levels from rank 0's head arena, then each partitioned level from
    // every partition's arena (a partition's whole arena prefix broadcast by its owner rank).
    void gather_visits() {
        vst_.clear();
        vlev_.clear();
        if (!o_.record_visits) return;
        // levels 0..max_depth hold states; after a target_state_count stop the last of them was
        // generated but never popped, and the reference visits a state at its pop (bfs.rs:188)
        const u32 md = max_depth.load(), last = target_stop_ && md > 0 ? md - 1 : md;
        auto fetch = [&](const u64* dev, u64 words, int root) {
            std::vector<u64> h(words);
            if (!words) return h;
            if (!comm_) {
                SR_HIP(hipMemcpy(h.data(), dev, words * 8, hipMemcpyDeviceToHost));
                return h;
            }
            DBuf<u64> buf;
            buf.alloc(o_.device, words);
            if (comm_->rank == root) SR_HIP(hipMemcpyAsync(buf.p, dev, words * 8, hipMemcpyDeviceToDevice, stream_));
            comm_->broadcast(buf.p, words, root, stream_);
            SR_HIP(hipMemcpyAsync(h.data(), buf.p, words * 8, hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            return h;
        };
        SR_HIP(stream_sync(stream_));
        const u32 head_levels = head_done_ ? last + 1 : lvl0_;
        if (head_levels) {
            const u64 hn = hlstart_[std::min<size_t>(head_levels, hlstart_.size() - 1)];
            const std::vector<u64> h = fetch(harena_.p, hn * W, 0);
            for (u32 d = 0; d < head_levels && d + 1 < hlstart_.size(); ++d) {
                vlev_.push_back(hlstart_[d + 1] - hlstart_[d]);
                vst_.insert(vst_.end(), h.begin() + (i64)(hlstart_[d] * W), h.begin() + (i64)(hlstart_[d + 1] * W));
            }
        }
        if (head_done_) return;
        std::vector<std::vector<u64>> arenas(T_);
        for (u32 q = 0; q < T_; ++q) {
            const Part* pp = nullptr;
            for (auto& p : parts_)
                if (p.id == q) pp = &p;
            arenas[q] = fetch(pp ? pp->arena.p : nullptr, gl_off_[q] * W, (int)q);
        }
        for (u32 d = lvl0_; d <= last; ++d) {
            u64 n = 0;
            for (u32 q = 0; q < T_; ++q) {
                const size_t k = d - lvl0_;
                const u64 lo = gl_lstart_[q][k], hi = k + 1 < gl_lstart_[q].size() ? gl_lstart_[q][k + 1] : gl_off_[q];
                vst_.insert(vst_.end(), arenas[q].begin() + (i64)(lo * W), arenas[q].begin() + (i64)(hi * W));
                n += hi - lo;
            }
            vlev_.push_back(n);
        }
    }
    std::vector<u64> vst_;   // visited states (gather_visits)
    std::vector<u64> vlev_;  // visited states per level

    bool path_states(int p, std::vector<u64>& st) {
        if (p < 0 || p >= M::NPROPS) return false;
        if (paths_ready_) {
            st = paths_[p];
            return !st.empty();
        }
        return tree_path(p, st);
    }

    // `reconstruct_path` across partitions: walk parent gids.
    int chain(int p, std::vector<u64>& out) override {
        out.clear();
        std::vector<u64> st;
        if (!path_states(p, st)) return 0;
        return fingerprint_chain(m_, st, out);
    }
    int path(int p, std::vector<i64>& actions, std::vector<i64>& states) override {
        std::vector<u64> st;
        if (!path_states(p, st)) return -1;
        return concrete_path(m_, st, actions, states);
    }
  private:
    struct DiscAt {
        bool found = false;
        u32 level = 0, part = 0, rank = 0;
        bool head = false;  // found in the replicated head: rank is in the head arena's level
    };

    // ---- exchange ---------------------------------------------------------------------------
    // Waits for rows_publish and copies the gathered rows out of pinned memory.
    void wait_rows(u32 seq, size_t words) {
        volatile u32* flag = reinterpret_cast<volatile u32*>(ctx_->hrows);
        for (u64 spin = 1;; ++spin) {
            if (*flag == seq) break;
            if ((spin & 4095) == 0) {
                hipError_t e = hipStreamQuery(stream_);
                if (e != hipSuccess && e != hipErrorNotReady) SR_HIP(e);
                if (e == hipSuccess && *flag != seq) {
                    if (*flag == seq) break;
                    throw Error(SR_ERR_HIP, "level finished without publishing its rows");
                }
            }
            _mm_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        rows_.assign(words, 0);
        std::memcpy(rows_.data(), (const void*)(ctx_->hrows + 8), words * 8);
    }

    void wait(Part& p) {
        volatile u32* flag = &p.hc->seq;
        for (u64 spin = 1;; ++spin) {
            if (*flag == p.seq) break;
            if ((spin & 4095) == 0) {
                hipError_t e = hipStreamQuery(stream_);
                if (e != hipSuccess && e != hipErrorNotReady) SR_HIP(e);
                if (e == hipSuccess && *flag != p.seq) {
                    if (*flag == p.seq) break;
                    throw Error(SR_ERR_HIP, "launch finished without publishing its counters");
                }
            }
            _mm_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        std::memcpy(&p.last, (const void*)p.hc, sizeof(HostCounters));
    }

    // Grows partition p's arena to hold `states`, preserving its first `used` states.
    void ensure_arena(Part& p, u64 states, u64 used) {
        if (p.arena_cap >= states) return;
        u64 cap = std::max<u64>(states, p.arena_cap * 2);
        used = std::min<u64>(used, p.arena_cap);
        DBuf<u64> na, np;
        na.alloc(o_.device, cap * W);
        np.alloc(o_.device, cap);
        if (used) {
            SR_HIP(hipMemcpyAsync(na.p, p.arena.p, used * W * 8, hipMemcpyDeviceToDevice, stream_));
            SR_HIP(hipMemcpyAsync(np.p, p.apar.p, used * 8, hipMemcpyDeviceToDevice, stream_));
        }
        p.arena.swap(na);
        p.apar.swap(np);
        p.arena_cap = cap;
        arena_grows_++;
        SR_HIP(stream_sync(stream_));
    }

    hipEvent_t event(size_t i) {
        auto& ev = ctx_->events;
        while (ev.size() <= i) {
            hipEvent_t e;
            SR_HIP(hipEventCreate(&e));
            ev.push_back(e);
        }
        return ev[i];
    }

    // The load at which a partition's visited set grows: the probe limit's (lmax) for a hinted
    // check, whose tables are planned at part_load_ from the start; without a hint the tables start
    // at the default size and grow once a level would take them past 1.5 part_load_ (to part_load_,
    // in one step: want = the states the level may leave in it), rather than running the rest of
    // the check at up to lmax (2pc N=9 on one rank ended at 0.62 load: expand_route 2.61 ms per
    // check against 1.98 hinted, profiles/r06_partitioned_nohint.txt).
    double grow_at(u64 cap) const {
        return o_.capacity_hint ? lmax(cap) : std::min(lmax(cap), 1.5 * part_load_);
    }
    void grow_table(Part& p, u64 want = 0) {
        DBuf<u64> ok;
        ok.swap(p.keys);
        const u64 old_cap = p.cap;
        u64 f = 2;
        if (!o_.capacity_hint)
            while ((double)want > std::min(part_load_, lmax(old_cap * f)) * (double)(old_cap * f) && f < 64) f *= 2;
        p.cap = old_cap * f;
        const TableView from = make_table_view(m_, ok.p, nullptr, old_cap), to0 = make_table_view(m_, nullptr, nullptr, p.cap);
        u32 lg = 0;
        while ((1ull << lg) < f) ++lg;
        const u64 S = to0.s32 ? rebuild_slots<u32>() : rebuild_slots<u64>();
        // range by range as in Engine::launch_rehash (no clear of the new table), else clear + CAS
        const bool ranges = from.qbits && to0.qbits && from.qbits == to0.qbits + lg && f <= S && p.cap % S == 0;
        p.keys.alloc(o_.device, p.words());
        if (ranges) {
            const u64 nranges = p.cap / S, spill_cap = nranges + 65536;
            if (spill_.n < spill_cap + 1) spill_.alloc(o_.device, spill_cap + 1);
            SR_HIP(hipMemsetAsync(spill_.p, 0, sizeof(u64), stream_));
            if (to0.s32)
                rehash_ranges<u32><<<(u32)nranges, REBUILD_BLOCK, 0, stream_>>>(from, old_cap, p.view(), lg, spill_.p,
                                                                               spill_cap, &p.lc->err);
            else
                rehash_ranges<u64><<<(u32)nranges, REBUILD_BLOCK, 0, stream_>>>(from, old_cap, p.view(), lg, spill_.p,
                                                                               spill_cap, &p.lc->err);
            SR_HIP(hipGetLastError());
            rehash_spill<<<256, 256, 0, stream_>>>(from, p.view(), spill_.p, spill_cap, &p.lc->err);
        } else {
            SR_HIP(hipMemsetAsync(p.keys.p, 0, p.words() * 8, stream_));
            rehash<<<blocks_for(old_cap, 256), 256, 0, stream_>>>(from, old_cap, p.view(), &p.lc->err);
        }
        SR_HIP(hipGetLastError());
        SR_HIP(stream_sync(stream_));
        stats.rehashes++;
    }
    DBuf<u64> spill_;  // rehash_ranges' spill list

    void init_counters(Part& p) {
        LevelCounters z;
        std::memset(&z, 0, sizeof(z));
        for (auto& d : z.disc) d = ~0u;
        SR_HIP(hipMemcpyAsync(p.lc, &z, sizeof(z), hipMemcpyHostToDevice, stream_));
    }

    void run_once() {
        auto t_start = Clock::now();
        state_count = 0;
        unique = 0;
        target_stop_ = false;
        max_depth = 0;
        reference_done = false;
        early_exit_ = false;
        for (auto& d : disc) d = DiscoveryRec{};
        disc_at_.assign(M::NPROPS, DiscAt{});
        stats = sr_stats{};
        stats.words_per_state = W;
        stats.order_used = SR_ORDER_FAST;
        stats.restarts = restarts_;
        stats.exchange_fallbacks = exchange_fallbacks_;
        stats.owner_key = okey_ ? 1u : 0u;
        stats.pipelined = lag_ ? 1u : 0u;
        const u64 hint = o_.capacity_hint ? o_.capacity_hint : (u64)1 << 22;
        gl_lstart_.assign(T_, {});
        gl_off_.assign(T_, 0);
        lvl0_ = 0;
        head_done_ = false;
        head_undiscovered_ = (1u << M::NPROPS) - 1;
        const bool use_head = head_max_ > 0 && head_ok_ && T_ > 1;  // one partition: nothing to save
        const u64 per_part = hint / T_ + 1;

        // ---- partitions: visited sets, arenas, level 0 ----
        const std::vector<u64> inits = init_states_of(m_);
        const int k = (int)(inits.size() / W);
        std::vector<u64> rev(k * W);
        for (int i = 0; i < k; ++i) std::copy(&inits[i * W], &inits[i * W] + W, &rev[(k - 1 - i) * W]);
        DBuf<u64> dinit;
        DBuf<u32> dn;
        dinit.alloc(o_.device, k * W);
        dn.alloc(o_.device, 1);
        SR_HIP(hipMemcpyAsync(dinit.p, rev.data(), rev.size() * 8, hipMemcpyHostToDevice, stream_));
        const size_t RW = T_ + 6 + M::NPROPS;
        rows_all_.alloc(o_.device, RW * T_);
        if (comm_) rows_mine_.alloc(o_.device, RW);
        for (auto& p : parts_) {
            u64 cap = std::max<u64>((u64)(1u << 16) * grow_factor_, min_table_cap(m_));
            while ((double)cap * std::min(part_load_, lmax(cap)) < (double)per_part * grow_factor_) cap <<= 1;
            p.uniq = 0;
            p.cap = cap;
            p.keys.alloc(o_.device, p.words());
            SR_HIP(hipMemsetAsync(p.keys.p, 0, p.words() * 8, stream_));
            p.arena_cap = 0;
            p.last = HostCounters{};
            p.lstart.assign(1, 0);
            ensure_arena(p, (per_part + per_part / 8 + 4096) * grow_factor_, 0);
            p.sendc.alloc(o_.device, (size_t)T_ * SENDC_STRIDE);
            SR_HIP(hipMemsetAsync(p.sendc.p, 0, (size_t)T_ * SENDC_STRIDE * 4, stream_));
            // sent cache: with few partitions a sender generates each remote state several times
            // per level (in-degree / T), and every copy would cross the link
            p.sent_mask = 0;
            if (T_ >= 2 && T_ <= send_cache_max_parts_) {
                u64 sc = 1u << 16;
                while (sc < 2 * per_part * grow_factor_ && sc < ((u64)1 << 28)) sc <<= 1;
                if (p.sent.n < sc) p.sent.alloc(o_.device, sc);
                SR_HIP(hipMemsetAsync(p.sent.p, 0, sc * 8, stream_));
                p.sent_mask = sc - 1;
            }
            init_counters(p);
            if (use_head) continue;  // the replicated head seeds the partitions (run_head)
            insert_roots_part<M><<<1, 64, 0, stream_>>>(m_, p.view(), dinit.p, (u32)k, p.id, T_, p.arena.p, p.apar.p, dn.p, p.lc);
            u32 n0 = 0;
            SR_HIP(hipMemcpyAsync(&n0, dn.p, 4, hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            p.n = n0;
            if (n0) eval_roots<M><<<blocks_for(n0, 64), 64, 0, stream_>>>(m_, p.arena.p, n0, p.lc, (1u << M::NPROPS) - 1);
            p.seq++;
            publish_kernel<<<1, 64, 0, stream_>>>(p.lc, p.hc_dev, p.seq, 1, nullptr);
            SR_HIP(hipGetLastError());
            wait(p);
            // the level-0 control block: frontier = the queued roots, discoveries among them
            DistCtl c0;
            std::memset(&c0, 0, sizeof(c0));
            c0.n = n0;
            c0.roots = p.last.claims;
            for (int pr = 0; pr < MAX_PROPS; ++pr) c0.disc_prev[pr] = pr < M::NPROPS ? p.last.disc[pr] : ~0u;
            SR_HIP(hipMemcpyAsync(p.ctl, &c0, sizeof(c0), hipMemcpyHostToDevice, stream_));
            SR_HIP(stream_sync(stream_));
            p.uniq = p.last.claims;
            p.n_hi = n0;
            p.n_est = n0;
        }
        SR_HIP(stream_sync(stream_));
        state_count = (u64)k;
        u64 unique_total = 0;
        if (use_head) run_head(rev, k, unique_total);
        u64 glob_est = 0;  // estimated global frontier size of the level being expanded
        for (auto& p : parts_) glob_est += p.n;  // virtual mode: exact; RCCL: own share
        if (comm_) glob_est *= T_;
        u32 undiscovered = head_undiscovered_;
        double ratio = (double)D_;  // non-self-loop successors per parent, last level
        double new_frac = 1.0;      // received records that were new, last level
        double growth = 2.0;        // global frontier growth, last level
        u64 prev_glob_n = 0;
        auto t_loop = Clock::now();

        // One host synchronisation per level: the all-gathered rows of expand_route. The exchange,
        // insert_recv and the NEXT level's expand_route are enqueued right after it; the next
        // expand reads its frontier size from the device (DistCtl), so the GPU never waits for
        // the host between the insert and the next expansion.
        if (head_done_) {
            // the replicated head explored everything (or discovered every property)
        } else if (lag_) lag_loop(unique_total, undiscovered);
        else for (u32 level = lvl0_;; ++level) {
            const bool target_hit = o_.target_state_count && level > lvl0_ && state_count >= o_.target_state_count;
            // ---- 1. expand + route (grid sized from an upper bound of the frontier) ----
            const u64 d_eff = pessimistic_ ? D_ : std::min<u64>(D_, (u64)std::ceil(1.5 * ratio + 1.0));
            for (auto& p : parts_) {
                // keep each visited-set partition under 75% load for this level's share of new states
                // new states of a level ~ the frontier times its growth (not its successor count:
                // most successors are duplicates)
                const double g = std::min((double)d_eff, std::max(1.0, growth) * 1.5);
                const u64 expect_new = (u64)((double)glob_est * g / (double)T_) + 1024;
                const u64 want = p.uniq + p.n_hi + expect_new;
                while ((double)want > grow_at(p.cap) * (double)p.cap) grow_table(p, want);
                const u64 nb = p.lstart.back();  // arena offset of the frontier being expanded
                const u64 n_plan = pessimistic_ ? p.n_hi : std::min(p.n_hi, p.n_est * 2 + 1024);
                // records per destination: last level's records per parent (measured), with slack
                const double rpp = std::min((double)d_eff, 1.5 * rec_ratio_ + 1.0);
                u64 bcap = (u64)((double)n_plan * rpp / (double)std::max<u32>(1, T_ - 1) * 1.5) + 4096;
                if (pessimistic_) bcap = p.n_hi * D_ + 4096;
                if (p.bucket_cap < bcap) {
                    p.bucket_cap = bcap;
                    p.send.alloc(o_.device, bcap * T_ * REC);
                }
                // local new states of this level: ~ the frontier times its growth (an overflow
                // restarts the check pessimistically)
                const double npp = pessimistic_ ? (double)d_eff : std::min((double)d_eff, std::max(4.0, 2.0 * growth));
                ensure_arena(p, nb + p.n_hi + (u64)((double)n_plan * npp) + 4096, nb + p.n_hi);
                if (o_.profile) SR_HIP(hipEventRecord(event(2 * stats.expand_launches), stream_));
                const u32 ppw_log2 = route_ppw_env_ >= 0 ? (u32)route_ppw_env_ : ppw_for(p.n_est);
                const u32 grid = (u32)std::min<u64>(std::max<u64>(1, blocks_for(p.n_hi, 4u << ppw_log2)), route_grid_cap());
                u64* row = comm_ ? rows_mine_.p : rows_all_.p + (u64)p.id * RW;
                auto route = route_kernel(p);
                route<<<grid, 256, route_lds(), stream_>>>(
                    m_, p.arena.p, p.apar.p, nb, p.arena_cap, p.view(), p.id, T_, p.send.p, (u32)p.bucket_cap,
                    p.sendc.p, p.lc, p.ctl, undiscovered, row, ppw_log2, filt_log2_, p.bucket_cap * REC, 0u,
                    p.sent_mask ? p.sent.p : nullptr, p.sent_mask, rstage_recs(), nullptr, nullptr, 0u, rflags(), nullptr, 0u);
                SR_HIP(hipGetLastError());
                if (o_.profile) SR_HIP(hipEventRecord(event(2 * stats.expand_launches + 1), stream_));
                stats.expand_launches++;
            }
            // ---- 2. all-gather one row per partition; the host waits for it ----
            if (comm_) comm_->all_gather(rows_mine_.p, rows_all_.p, RW, stream_);
            const u32 rseq = ++ctx_->rows_seq;
            u32* hseq = reinterpret_cast<u32*>(ctx_->hrows_dev);
            rows_publish<<<1, 64, 0, stream_>>>(rows_all_.p, ctx_->hrows_dev + 8, (u32)(RW * T_), hseq, rseq);
            SR_HIP(hipGetLastError());
            wait_rows(rseq, RW * T_);
            const std::vector<u64>& all = rows_;
            const LevelPlan::Sums sm = LevelPlan::sums(all.data(), T_, RW);
            const u64 glob_n = sm.n, glob_succ = sm.succ, glob_roots = sm.roots, glob_enabled = sm.enabled;
            for (u32 q = 0; q < T_; ++q) {
                gl_lstart_[q].push_back(gl_off_[q]);  // arena offset of this level in partition q
                gl_off_[q] += all[q * RW + T_ + ROW_N];
            }
            throw_row_errors(sm.err, level);
            for (auto& p : parts_) {
                const u64* row = &all[p.id * RW];
                if (level > lvl0_) {
                    // the frontier just expanded is exact now: what the last insert_recv received new
                    const u64 recv_new = row[T_ + 0] - std::min<u64>(row[T_ + 0], p.local_prev);
                    if (p.nrec_prev) new_frac = std::min(1.0, (double)recv_new / (double)p.nrec_prev);
                    p.uniq += row[T_ + 0];
                }
                p.n = row[T_ + 0];
                p.lstart.push_back(p.lstart.back() + p.n);  // where the next frontier starts
            }
            if (level == 0) unique_total = glob_roots;  // (a replicated head sets it instead)
            if (target_hit && glob_n) {
                // the last level took state_count to the target: its successors are all inserted
                // (this frontier, generated but never popped: no discovery among them counts),
                // this expansion is not counted, and the check is not done
                unique_total += glob_n;
                max_depth = level;
                unique = unique_total;
                reference_done = false;
                early_exit_ = true;
                target_stop_ = true;
                break;
            }
            // discoveries among this level's states: the lowest (partition, rank) per property
            u32 newly = 0;
            for (int pr = 0; pr < M::NPROPS; ++pr) {
                if (!(undiscovered >> pr & 1)) continue;
                for (u32 q = 0; q < T_; ++q) {
                    u32 rk = (u32)all[q * RW + T_ + 6 + pr];
                    if (rk != ~0u) {
                        disc_at_[pr] = DiscAt{true, level, q, rk};
                        disc[pr].found = true;
                        disc[pr].level = level;
                        disc[pr].rank = rk;
                        newly |= 1u << pr;
                        break;
                    }
                }
            }
            undiscovered &= ~newly;
            if (trace_) {
                const double us = std::chrono::duration<double, std::micro>(Clock::now() - t_trace_).count();
                std::fprintf(stderr, "[sr-dist] level %u n=%llu succ=%llu  %.1f us since last row  grows=%llu arena=%llu\n",
                             level, (unsigned long long)glob_n, (unsigned long long)glob_succ, us,
                             (unsigned long long)stats.rehashes, (unsigned long long)arena_grows_);
                t_trace_ = Clock::now();
            }
            if (prev_glob_n) growth = (double)glob_n / (double)prev_glob_n;
            if (glob_n) en_ratio_ = std::max(1.0, (double)glob_enabled / (double)glob_n);
            if (glob_n) {
                u64 recs = 0;
                for (u32 q = 0; q < T_; ++q)
                    for (u32 d = 0; d < T_; ++d) recs += all[q * RW + d];
                rec_ratio_ = (double)recs / (double)glob_n;
                stats.records_routed += recs;
            }
            prev_glob_n = glob_n;
            if (glob_n == 0) {  // frontier exhausted everywhere: `is_done` (bfs.rs:307-311)
                reference_done = true;
                break;
            }
            if (level > lvl0_) unique_total += glob_n;  // every state is in exactly one frontier
            max_depth = level;
            unique = unique_total;
            if (M::NPROPS == 0 || (newly && undiscovered == 0)) {
                // Early exit: every property discovered in this level (order-dependent in FAST);
                // this level's (speculative) expansion is not counted.
                reference_done = true;
                early_exit_ = true;
                break;
            }
            state_count += glob_succ;
            stats.successors += glob_succ;
            ratio = glob_n ? (double)glob_succ / (double)glob_n : ratio;

            // ---- 3. all-to-all of the records ----
            exchange(all, RW);

            // ---- 4. owners insert what they received (closes the level on the device) ----
            glob_est = 0;
            for (auto& p : parts_) {
                u64 nrec = 0;
                for (u32 q = 0; q < T_; ++q) nrec += all[q * RW + p.id];
                const u64 local_new = all[p.id * RW + T_ + 2];
                const u64 nb = p.lstart.back();  // start of the next frontier
                ensure_arena(p, nb + local_new + nrec + 1, nb + local_new);
                const u32 ncap = (u32)std::min<u64>(p.arena_cap - nb, 0xffffffffu);
                // a capped grid: every workgroup reserves its span of the frontier at least once
                insert_recv<M><<<(u32)std::min<u64>(std::max<u32>(1, blocks_for(nrec, 256)), INSERT_GRID_MAX), 256, 0, stream_>>>(
                    m_, p.recv.p, (u32)nrec, p.view(), p.arena.p + nb * W, p.apar.p + nb, ncap, p.lc, undiscovered, p.ctl);
                SR_HIP(hipGetLastError());
                p.local_prev = local_new;
                p.nrec_prev = nrec;
                p.n_hi = local_new + nrec;  // exact upper bound of the next frontier
                p.n_est = std::min<u64>(p.n_hi, local_new + (u64)std::ceil((double)nrec * std::min(1.0, 2.0 * new_frac + 0.02)));
                glob_est += p.n_est;
            }
            if (comm_) glob_est *= T_;
            stats.levels++;
        }
        unique = unique_total;
        auto t_end = Clock::now();
        if (o_.profile && stats.expand_launches) {
            SR_HIP(hipEventSynchronize(event(2 * stats.expand_launches - 1)));
            double ms = 0;
            for (u64 i = 0; i < stats.expand_launches; ++i) {
                float t = 0;
                SR_HIP(hipEventElapsedTime(&t, event(2 * i), event(2 * i + 1)));
                ms += t;
            }
            stats.expand_kernel_ms = ms;
        }
        stats.algorithmic_bytes = stats.successors * 8 + (unique_total) * (16 + 8 * W) + unique_total * 8 * W;
        stats.level_loop_sec = secs(t_loop, t_end);
        stats.total_sec = secs(t_start, t_end);
        stats.table_capacity = parts_[0].cap * T_;
        stats.displacement_limit = parts_[0].view().plimit;
    }

    // ---- pipelined level loop ------------------------------------------------------------------
    // No host wait inside a level. Level L is enqueued as expand_route -> ONE all-to-all of
    // fixed-capacity buckets (C records each, the sender's row in a header) -> insert_recv_lag,
    // whose last workgroup closes the level on the device and publishes every row to pinned host
    // memory. The host enqueues level L+1 BEFORE it reads level L's rows, planning L+1 from the
    // rows of level L-1 (identical on every rank, so every rank makes the same collective-size
    // decision). An under-estimated bucket, arena or table shows up as an error bit in the rows of
    // that level or the next one on every rank, and all ranks restart together in the synchronous
    // mode (`run`).
    // ---- replicated head -----------------------------------------------------------------------
    // The first levels are tiny, and partitioning them buys nothing but one all-to-all each. Every
    // rank (or, with virtual partitions, the process once) runs them as a one-GPU search on a
    // scratch visited set and a head arena (expand_fast, one host wait per level, no collective):
    // the counts of a level do not depend on the order inside it, so every rank agrees. When the
    // next frontier exceeds head_max_ states, each partition takes its owned share: the owned
    // states of every head level into its visited set, the owned states of the last level as its
    // first frontier (parent PAR_SEARCH: a path through them searches the head arena).
    void run_head(const std::vector<u64>& rev, int k, u64& unique_total) {
        Part& p0 = parts_[0];
        const u64 cap_states = head_max_ * (u64)(D_ + 4) * 2 + 4096;
        u64 hcap = std::max<u64>(1u << 12, min_table_cap(m_));
        while ((double)hcap * std::min(0.5, lmax(hcap)) < (double)cap_states) hcap <<= 1;
        const u64 hwords = table_words(make_table_view(m_, nullptr, nullptr, hcap), hcap);
        if (hkeys_.n < hwords) hkeys_.alloc(o_.device, hwords);
        if (harena_.n < cap_states * W) {
            harena_.alloc(o_.device, cap_states * W);
            hpar_.alloc(o_.device, cap_states);
        }
        SR_HIP(hipMemsetAsync(hkeys_.p, 0, hwords * 8, stream_));
        const TableView hv = make_table_view(m_, hkeys_.p, nullptr, hcap);
        hlstart_.assign(1, 0);
        SR_HIP(hipMemcpyAsync(harena_.p, rev.data(), rev.size() * 8, hipMemcpyHostToDevice, stream_));
        SR_HIP(hipMemsetAsync(hpar_.p, 0xff, (size_t)k * 4, stream_));
        init_counters(p0);
        insert_roots<M><<<blocks_for(k, 64), 64, 0, stream_>>>(m_, hv, harena_.p, (u32)k, p0.lc);
        u32 und = (1u << M::NPROPS) - 1;
        eval_roots<M><<<blocks_for(k, 64), 64, 0, stream_>>>(m_, harena_.p, (u32)k, p0.lc, und);
        p0.seq++;
        publish_kernel<<<1, 64, 0, stream_>>>(p0.lc, p0.hc_dev, p0.seq, 1, nullptr);
        SR_HIP(hipGetLastError());
        wait(p0);
        unique_total = p0.last.claims;
        u64 n = (u64)k;
        hlstart_.push_back(n);
        auto discover = [&](u32 level) {
            u32 newly = 0;
            for (int pr = 0; pr < M::NPROPS; ++pr) {
                if (!(und >> pr & 1) || p0.last.disc[pr] == ~0u) continue;
                disc_at_[pr] = DiscAt{true, level, 0, p0.last.disc[pr], true};
                disc[pr].found = true;
                disc[pr].level = level;
                disc[pr].rank = p0.last.disc[pr];
                newly |= 1u << pr;
            }
            und &= ~newly;
            return newly;
        };
        u32 newly = discover(0);
        u32 level = 0;
        for (;;) {
            if (M::NPROPS == 0 || (newly && und == 0)) {  // early exit inside the head
                reference_done = true;
                early_exit_ = true;
                head_done_ = true;
                break;
            }
            if (n > head_max_) break;  // this level is partitioned
            // expand level `level` (n states at hlstart_[level]) into the head arena
            const u64 fb = hlstart_[level], nb = fb + n;
            const u32 ncap = (u32)std::min<u64>(cap_states - nb, 0xffffffffu);
            const u32 ppw_log2 = std::max<u32>(2, std::min<u32>(6, ppw_for(n)));
            const u32 grid = std::max<u32>(1, blocks_for((n + (1u << ppw_log2) - 1) >> ppw_log2, (u32)expand_wpb<M>()));
            p0.seq++;
            expand_fast<M, 1, 0><<<grid, 64 * expand_wpb<M>(), filt_log2_ ? (8u << filt_log2_) : 0u, stream_>>>(
                m_, harena_.p + fb * W, 0u, (u32)n, hv, harena_.p + nb * W, hpar_.p + nb, ncap, p0.lc, und, p0.hc_dev, p0.seq,
                1u, ppw_log2, filt_log2_, SlotWork{});
            SR_HIP(hipGetLastError());
            wait(p0);
            if (p0.last.err) {
                head_failed_ = true;
                throw Error(SR_ERR_CAPACITY, "replicated head: scratch buffers too small");
            }
            state_count += p0.last.successors;
            stats.successors += p0.last.successors;
            stats.levels++;
            const u64 produced = p0.last.claims;
            if (produced == 0) {  // exhausted inside the head
                reference_done = true;
                head_done_ = true;
                break;
            }
            ++level;
            unique_total += produced;
            max_depth = level;
            hlstart_.push_back(nb + produced);
            head_growth_ = (double)produced / (double)n;
            head_spp_ = (double)p0.last.successors / (double)n;
            head_prev_n_ = n;
            n = produced;
            newly = discover(level);
        }
        head_undiscovered_ = und;
        unique = unique_total;
        init_counters(p0);
        if (head_done_) return;
        // ---- hand-over: level `level` (n states) is the first partitioned level ----
        lvl0_ = level;
        head_n_ = n;
        const u64 total = hlstart_[level] + n;  // head states, every level
        DBuf<u32> cnt;
        cnt.alloc(o_.device, 2);
        for (auto& p : parts_) {
            // sized from the global head (the same on every rank): a rank-local overflow here would
            // leave the other ranks waiting in the first all-to-all
            while ((double)total > std::min(part_load_, lmax(p.cap)) * (double)p.cap) grow_table(p);
            ensure_arena(p, n + n / 4 + 4096, 0);
            SR_HIP(hipMemsetAsync(cnt.p, 0, 8, stream_));
            take_owned<M><<<blocks_for(total, 256), 256, 0, stream_>>>(m_, harena_.p, (u32)total, (u32)hlstart_[level], p.id, T_,
                                                                      p.view(), p.arena.p, p.apar.p, (u32)p.arena_cap, cnt.p,
                                                                      p.lc);
            SR_HIP(hipGetLastError());
            u32 h[2];
            SR_HIP(hipMemcpyAsync(h, cnt.p, 8, hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            if (h[0] > p.arena_cap) throw Error(SR_ERR_CAPACITY, "replicated head: arena of a partition too small");
            p.n = h[0];
            p.uniq = h[1];
            p.n_hi = p.n_est = p.n;
            DistCtl c0;
            std::memset(&c0, 0, sizeof(c0));
            c0.n = h[0];
            for (int pr = 0; pr < MAX_PROPS; ++pr) c0.disc_prev[pr] = ~0u;  // evaluated in the head
            SR_HIP(hipMemcpyAsync(p.ctl, &c0, sizeof(c0), hipMemcpyHostToDevice, stream_));
        }
        SR_HIP(stream_sync(stream_));
        stats.head_levels = level;
    }

    u64 lag_S(u64 C) const { return DIST_HDR + C * REC; }

    // Growth threshold of a partition's visited set of `cap` slots: 0.75 load, lower for a
    // quotient-mode table whose probe limit would be reached sooner (kernels.hpp max_load_for).
    double lmax(u64 cap) const {
        return max_load_for(make_table_view(m_, nullptr, nullptr, cap, true).plimit, (double)cap, 0.75);
    }

    void lag_enqueue(u32 level, u64 C, u32 undiscovered, const std::vector<u64>& n_plan) {
        const u64 S = lag_S(C);
        const size_t RW = T_ + 6 + M::NPROPS;
        const u32 fseq = direct_ ? ++ctx_->dx.fseq : 0, par = fseq & 1;
        if (direct_) {
            direct_buffers(S);
        } else {
            bool sync = false;
            for (auto& p : parts_) {
                if (p.send_words < S * T_ || p.recv_words < S * T_) {
                    if (!sync) SR_HIP(stream_sync(stream_));  // in-flight levels use the old buffers
                    sync = true;
                    const u64 words = std::max<u64>(S * T_, p.send_words * 2);
                    p.send.alloc(o_.device, words);
                    p.recv.alloc(o_.device, words);
                    p.send_words = p.recv_words = words;
                }
            }
        }
        for (auto& p : parts_) {
            if (o_.profile) SR_HIP(hipEventRecord(event(2 * stats.expand_launches), stream_));
            const u32 ppw_log2 = route_ppw_env_ >= 0 ? (u32)route_ppw_env_ : ppw_for(n_plan[p.id]);
            const u32 grid = (u32)std::min<u64>(std::max<u64>(1, blocks_for(n_plan[p.id], 4u << ppw_log2)), route_grid_cap());
            u64* row = comm_ ? rows_mine_.p : rows_all_.p + (u64)p.id * RW;
            auto route = route_kernel(p);
            route<<<grid, 256, route_lds(), stream_>>>(
                m_, p.arena.p, p.apar.p, 0, p.arena_cap, p.view(), p.id, T_, direct_ ? nullptr : p.send.p + DIST_HDR,
                (u32)C, p.sendc.p, p.lc, p.ctl, undiscovered, row, ppw_log2, filt_log2_, S, 1u,
                p.sent_mask ? p.sent.p : nullptr, p.sent_mask, rstage_recs(), direct_ ? ctx_->parts[p.res].ptab[par].p : nullptr,
                dflags_ ? ctx_->dx.ftab.p : nullptr, fseq, rflags(), dcheck() ? ctx_->parts[p.res].dsum.p : nullptr,
                flush_at(ppw_log2));
            SR_HIP(hipGetLastError());
            if (o_.profile) SR_HIP(hipEventRecord(event(2 * stats.expand_launches + 1), stream_));
            stats.expand_launches++;
        }
        if (direct_) {
            // the records are in the owners' buffers already; ranks on their own streams wait for
            // every source's flag (virtual partitions share this stream: the routes ran before)
            const bool corrupt = corrupt_level_ == (i64)level && (!comm_ || comm_->rank == 0);
            if (dflags_ && (!fused_wait_ || corrupt)) {
                peer_wait<<<1, 64, 0, stream_>>>(ctx_->dx.flags.p, T_, fseq, parts_[0].lc, peer_timeout_);
                SR_HIP(hipGetLastError());
            }
            if (corrupt) {
                corrupt_level_ = -1;
                dx_corrupt<<<1, 64, 0, stream_>>>(ctx_->parts[parts_[0].res].drecv[par].p, S, (u32)C, parts_[0].id, T_);
                SR_HIP(hipGetLastError());
            }
        } else if (comm_) {
            comm_->all_to_all(parts_[0].send.p, parts_[0].recv.p, S, stream_);
        } else {
            for (auto& dst : parts_)
                for (auto& src : parts_)
                    SR_HIP(hipMemcpyAsync(dst.recv.p + (u64)src.id * S, src.send.p + (u64)dst.id * S, S * 8,
                                          hipMemcpyDeviceToDevice, stream_));
        }
        const u32 ig = insert_grid((u64)T_ * C);
        for (auto& p : parts_) {
            p.seq++;
            auto& r = ctx_->parts[p.res];
            // four records per thread on the large grid (insert_grid), one otherwise; the four as
            // parallel probe state machines (-4) unless SR_INSERT_MACHINES=0
            auto kern = ig > INSERT_GRID_MAX && W <= 2 ? (insert_machines_ ? insert_recv_lag<M, -4> : insert_recv_lag<M, 4>)
                                                         : insert_recv_lag<M, 1>;
            kern<<<ig, 256, 0, stream_>>>(m_, direct_ ? r.drecv[par].p : p.recv.p, S, (u32)C, p.id, T_, p.view(),
                                          p.arena.p, p.apar.p, p.arena_cap, p.lc, undiscovered, p.ctl,
                                          r.pub_dev[p.seq & 1], p.seq, dflags_ && fused_wait_ ? ctx_->dx.flags.p : nullptr,
                                          fseq, peer_timeout_, dcheck() ? 1u : 0u);
            SR_HIP(hipGetLastError());
        }
    }
    // The exchange check guards what crosses from one partition's kernels to another's inside
    // running kernels. With ONE partition in all (a one-rank communicator) every
    // record is its own, written and read by consecutive launches of one stream: ordered by the
    // kernel boundary, nothing to check (-0.07 ms per 2pc N=9 check, profiles/r05_rccl1_attribution.txt).
    bool dcheck() const { return direct_ && xcheck_ && T_ > 1; }
    // memory of the direct exchange's flags and receive buffers (SR_DX_FINE=0: ordinary device
    // memory, measurements only)
    static int dx_kind() {
        const char* e = std::getenv("SR_DX_FINE");
        return e && std::atoi(e) == 0 ? 0 : 1;
    }

    // Direct exchange: receive buffers of T slots of S words for both level parities, and every
    // partition's table of the owners' buffers. They grow (doubling) when a level needs larger
    // slots; every rank takes that decision at the same level (the plan is the same everywhere), and
    // first waits until no level is in flight ANYWHERE (a collective barrier: peers may still be
    // storing into the old buffers), then shares the new buffers' addresses.
    void direct_buffers(u64 S) {
        auto R = [&](Part& p) -> DistContext::PartRes& { return ctx_->parts[p.res]; };
        bool grow = false;
        for (auto& p : parts_) grow |= R(p).drecv_words < S * T_;
        if (!grow) return;
        if (comm_) comm_->barrier(stream_);
        else SR_HIP(stream_sync(stream_));
        for (auto& p : parts_) {
            const u64 words = std::max<u64>(S * T_, R(p).drecv_words * 2);
            for (int k = 0; k < 2; ++k) R(p).drecv[k].alloc(o_.device, words, dx_kind());
            R(p).drecv_words = words;
        }
        for (int k = 0; k < 2; ++k) {
            std::vector<u64*> owners(T_);
            if (comm_) {
                comm_->peer_addresses(R(parts_[0]).drecv[k].p, owners, stream_);
            } else {
                for (auto& q : parts_) owners[q.id] = R(q).drecv[k].p;
            }
            for (auto& o : owners) o += DIST_HDR;
            for (auto& p : parts_) {
                if (R(p).ptab[k].n < T_) R(p).ptab[k].alloc(o_.device, T_);
                SR_HIP(hipMemcpyAsync(R(p).ptab[k].p, owners.data(), T_ * sizeof(u64*), hipMemcpyHostToDevice, stream_));
            }
        }
        SR_HIP(stream_sync(stream_));  // the host tables may go
        direct_grows_++;
    }

    // The direct exchange's state at the start of a check (lag_loop). It is kept in the pooled
    // context across checks; a check reuses it only if EVERY rank holds it for this communicator
    // with the same flag sequence number (one small collective), and otherwise every rank sets it
    // up again: its flag words cleared before any peer may store into them (the address share is
    // collective and follows the clear on every rank), the table of this rank's word in every
    // owner's flags, and receive buffers grown (and shared) at the first level.
    void direct_setup() {
        auto& d = ctx_->dx;
        const u64 uid = comm_ ? comm_->uid : 0;
        bool reuse = d.valid && d.comm_uid == uid && d.T == T_;
        u64 gen = d.gen + 1;
        if (comm_) {
            // min over the ranks of: held, sequence number, ~sequence number, set-up generation and
            // ~generation. A rank may be handed another pooled context than last time, holding the
            // state of an OLDER set-up of this communicator (its peers' addresses stale): the
            // generation, agreed at every set-up, tells it apart even when the sequence numbers match.
            u64 v[5] = {reuse ? 1ull : 0ull, (u64)d.fseq, ~(u64)d.fseq, d.gen, ~d.gen};
            DBuf<u64> dv;
            dv.alloc(o_.device, 5);
            SR_HIP(hipMemcpyAsync(dv.p, v, sizeof(v), hipMemcpyHostToDevice, stream_));
            comm_->all_reduce(dv.p, 5, RedOp::Min, stream_);
            SR_HIP(hipMemcpyAsync(v, dv.p, sizeof(v), hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            reuse = v[0] == 1 && v[1] == ~v[2] && v[3] == ~v[4];  // everyone holds the same set-up
            gen = ~v[4] + 1;  // a new set-up's generation: past every rank's
        }
        if (trace_)
            std::fprintf(stderr, "[sr-direct] rank %d: %s (uid %llu/%llu, T %u, fseq %u, gen %llu, ctx %p)\n",
                         comm_ ? comm_->rank : 0, reuse ? "reuse" : "set up", (unsigned long long)d.comm_uid,
                         (unsigned long long)uid, d.T, d.fseq, (unsigned long long)d.gen, (void*)ctx_);
        d.fseq_start = d.fseq;
        d.reused = reuse;
        if (reuse) return;
        d.valid = false;
        for (auto& p : parts_) ctx_->parts[p.res].drecv_words = 0;  // grown and shared at level one
        d.gen = gen;
        d.comm_uid = uid;
        d.T = T_;
        d.fseq = 0;
        if (comm_) {
            d.flags.alloc(o_.device, T_, dx_kind());
            flags_clear<<<1, 64, 0, stream_>>>(d.flags.p, T_);
            SR_HIP(hipGetLastError());
            std::vector<u64*> owners;
            comm_->peer_addresses(d.flags.p, owners, stream_);
            std::vector<u32*> ft(T_);
            for (u32 q = 0; q < T_; ++q) ft[q] = reinterpret_cast<u32*>(owners[q]) + comm_->rank;
            d.ftab.alloc(o_.device, T_);
            SR_HIP(hipMemcpyAsync(d.ftab.p, ft.data(), T_ * sizeof(u32*), hipMemcpyHostToDevice, stream_));
            SR_HIP(stream_sync(stream_));
        }
        d.valid = true;
    }

    // Waits for partition p's publish of the level tagged `seq`.
    const LagPub* lag_wait(Part& p, u32 seq) {
        auto& r = ctx_->parts[p.res];
        const LagPub* pub = r.pub[seq & 1];
        volatile const u32* flag = &pub->seq;
        for (u64 spin = 1;; ++spin) {
            if (*flag == seq) break;
            if ((spin & 4095) == 0) {
                hipError_t e = hipStreamQuery(stream_);
                if (e != hipSuccess && e != hipErrorNotReady) SR_HIP(e);
                if (e == hipSuccess && *flag != seq) {
                    if (*flag == seq) break;
                    throw Error(SR_ERR_HIP, "pipelined level finished without publishing its rows");
                }
            }
            _mm_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return pub;
    }

    void lag_loop(u64& unique_total, u32& undiscovered) {
        const size_t RW = T_ + 6 + M::NPROPS;
        for (auto& p : parts_) ctx_->ensure_pub(p.res, RW * T_);
        // the exchange of this check's levels (every rank decides the same: probe_direct is collective)
        direct_ = direct_env_on() && !direct_off_ && (comm_ ? comm_->probe_direct(stream_) : T_ > 1);
        dflags_ = direct_ && comm_ != nullptr;
        fused_wait_ = dflags_ && comm_->distinct_devices() && fused_env_on();
        stats.pipelined = direct_ ? 2u : 1u;
        if (direct_) direct_setup();
        if (dcheck())
            for (auto& p : parts_) {
                auto& ds = ctx_->parts[p.res].dsum;
                if (!ds.p) ds.alloc(o_.device, (size_t)NSHARD * MAX_PARTS);
                SR_HIP(hipMemsetAsync(ds.p, 0, (size_t)NSHARD * MAX_PARTS * 8, stream_));
            }
        const u64 cmin = lag_cmin_;
        // What the plan knows, the same on every rank (LevelPlan).
        LevelPlan lp;
        lp.n_last.assign(T_, 0);
        lp.n_hi.assign(T_, 0);
        std::vector<u64>& n_last = lp.n_last;
        std::vector<u64>& n_hi = lp.n_hi;
        std::vector<u64> n_plan(T_, 0);
        u64 glob0 = 0;
        for (auto& p : parts_) glob0 += p.n;
        if (comm_) glob0 *= T_;  // level 0 (roots): a rank knows only its own share
        for (u32 q = 0; q < T_; ++q) n_last[q] = std::max<u64>(1, glob0 / T_);
        lp.growth = (double)std::min<u32>(D_, 32);  // first levels: no measurement yet
        u64 C0 = cmin;
        const bool head_start = lvl0_ > 0;
        if (head_start) {
            // the head measured the first partitioned level exactly, its growth and its successors
            // per parent: plan as if its rows had been read
            for (u32 q = 0; q < T_; ++q) {
                n_last[q] = head_n_ / T_ + 1;
                n_hi[q] = (u64)((double)n_last[q] * std::max(1.0, head_growth_) * 2.0) + 64;
            }
            lp.growth = head_growth_;
            lp.pair_ratio = head_spp_ / ((double)T_ * (double)T_);
            lp.have_rows = true;
            lp.glob_prev = head_prev_n_;  // the level before: the growth of the first rows is measured from it
            C0 = std::max<u64>(cmin, (u64)(lp.pair_ratio * (double)head_n_ * 1.3) + 256);
        }
        const bool& have_rows = lp.have_rows;
        const double& growth = lp.growth;
        for (u32 q = 0; q < T_; ++q) n_plan[q] = n_last[q];
        lag_enqueue(0, C0, undiscovered, n_plan);
        std::vector<u32> seq0(parts_.size());
        for (size_t i = 0; i < parts_.size(); ++i) seq0[i] = parts_[i].seq;  // level L: seq0 + L
        // Plan and enqueue the next level, `ahead` levels past the last rows read (1 or 2).
        u32 enq = lvl0_ + 1;  // the next level to enqueue
        u64 C = C0;
        auto plan_enqueue = [&](u32 ahead) {
            // growth of the last exact step with a margin (no floor at 1: shrinking tails shrink the
            // buckets too); it compounds once per level of look-ahead
            const double gc = std::max(1.0, growth) * 1.3;  // capacities: cheap, so generous
            for (auto& p : parts_) {
                // the frontier after the last rows (<= its upper bound), the target level's
                // frontier and the states it will claim
                const u64 hi = have_rows ? n_hi[p.id] : (u64)((double)n_last[p.id] * gc) + 64;
                const u64 c1 = std::min<u64>(hi, (u64)((double)n_last[p.id] * gc) + 64);
                const u64 fr = ahead == 2 ? (u64)((double)c1 * gc) + 1024 : c1;
                const u64 nw = (u64)((double)fr * gc) + 1024;
                const u64 before = ahead == 2 ? hi : 0;  // a frontier between the rows and the target
                const u64 want = p.uniq + before + hi + fr + nw;
                while ((double)want > grow_at(p.cap) * (double)p.cap) grow_table(p, want);
                const u64 need = p.lstart.back() + hi + (ahead == 2 ? fr : 0) + nw + 1024;
                if (p.arena_cap < need) ensure_arena(p, std::max<u64>(need + need / 4, p.arena_cap * 2), p.arena_cap);
                n_plan[p.id] = fr;
            }
            C = lp.bucket_cap(ahead, cmin);
            lag_enqueue(enq++, C, undiscovered, n_plan);
        };
        for (u32 level = lvl0_;; ++level) {
            // ---- level+1 is enqueued before the rows of `level` are read, unless it is big: then
            // its buckets are planned one level closer (one host round trip, tighter buckets) ----
            u64 glob_last = 0;
            for (u32 q = 0; q < T_; ++q) glob_last += n_last[q];
            const bool big = have_rows && (double)glob_last * growth * growth >= (double)lag_big_;
            if (enq == level + 1 && !big) plan_enqueue(have_rows && !(head_start && level == lvl0_) ? 2 : 1);

            // ---- the rows of `level` ----
            const LagPub* pub = nullptr;
            for (size_t i = 0; i < parts_.size(); ++i) {
                const LagPub* pb = lag_wait(parts_[i], seq0[i] + (level - lvl0_));
                if (i == 0) pub = pb;
            }
            rows_.assign(pub->rows, pub->rows + RW * T_);
            const std::vector<u64>& all = rows_;
            const LevelPlan::Sums sm = LevelPlan::sums(all.data(), T_, RW);
            const u64 glob_n = sm.n, glob_succ = sm.succ, glob_err = sm.err, recs = sm.recs;
            for (u32 q = 0; q < T_; ++q) {
                gl_lstart_[q].push_back(gl_off_[q]);
                gl_off_[q] += all[q * RW + T_ + ROW_N];
            }
            // A failed exchange check, a bucket over its capacity, an arena or a visited set too
            // small: the sender's (or, one level later, the receiver's) error bit is in these rows on
            // every rank, so every rank throws at the SAME level. The owner of a corrupt slot knows
            // one level earlier (its insert's own err word) but does not act on it then: its peers
            // have enqueued waits for its flags of the next level, and leaving them unanswered would
            // stall the vote until SR_PEER_TIMEOUT_MS. An exchange error wins over a
            // capacity error (a corrupt record can overflow a bucket; a capacity restart would keep
            // the direct exchange).
            throw_row_errors(glob_err, level);
            // The last level's insert has no later rows: its own check is read where the search
            // ends (the vote then makes every rank redo the check).
            auto own_exchange_check = [&] {
                u32 own_err = 0;
                for (size_t i = 0; i < parts_.size(); ++i) own_err |= ctx_->parts[parts_[i].res].pub[(seq0[i] + (level - lvl0_)) & 1]->err;
                throw_row_errors(own_err & ERR_EXCHANGE, level);
            };
            if (glob_err & ERR_PEER_TIMEOUT) {
                auto& d = ctx_->dx;
                d.valid = false;
                std::string fl;
                if (d.flags.p) {  // what this rank's flag words hold against the last sequence enqueued
                    std::vector<u32> f(T_);
                    SR_HIP(stream_sync(stream_));
                    SR_HIP(hipMemcpy(f.data(), d.flags.p, T_ * 4, hipMemcpyDeviceToHost));
                    for (u32 q = 0; q < T_; ++q) fl += (q ? "," : "") + std::to_string(f[q]);
                }
                throw Error(ERR_CODE_EXCHANGE, "direct exchange: a source's records did not arrive within SR_PEER_TIMEOUT_MS "
                                        "(level " + std::to_string(level) + ", rank " + std::to_string(comm_ ? comm_->rank : 0) +
                                        ", last sequence " + std::to_string(d.fseq) + ", flags [" + fl + "], check started at " +
                                        std::to_string(d.fseq_start) + (d.reused ? " reusing" : " after set-up") + ")");
            }
            lp.absorb(all.data(), T_, RW, sm);  // n_last, n_hi; growth and pair ratio when the level had states
            for (auto& p : parts_) {
                if (level > lvl0_) p.uniq += n_last[p.id];
                p.n = n_last[p.id];
                p.lstart.push_back(p.lstart.back() + p.n);
            }
            if (level == 0) unique_total = sm.roots;  // (a replicated head sets it instead)
            u32 newly = 0;
            for (int pr = 0; pr < M::NPROPS; ++pr) {
                if (!(undiscovered >> pr & 1)) continue;
                for (u32 q = 0; q < T_; ++q) {
                    u32 rk = (u32)all[q * RW + T_ + 6 + pr];
                    if (rk != ~0u) {
                        disc_at_[pr] = DiscAt{true, level, q, rk};
                        disc[pr].found = true;
                        disc[pr].level = level;
                        disc[pr].rank = rk;
                        newly |= 1u << pr;
                        break;
                    }
                }
            }
            undiscovered &= ~newly;
            if (trace_) {
                const double us = std::chrono::duration<double, std::micro>(Clock::now() - t_trace_).count();
                std::fprintf(stderr, "[sr-lag] level %u n=%llu succ=%llu maxpair=%llu C(next)=%llu  %.1f us since last\n",
                             level, (unsigned long long)glob_n, (unsigned long long)glob_succ,
                             (unsigned long long)sm.maxpair, (unsigned long long)C, us);
                t_trace_ = Clock::now();
            }
            stats.records_routed += recs;
            if (glob_n) {
                en_ratio_ = std::max(1.0, (double)sm.enabled / (double)glob_n);
                rec_ratio_ = (double)recs / (double)glob_n;
                lnew_ratio_ = (double)sm.local / (double)glob_n;
            }
            if (glob_n == 0) {  // frontier exhausted everywhere: `is_done` (bfs.rs:307-311)
                own_exchange_check();
                reference_done = true;
                break;
            }
            if (level > lvl0_) unique_total += glob_n;
            max_depth = level;
            unique = unique_total;
            if (M::NPROPS == 0 || (newly && undiscovered == 0)) {
                own_exchange_check();
                reference_done = true;
                early_exit_ = true;
                break;
            }
            state_count += glob_succ;
            stats.successors += glob_succ;
            stats.levels++;
            if (enq == level + 1) plan_enqueue(1);
        }
        SR_HIP(stream_sync(stream_));  // the speculative level enqueued past the end
    }

    void exchange(const std::vector<u64>& all, size_t RW) {
        // receive buffers
        for (auto& p : parts_) {
            u64 nrec = 0;
            for (u32 q = 0; q < T_; ++q) nrec += all[q * RW + p.id];
            if (p.recv_cap < nrec + 1) {
                p.recv_cap = std::max<u64>(nrec + 1, p.recv_cap * 2);
                p.recv.alloc(o_.device, p.recv_cap * REC);
            }
        }
        if (!comm_) {
            // virtual partitions: device copies, source-major order
            for (auto& dst : parts_) {
                u64 off = 0;
                for (auto& src : parts_) {
                    u64 c = all[src.id * RW + dst.id];
                    if (c) SR_HIP(hipMemcpyAsync(dst.recv.p + off * REC, src.send.p + (u64)dst.id * src.bucket_cap * REC,
                                                 c * REC * 8, hipMemcpyDeviceToDevice, stream_));
                    off += c;
                }
            }
            return;
        }
        Part& p = parts_[0];
        const int me = comm_->rank, world = comm_->world;
        std::vector<const u64*> sp(world);
        std::vector<u64*> rp(world);
        std::vector<u64> sc(world), rc(world);
        u64 off = 0;
        for (int peer = 0; peer < world; ++peer) {
            sc[peer] = all[(u64)me * RW + peer] * REC;  // words I send to peer
            rc[peer] = all[(u64)peer * RW + me] * REC;  // words peer sends to me (source-major)
            sp[peer] = p.send.p + (u64)peer * p.bucket_cap * REC;
            rp[peer] = p.recv.p + off;
            off += rc[peer];
        }
        comm_->exchange(sp, sc, rp, rc, stream_);
    }

    bool tree_path(int pr, std::vector<u64>& st) {
        if (pr < 0 || pr >= M::NPROPS || !disc_at_.size() || !disc_at_[pr].found) return false;
        SR_HIP(hipSetDevice(o_.device));
        const DiscAt d = disc_at_[pr];
        u32 level = d.level;
        // gid of the discovered state (partitioned levels) or its index in the head arena
        u64 gid = d.head ? 0 : ((u64)d.part << GID_SHIFT) | (part_lstart(d.part, d.level) + d.rank);
        bool in_head = d.head;
        u64 hidx = d.head ? hlstart_[level] + d.rank : 0;
        std::vector<u64> rev;
        DBuf<u64> buf;
        DBuf<unsigned long long> best;
        buf.alloc(o_.device, TREC);
        best.alloc(o_.device, 1);
        for (int guard = 0; guard < (1 << 20); ++guard) {
            if (in_head) {
                // the replicated head is local to every rank (no collective)
                u64 hs[W];
                u32 prank = 0;
                SR_HIP(hipMemcpy(hs, harena_.p + hidx * W, W * 8, hipMemcpyDeviceToHost));
                SR_HIP(hipMemcpy(&prank, hpar_.p + hidx, 4, hipMemcpyDeviceToHost));
                rev.insert(rev.end(), hs, hs + W);
                if (level == 0) break;
                --level;
                hidx = hlstart_[level] + prank;
                continue;
            }
            const u32 owner = (u32)(gid >> GID_SHIFT);
            const u64 idx = gid & (((u64)1 << GID_SHIFT) - 1);
            u64 rec[TREC];
            if (!comm_) {
                Part& p = parts_[owner];
                SR_HIP(hipMemcpy(buf.p, p.arena.p + idx * W, W * 8, hipMemcpyDeviceToDevice));
                SR_HIP(hipMemcpy(buf.p + W, p.apar.p + idx, 8, hipMemcpyDeviceToDevice));
                SR_HIP(hipMemcpy(rec, buf.p, TREC * 8, hipMemcpyDeviceToHost));
            } else {
                if (owner == (u32)comm_->rank) {
                    Part& p = parts_[0];
                    SR_HIP(hipMemcpyAsync(buf.p, p.arena.p + idx * W, W * 8, hipMemcpyDeviceToDevice, stream_));
                    SR_HIP(hipMemcpyAsync(buf.p + W, p.apar.p + idx, 8, hipMemcpyDeviceToDevice, stream_));
                }
                comm_->broadcast(buf.p, TREC, (int)owner, stream_);
                SR_HIP(hipMemcpyAsync(rec, buf.p, TREC * 8, hipMemcpyDeviceToHost, stream_));
                SR_HIP(stream_sync(stream_));
            }
            rev.insert(rev.end(), rec, rec + W);
            if (rec[W] == NONE) break;
            if (rec[W] == PAR_SEARCH && level == lvl0_ && lvl0_ > 0) {
                // handed over by the replicated head: a generator in the head's last level
                const u64 lo = hlstart_[level - 1], n = hlstart_[level] - lo;
                const unsigned long long init = ~0ull;
                SR_HIP(hipMemcpyAsync(best.p, &init, 8, hipMemcpyHostToDevice, stream_));
                find_pred<M><<<blocks_for(n, 256), 256, 0, stream_>>>(m_, harena_.p + lo * W, (u32)n, buf.p, best.p);
                SR_HIP(hipGetLastError());
                unsigned long long h = ~0ull;
                SR_HIP(hipMemcpyAsync(&h, best.p, 8, hipMemcpyDeviceToHost, stream_));
                SR_HIP(stream_sync(stream_));
                if (h == ~0ull) throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path` into the replicated head");
                in_head = true;
                --level;
                hidx = lo + h;
                continue;
            }
            if (rec[W] == PAR_SEARCH) {
                // inserted from a record: a generator in the previous level, the lowest gid among
                // every partition's candidates (the same on every rank)
                if (level == 0) throw Error(SR_ERR_NONDETERMINISM, "record state at level 0");
                u64 found = NONE;
                for (auto& p : parts_) {
                    const u64 lo = part_lstart(p.id, level - 1), n = part_lstart(p.id, level) - lo;
                    const unsigned long long init = ~0ull;
                    SR_HIP(hipMemcpyAsync(best.p, &init, 8, hipMemcpyHostToDevice, stream_));
                    if (n) find_pred<M><<<blocks_for(n, 256), 256, 0, stream_>>>(m_, p.arena.p + lo * W, (u32)n, buf.p, best.p);
                    SR_HIP(hipGetLastError());
                    unsigned long long h = ~0ull;
                    if (comm_) {
                        // local candidate as a gid, then the minimum over the ranks
                        DBuf<unsigned long long> g;
                        g.alloc(o_.device, 1);
                        SR_HIP(hipMemcpyAsync(&h, best.p, 8, hipMemcpyDeviceToHost, stream_));
                        SR_HIP(stream_sync(stream_));
                        unsigned long long lg = h == ~0ull ? ~0ull : (((u64)p.id << GID_SHIFT) | (lo + h));
                        SR_HIP(hipMemcpyAsync(g.p, &lg, 8, hipMemcpyHostToDevice, stream_));
                        comm_->all_reduce(reinterpret_cast<u64*>(g.p), 1, RedOp::Min, stream_);
                        SR_HIP(hipMemcpyAsync(&h, g.p, 8, hipMemcpyDeviceToHost, stream_));
                        SR_HIP(stream_sync(stream_));
                        found = std::min<u64>(found, h);
                    } else {
                        SR_HIP(hipMemcpyAsync(&h, best.p, 8, hipMemcpyDeviceToHost, stream_));
                        SR_HIP(stream_sync(stream_));
                        if (h != ~0ull) found = std::min<u64>(found, ((u64)p.id << GID_SHIFT) | (lo + h));
                    }
                }
                if (found == NONE) throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path` across partitions");
                gid = found;
            } else {
                gid = rec[W];
            }
            --level;
        }
        const size_t len = rev.size() / W;
        st.resize(rev.size());
        for (size_t i = 0; i < len; ++i) std::copy(&rev[(len - 1 - i) * W], &rev[(len - i) * W], &st[i * W]);
        return true;
    }

    // arena offset of `level` in partition `part`, as known on every rank (lstart of remote
    // partitions is rebuilt from the all-gathered frontier sizes)
    u64 part_lstart(u32 part, u32 level) { return gl_lstart_[part][level - lvl0_]; }

    M m_;
    sr_opts o_;
    Comm* comm_;
    u32 D_;
    u32 T_ = 1;
    std::vector<Part> parts_;
    hipStream_t stream_ = nullptr;
    bool pessimistic_ = false;
    bool lag_ = std::getenv("SR_DIST_SYNC") == nullptr;  // pipelined levels (synchronous on restart)
    u64 lag_cmin_ = 8192;      // minimum bucket capacity (records) of the pipelined mode
    u64 lag_big_ = std::getenv("SR_LAG_BIG") ? std::strtoull(std::getenv("SR_LAG_BIG"), nullptr, 10) : 262144;
                               // global frontier from which a level is planned after the previous one's rows
    u32 restarts_ = 0;
    u32 exchange_fallbacks_ = 0;
    bool direct_off_ = false;  // the direct exchange failed once: the collective exchange from then on
    // test hook (SR_DX_CORRUPT_LEVEL): corrupt one received slot of this level (enqueue index, first
    // partition of rank 0 only, once per engine) after its sources checksummed it
    i64 corrupt_level_ = std::getenv("SR_DX_CORRUPT_LEVEL") ? std::atoll(std::getenv("SR_DX_CORRUPT_LEVEL")) : -1;
    // the exchange check (SR_DX_CHECK=0 turns it off: measurements only)
    bool xcheck_ = !(std::getenv("SR_DX_CHECK") && std::atoi(std::getenv("SR_DX_CHECK")) == 0);
    // the outcome vote of the direct exchange (SR_DX_VOTE=0 skips it: measurements only)
    bool vote_ = !(std::getenv("SR_DX_VOTE") && std::atoi(std::getenv("SR_DX_VOTE")) == 0);
    u32 send_cache_max_parts_ = std::getenv("SR_SEND_CACHE") ? (u32)std::atoi(std::getenv("SR_SEND_CACHE")) : 4;
    // replicated head (SR_HEAD_MAX: largest head frontier; 0 disables)
    u64 head_max_ = std::getenv("SR_HEAD_MAX") ? std::strtoull(std::getenv("SR_HEAD_MAX"), nullptr, 10) : 65536;
    bool head_ok_ = true, head_failed_ = false, head_done_ = false;
    u32 lvl0_ = 0;                      // first partitioned level
    u64 head_n_ = 0, head_prev_n_ = 0;  // its global frontier size, and the head's last one
    double head_growth_ = 1.0, head_spp_ = 1.0;  // last head level: growth, successors per parent
    u32 head_undiscovered_ = (1u << M::NPROPS) - 1;
    DBuf<u64> hkeys_, harena_;          // head: scratch visited set, every head level's states
    DBuf<u32> hpar_;                    // head: parent rank in the previous head level
    std::vector<u64> hlstart_;          // head arena offset of each head level
    u64 grow_factor_ = 1;
    bool early_exit_ = false;
    bool target_stop_ = false;  // the search stopped at a target_state_count level boundary
    std::vector<DiscAt> disc_at_;
    std::vector<std::vector<u64>> gl_lstart_;  // per partition: arena offset of each level
    std::vector<u64> gl_off_;
    DBuf<u64> rows_all_, rows_mine_;  // gathered rows (T x RW) / this rank's row (RCCL mode)
    DistContext* ctx_ = nullptr;      // pooled stream, counters, pinned mirrors, events
    double en_ratio_ = 8.0;  // enabled action slots per parent, last level
    u32 filt_log2_ = std::getenv("SR_FILTER_LOG2") ? (u32)std::atoi(std::getenv("SR_FILTER_LOG2")) : (W >= 4 ? 10 : 9);

    // Parents per wave (log2) for a frontier of ~c states (the single-GPU engine's rule,
    // Engine::ppw_for): ~16 successor rounds per wave for 1-2 word states, 4 for wider ones, and
    // fewer parents per wave until ~1K waves are in flight.
    u32 ppw_for(u64 c) const {
        const double rounds = W >= 4 ? 4.0 : 16.0;
        const double ppw = 64.0 * rounds / en_ratio_;
        u32 l = 2;
        while (l < 6 && (double)(2u << l) <= ppw) ++l;
        while (l > 2 && ((c + (1u << l) - 1) >> l) < 1024) --l;
        // a chunk (4 waves) must fit the LDS record stage (one partition stages no records: the
        // clamp would force 4 parents per wave, one partly filled round each)
        if (const u32 rs = rstage_recs())
            while (l > 2 && 4.0 * (double)(1u << l) * rec_ratio_ * 1.3 > (double)rs) --l;
        // ... and, with an owner key, its local new states the local stage
        if (okey_)
            while (l > 2 && 4.0 * (double)(1u << l) * lnew_ratio_ * 1.3 > (double)route_local_stage(T_, W, rflags())) --l;
        return l;
    }
    // expand_route's flush thresholds for parents per wave 2^l: a stage is flushed once its fill
    // exceeds its size minus a chunk's bound (the bound ppw_for sized the chunk by)
    u32 flush_at(u32 l) const {
        const double chunk = 4.0 * (double)(1u << l) * 1.3;
        const double rs = (double)rstage_recs(), ls = (double)route_local_stage(T_, W, rflags());
        const u32 fr = (u32)std::max(0.0, rs - chunk * rec_ratio_), fl = (u32)std::max(0.0, ls - chunk * lnew_ratio_);
        return std::min<u32>(fl, 0xffffu) << 16 | std::min<u32>(fr, 0xffffu);
    }
    double rec_ratio_ = 4.0;   // remote records per parent, last level
    double lnew_ratio_ = 2.0;  // new states claimed in place per parent, last level
    // Records staged per chunk in LDS (none with one partition), and expand_route's dynamic LDS.
    u32 rstage_recs() const { return T_ > 1 ? rstage_words() / REC : 0u; }
    // expand_route turns local successors into records to itself from this many partitions on
    // (SR_SELF_RECORDS_MIN; 0 = never): its rounds then wait on no visited-set probe
    // (not with an owner key: most successors are then local, and probing them in place is cheaper)
    u32 self_rec() const { return !okey_ && self_rec_min_ && T_ >= self_rec_min_ ? 1u : 0u; }
    // The route kernel's form: self records (no probes), or probes of the local successors in
    // rounds, or in per-lane queues (expand_fast's probe_loop rule: fingerprint-mode narrow states,
    // a partition table of >= 2^27 slots, and here no sent cache). SR_ROUTE_QUEUE=0/1 forces it.
    using RouteKernel = decltype(&expand_route<M, 1, false>);
    RouteKernel route_kernel(const Part& p) const {
        if (self_rec()) return expand_route<M, 1, true>;
        constexpr bool queue_ok = W == 1 || !has_qkey<M>::value;  // not multi-word quotient tables
        if constexpr (queue_ok && W < 4) {
            const bool big = p.view().mask + 1 >= (1ull << 27);
            if (!p.sent_mask && (route_queue_env_ < 0 ? big : route_queue_env_ > 0)) return expand_route<M, -4, false>;
        }
        return expand_route<M, 1, false>;
    }
    bool insert_machines_ = !(std::getenv("SR_INSERT_MACHINES") && std::atoi(std::getenv("SR_INSERT_MACHINES")) == 0);
    int route_queue_env_ = std::getenv("SR_ROUTE_QUEUE") ? std::atoi(std::getenv("SR_ROUTE_QUEUE")) : -1;
    u32 rflags() const {
        // SR_LSTAGE_WORDS: the local stage's size; with an owner key 512 words for narrow states (more
        // blocks per CU: config 4 at T = 8 13.4 -> 12.6 ms per rank, T = 4 29.6 -> 24.6 ms,
        // profiles/r06_config4_stages.txt)
        const u32 lw = lstage_words_ ? lstage_words_ : okey_ && W <= 2 ? 512u : 0u;
        const u32 ls = lw ? lw / W : 0u;
        return self_rec() | (okey_ ? (u32)RF_LOCAL : 0u) | (ordered_flush() ? (u32)RF_ORDERED : 0u) | ls << RF_LSTAGE_SHIFT;
    }
    // The owner-ordered record flush when the owners are other devices (RF_ORDERED; SR_ORDERED_FLUSH
    // = 0 / 1 forces it off / on, e.g. to test it on one device).
    bool ordered_flush() const {
        if (ordered_env_ >= 0) return ordered_env_ > 0;
        return comm_ && comm_->world > 1 && comm_->distinct_devices();
    }
    int ordered_env_ = std::getenv("SR_ORDERED_FLUSH") ? std::atoi(std::getenv("SR_ORDERED_FLUSH")) : -1;
    u32 lstage_words_ = std::getenv("SR_LSTAGE_WORDS") ? (u32)std::atoi(std::getenv("SR_LSTAGE_WORDS")) : 0u;
    // planned load of a partition's visited set at its share of the hint (SR_PART_LOAD): 0.3, like the
    // one-GPU table (config 4 at T = 8: 12.58 -> 11.65 ms per rank, T = 4: 21.3 -> 19.7;
    // profiles/r06_table_load.txt)
    double part_load_ = std::getenv("SR_PART_LOAD") ? std::atof(std::getenv("SR_PART_LOAD")) : 0.3;
    const bool okey_ = uses_owner_key(m_);  // states owned by the model's owner key (kernels_dist.hpp part_of)
    u32 self_rec_min_ = std::getenv("SR_SELF_RECORDS_MIN") ? (u32)std::atoi(std::getenv("SR_SELF_RECORDS_MIN")) : 5u;
    size_t route_lds() const {
        const size_t rs = rstage_recs();
        return (filt_log2_ ? (8u << filt_log2_) : 0u) + rs * (REC * 8 + 2) + ((rs + 1) & ~(size_t)1) +
               (ordered_flush() ? rs * 2 : 0) + (size_t)route_local_stage(T_, W, rflags()) * (W * 8 + 4);
    }
    // expand_route's grid: two device residencies at its LDS footprint (expand_fast's rule); the
    // kernel strides over further parents. SR_ROUTE_GRID_MAX > 0 overrides it.
    u32 route_grid_cap() {
        if (route_grid_max_) return route_grid_max_;
        if (const char* e = std::getenv("SR_ROUTE_GRID_MAX"))
            if (std::atoi(e) > 0) return route_grid_max_ = (u32)std::atoi(e);
        int per_cu = 0, cus = 0;
        const void* k = self_rec() ? (const void*)expand_route<M, 1, true> : (const void*)expand_route<M, 1, false>;
        SR_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, route_lds()));
        SR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, o_.device));
        route_grid_max_ = per_cu > 0 && cus > 0 ? (u32)(2 * per_cu * cus) : 8192u;
        return route_grid_max_;
    }
    u32 route_grid_max_ = 0;
    // insert kernels: workgroups at most (each reserves frontier space with a same-line atomic,
    // ~11 ns apiece; 512 x 256 threads keep enough probes in flight)
    static constexpr u32 INSERT_GRID_MAX = 512;
    // The insert grid for up to `recs` records: at most INSERT_GRID_MAX workgroups (each one's
    // final flush is a same-line claims atomic, so inserts of a few million records keep few of
    // them: 2pc N=9 at T = 2 / 8 is 15% / 6% slower on more), and for inserts of more than 8 M
    // records up to insert_grid_big_ workgroups with four records per thread (insert_records
    // batches the probes): 2pc N=11 at T = 8 inserts in 59.5
    // instead of 76.6 ms per check (profiles/r02_insert_ab.txt).
    u32 insert_grid(u64 recs) const {
        const u64 small = std::max<u64>(1, blocks_for(recs, 256));
        if (recs <= insert_batch_min_) return (u32)std::min<u64>(small, INSERT_GRID_MAX);
        return (u32)std::min<u64>(insert_grid_big_, std::max<u64>(INSERT_GRID_MAX, blocks_for(recs, 1024)));
    }
    // planned records above which the batched insert runs (SR_INSERT_BATCH_MIN; tests force it low)
    u64 insert_batch_min_ = std::getenv("SR_INSERT_BATCH_MIN") ? std::strtoull(std::getenv("SR_INSERT_BATCH_MIN"), nullptr, 10)
                                                               : (8ull << 20);
    u32 insert_grid_big_ = std::getenv("SR_INSERT_GRID") && std::atoi(std::getenv("SR_INSERT_GRID")) > 0
                               ? (u32)std::atoi(std::getenv("SR_INSERT_GRID")) : 4096u;
    // record stage of expand_route (words): twice as large with self records (no local stage, and a
    // chunk of 4 x 32 parents then fits: 2pc N=11 at T = 8 routes in 41 instead of 69 ms per check)
    // (0 = that default; SR_RSTAGE_WORDS overrides)
    u32 rstage_words_ = std::getenv("SR_RSTAGE_WORDS") ? (u32)std::atoi(std::getenv("SR_RSTAGE_WORDS")) : 0u;
    u32 rstage_words() const { return rstage_words_ ? rstage_words_ : self_rec() ? 2048u : okey_ && W <= 2 ? 512u : 1024u; }
    int route_ppw_env_ = std::getenv("SR_ROUTE_PPW_LOG2") ? std::atoi(std::getenv("SR_ROUTE_PPW_LOG2")) : -1;
    bool trace_ = std::getenv("SR_DIST_TRACE") != nullptr;
    Clock::time_point t_trace_ = Clock::now();
    u64 arena_grows_ = 0;
    // direct exchange (lag_loop): on for this check, with device flags (comm ranks); buffer growths
    // (the flags, buffers and tables live in the pooled context: DistContext::Direct)
    bool direct_ = false, dflags_ = false;
    bool fused_wait_ = false;  // the insert grid polls the flags itself (ranks on distinct devices)
    static bool fused_env_on() {
        const char* e = std::getenv("SR_FUSED_WAIT");
        return !(e && std::atoi(e) == 0);
    }
    u64 peer_timeout_ = peer_timeout_ticks();
    u64 direct_grows_ = 0;
    std::vector<u64> rows_;
    std::vector<std::vector<u64>> paths_;  // per property: the discovery path's states (gather_paths)
    bool paths_ready_ = false;
};

}  // namespace sr
