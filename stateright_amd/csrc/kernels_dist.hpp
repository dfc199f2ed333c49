// Kernels of the PARTITIONED search: the visited set and the frontier are split
// into T partitions by fingerprint owner, one partition per GPU (RCCL all-to-all over xGMI each
// level) or T virtual partitions on one GPU (device-copy exchange; used to test the protocol on a
// single device).
//
// Per level and partition:
//   expand_route  expands the local frontier; a successor owned by this partition is inserted
//                 directly (probe / CAS claim / append), one owned elsewhere becomes a record
//                 {state[W], parent gid} in the send bucket of its owner (LDS-staged per owner,
//                 one global atomic per (workgroup, owner));
//   insert_recv   inserts the records received from every partition.
// A parent gid is (partition << 40) | arena index: the BFS tree spans partitions. A record carries
// the state only (8 B for one-word states): the xGMI link is the scarce resource at small T. A
// state inserted from a record gets the parent PAR_SEARCH, and a discovery path that reaches it
// finds a parent in the previous level with find_pred (any generator is a valid FAST-order parent).
#pragma once
#include "kernels.hpp"

namespace sr {

constexpr int GID_SHIFT = 40;
// expand_route's per-owner record counters, one 128-byte line each (u32 stride): every workgroup
// reserves its span of each owner's slot with a returning atomic, and atomics to one line
// serialise at ~11 ns apiece whatever the addresses inside it (kernels.hpp LevelCounters).
constexpr u32 SENDC_STRIDE = 32;
constexpr u64 PAR_SEARCH = ~0ull - 1;  // parent not recorded: search the previous level

// Owner partition of a fingerprint: the high 32 bits scaled to [0, T) (any T, uniform).
__device__ __host__ __forceinline__ u32 owner_of(u64 fp, u32 nparts) { return (u32)(((fp >> 32) * (u64)nparts) >> 32); }
// Owner partition of an owner key (a model's projection of the state): a multiplicative hash of the
// key's 32-bit halves, scaled to [0, T). Round 6: against fmix64 of the key (SR_OKEY_HASH=0, a
// build-time variant) it balances config 4's partitions better (max/mean 1.09 -> 1.03 at T = 8)
// and costs fewer instructions per successor: critical path per rank T = 8 11.68 -> 10.83 ms,
// T = 4 19.78 -> 18.66 (profiles/r06_config4_stages.txt).
#ifndef SR_OKEY_HASH
#define SR_OKEY_HASH 1
#endif
__device__ __host__ __forceinline__ u32 key_owner(u64 key, u32 nparts) {
#if SR_OKEY_HASH
    const u32 h = (u32)key * 0x9E3779B1u ^ (u32)(key >> 32) * 0x85EBCA77u;
    return (u32)(((u64)h * nparts) >> 32);
#else
    return owner_of(fmix64(key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull), nparts);
#endif
}
// Owner partition of state s (fingerprint fp): by the model's owner key when it has one
// (models.hpp has_owner_key; mixed, then scaled like a fingerprint), else by the fingerprint.
template <class M>
__device__ __host__ __forceinline__ u32 part_of(const M& m, const u64* s, u64 fp, u32 nparts) {
    if constexpr (has_owner_key<M>::value) {
        u64 key;
        if (m.owner_key(s, &key)) return key_owner(key, nparts);
    }
    return owner_of(fp, nparts);
}
// The route kernel's key of a successor for the LDS filter and the sent cache, and its owner. The
// key must be injective wherever those are on: the fingerprint in fingerprint mode (the slot value),
// the permuted key + 1 for one-word quotient tables (filter_key: no second hash per successor), the
// fingerprint for multi-word quotient tables (their filter and sent cache are off; it serves the
// owner only). The owner is part_of's, with the fingerprint computed only when it is needed (no
// owner key) and the key is not already it.
template <class M>
__device__ __forceinline__ u64 route_key(const M&, const TableView& t, const ProbeKey& pk, const u64* s) {
    if (!t.qbits) return pk.tag;
    if (M::W == 1) return filter_key(t, pk);
    return state_fp<M>(s);
}
template <class M>
__device__ __forceinline__ u32 route_owner(const M& m, const TableView& t, const u64* s, u64 key, u32 nparts) {
    if constexpr (has_owner_key<M>::value) {
        u64 k;
        if (m.owner_key(s, &k)) return key_owner(k, nparts);
    }
    return owner_of(t.qbits && M::W == 1 ? state_fp<M>(s) : key, nparts);
}
template <class M>
inline bool uses_owner_key(const M& m) {
    if constexpr (has_owner_key<M>::value) {
        u64 s[M::W] = {}, key;
        return m.owner_key(s, &key);
    }
    return false;
}

// Device-side control block of one partition: the size of the frontier being expanded and the
// discovery ranks among it. The last workgroup of insert_recv writes it for the next level, so the
// host can enqueue the next expand_route before it knows the frontier size (one host
// synchronisation per level: the all-gathered rows).
struct DistCtl {
    u32 n;
    u32 roots;                   // distinct init states claimed here (level 0 only)
    u64 nb;                      // arena offset of that frontier (pipelined mode: kept on the device)
    u32 pad0[28];
    u32 disc_prev[MAX_PROPS];
};

// Pipelined mode: every send bucket starts with a header of HDR words holding the sender's row, so
// the all-to-all also delivers every partition's row to every rank (no separate all-gather, no
// host wait inside a level). Bucket q of a sender = [HDR words: row][C records].
constexpr u32 DIST_HDR = 128;
// Direct exchange: the last two header words of a slot are the level's flag sequence number and a
// checksum: the wrapping sum of every record word the source stored into that slot plus every row
// word of the header. The owner's insert recomputes both (ERR_EXCHANGE on a mismatch), so a slot
// read with a stale cached line, a late or a lost store cannot turn into a silently wrong count:
// the sequence tag shares a line with the checksum, and the checksum covers every other line.
constexpr u32 HDR_SEQ = DIST_HDR - 2, HDR_SUM = DIST_HDR - 1;
static_assert(MAX_PARTS + 6 + MAX_PROPS <= (int)HDR_SEQ, "the row fits the header before its tag");

// Row published by the last workgroup of expand_route (u64 words; RW = T + 6 + NPROPS):
//   [0, T)  records routed to each partition      T     frontier size n
//   T+1     successors within boundary             T+2   local claims (new states inserted here)
//   T+3     error bits    T+4 enabled slots        T+5   distinct roots (level 0)
//   T+6+p discovery rank of property p in the frontier
template <int NP>
__device__ __forceinline__ bool last_workgroup(LevelCounters* lc) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x != 0) return false;
#if SR_TICKET_FENCE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
    if (!take_ticket(lc)) return false;
#if SR_TICKET_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    return true;
}

// Pipelined mode: the last workgroup of a launch, told to every thread of that workgroup.
// `sysrel`: the workgroup's stores went (also) to another device's memory (direct exchange), so
// they are released at system scope before the ticket, and the last workgroup acquires them.
// `sysacq`: the last workgroup acquires at system scope whatever its own stores were (it then
// raises flags that publish every workgroup's remote stores).
__device__ __forceinline__ bool last_block(LevelCounters* lc, bool sysrel = false, bool sysacq = false) {
    __shared__ u32 is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (sysrel) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        is_last = take_ticket(lc);
        if ((sysrel || sysacq) && is_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    return is_last != 0;
}

// Direct exchange: the records of a level are stored by the SOURCE's expand_route
// straight into slot `source` of every owner's receive buffer (a peer pointer: the same device, a
// peer device in this process, or another process's memory through IPC), and its last workgroup
// then stores the level's flag sequence number into every owner's flag word for that source. The
// owner waits for every source's flag with this one-wave kernel before its insert (a spinning
// insert grid could starve the sources' expand grids of the same device), then acquires at system
// scope. A flag is a monotonic sequence number, so a source that is already a level ahead also
// satisfies the wait (its next level writes the other buffer parity). Bounded: after `timeout`
// ticks of the 100 MHz real-time counter the wait gives up and sets ERR_PEER_TIMEOUT, which
// reaches every rank through the next level's rows.
template <int = 0> __global__ void peer_wait(const u32* flags, u32 nparts, u32 seq, LevelCounters* lc, u64 timeout) {
    const u32 q = threadIdx.x;
    bool ok = q >= nparts;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    while (!ok) {
        const u32 v = __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int)(v - seq) >= 0) {
            ok = true;
            break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) atomicOr(&lc->err, (u32)ERR_PEER_TIMEOUT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// Local new states expand_route stages per chunk (states of W words): a partition keeps ~1/T of its
// new states (a growth level of 2pc makes ~3 per parent, 768 per 256-parent chunk), so the stage
// shrinks with T and leaves its LDS to the record stage: LDS per block sets residency, and the
// probes of this kernel are latency-bound.
// With self records (below) nothing is inserted locally: no stage. With an owner key most new
// states are local: the stage of one partition.
// rflags: RF_SELF (self records), RF_LOCAL (owner key: most successors stay local), and from bit 8
// on the local stage's size in states when the host sets one (RF_LSTAGE_SHIFT; 0 = this default).
// RF_ORDERED: the record flush writes each owner's records as one contiguous run from consecutive
// threads (owner-ordered): taken when the owners are other devices (stores over
// xGMI into fine-grained peer memory); same-device owners keep the stage-order flush.
enum RouteFlags : u32 { RF_SELF = 1, RF_LOCAL = 2, RF_ORDERED = 4, RF_LSTAGE_SHIFT = 8 };
__host__ __device__ __forceinline__ u32 route_local_stage(u32 nparts, int W, u32 rflags) {
    if (rflags & RF_SELF) return 0u;
    if (rflags >> RF_LSTAGE_SHIFT) return rflags >> RF_LSTAGE_SHIFT;
    return (nparts <= 1 || (rflags & RF_LOCAL) ? 1024u : nparts == 2 ? 512u : 256u) / (u32)W;
}

// Expands the frontier of this partition (its size n is read from ctl). Same structure as
// expand_fast (kernels.hpp): waves of ppw parents, successors load-balanced over the lanes, PB
// successors per lane per round with their probes issued back to back, and the block-local LDS
// duplicate filter. A successor owned by another partition becomes a record {state[W], parent
// gid} for that owner's send bucket.
//
// The launch is grid-strided over chunks of 4 waves x ppw parents (sized on the host from an upper
// bound of n, and ppw so that a chunk's records fit the LDS stages). New local states and remote
// records are staged in LDS per chunk, then flushed by the whole block: a block-local counting
// sort by owner and ONE global atomic per (chunk, owner) reserves each owner's span. The global
// bucket counters are the only same-address atomics, so they must be rare: per-successor or
// per-wave reservations serialise at the L2 when every wave of the GPU targets T addresses.
// A stage that overflows (a chunk larger than planned) falls back to per-wave reservations.
// Six waves per SIMD (<= 80 VGPRs) for narrow states: the kernel waits on memory, and at its
// natural 83 VGPRs it ran five (2pc N=11 at T = 8 with an owner key, where it probes most
// successors in place). Wide states (paxos) are bound by their LDS stages instead.
template <class M, int PB, bool SELF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(M::W <= 2 ? 6 : 1))) expand_route(M m, u64* __restrict__ arena, u64* __restrict__ apar, u64 nb,
                                                    u64 arena_cap, TableView t, u32 my_part, u32 nparts,
                                                    u64* __restrict__ send, u32 bucket_cap, u32* send_counts,
                                                    LevelCounters* lc, DistCtl* ctl, u32 undiscovered, u64* row,
                                                    u32 ppw_log2, u32 filt_log2, u64 bucket_stride, u32 lag,
                                                    u64* __restrict__ sent, u64 sent_mask, u32 rs,
                                                    u64* const* ptab, u32* const* ftab, u32 fseq, u32 rflags,
                                                    u64* dsum, u32 flush_at) {
    // dsum (direct exchange): [NSHARD][MAX_PARTS] per-owner sums of the record words this launch
    // stores, accumulated per chunk flush into shard blockIdx % NSHARD (non-returning atomics, spread
    // like the statistics); the last workgroup folds them into each owner's slot checksum (HDR_SUM).
    // self_rec: successors owned by this partition become records too (to its own slot), so this
    // kernel probes nothing and has no global round trip per round of successors: with many
    // partitions 1/T of the lanes probed and the whole wave waited for them. The insert kernel
    // then probes every successor, with its batched probes. SELF = the same, fixed at compile time:
    // the instantiation for self records has no probe, claim, local stage or sent-cache code at all
    // (the kernel is instruction-bound there: profiles/r03_pmc_instruction_mix.txt).
    u32 self_rec = rflags & RF_SELF;
    if constexpr (SELF) {
        self_rec = 1;
        sent = nullptr;
    }
    // Destinations. Exchanged buckets (ptab == nullptr): owner q's records go to this partition's
    // own send bucket q, send + q * bucket_stride. Direct exchange: straight into slot my_part of
    // owner q's receive buffer, ptab[q] + my_part * bucket_stride (both past the header; the row
    // goes into the HDR words before it), and with ftab the level's flag to every owner at the end.
    constexpr int W = M::W, MW = M::MW, REC = W;
    __shared__ u64* sdst[MAX_PARTS];
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x)
        sdst[q] = ptab ? ptab[q] + (u64)my_part * bucket_stride : send + (u64)q * bucket_stride;
    // Dynamic LDS: [filter: 2^filt_log2 fingerprints][record stage: rs x REC words][local stage:
    // ls x W words][its parents' frontier ranks: ls u32][record ranks: rs u16][record owners: rs u8]
    // and, with RF_ORDERED, [the records in owner order: rs u16].
    // rs (records staged per chunk, all owners) is chosen on the host: 0 with one partition, so the
    // one-partition launch keeps expand_fast's occupancy; ls = route_local_stage(nparts).
    extern __shared__ u64 dyn[];
    const u32 RSTAGE = rs, STAGE = route_local_stage(nparts, W, SELF ? (u32)RF_SELF : rflags);
    u64* filt = dyn;
    u64* rstage = dyn + (filt_log2 ? (1u << filt_log2) : 0u);
    u64* stage = rstage + (u64)rs * REC;
    u32* stage_par = reinterpret_cast<u32*>(stage + (u64)STAGE * W);  // the gid is formed at flush
    u16* rrank = reinterpret_cast<u16*>(stage_par + STAGE);
    u8* rown = reinterpret_cast<u8*>(rrank + rs);
    u16* rperm = reinterpret_cast<u16*>(rown + ((rs + 1) & ~1u));  // RF_ORDERED only
    const bool ordered = (rflags & RF_ORDERED) != 0;
    __shared__ u32 ocnt[MAX_PARTS], obase[MAX_PARTS], lbase[MAX_PARTS + 1];
    __shared__ u64 ocsum[MAX_PARTS];  // the chunk's record-word sum per owner (dsum)
    __shared__ u64 pst[4][64 * W];
    // the wave's successor list, (parent, action) per successor (see expand_fast), in windows
    constexpr u32 MAPCAP = 512;
    static_assert(MW * 64 <= 1024, "action ids must fit 10 bits");
    __shared__ u16 smap[4][MAPCAP];
    __shared__ u32 stage_n, rstage_n, base, scratch[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const u64 lanes_below = (1ull << lane) - 1;
    const u64 n = ctl->n;                   // written by the previous level's insert_recv
    if (lag) nb = ctl->nb;                  // pipelined: the arena offset is tracked on the device
    const u64* frontier = arena + nb * W;
    u64* next = arena + (nb + n) * W;
    u64* next_par = apar + nb + n;
    const u32 next_cap = (u32)min<u64>(arena_cap > nb + n ? arena_cap - nb - n : 0, 0xffffffffull);
    const u64 gid_base = ((u64)my_part << GID_SHIFT) + nb;
    const u32 ppw = 1u << ppw_log2;
    const u32 fmask = filt_log2 ? (1u << filt_log2) - 1 : 0;
    __shared__ u32 sent_any;  // this workgroup stored records (direct exchange: release them)
    if (threadIdx.x == 0) stage_n = rstage_n = sent_any = 0;
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) ocnt[q] = 0, ocsum[q] = 0;
    for (u32 i = threadIdx.x; i < (fmask ? fmask + 1 : 0u); i += blockDim.x) filt[i] = 0;
    u64* const my_dsum = dsum ? dsum + (u64)(blockIdx.x % NSHARD) * MAX_PARTS : nullptr;

    // Block flush of the stages (every thread; fl / fr uniform): local new states get ONE claims
    // reservation, records are counting-sorted by owner and get one reservation per owner.
    auto flush = [&](bool fl, bool fr) {
        const u32 nl = fl ? min(stage_n, (u32)STAGE) : 0u;
        const u32 nr = fr ? min(rstage_n, RSTAGE) : 0u;
        if (nr && threadIdx.x == 0) sent_any = 1;
        for (u32 i = threadIdx.x; i < nr; i += blockDim.x) {
            rrank[i] = (u16)atomicAdd(&ocnt[rown[i]], 1u);
            if (my_dsum) {
                u64 v = 0;
#pragma unroll
                for (int x = 0; x < REC; ++x) v += rstage[i * REC + x];
                atomicAdd(reinterpret_cast<unsigned long long*>(&ocsum[rown[i]]), (unsigned long long)v);
            }
        }
        if (threadIdx.x == 0 && nl) base = atomicAdd(&lc->claims, nl);
        __syncthreads();
        if (threadIdx.x == 0) {
            if (fl) stage_n = 0;
            if (fr) rstage_n = 0;
        }
        if (nr && ordered && threadIdx.x < 64) {  // the owners' runs in the chunk: exclusive prefix
            const u32 c = threadIdx.x < nparts ? ocnt[threadIdx.x] : 0u;
            u32 incl = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const u32 y = __shfl_up(incl, d, 64);
                if ((int)threadIdx.x >= d) incl += y;
            }
            if (threadIdx.x < nparts) lbase[threadIdx.x] = incl - c;
        }
        if (nr)
            for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) {
                const u32 c = ocnt[q];
                obase[q] = c ? atomicAdd(&send_counts[q * SENDC_STRIDE], c) : 0;
                ocnt[q] = 0;
                if (my_dsum && c) {
                    atomicAdd(reinterpret_cast<unsigned long long*>(&my_dsum[q]), (unsigned long long)ocsum[q]);
                    ocsum[q] = 0;
                }
            }
        if (nr && ordered) {
            __syncthreads();  // lbase
            for (u32 i = threadIdx.x; i < nr; i += blockDim.x) rperm[lbase[rown[i]] + rrank[i]] = (u16)i;
        }
        for (u32 i = threadIdx.x; i < nl; i += blockDim.x) {
            const u32 pos = base + i;
            u64 ns[W];
#pragma unroll
            for (int x = 0; x < W; ++x) ns[x] = stage[i * W + x];
            if (pos < next_cap) {
                store_state<W>(next, pos, ns);
                next_par[pos] = gid_base + stage_par[i];
            } else {
                atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
            }
            eval_props(m, ns, pos, undiscovered, lc);
        }
        __syncthreads();
        for (u32 i = threadIdx.x; i < nr * REC; i += blockDim.x) {
            // ordered: thread i takes word x of the k-th record in owner order, so consecutive
            // threads store consecutive words of one owner's run; else the k-th staged record
            const u32 k = i / REC, x = i - k * REC;
            const u32 rr = ordered ? rperm[k] : k;
            const u32 q = rown[rr];
            const u32 pos = obase[q] + rrank[rr];
            if (pos < bucket_cap) sdst[q][(u64)pos * REC + x] = rstage[rr * REC + x];
            else if (x == 0) atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
        __syncthreads();  // the stages are read before any later append
    };

    u32 succ = 0, enabled = 0;
    const u64 chunk = (u64)(blockDim.x >> 6) * ppw;
    const u64 cstride = (u64)gridDim.x * chunk;
    u64 nxt[W];  // the wave's parents of the next chunk, loaded one chunk ahead
    if (lane < (int)ppw && (u64)blockIdx.x * chunk + (u64)wid * ppw + lane < n)
        load_state<W>(frontier, (u64)blockIdx.x * chunk + (u64)wid * ppw + lane, nxt);
    for (u64 c0 = (u64)blockIdx.x * chunk; c0 < n; c0 += cstride) {
        const u64 wave0 = c0 + (u64)wid * ppw;  // first parent of the wave
        const u64 r = wave0 + lane;
        u32 cnt = 0;
        u64 s[W], mk[MW];
#pragma unroll
        for (int i = 0; i < W; ++i) s[i] = nxt[i];
#pragma unroll
        for (int i = 0; i < MW; ++i) mk[i] = 0;
        if (lane < (int)ppw && r + cstride < n) load_state<W>(frontier, r + cstride, nxt);
        __syncthreads();  // the previous chunk's parents and stages are no longer read
        if (lane < (int)ppw && r < n) {
            m.enabled(s, mk);
            if constexpr (has_self_loops<M>::value) {  // counted, never generated
                u64 sl[MW];
                m.self_loops(s, mk, sl);
#pragma unroll
                for (int i = 0; i < MW; ++i) {
                    succ += __popcll(sl[i]);
                    mk[i] &= ~sl[i];
                }
            }
#pragma unroll
            for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = s[i];
#pragma unroll
            for (int i = 0; i < MW; ++i) cnt += __popcll(mk[i]);
        }
        const u32 incl = wave_incl_scan(cnt);
        u32 nidx = incl - cnt;
        const u32 total = lane_u32(incl, 63);
        if (lane == 0) enabled += total;

        for (u32 w0 = 0; w0 < total; w0 += MAPCAP) {
        const u32 wend = min(total, w0 + MAPCAP);
        while (nidx < wend && nidx < incl) {
            u32 a = 0;
#pragma unroll
            for (int w = MW - 1; w >= 0; --w)
                if (mk[w]) a = (u32)w * 64 + (u32)__builtin_ctzll(mk[w]);
            mk[a >> 6] &= mk[a >> 6] - 1;
            smap[wid][nidx - w0] = (u16)((u32)lane | a << 6);
            ++nidx;
        }
        wave_lds_sync();  // pst and the map are the wave's own

        if constexpr (PB < 0) {
            // Per-lane probe queues (expand_fast's, kernels.hpp; the host takes this form for big
            // fingerprint-mode tables without a sent cache): R rounds expanded with every lane
            // busy, remote successors staged as records at once, the local ones' keys kept in
            // registers and probed one visited-set access per lane and iteration.
            static_assert(!SELF, "self records probe nothing");
            constexpr int R = -PB;
            constexpr bool FP_ONLY = !has_qkey<M>::value;
            for (u32 s0 = w0; s0 < wend; s0 += 64u * R) {
                u64 kh[FP_ONLY ? 1 : R], kt[R];
                u32 vmask = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (!FP_ONLY) kh[FP_ONLY ? 0 : r] = 0;
                    kt[r] = 0;
                    const u32 i = s0 + (u32)r * 64u + (u32)lane;
                    u64 q[W];
                    bool ok = false, rem = false;
                    u32 own = my_part;
                    if (i < wend) {
                        const u32 e = smap[wid][i - w0];
                        const u32 p = e & 63, a = e >> 6;
                        u64 ps[W];
#pragma unroll
                        for (int x = 0; x < W; ++x) ps[x] = pst[wid][p * W + x];
                        ok = m.apply(ps, (int)a, q);
                        if (ok) {
                            ++succ;
                            ok = !same_state<W>(q, ps);  // self-loop: counted, never routed
                        }
                        if (ok) {
                            const ProbeKey pk = probe_key(m, t, q);
                            const u64 key = route_key(m, t, pk, q);
                            if (fmask) {  // block-local duplicate filter (see expand_fast)
                                const u64 old = atomicExch(reinterpret_cast<unsigned long long*>(&filt[filter_index(t, key) & fmask]),
                                                           (unsigned long long)key);
                                ok = old != key;
                            }
                            if (ok) {
                                own = route_owner(m, t, q, key, nparts);
                                rem = self_rec || own != my_part;
                                if (!rem) {
                                    vmask |= 1u << r;
                                    kt[r] = pk.tag;
                                    if (!FP_ONLY) kh[FP_ONLY ? 0 : r] = pk.home;
                                }
                            }
                        }
                    }
                    // remote records -> the chunk's record stage (one LDS atomic per wave)
                    const u64 rmask = __ballot(rem);
                    if (!rmask) continue;
                    const u32 rcnt = __popcll(rmask);
                    const u32 rbelow = __popcll(rmask & lanes_below);
                    const int rleader = __builtin_ctzll(rmask);
                    u32 rsb = 0;
                    if (lane == rleader) rsb = atomicAdd(&rstage_n, rcnt);
                    rsb = lane_u32(rsb, (u32)rleader);
                    const u32 rin = rsb >= RSTAGE ? 0u : min(rcnt, RSTAGE - rsb);
                    if (rem && rbelow < rin) {
                        const u32 kk = rsb + rbelow;
#pragma unroll
                        for (int x = 0; x < W; ++x) rstage[kk * REC + x] = q[x];
                        rown[kk] = (u8)own;
                    }
                    u64 om = __ballot(rem && rbelow >= rin);  // overflow (rare): per-wave reservations
                    if (om && lane == 0) sent_any = 1;
                    while (om) {
                        const int leader = __builtin_ctzll(om);
                        const u32 qo = lane_u32(own, (u32)leader);
                        const bool mine = rem && rbelow >= rin && own == qo;
                        const u64 qm = __ballot(mine);
                        om &= ~qm;
                        u32 gb = 0;
                        if (lane == leader) gb = atomicAdd(&send_counts[qo * SENDC_STRIDE], (u32)__popcll(qm));
                        gb = lane_u32(gb, (u32)leader);
                        if (mine) {
                            const u32 pos = gb + __popcll(qm & lanes_below);
                            if (pos < bucket_cap) {
                                u64* rec = sdst[qo] + (u64)pos * REC;
                                u64 v = 0;
#pragma unroll
                                for (int x = 0; x < W; ++x) rec[x] = q[x], v += q[x];
                                if (my_dsum) atomicAdd(reinterpret_cast<unsigned long long*>(&my_dsum[qo]), (unsigned long long)v);
                            } else {
                                atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                            }
                        }
                    }
                }
                // the local successors' probes, one access per lane and iteration
                u32 nmask = 0, st = 0, cr = 0, disp = 0;
                u64 si = 0, tag = 0;
                const u64 step = probe_step(t);
                for (;;) {
                    if (st == 0 && vmask) {
                        cr = (u32)__builtin_ctz(vmask);
                        vmask &= vmask - 1;
                        tag = kt[0];
#pragma unroll
                        for (int r = 1; r < R; ++r)
                            if (cr == (u32)r) tag = kt[r];
                        if constexpr (FP_ONLY) {
                            si = tag & t.mask;
                        } else {
                            si = kh[0];
#pragma unroll
                            for (int r = 1; r < R; ++r)
                                if (cr == (u32)r) si = kh[FP_ONLY ? 0 : r];
                        }
                        st = 1;
                        disp = 0;
                    }
                    if (!__ballot(st != 0)) break;
                    u64 v = 0;
                    if (st == 1) v = slot_load<0>(t, si);
                    if (st == 2) v = slot_cas(t, si, tag);
                    if (st != 0) {
                        if (v == tag) {
                            st = 0;
                        } else if (v == 0) {
                            if (st == 2) nmask |= 1u << cr;
                            st = st == 1 ? 2u : 0u;
                        } else if (++disp >= t.plimit) {
                            atomicOr(&lc->err, (u32)ERR_TABLE_FULL);
                            st = 0;
                        } else {
                            si = (si + 1) & t.mask;
                            tag += step;
                            st = 1;
                        }
                    }
                }
                // local new states -> the chunk's stage (their states recomputed from the map)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool nw = nmask >> r & 1;
                    const u64 mask = __ballot(nw);
                    if (!mask) continue;
                    u64 q[W];
                    u32 p = 0;
                    if (nw) {
                        const u32 e = smap[wid][s0 + (u32)r * 64u + (u32)lane - w0];
                        p = e & 63;
                        u64 ps[W];
#pragma unroll
                        for (int x = 0; x < W; ++x) ps[x] = pst[wid][p * W + x];
                        m.apply(ps, (int)(e >> 6), q);
                    }
                    const u32 cnt = __popcll(mask);
                    const u32 below = __popcll(mask & lanes_below);
                    const int leader = __builtin_ctzll(mask);
                    u32 sb = 0;
                    if (lane == leader) sb = atomicAdd(&stage_n, cnt);
                    sb = lane_u32(sb, (u32)leader);
                    const u32 in_stage = sb >= (u32)STAGE ? 0u : min(cnt, (u32)STAGE - sb);
                    u32 gb = 0;
                    if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
                    gb = lane_u32(gb, (u32)leader);
                    if (!nw) continue;
                    if (below < in_stage) {
                        const u32 kk = sb + below;
#pragma unroll
                        for (int x = 0; x < W; ++x) stage[kk * W + x] = q[x];
                        stage_par[kk] = (u32)(wave0 + p);
                    } else {
                        const u32 pos = gb + (below - in_stage);
                        if (pos < next_cap) {
                            store_state<W>(next, pos, q);
                            next_par[pos] = gid_base + wave0 + p;
                        } else {
                            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                        }
                        eval_props(m, q, pos, undiscovered, lc);
                    }
                }
            }
        } else
        for (u32 it = w0; it < wend; it += 64 * PB) {
            u64 ns[PB][W], key[PB], cur[PB];
            ProbeKey pk[PB];
            u32 par[PB], own[PB];
            bool ok[PB], rem[PB];
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                const u32 i = it + j * 64 + lane;
                ok[j] = i < wend;
                par[j] = 0;
                if (ok[j]) {
                    const u32 e = smap[wid][i - w0];
                    const u32 p = e & 63, a = e >> 6;
                    u64 ps[W];
#pragma unroll
                    for (int x = 0; x < W; ++x) ps[x] = pst[wid][p * W + x];
                    ok[j] = m.apply(ps, (int)a, ns[j]);
                    par[j] = p;
                    if (ok[j] && same_state<W>(ns[j], ps)) {  // self-loop: counted, never routed
                        ++succ;
                        ok[j] = false;
                    }
                }
                // key = the fingerprint (owner, filter, sent cache); pk = the visited-set probe
                // (the same value in fingerprint mode; the host turns the filter and the sent
                // cache off for a quotient-mode table)
                pk[j] = ok[j] ? probe_key(m, t, ns[j]) : ProbeKey{0, 0};
                key[j] = !ok[j] ? 0 : route_key(m, t, pk[j], ns[j]);
                if (fmask && ok[j]) {  // block-local duplicate filter (see expand_fast)
                    const u64 old = atomicExch(reinterpret_cast<unsigned long long*>(&filt[filter_index(t, key[j]) & fmask]),
                                               (unsigned long long)key[j]);
                    if (old == key[j]) {
                        ++succ;
                        ok[j] = false;
                    }
                }
                own[j] = ok[j] ? route_owner(m, t, ns[j], key[j], nparts) : my_part;
                rem[j] = ok[j] && (SELF || self_rec || own[j] != my_part);
            }
            // One memory round trip per round: a local successor's visited-set probe and a remote
            // one's sent-cache lookup are issued together (the lookup used to be resolved before
            // the probes were issued: two dependent round trips per round).
            // Sent cache (small T): a lossy direct-mapped record of the fingerprints this
            // partition already routed in this check. A hit is skipped: its owner received that
            // state in this level's exchange or an earlier one, so it is visited. A miss, an
            // eviction or a race only re-sends (the owner dedups).
#pragma unroll
            for (int j = 0; j < PB; ++j)
                cur[j] = SELF || !ok[j] ? 0 : !rem[j] ? slot_load<0>(t, pk[j].home) : sent ? sent[key[j] & sent_mask] : 0;
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                if (SELF || !(sent && rem[j])) continue;
                if (cur[j] == key[j]) {
                    ++succ;
                    ok[j] = rem[j] = false;
                } else {
                    sent[key[j] & sent_mask] = key[j];
                }
            }
            bool nw[PB];
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                nw[j] = false;
                if (!ok[j]) continue;
                ++succ;
                if (SELF || rem[j] || cur[j] == pk[j].tag) continue;
                find_or_claim_from<0>(t, pk[j], cur[j], &nw[j], &lc->err);
            }
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                const u64 pg = gid_base + wave0 + par[j];
                // local new states -> the chunk's stage (one LDS atomic per wave)
                const u64 mask = SELF ? 0ull : __ballot(nw[j]);
                if (mask) {
                    const u32 cnt = __popcll(mask);
                    const u32 below = __popcll(mask & lanes_below);
                    const int leader = __builtin_ctzll(mask);
                    u32 sb = 0;
                    if (lane == leader) sb = atomicAdd(&stage_n, cnt);
                    sb = lane_u32(sb, (u32)leader);
                    const u32 in_stage = sb >= (u32)STAGE ? 0u : min(cnt, (u32)STAGE - sb);
                    u32 gb = 0;
                    if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
                    gb = lane_u32(gb, (u32)leader);
                    if (nw[j]) {
                        if (below < in_stage) {
                            const u32 kk = sb + below;
#pragma unroll
                            for (int x = 0; x < W; ++x) stage[kk * W + x] = ns[j][x];
                            stage_par[kk] = (u32)(wave0 + par[j]);
                        } else {
                            const u32 pos = gb + (below - in_stage);
                            if (pos < next_cap) {
                                store_state<W>(next, pos, ns[j]);
                                next_par[pos] = pg;
                            } else {
                                atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                            }
                            eval_props(m, ns[j], pos, undiscovered, lc);
                        }
                    }
                }
                // remote records -> the chunk's record stage (one LDS atomic per wave)
                const u64 rmask = __ballot(rem[j]);
                if (!rmask) continue;
                const u32 rcnt = __popcll(rmask);
                const u32 rbelow = __popcll(rmask & lanes_below);
                const int rleader = __builtin_ctzll(rmask);
                u32 rsb = 0;
                if (lane == rleader) rsb = atomicAdd(&rstage_n, rcnt);
                rsb = lane_u32(rsb, (u32)rleader);
                const u32 rin = rsb >= RSTAGE ? 0u : min(rcnt, RSTAGE - rsb);
                if (rem[j] && rbelow < rin) {
                    const u32 kk = rsb + rbelow;
#pragma unroll
                    for (int x = 0; x < W; ++x) rstage[kk * REC + x] = ns[j][x];
                    rown[kk] = (u8)own[j];
                }
                // overflow (rare): per-wave reservations, owner by owner
                u64 om = __ballot(rem[j] && rbelow >= rin);
                if (om && lane == 0) sent_any = 1;
                while (om) {
                    const int leader = __builtin_ctzll(om);
                    const u32 q = lane_u32(own[j], (u32)leader);
                    const bool mine = rem[j] && rbelow >= rin && own[j] == q;
                    const u64 qm = __ballot(mine);
                    om &= ~qm;
                    u32 gb = 0;
                    if (lane == leader) gb = atomicAdd(&send_counts[q * SENDC_STRIDE], (u32)__popcll(qm));
                    gb = lane_u32(gb, (u32)leader);
                    if (mine) {
                        const u32 pos = gb + __popcll(qm & lanes_below);
                        if (pos < bucket_cap) {
                            u64* rec = sdst[q] + (u64)pos * REC;
                            u64 v = 0;
#pragma unroll
                            for (int x = 0; x < W; ++x) rec[x] = ns[j][x], v += ns[j][x];
                            if (my_dsum) atomicAdd(reinterpret_cast<unsigned long long*>(&my_dsum[q]), (unsigned long long)v);
                        } else {
                            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                        }
                    }
                }
            }
        }

        wave_lds_sync();  // the window's map is read before the next window overwrites it
        }

        // ---- the stages persist across the block's chunks: a stage is flushed (by the whole
        // block) once it could not hold another chunk's output, flush_at = (local fill << 16 |
        // record fill) thresholds from the host's per-chunk bound (ppw_for sizes a chunk to fit a
        // whole stage). With few records per chunk (an owner key) a flush, its claims reservation
        // and its reservation per owner are shared by several chunks ----
        __syncthreads();
        const bool fl = stage_n > (flush_at >> 16), fr = rstage_n > (flush_at & 0xffffu);
        if (fl || fr) flush(fl, fr);
    }
    __syncthreads();
    flush(true, true);
    u32 total_succ = block_sum(succ, scratch);
    u32 total_enabled = block_sum(enabled, scratch);
    if (threadIdx.x == 0) add_stats(lc, total_succ, total_enabled);
    if (!last_block(lc, ftab != nullptr && sent_any, ftab != nullptr)) return;
    // The row, one word per thread (every source word is a round trip to the coherence point: one
    // thread loading them in turn was the floor of a small level), staged in LDS for the headers.
    __shared__ u64 srow[MAX_PARTS + 6 + MAX_PROPS];
    __shared__ u64 sstat[4];  // the statistics summed over their shards
    __shared__ u64 hsum[MAX_PARTS];  // dsum: each owner's record-word sum over the shards
    if (threadIdx.x < 64) {
        const u64 v = gather_stats(lc, threadIdx.x);
        if ((threadIdx.x & 15) == 0) sstat[threadIdx.x >> 4] = v;
    }
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) hsum[q] = 0;
    __syncthreads();
    if (dsum && lag) {  // the shards' loads are issued together with the row's below (one round trip)
        for (u32 i = threadIdx.x; i < NSHARD * nparts; i += blockDim.x) {
            u64* a = dsum + (u64)(i / nparts) * MAX_PARTS + (i % nparts);
            const u64 v = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&hsum[i % nparts]), (unsigned long long)v);
                *a = 0;  // for the next level (a later launch)
            }
        }
    }
    const u32 rw = nparts + 6 + M::NPROPS;
    for (u32 w = threadIdx.x; w < rw; w += blockDim.x) {
        const u32 f = w - nparts;  // row fields after the per-destination counts
        const u32* src = w < nparts ? send_counts + w * SENDC_STRIDE
                         : f == 2   ? &lc->claims
                         : f == 3   ? &lc->err
                         : f == 5   ? &ctl->roots
                         : f >= 6   ? &ctl->disc_prev[f - 6]
                                    : &lc->claims;  // f == 0 (the frontier size n), 1, 4: no load needed
        const u64 ld = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 v = w < nparts ? ld : f == 0 ? n : f == 1 ? sstat[0] : f == 4 ? sstat[1] : ld;
        srow[w] = v;
        row[w] = v;
    }
    __syncthreads();
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) send_counts[q * SENDC_STRIDE] = 0;  // for the next level
    if (lag)  // the row travels in the header of every bucket (and so reaches every rank)
        for (u32 i = threadIdx.x; i < nparts * rw; i += blockDim.x) {
            const u32 q = i / rw, w = i - q * rw;
            (sdst[q] - DIST_HDR)[w] = srow[w];
        }
    if (dsum && lag)  // each slot's sequence tag and checksum (records + row words)
        for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) {
            u64 rs = 0;
            for (u32 w = 0; w < rw; ++w) rs += srow[w];
            u64* hdr = sdst[q] - DIST_HDR;
            hdr[HDR_SEQ] = fseq;
            hdr[HDR_SUM] = hsum[q] + rs;
        }
    if (threadIdx.x < 64) reset_stats_tickets(lc, threadIdx.x, true);
    if (!ftab) return;
    // direct exchange: the headers (and, before the ticket, every workgroup's records) reach the
    // owners before their flags
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x)
        __hip_atomic_store(ftab[q], fseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Inserts received records [0, total) (record g at rec_at(g)), grid-strided over the workgroups:
// probe / CAS claim, then the new states are appended per wave into an LDS stage (its parent is
// PAR_SEARCH: a received state's generator is found by find_pred) that is flushed with ONE claims
// reservation when half full and at the end. The old form reserved once per workgroup and round:
// with up to 2048 workgroups that was ~2 K same-line atomics per level (~22 us at ~11 ns each,
// scripts/microbench_atomics.hip), the whole duration of a typical insert launch.
template <int IPB, class M, class RecAt>
__device__ __forceinline__ void insert_records(const M& m, RecAt rec_at, u32 total, const TableView& t, u64* next,
                                               u64* next_par, u32 next_cap, LevelCounters* lc, u32 undiscovered,
                                               u64* stage, u32 STAGE, u32& stage_n, u32& base, u64& rsum) {
    constexpr int W = M::W;
    const int lane = threadIdx.x & 63;
    auto flush = [&](u32 nl) {
        if (threadIdx.x == 0) base = atomicAdd(&lc->claims, nl);
        __syncthreads();
        for (u32 k = threadIdx.x; k < nl; k += blockDim.x) {
            const u32 pos = base + k;
            u64 ns[W];
#pragma unroll
            for (int x = 0; x < W; ++x) ns[x] = stage[k * W + x];
            if (pos < next_cap) {
                store_state<W>(next, pos, ns);
                next_par[pos] = PAR_SEARCH;
            } else {
                atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
            }
            eval_props(m, ns, pos, undiscovered, lc);
        }
        __syncthreads();
        if (threadIdx.x == 0) stage_n = 0;
    };
    // IPB records per thread and round: their probes and claims are issued back to back before any
    // is resolved (one round of barriers per IPB x blockDim records). The host takes 4 for large
    // inserts; small ones, latency-bound, keep one (a separate instantiation: the batched form's
    // registers would lower the occupancy of the small ones).
    // IPB < 0: R = -IPB records per thread and round, each with a probe state machine of its own
    // (home load, linear-probe step or claim CAS); every iteration issues the next access of EVERY
    // unresolved record together, so a round costs its longest chain, not the sum of its records'
    // chains (IPB > 1 resolves them one after the other).
    if constexpr (IPB < 0) {
        constexpr int R = -IPB;
        const u64 per_round = (u64)gridDim.x * blockDim.x * R;
        const u64 step = probe_step(t);
        for (u64 g0 = (u64)blockIdx.x * blockDim.x * R; g0 < total; g0 += per_round) {
            __syncthreads();  // every thread read the last fill (and the stage was reset) before appends
            u64 ns[R][W], si[R], tag[R];
            u32 st[R], disp[R];
            bool nws[R];
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const u64 g = g0 + (u64)j * blockDim.x + threadIdx.x;
                st[j] = g < total ? 1u : 0u;
                disp[j] = 0;
                nws[j] = false;
                si[j] = tag[j] = 0;
                if (st[j]) {
                    const u64* rec = rec_at((u32)g);
#pragma unroll
                    for (int x = 0; x < W; ++x) ns[j][x] = rec[x], rsum += rec[x];
                    const ProbeKey pk = probe_key(m, t, ns[j]);
                    si[j] = pk.home;
                    tag[j] = pk.tag;
                }
            }
            for (;;) {
                u32 live = 0;
#pragma unroll
                for (int j = 0; j < R; ++j) live |= st[j];
                if (!__ballot(live != 0)) break;
                u64 v[R];
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    v[j] = 0;
                    if (st[j] == 1) v[j] = slot_load(t, si[j]);
                    if (st[j] == 2) v[j] = slot_cas(t, si[j], tag[j]);
                }
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    if (!st[j]) continue;
                    if (v[j] == tag[j]) {
                        st[j] = 0;
                    } else if (v[j] == 0) {
                        nws[j] = st[j] == 2;
                        st[j] = st[j] == 1 ? 2u : 0u;
                    } else if (++disp[j] >= t.plimit) {
                        atomicOr(&lc->err, (u32)ERR_TABLE_FULL);
                        st[j] = 0;
                    } else {
                        si[j] = (si[j] + 1) & t.mask;
                        tag[j] += step;
                        st[j] = 1;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const bool nw = nws[j];
                const u64 mask = __ballot(nw);
                if (!mask) continue;
                const u32 cnt = __popcll(mask), below = __popcll(mask & ((1ull << lane) - 1));
                const int leader = __builtin_ctzll(mask);
                u32 sb = 0;
                if (lane == leader) sb = atomicAdd(&stage_n, cnt);
                sb = lane_u32(sb, (u32)leader);
                const u32 in_stage = sb >= STAGE ? 0u : min(cnt, STAGE - sb);
                u32 gb = 0;
                if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
                gb = lane_u32(gb, (u32)leader);
                if (!nw) continue;
                if (below < in_stage) {
#pragma unroll
                    for (int x = 0; x < W; ++x) stage[(sb + below) * W + x] = ns[j][x];
                } else {
                    const u32 pos = gb + (below - in_stage);
                    if (pos < next_cap) {
                        store_state<W>(next, pos, ns[j]);
                        next_par[pos] = PAR_SEARCH;
                    } else {
                        atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                    }
                    eval_props(m, ns[j], pos, undiscovered, lc);
                }
            }
            __syncthreads();
            const u32 sn = min(stage_n, STAGE);
            if (sn >= STAGE / 2) flush(sn);
        }
        __syncthreads();
        const u32 sn = min(stage_n, STAGE);
        if (sn) flush(sn);
        return;
    }
    constexpr int PBI = IPB < 1 ? 1 : IPB;  // (the batched-round form below)
    const u64 per_round = (u64)gridDim.x * blockDim.x * PBI;
    for (u64 g0 = (u64)blockIdx.x * blockDim.x * PBI; g0 < total; g0 += per_round) {
        __syncthreads();  // every thread read the last fill (and the stage was reset) before appends
        u64 ns[PBI][W], cur[PBI];
        ProbeKey pk[PBI];
        bool ok[PBI];
#pragma unroll
        for (int j = 0; j < PBI; ++j) {
            const u64 g = g0 + (u64)j * blockDim.x + threadIdx.x;
            ok[j] = g < total;
            pk[j] = ProbeKey{0, 0};
            if (ok[j]) {
                const u64* rec = rec_at((u32)g);
#pragma unroll
                for (int x = 0; x < W; ++x) ns[j][x] = rec[x], rsum += rec[x];
                pk[j] = probe_key(m, t, ns[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < PBI; ++j) cur[j] = ok[j] ? slot_load(t, pk[j].home) : 0;
        bool nws[PBI];  // every claim of the round before any append (their CASes overlap)
#pragma unroll
        for (int j = 0; j < PBI; ++j) {
            nws[j] = false;
            if (ok[j] && cur[j] != pk[j].tag) find_or_claim_from(t, pk[j], cur[j], &nws[j], &lc->err);
        }
#pragma unroll
        for (int j = 0; j < PBI; ++j) {
            const bool nw = nws[j];
            const u64 mask = __ballot(nw);
            if (!mask) continue;  // wave-aggregated: one LDS atomic, the overflow with one claims atomic per wave
            const u32 cnt = __popcll(mask), below = __popcll(mask & ((1ull << lane) - 1));
            const int leader = __builtin_ctzll(mask);
            u32 sb = 0;
            if (lane == leader) sb = atomicAdd(&stage_n, cnt);
            sb = lane_u32(sb, (u32)leader);
            const u32 in_stage = sb >= STAGE ? 0u : min(cnt, STAGE - sb);
            u32 gb = 0;
            if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
            gb = lane_u32(gb, (u32)leader);
            if (!nw) continue;
            if (below < in_stage) {
#pragma unroll
                for (int x = 0; x < W; ++x) stage[(sb + below) * W + x] = ns[j][x];
            } else {
                const u32 pos = gb + (below - in_stage);
                if (pos < next_cap) {
                    store_state<W>(next, pos, ns[j]);
                    next_par[pos] = PAR_SEARCH;
                } else {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                }
                eval_props(m, ns[j], pos, undiscovered, lc);
            }
        }
        __syncthreads();
        const u32 sn = min(stage_n, STAGE);  // the same value in every thread (no append until the next barrier)
        if (sn >= STAGE / 2) flush(sn);
    }
    __syncthreads();
    const u32 sn = min(stage_n, STAGE);
    if (sn) flush(sn);
}

// Insert the records this partition received (state + parent gid); new states continue the next
// frontier after the ones expand_route produced locally. The last workgroup closes the level:
// ctl = {next frontier size, discoveries among it}, counters reset for the next level.
template <class M>
__global__ void __launch_bounds__(256) insert_recv(M m, const u64* __restrict__ recv, u32 nrec, TableView t,
                                                   u64* __restrict__ next, u64* __restrict__ next_par, u32 next_cap,
                                                   LevelCounters* lc, u32 undiscovered, DistCtl* ctl) {
    constexpr int W = M::W, REC = W;
    constexpr u32 STAGE = 1024 / W;
    __shared__ u64 stage[STAGE * W];
    __shared__ u32 stage_n, base;
    if (threadIdx.x == 0) stage_n = 0;
    u64 rsum = 0;  // (unchecked: RCCL's exchange)
    insert_records<1>(m, [&](u32 g) { return recv + (u64)g * REC; }, nrec, t, next, next_par, next_cap, lc, undiscovered,
                   stage, STAGE, stage_n, base, rsum);
    if (!last_workgroup<M::NPROPS>(lc)) return;
    const u32 claims = __hip_atomic_load(&lc->claims, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctl->n = min(claims, next_cap);
#pragma unroll
    for (int p = 0; p < M::NPROPS; ++p) {
        ctl->disc_prev[p] = __hip_atomic_load(&lc->disc[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lc->disc[p] = ~0u;
    }
    ctl->roots = 0;
    lc->claims = 0;
    for (u32 g = 0; g < NSHARD; ++g) lc->gticket[g][0] = 0;
    lc->ticket = 0;
}

// Host-visible outcome of one pipelined level (pinned, two slots per partition): the rows of
// every partition (from the bucket headers) and this partition's close.
struct LagPub {
    u32 seq;           // written last
    u32 claims;        // next frontier of this partition (local + received new states)
    u32 err;
    u32 pad;
    u64 rows[1];       // nparts x RW words
};

// Pipelined insert: the records of source q sit in recv[q * S + HDR ...], their count in the
// header (source q's row, word `me`). Grid-strided over the T x C slots (counts are known only on
// the device). The last workgroup closes the level on the device (ctl: arena offset, frontier
// size, discoveries) and publishes every row plus the close to pinned host memory.
template <class M, int IPB = 1>
__global__ void __launch_bounds__(256) insert_recv_lag(M m, const u64* __restrict__ recv, u64 S, u32 C, u32 me,
                                                       u32 nparts, TableView t, u64* __restrict__ arena,
                                                       u64* __restrict__ apar, u64 arena_cap, LevelCounters* lc,
                                                       u32 undiscovered, DistCtl* ctl, LagPub* pub, u32 seq,
                                                       const u32* wflags, u32 wseq, u64 wtimeout, u32 xcheck) {
    // xcheck (direct exchange): verify every source's slot against its sequence tag and checksum
    // (HDR_SEQ / HDR_SUM); the record words this launch read are summed per workgroup into the
    // statistics shards' xsum word, and the last workgroup compares. ERR_EXCHANGE on a mismatch.
    constexpr int W = M::W, REC = W;
    constexpr u32 STAGE = 1024 / W;
    __shared__ u64 stage[STAGE * W];
    __shared__ u32 qoff[MAX_PARTS + 1];  // exclusive prefix of the received counts per source
    __shared__ u32 stage_n, base;
    if (wflags) {
        // Direct exchange with every rank on its own device: peer_wait's poll is this grid's first
        // step (no launch of its own), one source flag per lane of wave 0, then one acquire per
        // workgroup before any record or header is read. Bounded like peer_wait. (Ranks that share
        // a device keep the separate one-wave wait: a spinning insert grid could hold the CUs a
        // source's expand grid needs.)
        if (threadIdx.x < nparts) {
            const u64 t0 = __builtin_amdgcn_s_memrealtime();
            bool ok = false;
            for (;;) {
                const u32 v = __hip_atomic_load(&wflags[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((int)(v - wseq) >= 0) {
                    ok = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > wtimeout) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (!ok) atomicOr(&lc->err, (u32)ERR_PEER_TIMEOUT);
        }
        __syncthreads();
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const u64 nb = ctl->nb, n = ctl->n;
    u64* next = arena + (nb + n) * W;
    u64* next_par = apar + nb + n;
    const u32 next_cap = (u32)min<u64>(arena_cap > nb + n ? arena_cap - nb - n : 0, 0xffffffffull);
    if (threadIdx.x < 64) {  // counts from the bucket headers (source q's row, word `me`), scanned in wave 0
        const u32 lane = threadIdx.x;
        u32 c = 0;
        if (lane < nparts) c = (u32)min<u64>(recv[(u64)lane * S + me], C);
        u32 incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += y;
        }
        if (lane < nparts) qoff[lane] = incl - c;
        if (lane == nparts - 1) qoff[nparts] = incl;
        if (lane == 0) stage_n = 0;
    }
    __syncthreads();
    const u32 total = qoff[nparts];
    // record g: source q = the last with qoff[q] <= g (binary search over <= 64 sources)
    auto rec_at = [&](u32 g) {
        u32 q = 0;
#pragma unroll
        for (u32 step = MAX_PARTS / 2; step >= 1; step >>= 1)
            if (q + step < nparts && qoff[q + step] <= g) q += step;
        return recv + (u64)q * S + DIST_HDR + (u64)(g - qoff[q]) * REC;
    };
    u64 rsum = 0;
    insert_records<IPB>(m, rec_at, total, t, next, next_par, next_cap, lc, undiscovered, stage, STAGE, stage_n, base, rsum);
    __shared__ u64 sc64[4];
    if (xcheck) {
        const u64 bs = block_sum64(rsum, sc64);
        if (threadIdx.x == 0 && bs) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->stat[blockIdx.x % NSHARD].pad[0]),
                                              (unsigned long long)bs);
    }
    if (!last_block(lc)) return;
    // every row (the bucket headers) to the host, then the close
    const u32 rw = nparts + 6 + M::NPROPS;
    u64 rows_sum = 0;
    for (u32 w = threadIdx.x; w < nparts * rw; w += blockDim.x) {
        const u32 q = w / rw;
        const u64 v = recv[(u64)q * S + (w - q * rw)];
        pub->rows[w] = v;
        rows_sum += v;
    }
    __shared__ u32 xbad;
    if (xcheck) {
        // got = every record word read + every row word; want = the sources' checksums; each tag =
        // this level's sequence number. A source that overflowed its slot (count > C) is a capacity
        // error of its own row, not a corrupt exchange.
        __shared__ u64 xacc[2];
        __shared__ u32 xseq_bad, xover;
        if (threadIdx.x == 0) xacc[0] = xacc[1] = 0, xseq_bad = xover = 0;
        const u64 rs = block_sum64(rows_sum, sc64);  // (its barriers order the resets above)
        for (u32 i = threadIdx.x; i < NSHARD + 2 * nparts; i += blockDim.x) {
            if (i < NSHARD) {
                u64* a = &lc->stat[i].pad[0];
                const u64 v = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&xacc[0]), (unsigned long long)v), *a = 0;
            } else if (i < NSHARD + nparts) {
                const u32 q = i - NSHARD;
                if (recv[(u64)q * S + HDR_SEQ] != (u64)wseq) xseq_bad = 1;
                if (recv[(u64)q * S + me] > (u64)C) xover = 1;
            } else {
                const u32 q = i - NSHARD - nparts;
                atomicAdd(reinterpret_cast<unsigned long long*>(&xacc[1]), (unsigned long long)recv[(u64)q * S + HDR_SUM]);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) xbad = !xover && (xseq_bad || xacc[0] + rs != xacc[1]);
    } else if (threadIdx.x == 0) {
        xbad = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x >= 64) return;
    if (threadIdx.x == 0 && xbad) atomicOr(&lc->err, (u32)ERR_EXCHANGE);  // persists into the next rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the close, one counter per lane of wave 0: lane 0 claims, 1 err, 2 + p disc[p]
    const u32 lane = threadIdx.x;
    const bool live = lane < 2u + (u32)M::NPROPS;
    const u32* src = lane == 0 ? &lc->claims : lane == 1 ? &lc->err : &lc->disc[live ? lane - 2 : 0];
    const u32 v = live ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const u32 claims = __shfl(v, 0, 64), err = __shfl(v, 1, 64) | (xbad ? (u32)ERR_EXCHANGE : 0u);
    if (lane >= 2 && live) {
        ctl->disc_prev[lane - 2] = v;
        lc->disc[lane - 2] = ~0u;
    }
    if (lane == 0) {
        pub->claims = claims;
        pub->err = err;
        ctl->nb = nb + n;
        ctl->n = min(claims, next_cap);
        ctl->roots = 0;
        lc->claims = 0;
    }
    reset_stats_tickets(lc, lane, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: host memory
    if (lane == 0) __hip_atomic_store(&pub->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Copies the all-gathered rows to pinned host memory and then stores `seq` (the host spins on it).
template <int = 0> __global__ void rows_publish(const u64* rows, u64* host_rows, u32 words, u32* host_seq, u32 seq) {
    for (u32 i = threadIdx.x; i < words; i += blockDim.x) host_rows[i] = rows[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: host memory
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(host_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Test hook of the exchange check (SR_DX_CORRUPT_LEVEL): flips one bit of the first record some
// source stored into this owner's receive slots, or of a header row word when no source sent any,
// AFTER the sources computed their checksums. The owner's insert must report ERR_EXCHANGE.
template <int = 0> __global__ void dx_corrupt(u64* recv, u64 S, u32 C, u32 me, u32 nparts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (u32 q = 0; q < nparts; ++q) {
        const u64 c = recv[(u64)q * S + me];
        if (c && c <= C) {
            recv[(u64)q * S + DIST_HDR] ^= 1;
            return;
        }
    }
    recv[nparts + 4] ^= 1;  // source 0's row: enabled slots (statistics only)
}

// Init states owned by this partition (insert + level-0 properties), in visit order.
template <class M>
__global__ void insert_roots_part(M m, TableView t, const u64* states, u32 n, u32 my_part, u32 nparts, u64* out, u64* out_par,
                                  u32* out_n, LevelCounters* lc) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;  // a handful of states: serial keeps init order
    u32 k = 0;
    for (u32 r = 0; r < n; ++r) {
        u64 s[M::W];
        load_state<M::W>(states, r, s);
        u64 key = state_fp<M>(s);
        if (part_of(m, s, key, nparts) != my_part) continue;
        bool is_new;
        find_or_claim(t, probe_key(m, t, s), &is_new, &lc->err);
        if (is_new) lc->claims += 1;
        store_state<M::W>(out, k, s);  // duplicates are queued too (bfs.rs:61-66)
        out_par[k] = ~0ull;
        ++k;
    }
    *out_n = k;
}

// Hand-over from the replicated head: this partition's share of every head state goes into its
// visited set (cnt[1] = claims) and its share of the last head level [first_front, total) becomes
// its first frontier (cnt[0] = size; parent PAR_SEARCH). Wave-aggregated counters.
template <class M>
__global__ void take_owned(M m, const u64* __restrict__ hstates, u32 total, u32 first_front, u32 my_part, u32 nparts,
                           TableView t, u64* __restrict__ arena, u64* __restrict__ apar, u32 arena_cap, u32* cnt,
                           LevelCounters* lc) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    bool mine = false, nw = false;
    u64 s[M::W];
    if (i < total) {
        load_state<M::W>(hstates, i, s);
        const u64 fp = state_fp<M>(s);
        mine = part_of(m, s, fp, nparts) == my_part;
        if (mine) find_or_claim(t, probe_key(m, t, s), &nw, &lc->err);
    }
    const u64 cm = __ballot(nw);
    if (cm && lane == __builtin_ctzll(cm)) atomicAdd(&cnt[1], (u32)__popcll(cm));
    const bool front = mine && i >= first_front;
    const u64 fm = __ballot(front);
    if (!fm) return;
    const int leader = __builtin_ctzll(fm);
    u32 base = 0;
    if (lane == leader) base = atomicAdd(&cnt[0], (u32)__popcll(fm));
    base = __shfl(base, leader, 64);
    if (!front) return;
    const u32 pos = base + __popcll(fm & ((1ull << lane) - 1));
    if (pos < arena_cap) {
        store_state<M::W>(arena, pos, s);
        apar[pos] = PAR_SEARCH;
    }
}

// Parent search for a state inserted from a record (PAR_SEARCH): the lowest frontier index of
// level [0, n) of this partition with a successor equal to `target` (within boundary), or ~0.
template <class M>
__global__ void find_pred(M m, const u64* __restrict__ level_states, u32 n, const u64* __restrict__ target_dev,
                          unsigned long long* best) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 target[M::W];
#pragma unroll
    for (int x = 0; x < M::W; ++x) target[x] = target_dev[x];
    u64 s[M::W];
    load_state<M::W>(level_states, r, s);
    bool hit = false;
    for_each_successor(m, s, [&](int, const u64* ns) { hit |= same_state<M::W>(ns, target); });
    if (hit) atomicMin(best, (unsigned long long)r);
}

}  // namespace sr
