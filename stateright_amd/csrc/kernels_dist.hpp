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
// A parent gid is (partition << 40) | arena index: the BFS tree spans partitions.
#pragma once
#include "kernels.hpp"

namespace sr {

constexpr int GID_SHIFT = 40;

// Owner partition of a fingerprint: the high 32 bits scaled to [0, T) (any T, uniform).
__device__ __host__ __forceinline__ u32 owner_of(u64 fp, u32 nparts) { return (u32)(((fp >> 32) * (u64)nparts) >> 32); }

template <class M>
__global__ void __launch_bounds__(256) expand_route(M m, const u64* __restrict__ frontier, u32 n, TableView t,
                                                    u32 my_part, u32 nparts, u64* __restrict__ next,
                                                    u64* __restrict__ next_par, u32 next_cap, u64 gid_base,
                                                    u64* __restrict__ send, u32 bucket_cap, u32* send_counts,
                                                    LevelCounters* lc, u32 undiscovered, HostCounters* hc, u32 seq) {
    constexpr int W = M::W, MW = M::MW, REC = W + 1;
    constexpr int STAGE = 512 / W;          // local new states staged per workgroup
    constexpr int RSTAGE = 1536 / REC;      // remote records staged per workgroup (split per owner)
    __shared__ u64 stage[STAGE * W];
    __shared__ u64 stage_par[STAGE];
    __shared__ u64 rstage[RSTAGE * REC];
    __shared__ u32 rcount[MAX_PARTS], rbase[MAX_PARTS];
    __shared__ u64 pst[4][64 * W];
    __shared__ u64 pmask[4][64 * MW];
    __shared__ u32 pexcl[4][64];
    __shared__ u32 stage_n, base, scratch[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const u32 seg = RSTAGE / nparts;        // LDS records per owner
    if (threadIdx.x == 0) stage_n = 0;
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) rcount[q] = 0;

    const u32 wave0 = (blockIdx.x * (blockDim.x >> 6) + wid) * 64;
    const u32 r = wave0 + lane;
    u32 cnt = 0;
    if (r < n) {
        u64 s[W], mk[MW];
        load_state<W>(frontier, r, s);
        m.enabled(s, mk);
#pragma unroll
        for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = s[i];
#pragma unroll
        for (int i = 0; i < MW; ++i) {
            pmask[wid][lane * MW + i] = mk[i];
            cnt += __popcll(mk[i]);
        }
    }
    u32 incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        u32 y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    pexcl[wid][lane] = incl - cnt;
    const u32 total = __shfl(incl, 63, 64);
    __syncthreads();

    u32 succ = 0;
    for (u32 it = 0; it < total; it += 64) {
        const u32 i = it + lane;
        if (i >= total) break;
        u32 p = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (pexcl[wid][p + step] <= i) p += step;
        u32 k = i - pexcl[wid][p];
        u32 a = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) {
            u64 mw = pmask[wid][p * MW + w];
            u32 c = __popcll(mw);
            if (k < c) {
                a = w * 64 + select_bit(mw, k);
                break;
            }
            k -= c;
        }
        u64 ps[W], ns[W];
#pragma unroll
        for (int x = 0; x < W; ++x) ps[x] = pst[wid][p * W + x];
        if (!m.apply(ps, (int)a, ns)) continue;
        ++succ;
        if (same_state<W>(ns, ps)) continue;  // self-loop
        const u64 key = fingerprint<W>(ns);
        const u32 owner = owner_of(key, nparts);
        const u64 pgid = gid_base + wave0 + p;
        if (owner == my_part) {
            bool is_new;
            find_or_claim(t, key, &is_new, &lc->err);
            if (!is_new) continue;
            u32 kk = atomicAdd(&stage_n, 1u);
            if (kk < (u32)STAGE) {
#pragma unroll
                for (int x = 0; x < W; ++x) stage[kk * W + x] = ns[x];
                stage_par[kk] = pgid;
            } else {
                u32 pos = atomicAdd(&lc->claims, 1u);
                if (pos < next_cap) {
                    store_state<W>(next, pos, ns);
                    next_par[pos] = pgid;
                } else {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                }
                eval_props(m, ns, pos, undiscovered, lc);
            }
        } else {
            u32 kk = atomicAdd(&rcount[owner], 1u);
            u64* rec;
            if (kk < seg) {
                rec = &rstage[(owner * seg + kk) * REC];
            } else {  // LDS segment full: append straight to the bucket
                u32 pos = atomicAdd(&send_counts[owner], 1u);
                if (pos >= bucket_cap) {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                    continue;
                }
                rec = &send[((u64)owner * bucket_cap + pos) * REC];
            }
#pragma unroll
            for (int x = 0; x < W; ++x) rec[x] = ns[x];
            rec[W] = pgid;
        }
    }
    u32 total_succ = block_sum(succ, scratch);
    const u32 nl = min(stage_n, (u32)STAGE);
    if (threadIdx.x == 0) {
        base = nl ? atomicAdd(&lc->claims, nl) : 0;
        if (total_succ) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->successors), (unsigned long long)total_succ);
    }
    for (u32 q = threadIdx.x; q < nparts; q += blockDim.x) {
        u32 c = min(rcount[q], seg);
        rbase[q] = c ? atomicAdd(&send_counts[q], c) : 0;
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < nl; i += blockDim.x) {
        u32 pos = base + i;
        u64 ns[W];
#pragma unroll
        for (int x = 0; x < W; ++x) ns[x] = stage[i * W + x];
        if (pos < next_cap) {
            store_state<W>(next, pos, ns);
            next_par[pos] = stage_par[i];
        } else {
            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
        eval_props(m, ns, pos, undiscovered, lc);
    }
    // flush staged remote records, owner by owner
    for (u32 q = 0; q < nparts; ++q) {
        const u32 c = min(rcount[q], seg);
        for (u32 i = threadIdx.x; i < c * REC; i += blockDim.x) {
            const u32 rec = i / REC, x = i % REC;
            const u32 pos = rbase[q] + rec;
            if (pos < bucket_cap) send[((u64)q * bucket_cap + pos) * REC + x] = rstage[(q * seg + rec) * REC + x];
            else if (x == 0) atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
    }
    publish<M::NPROPS>(lc, hc, seq, false, nullptr, send_counts, nparts);
}

// Insert the records this partition received (state + parent gid); new states continue the next
// frontier after the ones expand_route produced locally.
template <class M>
__global__ void __launch_bounds__(256) insert_recv(M m, const u64* __restrict__ recv, u32 nrec, TableView t,
                                                   u64* __restrict__ next, u64* __restrict__ next_par, u32 next_cap,
                                                   LevelCounters* lc, u32 undiscovered, HostCounters* hc, u32 seq) {
    constexpr int W = M::W, REC = W + 1;
    constexpr int STAGE = 1024 / W;
    __shared__ u64 stage[STAGE * W];
    __shared__ u64 stage_par[STAGE];
    __shared__ u32 stage_n, base;
    if (threadIdx.x == 0) stage_n = 0;
    __syncthreads();
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nrec) {
        u64 ns[W];
#pragma unroll
        for (int x = 0; x < W; ++x) ns[x] = recv[(u64)i * REC + x];
        const u64 pgid = recv[(u64)i * REC + W];
        bool is_new;
        find_or_claim(t, fingerprint<W>(ns), &is_new, &lc->err);
        if (is_new) {
            u32 kk = atomicAdd(&stage_n, 1u);
            if (kk < (u32)STAGE) {
#pragma unroll
                for (int x = 0; x < W; ++x) stage[kk * W + x] = ns[x];
                stage_par[kk] = pgid;
            } else {
                u32 pos = atomicAdd(&lc->claims, 1u);
                if (pos < next_cap) {
                    store_state<W>(next, pos, ns);
                    next_par[pos] = pgid;
                } else {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                }
                eval_props(m, ns, pos, undiscovered, lc);
            }
        }
    }
    __syncthreads();
    const u32 nl = min(stage_n, (u32)STAGE);
    if (threadIdx.x == 0) base = nl ? atomicAdd(&lc->claims, nl) : 0;
    __syncthreads();
    for (u32 k = threadIdx.x; k < nl; k += blockDim.x) {
        u32 pos = base + k;
        u64 ns[W];
#pragma unroll
        for (int x = 0; x < W; ++x) ns[x] = stage[k * W + x];
        if (pos < next_cap) {
            store_state<W>(next, pos, ns);
            next_par[pos] = stage_par[k];
        } else {
            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
        eval_props(m, ns, pos, undiscovered, lc);
    }
    publish<M::NPROPS>(lc, hc, seq, true, nullptr);
}

// Init states owned by this partition (insert + level-0 properties), in visit order.
template <class M>
__global__ void insert_roots_part(TableView t, const u64* states, u32 n, u32 my_part, u32 nparts, u64* out, u64* out_par,
                                  u32* out_n, LevelCounters* lc) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;  // a handful of states: serial keeps init order
    u32 k = 0;
    for (u32 r = 0; r < n; ++r) {
        u64 s[M::W];
        load_state<M::W>(states, r, s);
        u64 key = fingerprint<M::W>(s);
        if (owner_of(key, nparts) != my_part) continue;
        bool is_new;
        find_or_claim(t, key, &is_new, &lc->err);
        if (is_new) lc->claims += 1;
        store_state<M::W>(out, k, s);  // duplicates are queued too (bfs.rs:61-66)
        out_par[k] = ~0ull;
        ++k;
    }
    *out_n = k;
}

}  // namespace sr
