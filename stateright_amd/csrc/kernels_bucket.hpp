// Bucketed expansion of BIG levels: delayed duplicate detection inside a level.
//
// On a big 2pc level ~87% of the successors that reach the visited set are duplicates of a state
// generated earlier IN THE SAME LEVEL by another parent (2pc N=9 peak: 10.3 M probes for 1.36 M
// new states). The single-kernel path (expand_fast) pays one random 8-byte probe per successor,
// bound by the chip's random-transaction rate (~45-55 G/s, profiles/r01_microbench_random_access.txt).
// This path replaces them with streaming traffic plus ONE probe per distinct state:
//
//   expand_bucket  expands the frontier like expand_fast, but stages each non-self successor
//                  {state, parent rank} in LDS and flushes it into bucket b = top bits of its
//                  fingerprint: a counting sort in LDS, then each bucket's run is appended to the
//                  block's own region of that bucket (cursor in LDS: no global atomics). The grid
//                  is persistent-sized (NB blocks, grid-strided over the frontier), so a flush
//                  carries thousands of records and its runs are several records long.
//   bucket_insert  one 1024-thread workgroup per bucket: streams the bucket's records through an
//                  LDS hash set (8192 slots, 64-bit LDS CAS) that keeps the first parent of each
//                  distinct state, then probes/claims the visited set once per distinct state with
//                  8 probes in flight per lane, and appends the new states with ONE global
//                  reservation per bucket (properties evaluated at the append, as in expand_fast).
//
// Every occurrence of a state falls in the same bucket, so the LDS set sees all of them; a record
// that finds no room (region full, LDS probe limit) takes the direct path (probe / claim / append),
// so capacities only affect speed, never which states are new. FAST order only; one-word states
// (the LDS key is the state itself: s ^ 2^63, never 0, and the fingerprint is recomputed from it).
#pragma once
#include "kernels.hpp"

namespace sr {

constexpr u32 BK_MAXNB = 1024;   // expand blocks at most
constexpr int BK_RS = 3584;      // records staged per expand_bucket workgroup (LDS: two blocks per CU)
constexpr int BK_QS = 8192;      // LDS hash-set slots per bucket in bucket_insert
constexpr u32 BK_MAXB = 512;     // buckets at most (LDS histogram size)
constexpr u64 BK_HB = 0x8000000000000000ull;

// Bucket b of expand block k is region (b, k): appended by that block only (its cursor lives in
// LDS), so there are no global cursor atomics and a region's lines are written by one CU.
struct BucketView {
    u64* st;     // [B][NB][rcap] states
    u32* par;    // [B][NB][rcap] parent ranks
    u32* cnt;    // [B][NB] records in each region (written by every expand block for every bucket)
    u32 rcap;    // records per region
    u32 blog2;   // B = 2^blog2 buckets, bucket = top blog2 bits of the fingerprint
    u32 nb;      // expand blocks (NB <= 1024: one per bucket_insert thread)
};

__device__ __forceinline__ u32 bucket_of(u64 fp, u32 blog2) { return (u32)(fp >> (64 - blog2)); }

// The direct path of a record that found no room: probe / claim / append one state.
template <class M>
__device__ __forceinline__ void direct_insert(const M& m, const TableView& t, u64 s, u32 parent, u64* next,
                                              u32* next_par, u32 next_cap, LevelCounters* lc, u32 undiscovered) {
    bool nw;
    find_or_claim(t, fingerprint<1>(&s), &nw, &lc->err);
    if (!nw) return;
    const u32 pos = atomicAdd(&lc->claims, 1u);
    if (pos < next_cap) {
        next[pos] = s;
        next_par[pos] = parent;
    } else {
        atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
    }
    eval_props(m, &s, pos, undiscovered, lc);
}

// Phase 1: expand parents [lo, hi) (or the previous level's claims, dev_n) into the buckets.
template <class M>
__global__ void __launch_bounds__(256) expand_bucket(M m, const u64* __restrict__ frontier, u32 lo, u32 hi, TableView t,
                                                     BucketView bk, u64* __restrict__ next, u32* __restrict__ next_par,
                                                     u32 next_cap, LevelCounters* lc, u32 undiscovered, u32 ppw_log2,
                                                     u32 dev_n) {
    static_assert(M::W == 1, "bucketed expansion: one-word states");
    constexpr int MW = M::MW;
    __shared__ u64 st_s[BK_RS];
    __shared__ u32 st_p[BK_RS];
    __shared__ u16 st_b[BK_RS];
    __shared__ u16 st_r[BK_RS];
    __shared__ u16 sidx[BK_RS];
    __shared__ u32 hist[BK_MAXB], hbase[BK_MAXB], lcur[BK_MAXB], hexcl[BK_MAXB];
    __shared__ u64 pst[4][64];
    __shared__ u64 pmask[4][64 * MW];
    __shared__ u32 pexcl[4][64];
    __shared__ u32 stage_n, scratch[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const u32 B = 1u << bk.blog2;
    if (dev_n) {
        const u32 nn = lc->prev_claims;
        hi = lo + nn;
        next += nn;
        next_par += nn;
        next_cap = next_cap > nn ? next_cap - nn : 0u;
    }
    for (u32 i = threadIdx.x; i < B; i += blockDim.x) hist[i] = lcur[i] = 0;
    if (threadIdx.x == 0) stage_n = 0;

    // Counting sort of the staged records by bucket, one reservation per non-empty bucket, then
    // the records to their regions. Called by every thread of the block.
    auto flush = [&]() {
        __syncthreads();
        const u32 n = min(stage_n, (u32)BK_RS);
        for (u32 i = threadIdx.x; i < n; i += blockDim.x) st_r[i] = (u16)atomicAdd(&hist[st_b[i]], 1u);
        __syncthreads();
        {   // exclusive scan of the histogram (thread t owns buckets 2t, 2t+1; B <= 512)
            const u32 b0 = 2 * threadIdx.x, b1 = b0 + 1;
            const u32 h0 = b0 < B ? hist[b0] : 0u, h1 = b1 < B ? hist[b1] : 0u;
            const u32 v = h0 + h1;
            u32 incl = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const u32 y = __shfl_up(incl, d, 64);
                if (lane >= d) incl += y;
            }
            if (lane == 63) scratch[wid] = incl;
            __syncthreads();
            u32 wb = 0;
            for (int w = 0; w < wid; ++w) wb += scratch[w];
            const u32 ex = wb + incl - v;
            if (b0 < B) {
                hexcl[b0] = ex;
                hbase[b0] = lcur[b0];  // this block's region of bucket b: its own cursor
                lcur[b0] += h0;
                hist[b0] = 0;
            }
            if (b1 < B) {
                hexcl[b1] = ex + h0;
                hbase[b1] = lcur[b1];
                lcur[b1] += h1;
                hist[b1] = 0;
            }
        }
        __syncthreads();
        // sorted by bucket (LDS permutation), so consecutive lanes write consecutive addresses
        for (u32 i = threadIdx.x; i < n; i += blockDim.x) sidx[hexcl[st_b[i]] + st_r[i]] = (u16)i;
        __syncthreads();
        for (u32 j = threadIdx.x; j < n; j += blockDim.x) {
            const u32 i = sidx[j];
            const u32 b = st_b[i], pos = hbase[b] + st_r[i];
            if (pos < bk.rcap) {
                const u64 r = ((u64)b * bk.nb + blockIdx.x) * bk.rcap + pos;
                bk.st[r] = st_s[i];
                bk.par[r] = st_p[i];
            } else {
                direct_insert(m, t, st_s[i], st_p[i], next, next_par, next_cap, lc, undiscovered);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) stage_n = 0;
        __syncthreads();
    };

    const u32 ppw = 1u << ppw_log2;
    const u64 chunk = (u64)(blockDim.x >> 6) << ppw_log2;
    u32 succ = 0, enabled = 0, chunk0 = 0;
    for (u64 c0 = lo + (u64)blockIdx.x * chunk; c0 < hi; c0 += (u64)gridDim.x * chunk) {
        const u32 wave0 = (u32)(c0 + ((u64)wid << ppw_log2));
        const u32 r = wave0 + lane;
        u32 cnt = 0;
        __syncthreads();
        if (lane < (int)ppw && r < hi) {
            u64 mk[MW];
            const u64 s = frontier[r];
            m.enabled(&s, mk);
            pst[wid][lane] = s;
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
        if (lane == 0) enabled += total;
        __syncthreads();

        for (u32 it = 0; it < total; it += 64) {
            const u32 i = it + lane;
            bool ok = i < total;
            u32 p = 0;
            u64 ns = 0;
            if (ok) {
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1)
                    if (pexcl[wid][p + step] <= i) p += step;
                u32 k = i - pexcl[wid][p];
                u32 a = 0;
#pragma unroll
                for (int w = 0; w < MW; ++w) {
                    const u64 mw = pmask[wid][p * MW + w];
                    const u32 c = __popcll(mw);
                    if (k < c) {
                        a = w * 64 + select_bit(mw, k);
                        break;
                    }
                    k -= c;
                }
                const u64 ps = pst[wid][p];
                ok = m.apply(&ps, (int)a, &ns);
                if (ok) ++succ;  // within boundary: counted (bfs.rs:235)
                if (ok && ns == ps) ok = false;  // self-loop: a duplicate by construction
            }
            const u64 mask = __ballot(ok);
            if (!mask) continue;
            const u32 cw = __popcll(mask);
            const u32 below = __popcll(mask & ((1ull << lane) - 1));
            const int leader = __builtin_ctzll(mask);
            u32 sb = 0;
            if (lane == leader) sb = atomicAdd(&stage_n, cw);
            sb = __shfl(sb, leader, 64);
            if (ok) {
                const u32 kk = sb + below;
                const u32 pr = wave0 + p;
                if (kk < (u32)BK_RS) {
                    st_s[kk] = ns;
                    st_p[kk] = pr;
                    st_b[kk] = (u16)bucket_of(fingerprint<1>(&ns), bk.blog2);
                } else {
                    direct_insert(m, t, ns, pr, next, next_par, next_cap, lc, undiscovered);
                }
            }
        }
        __syncthreads();
        // uniform (read after the barrier): flush when another chunk like this one might not fit
        const u32 sn = stage_n;
        if (sn + 2 * (sn - chunk0) > (u32)BK_RS || sn >= (u32)BK_RS * 3 / 4) flush();
        chunk0 = min(stage_n, (u32)BK_RS);
    }
    __syncthreads();
    if (stage_n) flush();
    for (u32 b = threadIdx.x; b < B; b += blockDim.x) bk.cnt[(u64)b * bk.nb + blockIdx.x] = min(lcur[b], bk.rcap);
    const u32 ts = block_sum(succ, scratch);
    const u32 te = block_sum(enabled, scratch);
    if (threadIdx.x == 0) {
        if (ts) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->successors), (unsigned long long)ts);
        if (te) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->enabled), (unsigned long long)te);
    }
}

// LDS set insert of one-word state key k (= s ^ 2^63) with fingerprint fp: true when k is in the
// set afterwards (first occurrence: its parent recorded), false when the probe limit is hit.
__device__ __forceinline__ bool lds_set_insert(u64* set, u32* spar, u64 k, u64 fp, u32 parent) {
    u32 slot = (u32)fp & (BK_QS - 1);
#pragma unroll 1
    for (int pr = 0; pr < 64; ++pr) {
        const u64 old = atomicCAS(reinterpret_cast<unsigned long long*>(&set[slot]), 0ull, (unsigned long long)k);
        if (old == 0) {
            spar[slot] = parent;
            return true;
        }
        if (old == k) return true;
        slot = (slot + 1) & (BK_QS - 1);
    }
    return false;
}

// Phase 2: one workgroup per bucket (blockIdx.x). Publishes the level (ticket) like expand_fast.
template <class M>
__global__ void __launch_bounds__(1024) bucket_insert(M m, TableView t, BucketView bk, u64* __restrict__ next,
                                                      u32* __restrict__ next_par, u32 next_cap, LevelCounters* lc,
                                                      u32 undiscovered, HostCounters* hc, u32 seq, u32 reset, u32 dev_n) {
    static_assert(M::W == 1, "bucketed expansion: one-word states");
    constexpr int PER = BK_QS / 1024;  // set slots swept per thread
    __shared__ u64 set[BK_QS];
    __shared__ u32 spar[BK_QS];
    __shared__ u32 off[BK_MAXNB + 1];
    __shared__ u32 wsum[16], base;
    if (dev_n) {
        const u32 nn = lc->prev_claims;
        next += nn;
        next_par += nn;
        next_cap = next_cap > nn ? next_cap - nn : 0u;
    }
    const u32 b = blockIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (u32 i = threadIdx.x; i < (u32)BK_QS; i += blockDim.x) set[i] = 0;
    // region offsets: exclusive scan of the NB region counts (one per thread)
    {
        const u32 c = threadIdx.x < bk.nb ? bk.cnt[(u64)b * bk.nb + threadIdx.x] : 0u;
        u32 incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        u32 wb = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            wb += w < wid ? wsum[w] : 0u;
            tot += wsum[w];
        }
        if (threadIdx.x < bk.nb) off[threadIdx.x] = wb + incl - c;
        if (threadIdx.x == 0) off[bk.nb] = tot;
        __syncthreads();
    }
    const u32 R = off[bk.nb];
    const u64 rbase = (u64)b * bk.nb * bk.rcap;
    const u32 nbl = 32 - __builtin_clz(bk.nb - 1);  // ceil(log2(NB)) steps of the region search

    // pass 1: the bucket's records through the LDS set, 8 loads in flight per lane
    for (u32 i0 = 0; i0 < R; i0 += 8 * 1024) {
        u64 s[8];
        u32 pp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u32 i = i0 + j * 1024 + threadIdx.x;
            s[j] = BK_HB;
            pp[j] = 0;
            if (i < R) {
                u32 x = 0;  // last region whose offset is <= i
                for (u32 st = 1u << (nbl - 1); st; st >>= 1)
                    if (x + st < bk.nb && off[x + st] <= i) x += st;
                const u64 r = rbase + (u64)x * bk.rcap + (i - off[x]);
                s[j] = bk.st[r];
                pp[j] = bk.par[r];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (i0 + j * 1024 + threadIdx.x >= R) continue;
            const u64 k = s[j] ^ BK_HB;
            const u64 fp = fmix64(k);
            if (!lds_set_insert(set, spar, k, fp, pp[j]))
                direct_insert(m, t, s[j], pp[j], next, next_par, next_cap, lc, undiscovered);
        }
    }
    __syncthreads();

    // pass 2: one visited-set probe per distinct state, PER probes in flight per lane
    u64 key[PER], cur[PER];
    bool nw[PER];
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const u64 k = set[threadIdx.x * PER + j];
        key[j] = k ? fmix64(k) : 0;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) cur[j] = key[j] ? t.keys[key[j] & t.mask] : 0;
    // claims of the vacant home slots issued back to back (PER atomics in flight), then the rare
    // rest (occupied home slot, lost race) through the ordinary probe loop
    u64 prev[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j)
        prev[j] = (key[j] && cur[j] == 0)
                      ? atomicCAS(reinterpret_cast<unsigned long long*>(&t.keys[key[j] & t.mask]), 0ull,
                                  (unsigned long long)key[j])
                      : cur[j];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        nw[j] = false;
        if (key[j]) {
            if (cur[j] == 0 && prev[j] == 0) nw[j] = true;
            else if (prev[j] != key[j])
                find_or_claim_from<0>(t, key[j], (key[j] + 1) & t.mask, t.keys[(key[j] + 1) & t.mask], &nw[j], &lc->err);
        }
        c += nw[j];
    }
    // block-exclusive scan of the new-state counts, ONE reservation for the bucket
    __syncthreads();  // wsum is reused
    u32 incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    u32 wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        wbase += w < wid ? wsum[w] : 0u;
        tot += wsum[w];
    }
    if (threadIdx.x == 0) base = tot ? atomicAdd(&lc->claims, tot) : 0u;
    __syncthreads();
    u32 pos = base + wbase + incl - c;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!nw[j]) continue;
        const u32 slot = threadIdx.x * PER + j;
        const u64 s = set[slot] ^ BK_HB;
        if (pos < next_cap) {
            next[pos] = s;
            next_par[pos] = spar[slot];
        } else {
            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
        eval_props(m, &s, pos, undiscovered, lc);
        ++pos;
    }
    publish<M::NPROPS>(lc, hc, seq, reset != 0, nullptr);
}

}  // namespace sr
