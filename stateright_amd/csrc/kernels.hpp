// HIP kernels of one BFS level on CDNA4 (gfx950). See DESIGN.md §3 for the data layout and the
// roofline each kernel is priced against.
//
// Visited set (replaces `generated: DashMap<Fingerprint, Option<Fingerprint>>`,
// src/checker/bfs.rs:26): open addressing in HBM, struct-of-arrays so that probes touch only the
// key array:
//   keys[cap]    u64 fingerprint, 0 = vacant (fingerprints are non-zero, src/lib.rs:303)
//   parents[cap] u64 parent fingerprint, 0 = None (an init state)
//   meta[cap]    u64 (FIFO mode only) min over this level's generators of
//                (level+1) << 44 | (parent_rank * A + action_slot): the generator that the
//                reference's single-threaded FIFO would have seen first owns the new state.
// Linear probing from fp & mask; a probe reads the key with a plain load first (duplicates are
// ~92% of successors on 2pc and never need an atomic; a stale EMPTY only falls through to the
// CAS, which is the arbiter, because a slot goes EMPTY -> key exactly once), and only a vacant
// slot costs a 64-bit atomicCAS.
#pragma once
#include "models.hpp"

namespace sr {

constexpr u64 META_UNSET = ~0ull;
constexpr int META_SHIFT = 44;
constexpr u32 CAND_NONE = 0xffffffffu;
constexpr int MAX_PROBE = 1 << 16;
constexpr int MAX_PROPS = 32;

enum ErrBits { ERR_TABLE_FULL = 1, ERR_FRONTIER_OVERFLOW = 2 };

struct TableView {
    u64* keys;
    u64* parents;
    u64* meta;
    u64 mask;
};

// Per-level device counters, copied back once per chunk/level. The hot counters sit on separate
// 128-byte lines (one returning atomic per workgroup each).
struct LevelCounters {
    u64 successors;        // successors within boundary (state_count increments, bfs.rs:235)
    u64 pad0[15];
    u32 claims;            // new states inserted into the visited set (= next-frontier cursor)
    u32 pad1[31];
    u32 err;               // ErrBits
    u32 disc[MAX_PROPS];   // min rank of a discovering state in the frontier being produced
};

// Find `key` or claim a vacant slot for it. Returns the slot; *is_new tells whether we claimed it.
__device__ __forceinline__ u64 find_or_claim(const TableView& t, u64 key, bool* is_new, u32* err) {
    u64 i = key & t.mask;
    for (int probe = 0; probe < MAX_PROBE; ++probe) {
        u64 cur = t.keys[i];
        if (cur == key) {
            *is_new = false;
            return i;
        }
        if (cur == 0) {
            u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&t.keys[i]), 0ull,
                                 (unsigned long long)key);
            if (prev == 0) {
                *is_new = true;
                return i;
            }
            if (prev == key) {
                *is_new = false;
                return i;
            }
        }
        i = (i + 1) & t.mask;
    }
    atomicOr(err, (u32)ERR_TABLE_FULL);
    *is_new = false;
    return ~0ull;
}

// Lookup only (path reconstruction).
__device__ __forceinline__ u64 find_slot(const TableView& t, u64 key) {
    u64 i = key & t.mask;
    for (int probe = 0; probe < MAX_PROBE; ++probe) {
        u64 cur = t.keys[i];
        if (cur == key) return i;
        if (cur == 0) return ~0ull;
        i = (i + 1) & t.mask;
    }
    return ~0ull;
}

template <class M, class F>
__device__ __forceinline__ void for_each_successor(const M& m, const u64* s, F&& f) {
    u64 mask[M::MW];
    m.enabled(s, mask);
#pragma unroll
    for (int w = 0; w < M::MW; ++w) {
        u64 bits = mask[w];
        while (bits) {
            int a = w * 64 + __builtin_ctzll(bits);
            bits &= bits - 1;
            u64 ns[M::W];
            if (m.apply(s, a, ns)) f(a, ns);
        }
    }
}

template <int W>
__device__ __forceinline__ void load_state(const u64* base, u64 r, u64* s) {
    if constexpr (W == 2) {
        auto v = reinterpret_cast<const ulonglong2*>(base)[r];
        s[0] = v.x;
        s[1] = v.y;
    } else {
#pragma unroll
        for (int i = 0; i < W; ++i) s[i] = base[r * W + i];
    }
}
template <int W>
__device__ __forceinline__ void store_state(u64* base, u64 r, const u64* s) {
    if constexpr (W == 2) {
        reinterpret_cast<ulonglong2*>(base)[r] = make_ulonglong2(s[0], s[1]);
    } else {
#pragma unroll
        for (int i = 0; i < W; ++i) base[r * W + i] = s[i];
    }
}

// Insert the (distinct) init states with parent None (`generated.insert(fp, None)`, bfs.rs:47-51).
template <class M>
__global__ void insert_roots(TableView t, const u64* states, u32 n, LevelCounters* lc) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 s[M::W];
    load_state<M::W>(states, r, s);
    bool is_new;
    u64 slot = find_or_claim(t, fingerprint<M::W>(s), &is_new, &lc->err);
    if (is_new) {
        t.parents[slot] = 0;
        if (t.meta) t.meta[slot] = 0;  // level 0
        atomicAdd(&lc->claims, 1u);
    }
}

template <class M>
__device__ __forceinline__ void eval_props(const M& m, const u64* s, u32 rank, u32 undiscovered, LevelCounters* lc) {
    u32 und = undiscovered;
    while (und) {
        int p = __builtin_ctz(und);
        und &= und - 1;
        if (m.discovers(p, s)) atomicMin(&lc->disc[p], rank);
    }
}

// Sum of v over the workgroup, returned to every thread (one LDS round).
__device__ __forceinline__ u32 block_sum(u32 v, u32* scratch) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    u32 t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += scratch[w];
    __syncthreads();
    return t;
}

// FAST order: expand parents [lo, hi) of the frontier. Every successor within boundary counts
// toward state_count (bfs.rs:235); one that claims a vacant slot is new: its parent pointer is
// written and the state is staged in LDS. At the end the workgroup reserves its span of the next
// frontier with ONE global atomic, copies the staged states out contiguously, and evaluates the
// properties there (rank = frontier position). A workgroup that stages more than STAGE states
// appends the overflow directly (per-wave aggregated atomics).
template <class M>
__global__ void __launch_bounds__(256) expand_fast(M m, const u64* __restrict__ frontier, u32 lo, u32 hi,
                                                   TableView t, u64* __restrict__ next, u32 next_cap,
                                                   LevelCounters* lc, u32 undiscovered) {
    constexpr int STAGE = 2048 / M::W;
    __shared__ u64 stage[STAGE * M::W];
    __shared__ u32 stage_n, base, scratch[4];
    if (threadIdx.x == 0) stage_n = 0;
    __syncthreads();
    const u32 r = lo + blockIdx.x * blockDim.x + threadIdx.x;
    u32 succ = 0;
    if (r < hi) {
        u64 s[M::W];
        load_state<M::W>(frontier, r, s);
        const u64 pfp = fingerprint<M::W>(s);
        for_each_successor(m, s, [&](int, const u64* ns) {
            ++succ;
            bool is_new;
            u64 slot = find_or_claim(t, fingerprint<M::W>(ns), &is_new, &lc->err);
            if (!is_new) return;
            t.parents[slot] = pfp;
            u32 k = atomicAdd(&stage_n, 1u);
            if (k < (u32)STAGE) {
#pragma unroll
                for (int i = 0; i < M::W; ++i) stage[k * M::W + i] = ns[i];
            } else {
                u32 pos = atomicAdd(&lc->claims, 1u);
                if (pos < next_cap) store_state<M::W>(next, pos, ns);
                else atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                eval_props(m, ns, pos, undiscovered, lc);
            }
        });
    }
    u32 total_succ = block_sum(succ, scratch);
    const u32 n = min(stage_n, (u32)STAGE);
    if (threadIdx.x == 0) {
        base = n ? atomicAdd(&lc->claims, n) : 0;
        if (total_succ) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->successors), (unsigned long long)total_succ);
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < n; i += blockDim.x) {
        u32 pos = base + i;
        u64 ns[M::W];
#pragma unroll
        for (int w = 0; w < M::W; ++w) ns[w] = stage[i * M::W + w];
        if (pos < next_cap) store_state<M::W>(next, pos, ns);
        else atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        eval_props(m, ns, pos, undiscovered, lc);
    }
}

// FIFO order, pass 1: insert-or-find every successor and record (level, parent rank, slot) in
// meta with atomicMin, so that the minimum — the generator the reference's single-threaded queue
// sees first (push_front/pop_back, bfs.rs:183,263) — owns each new state. The plain load of meta
// first skips the atomic whenever it cannot lower the value (meta only decreases within a level).
// Candidates go to cand[a * n + r] (action-major, so passes 2-3 read it coalesced).
template <class M>
__global__ void __launch_bounds__(256) expand_fifo(M m, const u64* __restrict__ frontier, u32 lo, u32 hi, u32 n,
                                                   TableView t, u32* __restrict__ cand, u32 A, u32 level,
                                                   LevelCounters* lc) {
    __shared__ u32 scratch[4];
    const u32 r = lo + blockIdx.x * blockDim.x + threadIdx.x;
    u32 succ = 0, claims = 0;
    if (r < hi) {
        u64 s[M::W];
        load_state<M::W>(frontier, r, s);
        const u64 lvl = (u64)(level + 1) << META_SHIFT;
        for_each_successor(m, s, [&](int a, const u64* ns) {
            ++succ;
            bool is_new;
            u64 slot = find_or_claim(t, fingerprint<M::W>(ns), &is_new, &lc->err);
            if (slot == ~0ull) return;
            claims += is_new;
            const u64 tag = lvl | ((u64)r * A + (u64)a);
            u64 cur = is_new ? META_UNSET : t.meta[slot];
            if (cur != META_UNSET && (cur >> META_SHIFT) != (u64)(level + 1)) return;  // seen in an earlier level
            if (tag < cur) atomicMin(reinterpret_cast<unsigned long long*>(&t.meta[slot]), (unsigned long long)tag);
            cand[(u64)a * n + r] = (u32)slot;
        });
    }
    u32 ts = block_sum(succ, scratch);
    u32 tc = block_sum(claims, scratch);
    if (threadIdx.x == 0) {
        if (ts) atomicAdd(reinterpret_cast<unsigned long long*>(&lc->successors), (unsigned long long)ts);
        if (tc) atomicAdd(&lc->claims, tc);
    }
}

// FIFO pass 2: number of successors each parent owns.
template <class M>
__global__ void __launch_bounds__(256) own_count(const u32* __restrict__ cand, u32 n, u32 A, u32 level, TableView t,
                                                 u32* __restrict__ counts) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u64 lvl = (u64)(level + 1) << META_SHIFT;
    u32 c = 0;
    for (u32 a = 0; a < A; ++a) {
        u32 slot = cand[(u64)a * n + r];
        if (slot != CAND_NONE && t.meta[slot] == (lvl | ((u64)r * A + a))) ++c;
    }
    counts[r] = c;
}

// FIFO pass 3: write owned successors at offs[r] + j in (parent rank, action slot) order — the
// reference's FIFO order — set their parent pointer, and evaluate properties at that rank.
template <class M>
__global__ void __launch_bounds__(256) scatter_fifo(M m, const u64* __restrict__ frontier, const u32* __restrict__ cand,
                                                    const u32* __restrict__ offs, u32 n, u32 A, u32 level,
                                                    TableView t, u64* __restrict__ next, LevelCounters* lc,
                                                    u32 undiscovered) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u64 lvl = (u64)(level + 1) << META_SHIFT;
    u64 s[M::W];
    bool loaded = false;
    u64 pfp = 0;
    u32 j = offs[r];
    for (u32 a = 0; a < A; ++a) {
        u32 slot = cand[(u64)a * n + r];
        if (slot == CAND_NONE || t.meta[slot] != (lvl | ((u64)r * A + a))) continue;
        if (!loaded) {
            load_state<M::W>(frontier, r, s);
            pfp = fingerprint<M::W>(s);
            loaded = true;
        }
        u64 ns[M::W];
        m.apply(s, (int)a, ns);
        store_state<M::W>(next, j, ns);
        t.parents[slot] = pfp;
        eval_props(m, ns, j, undiscovered, lc);
        ++j;
    }
}

// Successor count per parent, without inserting (used only on the level where a
// `target_state_count` stop can fall, to find the exact 1500-pop block boundary, bfs.rs:113-135).
template <class M>
__global__ void __launch_bounds__(256) count_successors(M m, const u64* __restrict__ frontier, u32 n, u32* counts) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 s[M::W];
    load_state<M::W>(frontier, r, s);
    u32 c = 0;
    for_each_successor(m, s, [&](int, const u64*) { ++c; });
    counts[r] = c;
}

// Properties of level-0 states (init states), rank = frontier position.
template <class M>
__global__ void eval_roots(M m, const u64* frontier, u32 n, LevelCounters* lc, u32 undiscovered) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 s[M::W];
    load_state<M::W>(frontier, r, s);
    u32 und = undiscovered;
    while (und) {
        int p = __builtin_ctz(und);
        und &= und - 1;
        if (m.discovers(p, s)) atomicMin(&lc->disc[p], r);
    }
}

// Rehash into a table of twice the capacity (keys, parents and meta move together).
__global__ void rehash(TableView from, u64 from_cap, TableView to, LevelCounters* lc) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    u64 k = from.keys[i];
    if (!k) return;
    bool is_new;
    u64 slot = find_or_claim(to, k, &is_new, &lc->err);
    if (slot == ~0ull) return;
    to.parents[slot] = from.parents[i];
    if (to.meta) to.meta[slot] = from.meta[i];
}

// After a rehash: candidate slot indices of the old table -> slots of the new one.
__global__ void remap_slots(u32* cand, u64 n, const u64* old_keys, TableView to) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 s = cand[i];
    if (s == CAND_NONE) return;
    cand[i] = (u32)find_slot(to, old_keys[s]);
}

// Walks the parent chain of `fp` (reconstruct_path, bfs.rs:314-342); one thread.
__global__ void trace_chain(TableView t, u64 fp, u64* out, u32 cap, u32* len) {
    u32 k = 0;
    u64 cur = fp;
    while (k < cap) {
        u64 slot = find_slot(t, cur);
        if (slot == ~0ull) break;
        out[k++] = cur;
        u64 p = t.parents[slot];
        if (p == 0) break;
        cur = p;
    }
    *len = k;
}

// ---- exclusive scan of u32 counts (3-phase: tile sums, scan of sums, tile scan + carry) ----
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ u32 block_exclusive_scan(u32 v, u32* total) {
    __shared__ u32 wsum[SCAN_BLOCK / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        u32 y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    u32 base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / 64; ++w) {
        if (w < wid) base += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__global__ void __launch_bounds__(SCAN_BLOCK) scan_tile_sums(const u32* in, u32 n, u32* sums) {
    u64 base = (u64)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i)
        if (base + i < n) acc += in[base + i];
    u32 tot;
    block_exclusive_scan(acc, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_BLOCK) scan_sums(u32* sums, u32 nt, u32* grand_total) {
    // one block; sequential over chunks of SCAN_BLOCK tiles
    u32 carry = 0;
    for (u32 base = 0; base < nt; base += SCAN_BLOCK) {
        u32 i = base + threadIdx.x;
        u32 v = i < nt ? sums[i] : 0;
        u32 tot;
        u32 ex = block_exclusive_scan(v, &tot);
        if (i < nt) sums[i] = ex + carry;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *grand_total = carry;
}

__global__ void __launch_bounds__(SCAN_BLOCK) scan_tiles(const u32* in, u32 n, const u32* sums, u32* out) {
    u64 base = (u64)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    u32 v[SCAN_ITEMS];
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = base + i < n ? in[base + i] : 0;
        acc += v[i];
    }
    u32 tot;
    u32 ex = block_exclusive_scan(acc, &tot) + sums[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        if (base + i < n) out[base + i] = ex;
        ex += v[i];
    }
}

}  // namespace sr
