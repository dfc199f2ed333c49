// HIP kernels of one BFS level on CDNA4 (gfx950). See DESIGN.md §3 for the data layout and the
// roofline each kernel is priced against.
//
// Visited set (replaces `generated: DashMap<Fingerprint, Option<Fingerprint>>`,
// src/checker/bfs.rs:26): open addressing over a KEYS-ONLY array in HBM,
//   keys[cap]    u64 fingerprint, 0 = vacant (fingerprints are non-zero, src/lib.rs:303)
//   meta[cap]    u64 (FIFO order only) min over this level's generators of
//                (level+1) << 44 | (parent_rank * A + action_slot): the generator that the
//                reference's single-threaded FIFO would have seen first owns the new state.
// The `Option<Fingerprint>` parent half of the reference map lives in the BFS tree instead: every
// level's frontier is kept in one arena (states in visit order) next to a u32 array of parent
// ranks in the previous level, both written coalesced. A path is rank -> parent rank -> ... .
//
// Linear probing from fp & mask; a probe reads the key with a plain load first (duplicates are
// ~90% of successors on 2pc and never need an atomic; a stale EMPTY only falls through to the
// CAS, which is the arbiter, because a slot goes EMPTY -> key exactly once), and only a vacant
// slot costs a 64-bit atomicCAS. A successor equal to its parent (a self-loop: 37% of 2pc's
// successors) is a duplicate by construction and is counted without touching the table.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdlib>

#include "models.hpp"

namespace sr {

constexpr u64 META_UNSET = ~0ull;
constexpr int META_SHIFT = 44;
constexpr u32 CAND_NONE = 0xffffffffu;
constexpr int MAX_PROBE = 1 << 16;
constexpr int MAX_PROPS = 32;
constexpr int MAX_PARTS = 64;  // visited-set partitions (one per GPU, or virtual ones on one GPU)
// expand_fast's largest parents per wave (log2) for wide states (W >= 4).
#ifndef SR_WIDE_PPW_LOG2_MAX
#define SR_WIDE_PPW_LOG2_MAX 5
#endif
// expand_fast's LDS stage of new narrow states (W < 4), in states per 4 waves (its size sets the
// blocks per CU; until round 6 it was in 64-bit words, i.e. half as many two-word states).
#ifndef SR_STAGE_WORDS
#define SR_STAGE_WORDS 1024
#endif
// expand_fast's dynamic chunks: on a level of many chunks per workgroup (> DYN_MIN_RATIO), each
// workgroup takes three chunks statically and then pulls the next ones from a counter, so that the
// workgroups finish the level together (0: static striding only).
#ifndef SR_DYN_CHUNKS
#define SR_DYN_CHUNKS 1
#endif
constexpr u32 DYN_SHARDS = 8;
#ifndef DYN_MIN_RATIO
#define DYN_MIN_RATIO 6
#endif
// expand_fast's waves per workgroup for narrow states (W < 4): the block-local duplicate filter
// is shared by the workgroup, so its reach is the parents of a whole chunk (waves x ppw).
#ifndef SR_NARROW_WPB
#define SR_NARROW_WPB 4
#endif
template <class M>
constexpr int expand_wpb() { return M::W >= 4 ? 4 : SR_NARROW_WPB; }
// ... and for wide states (W >= 4), whose blocks per CU are set by registers, not LDS.
#ifndef SR_WIDE_STAGE_WORDS
#define SR_WIDE_STAGE_WORDS 2048
#endif
// expand_fast's waves per SIMD for wide states (their VGPR budget: 3 -> <= 168, 4 -> <= 128).
#ifndef SR_WIDE_WAVES
#define SR_WIDE_WAVES 3
#endif

// ERR_EXCHANGE: the direct exchange delivered a receive slot whose sequence tag or checksum does
// not match what its source stored (kernels_dist.hpp): the check is redone on the collective exchange.
// ERR_DEFERRED: a speculative launch found its frontier too large for the room the host left in the
// visited set or the arena and expanded nothing (the host grows them and launches the level again).
enum ErrBits { ERR_TABLE_FULL = 1, ERR_FRONTIER_OVERFLOW = 2, ERR_PEER_TIMEOUT = 4, ERR_EXCHANGE = 8, ERR_DEFERRED = 16 };

// Two slot encodings ("Visited set"):
//  * fingerprint mode (qbits == 0): a slot holds the 64-bit fingerprint. Exact for one-word states
//    (fingerprint<1> is a bijection); a 64-bit hash for wider states, like the reference's own
//    visited set (DashMap keyed by a 64-bit ahash fingerprint, src/checker/bfs.rs:26,245-247).
//  * quotient mode (qbits > 0, models with a packed key of B = bbits <= 120 bits, `qkey`): the key
//    goes through a bijection on B bits (qperm); its top k = log2(cap) bits are the HOME slot and
//    the slot stores the other qbits = B - k bits (the remainder) above dbits = 64 - qbits bits
//    holding 1 + the linear-probe displacement from home. A slot value determines the key exactly,
//    so the visited set is exact at 8 bytes per slot, for states far wider than 64 bits.
//  * narrow quotient mode (s32 = 1, one-word keys of B <= 62 bits whose remainder leaves >= 10
//    displacement bits in 32): the same encoding in 32-bit slots, dbits = 32 - qbits. 2pc N=9's
//    40-bit key in a 2^25-slot table is a 15-bit remainder + 17 displacement bits: 128 MiB instead
//    of 256, so the table and a level's streamed frontier fit the 256 MiB Infinity Cache together.
struct TableView {
    u64* keys;      // cap slots of 8 bytes, or of 4 bytes when s32 (then (cap + 1) / 2 words)
    u64* meta;
    u64 mask;
    u32 qbits = 0;  // quotient mode: remainder bits per slot (0: fingerprint mode)
    u32 dbits = 0;  // quotient mode: displacement bits (slot bits - qbits)
    u32 bbits = 0;  // quotient mode: key bits B
    u32 plimit = MAX_PROBE;  // probe limit: slots past home a probe may visit (quotient: 2^dbits - 2)
    u32 s32 = 0;    // 32-bit slots (narrow quotient mode)
};

// Visited-set slot access (8- or 4-byte slots; 0 = vacant in both). POL: probe_load's policy.
template <int POL, class T>
__device__ __forceinline__ T probe_load(const T* p);
template <int POL = 0>
__device__ __forceinline__ u64 slot_load(const TableView& t, u64 i) {
    if (t.s32) return (u64)probe_load<POL>(reinterpret_cast<const u32*>(t.keys) + i);
    return probe_load<POL>(t.keys + i);
}
__device__ __forceinline__ u64 slot_cas(const TableView& t, u64 i, u64 tag) {
    if (t.s32) return (u64)atomicCAS(reinterpret_cast<u32*>(t.keys) + i, 0u, (u32)tag);
    return atomicCAS(reinterpret_cast<unsigned long long*>(t.keys + i), 0ull, (unsigned long long)tag);
}
// u64 words that hold a table of cap slots
SR_HD u64 table_words(const TableView& t, u64 cap) { return t.s32 ? (cap + 1) / 2 : cap; }

// The probe limit of an encoding: quotient mode stores 1 + the displacement in dbits bits.
SR_HD u32 encoding_probe_limit(u32 qbits, u32 dbits) {
    return qbits && dbits < 17 ? (1u << dbits) - 2 : (u32)MAX_PROBE;
}

// Longest linear-probe displacement the table can be expected to hold at load `alpha` with `slots`
// slots: a run of L occupied slots starts at a given slot with probability ~exp(-L (alpha - 1 -
// ln alpha)) under uniform hashing, so the longest of them is ~ln(slots) / (alpha - 1 - ln alpha)
// (at increment_lock N=12's 0.61 load over 2^33 slots: ~220).
inline double expected_max_displacement(double alpha, double slots) {
    if (alpha <= 0) return 0;
    if (alpha >= 1) return 1e300;
    return std::log(std::max(2.0, slots)) / (alpha - 1.0 - std::log(alpha));
}
// The largest load at which that expectation stays within half the probe limit (the growth
// threshold of a quotient-mode table, whose probe limit is set by its displacement bits), capped
// at `cap_load`.
inline double max_load_for(u32 plimit, double slots, double cap_load) {
    if (plimit >= (u32)MAX_PROBE) return cap_load;
    double lo = 0.0, hi = cap_load;
    if (expected_max_displacement(hi, slots) <= plimit / 2.0) return hi;
    for (int i = 0; i < 60; ++i) {
        const double mid = 0.5 * (lo + hi);
        (expected_max_displacement(mid, slots) <= plimit / 2.0 ? lo : hi) = mid;
    }
    return lo;
}

// Where a key's probe sequence starts, and the value its slot holds at displacement 0; at
// displacement d the slot is (home + d) & mask and the value tag + d * step (step = 1 in quotient
// mode, 0 in fingerprint mode).
struct ProbeKey {
    u64 home;
    u64 tag;
};

using u128 = unsigned __int128;

// A bijection on B-bit integers (B <= 128): a 4-round unbalanced Feistel network over the top
// B - B/2 and the low B/2 bits (every round is invertible whatever its round function).
SR_HD u128 qperm(u128 x, u32 B) {
    const u32 hb = B / 2, ab = B - hb;
    const u64 mb = hb >= 64 ? ~0ull : (1ull << hb) - 1, ma = ab >= 64 ? ~0ull : (1ull << ab) - 1;
    u64 b = (u64)x & mb, a = (u64)(x >> hb) & ma;
    b ^= fmix64(a * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) & mb;
    a ^= fmix64(b * 0xC2B2AE3D27D4EB4Full + 0x165667B19E3779F9ull) & ma;
    b ^= fmix64(a * 0xD6E8FEB86659FD93ull + 0x94D049BB133111EBull) & mb;
    a ^= fmix64(b * 0xBF58476D1CE4E5B9ull + 0x7F4A7C159E3779B9ull) & ma;
    return ((u128)a << hb) | b;
}

// A bijection on B-bit integers (B <= 63) for one-word keys: the murmur3 finalizer's steps with
// every product taken mod 2^B (multiplying by an odd constant and x ^= x >> r are both invertible
// on B bits). Two multiplies instead of qperm's four 64-bit mixes: it runs once per successor.
SR_HD u64 qmix(u64 x, u32 B) {
    const u64 m = (1ull << B) - 1;
    const u32 r = (B + 1) / 2;
    x ^= x >> r;
    x = (x * 0xff51afd7ed558ccdull) & m;
    x ^= x >> r;
    x = (x * 0xc4ceb9fe1a85ec53ull) & m;
    x ^= x >> r;
    return x;
}

SR_HD u64 probe_step(const TableView& t) { return t.qbits ? 1ull : 0ull; }
SR_HD ProbeKey fp_probe(const TableView& t, u64 fp) { return ProbeKey{fp & t.mask, fp}; }
SR_HD ProbeKey quot_probe(const TableView& t, u128 h) {
    return ProbeKey{(u64)(h >> t.qbits), (((u64)h & ((1ull << t.qbits) - 1)) << t.dbits) | 1ull};
}
// Quotient mode: the permuted key held by slot i with value v.
SR_HD u128 quot_decode(const TableView& t, u64 i, u64 v) {
    const u64 d = (v & ((1ull << t.dbits) - 1)) - 1;
    return ((u128)((i - d) & t.mask) << t.qbits) | (v >> t.dbits);
}
// Slot value of a key in `from` re-expressed for `to` (rehash into a larger table).
SR_HD ProbeKey reprobe(const TableView& from, const TableView& to, u64 i, u64 v) {
    return from.qbits ? quot_probe(to, quot_decode(from, i, v)) : fp_probe(to, v);
}

// Host: the view of a table of `cap` (a power of two) slots for model M. Quotient mode whenever
// the model packs its states into a key (qkey) whose remainder fits a slot with >= 8 displacement
// bits; min_table_cap keeps every table of such a model in that mode from the start (a
// fingerprint cannot be turned back into a key when the table grows).
// SR_DISP_LIMIT (tests) lowers every table's probe limit, to force the overflow path.
inline u32 forced_probe_limit() {
    const char* e = std::getenv("SR_DISP_LIMIT");
    return e ? (u32)std::max(1, std::atoi(e)) : 0u;
}
// One-word keys (W == 1, B <= 62 bits; 2pc: 4N+4) take the narrow 32-bit slots whenever the
// remainder leaves >= SLOT32_DMIN displacement bits, else 8-byte quotient slots. Their remainder
// is max(1, B - k) bits: a table larger than the key space (2pc N=3's 16-bit key in the default
// 2^22 slots) homes its keys in the first 2^(B-1) slots, still exact. SR_SLOT32=0 (measurement
// knob) keeps one-word keys in 8-byte slots.
constexpr u32 SLOT32_DMIN = 10;
inline bool slot32_enabled() {
    static const bool on = !std::getenv("SR_SLOT32") || std::atoi(std::getenv("SR_SLOT32")) != 0;
    return on;
}
// Whether model M keys its visited set by its packed key (quotient mode) rather than by a
// fingerprint; fixed per model instance, since a fingerprint cannot be turned back into a key.
template <class M>
inline bool quotient_model(const M& m) {
    if constexpr (has_qkey<M>::value) {
        const int B = m.qkey_bits();
        if constexpr (M::W == 1) return B >= 2 && B <= 62;
        else return B <= 120;
    }
    (void)m;
    return false;
}
template <class M>
inline TableView make_table_view(const M& m, u64* keys, u64* meta, u64 cap, bool natural = false) {
    TableView v{keys, meta, cap - 1};
    if constexpr (has_qkey<M>::value) {
        const u32 B = (u32)m.qkey_bits();
        u32 k = 0;
        while ((1ull << k) < cap) ++k;
        if constexpr (M::W == 1) {
            if (quotient_model(m)) {
                v.qbits = B > k ? B - k : 1u;
                v.bbits = B;
                if (slot32_enabled() && v.qbits + SLOT32_DMIN <= 32) {
                    v.s32 = 1;
                    v.dbits = 32 - v.qbits;
                } else {
                    v.dbits = 64 - v.qbits;
                }
            }
        } else if (B <= 120 && B > k && B - k <= 56) {
            v.qbits = B - k;
            v.dbits = 64 - v.qbits;
            v.bbits = B;
        }
    }
    v.plimit = encoding_probe_limit(v.qbits, v.dbits);
    if (!natural && forced_probe_limit()) v.plimit = std::min(v.plimit, forced_probe_limit());
    return v;
}
template <class M>
inline u64 min_table_cap(const M& m) {
    if constexpr (has_qkey<M>::value) {
        const int B = m.qkey_bits();
        if (M::W == 1 && quotient_model(m) && B > 56) return 1ull << (B - 56);
        if (M::W >= 2 && B > 56 && B <= 96) return 1ull << (B - 56);
    }
    return 1;
}

// The permuted key of a quotient-mode table (a bijection of the packed key; its top bits are the
// home slot).
template <class M>
SR_HD u128 quot_hash(const M& m, const TableView& t, const u64* s) {
    if constexpr (M::W == 1) return qmix((u64)m.qkey(s), t.bbits);
    else return qperm(m.qkey(s), t.bbits);
}

template <class M>
SR_HD ProbeKey probe_key(const M& m, const TableView& t, const u64* s) {
    if constexpr (has_qkey<M>::value) {
        if (t.qbits) return quot_probe(t, quot_hash(m, t, s));
    }
    return fp_probe(t, state_fp<M>(s));
}

// Key of the block-local duplicate filter (expand_fast): injective on states wherever the host
// turns the filter on. Fingerprint mode: the slot value (a bijection of a one-word state).
// Quotient mode with B <= 63: the permuted key + 1 (home and remainder put back together).
SR_HD u64 filter_key(const TableView& t, const ProbeKey& k) {
    return t.qbits ? ((k.home << t.qbits) | (k.tag >> t.dbits)) + 1 : k.tag;
}
SR_HD u32 filter_index(const TableView& t, u64 fk) { return t.qbits ? (u32)fk : (u32)(fk >> 40); }
// Whether the duplicate filter is exact for M's tables (filter_key injective). Multi-word quotient
// tables (increment_lock N >= 9: every successor is new, nothing to filter) run without it.
template <class M>
inline bool filter_exact(const M& m) {
    const TableView v = make_table_view(m, nullptr, nullptr, min_table_cap(m), true);
    return !v.qbits || (M::W == 1 && v.bbits <= 63);
}
// Compact filter (expand_fast's filt_log2 argument | FILT_COMPACT): 4-byte entries for one-word
// quotient tables whose filter key fk (<= 2^B) loses at most 30 bits past the entry index: entry
// fk & (2^L - 1) holds (fk >> L) | 2^31 (never 0, the empty entry), exact for B - L <= 30. Twice the
// entries in the same LDS (2pc N=9, B = 40: 1024 entries in 4 KB instead of 512).
constexpr u32 FILT_COMPACT = 0x100;
template <class M>
inline bool filter_compact_ok(const M& m, u32 log2_entries) {
    if (M::W != 1 || !filter_exact(m)) return false;
    const TableView v = make_table_view(m, nullptr, nullptr, min_table_cap(m), true);
    return v.qbits && v.bbits <= 30 + log2_entries;
}
// The block-local filter's lookup-and-insert of key fk: whether fk was there (a duplicate).
__device__ __forceinline__ bool filter_seen(u64* filt, bool compact, u32 flog, u32 fmask, const TableView& t, u64 fk) {
    if (compact) {
        const u32 e = (u32)(fk >> flog) | 0x80000000u;
        return atomicExch(reinterpret_cast<u32*>(filt) + ((u32)fk & fmask), e) == e;
    }
    return atomicExch(reinterpret_cast<unsigned long long*>(&filt[filter_index(t, fk) & fmask]), (unsigned long long)fk) ==
           (unsigned long long)fk;
}

constexpr u32 NO_PARENT = 0xffffffffu;

// Per-level device counters. Atomics to one 128-byte line serialise at the coherence point at
// ~11 ns each whatever the addresses inside it (scripts/microbench_atomics.hip: 12 288 atomics to
// one line take 143 us; to 8 lines, 21 us), and the workgroups of a level finish together. So
// every counter that each workgroup updates is spread: the statistics over NSHARD lines (by
// blockIdx % NSHARD, summed by the publisher) and the ticket over NSHARD group tickets plus one
// top ticket. claims (one or two reservations per workgroup) keeps its own line. The last
// workgroup of a launch publishes a snapshot to pinned host memory, so the host learns the
// level's outcome without a copy or a stream sync.
constexpr u32 NSHARD = 16;
struct StatShard {
    u64 successors;        // successors within boundary (state_count increments, bfs.rs:235)
    u64 enabled;           // enabled action slots of the expanded parents (launch-shape statistic)
    u64 probes;            // visited-set slots loaded (first probe + linear-probe steps)
    u64 cas;               // 64-bit atomicCAS claims attempted on the visited set
    u64 pad[12];
};
struct LevelCounters {
    StatShard stat[NSHARD];
    u32 claims;            // new states inserted into the visited set (= next-frontier cursor)
    u32 err;               // ErrBits; next to claims: a pipelined launch loads both with one load
    u32 pad1[30];
    u32 ticket;            // groups of workgroups finished in this launch
    u32 pad2[31];
    u32 gticket[NSHARD][32];  // workgroups finished per group (blockIdx % NSHARD), one line each
    u32 disc[MAX_PROPS];   // min rank of a discovering state in the frontier being produced
    u32 pad3[32];
    u32 prev_claims;       // claims of the last level (set by a resetting publish): the size of the
                           // frontier a pipelined launch expands, read on the device
    u32 prev_err;          // always 0 (the err word a launch reading prev_claims sees)
    // Written by a slotted launch of the pipelined loop for a launch chained to it (SlotWork.chain):
    u64 next_base;         // arena offset of the frontier this launch produces
    u64 unique;            // unique states inserted before this launch's claims (its frontier included)
    // expand_fast's dynamic chunks (SR_DYN_CHUNKS): chunks handed out past the static ones, one
    // counter per XCD-sized shard of the workgroups (a line each), and the workgroups done with them
    // (the last one zeroes them all for the slot's next launch)
    alignas(128) u32 chunk_next[DYN_SHARDS][32];
    u32 chunk_done;
    u32 pad5[31];
};
static_assert(offsetof(LevelCounters, err) == offsetof(LevelCounters, claims) + 4, "claims/err pair");
static_assert(offsetof(LevelCounters, prev_err) == offsetof(LevelCounters, prev_claims) + 4, "prev pair");
static_assert(offsetof(LevelCounters, claims) % 8 == 0 && offsetof(LevelCounters, prev_claims) % 8 == 0, "u64 loads");

// A workgroup's statistics (one thread): into its shard.
__device__ __forceinline__ void add_stats(LevelCounters* lc, u32 succ, u32 en, u32 probes = 0, u32 cas = 0) {
    StatShard* sh = &lc->stat[blockIdx.x % NSHARD];
    if (succ) atomicAdd(reinterpret_cast<unsigned long long*>(&sh->successors), (unsigned long long)succ);
    if (en) atomicAdd(reinterpret_cast<unsigned long long*>(&sh->enabled), (unsigned long long)en);
    if (probes) atomicAdd(reinterpret_cast<unsigned long long*>(&sh->probes), (unsigned long long)probes);
    if (cas) atomicAdd(reinterpret_cast<unsigned long long*>(&sh->cas), (unsigned long long)cas);
}

// The workgroup's ticket (one thread, after its counter atomics have drained): true for the last
// workgroup of the launch. The last arrival of each group takes the top ticket; the group
// tickets chain the arrivals, so the last workgroup sees every counter update of the launch.
__device__ __forceinline__ bool take_ticket(LevelCounters* lc) {
    // a small grid (a small level) takes the top ticket directly: one round trip, not two
    if (gridDim.x <= 128) return atomicAdd(&lc->ticket, 1u) == gridDim.x - 1;
    const u32 g = blockIdx.x % NSHARD;
    const u32 gsize = (gridDim.x - g + NSHARD - 1) / NSHARD;
    if (atomicAdd(&lc->gticket[g][0], 1u) != gsize - 1) return false;
    return atomicAdd(&lc->ticket, 1u) == min(gridDim.x, NSHARD) - 1;
}

// Sums of the four statistics over the shards, gathered by the 64 lanes of one wave (lane 16c + s
// loads counter c of shard s); lane 16c returns the total of counter c.
__device__ __forceinline__ u64 gather_stats(const LevelCounters* lc, u32 lane) {
    const u64* w = reinterpret_cast<const u64*>(&lc->stat[lane & (NSHARD - 1)]) + (lane >> 4);
    u64 v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int d = 8; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Reset of the statistics and the tickets for the next launch (one wave, lane = 0..63).
__device__ __forceinline__ void reset_stats_tickets(LevelCounters* lc, u32 lane, bool stats) {
    if (stats) reinterpret_cast<u64*>(&lc->stat[lane & (NSHARD - 1)])[lane >> 4] = 0;
    if (lane < NSHARD) lc->gticket[lane][0] = 0;
    if (lane == 0) lc->ticket = 0;
}

// Host-visible snapshot (hipHostMalloc'd), written by the publishing workgroup.
struct HostCounters {
    u64 successors;
    u64 enabled;
    u64 probes;
    u64 cas;
    u32 claims;
    u32 err;
    u32 aux;               // launch-specific value (FIFO: number of owners from the scan)
    u32 disc[MAX_PROPS];
    u32 sendc[MAX_PARTS];  // partitioned search: records routed to each partition
    u32 seq;               // written last: the launch's sequence number
};

template <int NP>
__device__ __forceinline__ void reset_counters(LevelCounters* lc) {
    for (u32 i = 0; i < NSHARD; ++i) lc->stat[i] = StatShard{};
    lc->claims = 0;
    lc->err = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) lc->disc[p] = ~0u;
}

// Every counter the last workgroup reads is updated with device-scope atomics (performed at the
// coherence point, not in an XCD's L2) and read back with agent-scope atomic loads, so the ticket
// needs only each wave's drained vmcnt before it — no agent release (an L2 writeback, ≈2-6 µs per
// workgroup, MI355X_MICROARCH.md) and no acquire. The frontier data the workgroups write with plain
// stores is read only by later launches (kernel boundary). SR_TICKET_FENCE=1 restores both fences.
#ifndef SR_TICKET_FENCE
#define SR_TICKET_FENCE 0
#endif

// Called by every workgroup after its last counter update (all threads). The workgroup that
// arrives last copies the counters to host memory, optionally resets them for the next level,
// and finally stores `seq` (Guideline 16: release before the ticket, acquire after it). NP = the
// number of properties whose discovery ranks are live.
//
// The snapshot is gathered by the 64 lanes of wave 0 at once: lane i loads counter word i (every
// load is an agent-scope round trip to the coherence point, ≈1 µs; issued by one thread they
// were ~12 dependent round trips at the tail of EVERY level, the floor of a small level), then
// writes it to its host word. u64 counters move as two u32 words: no workgroup updates them any
// more once the ticket has been taken by the last one.
template <int NP>
__device__ __forceinline__ void publish(LevelCounters* lc, HostCounters* h, u32 seq, bool reset, const u32* aux,
                                        const u32* sendc = nullptr, u32 nparts = 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const u32 lane = threadIdx.x;
    u32 last = 0;
    if (lane == 0) {
#if SR_TICKET_FENCE
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = take_ticket(lc);
    }
    if (!__shfl(last, 0, 64)) return;
#if SR_TICKET_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    // statistics: summed over the shards (lane 16c holds counter c), written as two u32 words
    u32* hw = reinterpret_cast<u32*>(h);
    const u64 st = gather_stats(lc, lane);
    if ((lane & 15) == 0) {
        hw[(lane >> 4) * 2] = (u32)st;
        hw[(lane >> 4) * 2 + 1] = (u32)(st >> 32);
    }
    // word map: 0 claims, 1 err, 2 aux, 3 + p disc[p], 3 + NP + q sendc[q]
    const u32* lcw = reinterpret_cast<const u32*>(lc);
    constexpr u32 O_CLAIMS = offsetof(LevelCounters, claims) / 4, O_ERR = offsetof(LevelCounters, err) / 4;
    constexpr u32 O_DISC = offsetof(LevelCounters, disc) / 4;
    constexpr u32 H_CLAIMS = offsetof(HostCounters, claims) / 4, H_ERR = offsetof(HostCounters, err) / 4;
    constexpr u32 H_AUX = offsetof(HostCounters, aux) / 4, H_DISC = offsetof(HostCounters, disc) / 4;
    constexpr u32 H_SENDC = offsetof(HostCounters, sendc) / 4;
    static_assert(offsetof(HostCounters, successors) == 0 && offsetof(HostCounters, cas) == 24, "host stats layout");
    const u32 nwords = 3 + NP + nparts;
    u32 claims = 0;
    for (u32 i0 = 0; i0 < nwords; i0 += 64) {
        const u32 i = i0 + lane;
        const u32* src = nullptr;
        u32 dst = 0;
        if (i == 0) src = lcw + O_CLAIMS, dst = H_CLAIMS;
        else if (i == 1) src = lcw + O_ERR, dst = H_ERR;
        else if (i == 2) src = aux, dst = H_AUX;
        else if (i < 3 + NP) src = lcw + O_DISC + (i - 3), dst = H_DISC + (i - 3);
        else if (i < nwords) src = sendc + (i - 3 - NP), dst = H_SENDC + (i - 3 - NP);
        const u32 v = src ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        if (i < nwords) hw[dst] = v;
        if (i0 == 0) claims = __shfl(v, 0, 64);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every word read before any is reset
    if (reset) {
        if (lane == 0) lc->claims = 0;
        if (lane == 1) lc->err = 0;
        if (lane >= 3 && lane < 3 + NP) lc->disc[lane - 3] = ~0u;
        if (lane == 0) lc->prev_claims = claims;
    }
    reset_stats_tickets(lc, lane, reset);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the whole wave's host stores issued and acked
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");     // system scope: host memory
    if (lane == 0) __hip_atomic_store(&h->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Standalone publish (after kernels that do not publish themselves).
template <int = 0> __global__ void publish_kernel(LevelCounters* lc, HostCounters* h, u32 seq, u32 reset, const u32* aux) {
    publish<MAX_PROPS>(lc, h, seq, reset != 0, aux);
}

// ---- per-level counter slots (the pipelined FAST level loop) ----
// A level's publish (ticket, gather, host stores, system fence, seq) used to end every expand
// launch: ~4-6 dependent round trips between the level's last workgroup and the next level. In the
// pipelined loop each level instead counts into its own slot (a ring of SLOTS); the next level's
// launch reads its frontier size from the previous slot, and its workgroup 0 publishes that slot to
// the host in wave 0 while the rest of the grid expands. The wave also resets slot K-2 for reuse:
// it was published (by launch K-1 or by slot_publish_kernel) before launch K starts. When the
// host waits for a level without having enqueued its successor, slot_publish_kernel publishes it.
constexpr u32 SLOTS = 4;
enum SlotFlags : u32 {
    // Repair pass of a level whose first pass overflowed the visited set's probe limit (the table
    // has been doubled since): every successor is probed again, the states still missing are
    // claimed and appended after the ones the first pass appended; successors are not counted
    // again (the first pass counted every one of them).
    SLOT_REPAIR = 1,
};
struct SlotWork {
    const u32* prev_n;          // frontier size = the previous level's claims (nullptr: `hi` is exact);
                                // prev_n[1] is that level's err word: a launch behind a failed level
                                // expands nothing
    const LevelCounters* pub;   // slot to publish (nullptr: none)
    HostCounters* hc;           // its host mirror
    u32 seq;                    // its launch's sequence number
    LevelCounters* zero;        // slot to reset (nullptr: none)
    u32 flags = 0;              // SlotFlags
    // `eventually` properties in FAST order: the EventuallyBits each parent passes on (by frontier
    // rank) and those of the states appended, written by whichever generator claims a state (the
    // reference's first insertion, src/checker/bfs.rs:246-263, in a multi-threaded order)
    const u32* peb = nullptr;
    u32* naeb = nullptr;
    // Speculative launches (prev_n): the visited-set slots the host can still fill below its growth
    // threshold, and a bound on new states per parent (x 256). A frontier of nn states for which
    // nn * (1 + g) exceeds that room, or nn * g the arena left after it, is not expanded (ERR_DEFERRED):
    // the host's plan assumed a smaller frontier, and overfilling a linear-probe table makes every
    // probe walk long runs (increment_lock's x5 levels: a 4 M-slot table at 0.78 load, then past it).
    u64 room = 0;  // (absolute: the growth threshold; the device adds the unique states before the level)
    u32 gmul = 0;  // 0: no check
    // Slotted launches of the pipelined loop record their frontier's successor offset and the unique
    // count in their slot (LevelCounters.next_base / .unique; arena != nullptr). `fbase` is this launch's
    // frontier offset in the arena and `ubase` the unique states before that frontier, both known to
    // the host, unless the launch is CHAINED: enqueued two levels ahead (the host has not read the
    // level before it), it takes both from the previous slot `chain`, and its frontier, next frontier
    // and arena room from `arena` / `apar` / `arena_cap`.
    const LevelCounters* chain = nullptr;
    u64* arena = nullptr;
    u32* apar = nullptr;
    u64 arena_cap = 0;
    u64 fbase = 0;
    u64 ubase = 0;
};

// One wave (lane = 0..63): publish sw.pub to sw.hc, then reset sw.zero.
template <int NP>
__device__ __forceinline__ void slot_service(const SlotWork& sw, u32 lane) {
    if (sw.pub) {
        const LevelCounters* lc = sw.pub;
        u32* hw = reinterpret_cast<u32*>(sw.hc);
        const u64 st = gather_stats(lc, lane);
        if ((lane & 15) == 0) {
            hw[(lane >> 4) * 2] = (u32)st;
            hw[(lane >> 4) * 2 + 1] = (u32)(st >> 32);
        }
        // lane 0 claims, 1 err, 2 aux (0), 3 + p disc[p]
        const u32* src = lane == 0 ? &lc->claims : lane == 1 ? &lc->err : lane >= 3 && lane < 3 + NP ? &lc->disc[lane - 3] : nullptr;
        const u32 v = src ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        if (lane == 0) sw.hc->claims = v;
        if (lane == 1) sw.hc->err = v;
        if (lane == 2) sw.hc->aux = 0;
        if (lane >= 3 && lane < 3 + NP) sw.hc->disc[lane - 3] = v;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the whole wave's host stores issued and acked
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");     // system scope: host memory
        if (lane == 0) __hip_atomic_store(&sw.hc->seq, sw.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (sw.zero) {
        LevelCounters* z = sw.zero;
        reinterpret_cast<u64*>(&z->stat[lane & (NSHARD - 1)])[lane >> 4] = 0;
        if (lane == 0) z->claims = 0;
        if (lane == 1) z->err = 0;
        if (lane < MAX_PROPS) z->disc[lane] = ~0u;
    }
}

template <int NP>
__global__ void slot_publish_kernel(SlotWork sw) {
    slot_service<NP>(sw, threadIdx.x);
}

// Probe loads of the visited set. POL selects the cache policy of the plain probe load:
// 0 default, 1 agent-scope relaxed atomic load (sc1), 2 non-temporal, 3 system-scope (sc0 sc1).
template <int POL, class T>
__device__ __forceinline__ T probe_load(const T* p) {
    if constexpr (POL == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (POL == 2) return __builtin_nontemporal_load(p);
    else if constexpr (POL == 3) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else return *p;
}

// Find key k or claim a vacant slot for it, starting at its home slot whose value `cur` was
// already loaded. Returns the slot; *is_new tells whether we claimed it.
// *probes / *cas (optional) count the further slot loads and the CAS attempts.
template <int POL = 0>
__device__ __forceinline__ u64 find_or_claim_from(const TableView& t, const ProbeKey& k, u64 cur, bool* is_new,
                                                  u32* err, u32* probes = nullptr, u32* cas = nullptr) {
    const u64 step = probe_step(t);
    const int limit = (int)t.plimit;
    u64 i = k.home, key = k.tag;
    for (int probe = 0; probe < limit; ++probe) {
        if (cur == key) {
            *is_new = false;
            return i;
        }
        if (cur == 0) {
            if (cas) ++*cas;
            const u64 prev = slot_cas(t, i, key);
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
        key += step;
        cur = slot_load<POL>(t, i);
        if (probes) ++*probes;
    }
    atomicOr(err, (u32)ERR_TABLE_FULL);
    *is_new = false;
    return ~0ull;
}

__device__ __forceinline__ u64 find_or_claim(const TableView& t, const ProbeKey& k, bool* is_new, u32* err) {
    return find_or_claim_from(t, k, slot_load(t, k.home), is_new, err);
}

// Lookup only.
__device__ __forceinline__ u64 find_slot(const TableView& t, const ProbeKey& k) {
    const u64 step = probe_step(t);
    u64 i = k.home, key = k.tag;
    for (int probe = 0; probe < MAX_PROBE; ++probe) {
        const u64 cur = slot_load(t, i);
        if (cur == key) return i;
        if (cur == 0) return ~0ull;
        i = (i + 1) & t.mask;
        key += step;
    }
    return ~0ull;
}

template <class M, class F>
__host__ __device__ __forceinline__ void for_each_successor(const M& m, const u64* s, F&& f) {
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

template <int W>
__device__ __forceinline__ bool same_state(const u64* a, const u64* b) {
    bool eq = true;
#pragma unroll
    for (int i = 0; i < W; ++i) eq &= a[i] == b[i];
    return eq;
}

// Insert the (distinct) init states with parent None (`generated.insert(fp, None)`, bfs.rs:47-51).
template <class M>
__global__ void insert_roots(M m, TableView t, const u64* states, u32 n, LevelCounters* lc) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 s[M::W];
    load_state<M::W>(states, r, s);
    bool is_new;
    u64 slot = find_or_claim(t, probe_key(m, t, s), &is_new, &lc->err);
    if (is_new) {
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

// Orders one wave's LDS accesses across its lanes: the LDS runs a wave's operations in issue
// order, the wait retires the pending ones, and the clobber keeps the compiler from moving memory
// accesses across this point (lanes write what other lanes of the same wave read next).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Lane `src` of v, for a wave-uniform src: v_readlane into a scalar register (a __shfl is an LDS
// permute, one LDS round trip on the chain).
__device__ __forceinline__ u32 lane_u32(u32 v, u32 src) { return (u32)__builtin_amdgcn_readlane((int)v, (int)src); }

// Inclusive prefix sum of v over the 64 lanes of a wave, VALU only: DPP row shifts 1, 2, 4, 8 scan
// each row of 16 lanes, then row_bcast:15 adds row 0's total to row 1 (and row 2's to row 3) and
// row_bcast:31 adds rows 0-1 to rows 2-3 (GFX9 DPP). The __shfl_up form was six dependent LDS
// permutes (~0.5 us on a lone wave's chain).
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return (u32)x;
}
// Sum of v over the wave, in every lane.
__device__ __forceinline__ u32 wave_sum(u32 v) { return lane_u32(wave_incl_scan(v), 63); }

// Sum of v over the workgroup, returned to every thread (one LDS round).
__device__ __forceinline__ u32 block_sum(u32 v, u32* scratch) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    u32 t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += scratch[w];
    __syncthreads();
    return t;
}

// 64-bit sum of v over the workgroup, returned to every thread (one LDS round; sc: a u64 per wave).
__device__ __forceinline__ u64 block_sum64(u64 v, u64* sc) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = v;
    __syncthreads();
    u64 t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sc[w];
    __syncthreads();
    return t;
}

// Sums of a and b over the workgroup, returned to every thread (one LDS round for both).
__device__ __forceinline__ void block_sum2(u32 a, u32 b, u32* scratch, u32& ta, u32& tb) {
    a = wave_sum(a);
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0) {
        scratch[2 * (threadIdx.x >> 6)] = a;
        scratch[2 * (threadIdx.x >> 6) + 1] = b;
    }
    __syncthreads();
    ta = tb = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        ta += scratch[2 * w];
        tb += scratch[2 * w + 1];
    }
    __syncthreads();
}

// k-th set bit (0-based) of a 64-bit mask with popcount(m) > k.
__device__ __forceinline__ u32 select_bit(u64 m, u32 k) {
    // the half first, then five steps on 32 bits (u64 shifts and masks cost two VALU each)
    const u32 lo = (u32)m, clo = (u32)__popc(lo);
    const bool up = k >= clo;
    u32 x = up ? (u32)(m >> 32) : lo, pos = up ? 32u : 0u;
    k -= up ? clo : 0u;
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const u32 c = (u32)__popc(x & ((1u << w) - 1));
        const bool u = k >= c;
        k -= u ? c : 0u;
        x = u ? x >> w : x;
        pos += u ? (u32)w : 0u;
    }
    return pos;
}

// Diagnostic build only (SR_TIMELINE=1, scripts/build_timeline.sh): expand_fast's lane 0 of wave 0
// stamps s_memrealtime (a 100 MHz clock shared by every CU) at each link of its workgroup's chain
// of dependent round trips, after draining its memory counters, into g_timeline[launch seq % 64]
// [block][stamp]; scripts/timeline.py turns them into the per-level breakdown. The production
// library is built with SR_TIMELINE=0 and contains none of it.
#ifndef SR_TIMELINE
#define SR_TIMELINE 0
#endif
constexpr u32 TL_STAMPS = 16, TL_BLOCKS = 2048, TL_LAUNCHES = 64;
#if SR_TIMELINE
__device__ u64* g_timeline;
#define SR_TL(k)                                                            \
    do {                                                                    \
        if (tl_on) {                                                        \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");     \
            tl_ts[k] = __builtin_amdgcn_s_memrealtime();                    \
        }                                                                   \
    } while (0)
#else
#define SR_TL(k) \
    do {         \
    } while (0)
#endif

// FAST order: expand parents [lo, hi) of the frontier.
//
// Load-balanced over SUCCESSORS: each wave loads 64 parents, counts their enabled actions, and
// then its 64 lanes walk the concatenated successor list (parent found by binary search over the
// wave's prefix sums, action = k-th set bit of that parent's mask). Lanes stay busy whatever the
// out-degree spread, and a lone parent's successors are probed in parallel. Each lane takes
// PB successors per round and issues their first visited-set probes back to back (PB loads in
// flight per lane) before resolving any of them.
//
// Every successor within boundary counts toward state_count (bfs.rs:235); one that claims a
// vacant slot is new: its parent pointer is written and the state is staged in LDS. At the end
// the workgroup reserves its span of the next frontier with ONE global atomic, copies the staged
// states out contiguously, and evaluates the properties there (rank = frontier position). A
// workgroup that stages more than STAGE states appends the overflow directly.
// STATS = 1 also counts visited-set probes and CAS attempts (sr_opts.counters): a separate
// instantiation, because the per-lane counters cost registers (SGPR spills 8 -> 47) and ~20% of
// the kernel's time.
// Wide states (W >= 4: paxos, the actor models) run three waves per SIMD (<= 168 VGPRs): their
// levels are latency-bound, and paxos' device-side history search had pushed them to two.
template <class M, int PB, int POL, bool STATS = false, bool NOPF = false, bool DYN = false>
__global__ void __launch_bounds__(64 * expand_wpb<M>()) __attribute__((amdgpu_waves_per_eu(M::W >= 4 ? SR_WIDE_WAVES : PB < 0 ? 6 : 1))) expand_fast(M m, const u64* __restrict__ frontier, u32 lo, u32 hi,
                                                   TableView t, u64* __restrict__ next, u32* __restrict__ next_par,
                                                   u32 next_cap, LevelCounters* lc, u32 undiscovered,
                                                   HostCounters* hc, u32 seq, u32 reset, u32 ppw_log2,
                                                   u32 filt_log2, SlotWork sw) {
    constexpr int W = M::W, MW = M::MW;
    // (narrow states: SR_STAGE_WORDS states per 4 waves whatever W; increment_lock's two-word states,
    // every successor new, flush half as often as with that many words: N=10 3.63 -> 3.32 ms)
    constexpr int STAGE = W >= 4 ? SR_WIDE_STAGE_WORDS / W : SR_STAGE_WORDS * expand_wpb<M>() / 4;
    extern __shared__ u64 filt[];       // 2^filt_log2 fingerprints (dynamic LDS; 0 = no filter)
    __shared__ u64 stage[STAGE * W];
    __shared__ u32 stage_par[STAGE];
    // Parents per wave at most: wide states (paxos, W = 11) take few parents per wave (ppw_for), and
    // staging 64 of them cost 22.5 KB of LDS per block, which capped residency at 3 blocks per CU.
    constexpr u32 PPW_LOG2_MAX = W >= 4 ? SR_WIDE_PPW_LOG2_MAX : 6;
    constexpr int WPB = expand_wpb<M>();
    __shared__ u64 pst[WPB][(1 << PPW_LOG2_MAX) * W];     // parent states of each wave
    // The wave's successor list, one u16 per successor: parent (bits 0-5) | action << 6, written by
    // the parent lanes (a ctz loop over their enabled masks) in windows of MAPCAP successors. A
    // successor lane reads its (parent, action) with one LDS load; the binary search over the
    // parents' prefix sums (6 dependent LDS loads) and the k-th-set-bit select it replaces were
    // the largest per-successor costs.
#ifndef SR_MAPCAP
#define SR_MAPCAP 1024
#endif
    // (wide states: ~2 successors per parent and <= 32 parents per wave fill a quarter of it)
#ifndef SR_WIDE_MAPCAP
#define SR_WIDE_MAPCAP 256
#endif
    constexpr u32 MAPCAP = W >= 4 ? SR_WIDE_MAPCAP : SR_MAPCAP;
    static_assert(MW * 64 <= 1024, "action ids must fit 10 bits");
    __shared__ u16 smap[WPB][MAPCAP];
    __shared__ u32 stage_n, base, scratch[2 * WPB];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) stage_n = 0;
    // The previous level's publish and the slot reset (SlotWork) run in one extra workgroup, the
    // last of the grid: in a small level any workgroup that expands parents is on the critical
    // path, and the publish waits for its host stores to be acknowledged.
#if SR_TIMELINE
    // stamps: 0 entry, 1 frontier size known, 2 first parents loaded, 3 first successor map, 4 first
    // probes returned, 5 first claims done, 6 chunks done, 7 stage reserved, 8 stage written,
    // 9 exit (service workgroup: 0 entry, 9 exit)
    const bool tl_on = threadIdx.x == 0 && blockIdx.x < TL_BLOCKS && g_timeline;
    u64 tl_ts[TL_STAMPS];
#pragma unroll
    for (u32 k = 0; k < TL_STAMPS; ++k) tl_ts[k] = 0;
    bool tl_first_chunk = true, tl_first_round = true;
    auto tl_store = [&]() {
        if (!tl_on) return;
        u64* t = g_timeline + ((u64)(seq % TL_LAUNCHES) * TL_BLOCKS + blockIdx.x) * TL_STAMPS;
#pragma unroll
        for (u32 k = 0; k < TL_STAMPS; ++k) t[k] = tl_ts[k];
        t[TL_STAMPS - 1] = (u64)gridDim.x << 32 | (u64)(hi - lo);
    };
#endif
    SR_TL(0);
    const bool svc = sw.pub || sw.zero;
    if (svc && blockIdx.x == gridDim.x - 1) {
        if (threadIdx.x < 64) slot_service<M::NPROPS>(sw, threadIdx.x);
        SR_TL(9);
#if SR_TIMELINE
        tl_store();
#endif
        return;
    }
    const u32 nblk = gridDim.x - (svc ? 1u : 0u);  // workgroups that expand parents
    // Each wave takes ppw = 2^ppw_log2 <= 64 parents (small levels use fewer parents per wave so
    // that their successors spread over more waves: shorter per-lane probe chains). The grid
    // strides over chunks of 4 waves (a pipelined launch is sized from an estimate of the frontier).
    ppw_log2 = min(ppw_log2, PPW_LOG2_MAX);
    const u32 ppw = 1u << ppw_log2;
    const u64 chunk = (u64)(blockDim.x >> 6) << ppw_log2;
    // The wave's first parents. A pipelined launch issues their load before it knows the frontier
    // size (any row below next_cap is inside the arena; rows past the frontier are never used), so
    // the two round trips overlap instead of following each other.
    const u64 r_first = lo + (u64)blockIdx.x * chunk + ((u64)wid << ppw_log2) + lane;
    u64 nxt[W];  // the wave's parents of its next chunk (here: its first)
    const bool chained = sw.chain != nullptr;  // (its frontier's offset is read below)
    const bool spec_first = sw.prev_n && !chained && lane < (int)ppw && r_first < next_cap;
    if (spec_first) load_state<W>(frontier, r_first, nxt);
    if (sw.prev_n) {
        // Pipelined launch (enqueued before the host saw the previous level finish): the frontier
        // is the previous level's claims, and the next level starts right after it. Behind a level
        // that failed (its err word, loaded with its claims) it expands nothing: the host repairs
        // or restarts that level and its frontier is not final.
        const u64 ce = __hip_atomic_load(reinterpret_cast<const u64*>(sw.prev_n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        u64 fb = sw.fbase, ub = sw.ubase;
        if (chained) {
            fb = __hip_atomic_load(&sw.chain->next_base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ub = __hip_atomic_load(&sw.chain->unique, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            frontier = sw.arena + fb * W;
            next = sw.arena + fb * W;
            next_par = sw.apar + fb;
            next_cap = (u32)min(sw.arena_cap > fb ? sw.arena_cap - fb : 0ull, 0xffffffffull);
        }
        u32 nn = (ce >> 32) ? 0u : (u32)ce;
        if (sw.gmul && nn) {
            const u64 grow = ((u64)nn * sw.gmul) >> 8;
            const u64 left = next_cap > nn ? (u64)(next_cap - nn) : 0ull;
            if (ub + nn + grow > sw.room || grow > left) {
                nn = 0;
                if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&lc->err, (u32)ERR_DEFERRED);
            }
        }
        hi = lo + nn;
        next += (u64)nn * W;
        next_par += nn;
        next_cap = next_cap > nn ? next_cap - nn : 0u;
        if (sw.arena && blockIdx.x == 0 && threadIdx.x == 0) {  // for a launch chained to this one
            lc->next_base = fb + nn;
            lc->unique = ub + nn;
        }
    } else if (sw.arena && blockIdx.x == 0 && threadIdx.x == 0) {
        lc->next_base = sw.fbase + (hi - lo);
        lc->unique = sw.ubase + (hi - lo);
    }
    SR_TL(1);
    // (the compact filter only for one-word quotient tables: FILT_COMPACT)
    const bool fcompact = M::W == 1 && has_qkey<M>::value && (filt_log2 & FILT_COMPACT) != 0;
    filt_log2 &= FILT_COMPACT - 1;
    const u32 fmask = filt_log2 ? (1u << filt_log2) - 1 : 0;
    const u32 fwords = !fmask ? 0u : fcompact ? (fmask + 1) / 2 : fmask + 1;  // u64 words of LDS
    if (lo + (u64)blockIdx.x * chunk < hi)  // blocks past the frontier only take their ticket
        for (u32 i = threadIdx.x; i < fwords; i += blockDim.x) filt[i] = 0;
    // One level: parents [lo, hi) of `frontier` into `next`.
    auto level = [&](const u64* __restrict__ frontier, u32 lo, u32 hi, u64* __restrict__ next,
                     u32* __restrict__ next_par, u32 next_cap, LevelCounters* lc, u32 undiscovered) {
    u32 succ = 0, enabled = 0, probes = 0, cas = 0;
    // The wave's parents of the next chunk are loaded one chunk ahead: their latency overlaps this
    // chunk's probes instead of stalling the chunk start.
    const u64 cstride = (u64)nblk * chunk;
    if (!spec_first && lane < (int)ppw && r_first < hi) load_state<W>(frontier, r_first, nxt);
    // Wide states without the register prefetch (NOPF: PF false): the first chunk's parents go to
    // the wave's LDS copy here, later chunks load theirs at the chunk start. The W-word prefetch
    // holds 2W VGPRs through every probe round, and a wide kernel's residency is set by its VGPRs
    // (paxos C=3: 146 -> 124 VGPRs, 3 -> 4 blocks per CU). The host takes this form for levels
    // whose chunks all fit the grid (no block strides, so nothing is prefetched anyway).
    constexpr bool PF = W < 4 || !NOPF;
    const u64 c_first = lo + (u64)blockIdx.x * chunk;
    if constexpr (!PF) {
        if (lane < (int)ppw && r_first < hi) {
#pragma unroll
            for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = nxt[i];
        }
    }
    // Dynamic chunks (SR_DYN_CHUNKS): with more than three chunks per workgroup, chunks 0 .. 3 nblk - 1
    // are static (workgroup b takes b, b + nblk, b + 2 nblk) and later ones are pulled from the
    // workgroup's shard counter (blockIdx % DYN_SHARDS; shard x hands out chunks 3 nblk + x + 8 i).
    // Thread 0 issues a pull at the end of chunk j and uses its result at the end of chunk j + 1,
    // as the chunk after next, so no wave waits for it (a returning atomic in flight holds every
    // later vmcnt wait of its wave). The chunk after next reaches the workgroup through LDS at the
    // chunk-end barrier. c_next: the chunk whose parents the prefetch loads (hi: none).
    const u64 nchunks = hi > lo ? ((u64)hi - lo + chunk - 1) / chunk : 0;
    // (only on levels of more than DYN_MIN_RATIO chunks per workgroup: the pulls cost each workgroup
    // a little on every chunk, and with few chunks per workgroup the static stride balances well
    // enough: 2pc N=9's big levels, 3.1-3.5 chunks per workgroup, were 5-8 us slower with them)
    // (DYN: a separate instantiation, chosen by the host for levels it expects to be that deep, so the
    // other levels run a kernel without this code and its registers)
    const bool dyn = DYN && SR_DYN_CHUNKS && nblk >= DYN_SHARDS && nchunks > (u64)DYN_MIN_RATIO * nblk;  // (every shard has workgroups)
    const u32 dshard = blockIdx.x % DYN_SHARDS;
    __shared__ u64 s_cnext;
    u64 c_next = c_first + cstride;
    u32 kpend = 0;            // (thread 0) the pull in flight
    bool pend = false, first_chunk = true;
    for (u64 c0 = c_first; c0 < hi;) {
        const u32 wave0 = (u32)(c0 + ((u64)wid << ppw_log2));  // first parent of the wave
        const u32 r = wave0 + lane;
        u32 cnt = 0;
        u64 s[W];
        if constexpr (PF) {
#pragma unroll
            for (int i = 0; i < W; ++i) s[i] = nxt[i];
            const u64 rn = c_next + ((u64)wid << ppw_log2) + lane;
            if (lane < (int)ppw && rn < hi) load_state<W>(frontier, rn, nxt);
        } else if (c0 != c_first && lane < (int)ppw && r < hi) {
            load_state<W>(frontier, r, s);  // (the wave's previous parents were last read by its own rounds)
#pragma unroll
            for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = s[i];
        }
        // the stage's fill is read by every thread at the end of the previous chunk before any
        // wave appends again (and the wave's parents are no longer read)
        __syncthreads();
        u64 mk[MW];
#pragma unroll
        for (int i = 0; i < MW; ++i) mk[i] = 0;
        if constexpr (has_enabled_slot<M>::value) {
            // One lane per (parent, slot): PPP parents per pass, their masks assembled from the
            // pass's ballot (has_enabled_slot). The parents are read from the wave's LDS copy.
            static_assert(MW == 1 && M::ESLOTS <= 64 && 64 % M::ESLOTS == 0, "enabled_slot: ESLOTS must divide 64");
            static_assert(!has_self_loops<M>::value, "enabled_slot: no self_loops hook");
            constexpr u32 ES = M::ESLOTS, PPP = 64 / ES;
            if (PF && lane < (int)ppw && r < hi) {
#pragma unroll
                for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = s[i];
            }
            wave_lds_sync();
            const u32 np = hi > wave0 ? min(ppw, hi - wave0) : 0u;  // this wave's parents (uniform)
            u64 mine = 0;
            for (u32 p0 = 0; p0 < np; p0 += PPP) {
                const u32 p = p0 + (u32)lane / ES, k = (u32)lane % ES;
                const bool en = p < np && m.enabled_slot(&pst[wid][p * W], (int)k);
                const u64 b = __ballot(en);
                const u32 i = (u32)lane - p0;
                if ((u32)lane >= p0 && i < PPP) mine = ES == 64 ? b : (b >> (i * ES)) & ((1ull << (ES % 64)) - 1);
            }
            if (lane < (int)ppw && r < hi) {
                mk[0] = mine;
                cnt = (u32)__popcll(mine);
            }
#if SR_TIMELINE
            if (tl_first_chunk) SR_TL(2);
            if (tl_first_chunk) SR_TL(10);
#endif
        } else
        if (lane < ppw && r < hi) {
            if constexpr (!PF) {
#pragma unroll
                for (int i = 0; i < W; ++i) s[i] = pst[wid][lane * W + i];  // (this lane's own LDS words)
            }
            m.enabled(s, mk);
#if SR_TIMELINE
            if (tl_first_chunk) SR_TL(2);
#endif
            if constexpr (has_self_loops<M>::value) {
                // self-loops are counted here and never generated (has_self_loops)
                u64 sl[MW];
                m.self_loops(s, mk, sl);
#pragma unroll
                for (int i = 0; i < MW; ++i) {
                    succ += __popcll(sl[i]);
                    mk[i] &= ~sl[i];
                }
            }
            if constexpr (PF) {
#pragma unroll
                for (int i = 0; i < W; ++i) pst[wid][lane * W + i] = s[i];
            }
#pragma unroll
            for (int i = 0; i < MW; ++i) cnt += __popcll(mk[i]);
#if SR_TIMELINE
            if (tl_first_chunk) SR_TL(10);
#endif
        }
        // wave-inclusive scan of the counts
        const u32 incl = wave_incl_scan(cnt);
        u32 nidx = incl - cnt;  // this parent's next successor index (its entries are [excl, incl))
        const u32 total = lane_u32(incl, 63);
        if (lane == 0) enabled += total;
#if SR_TIMELINE
        if (tl_first_chunk) SR_TL(11);
#endif

        // Appends the wave's new states of one round: one LDS atomic reserves the wave's span of the
        // stage; what does not fit goes straight to the next frontier with ONE global atomic for the
        // wave (never one per state).
        auto append_new = [&](bool nw, const u64* ns, u32 par) {
            const u64 mask = __ballot(nw);
            if (!mask) return;
            const u32 cnt = __popcll(mask);
            const u32 below = __popcll(mask & ((1ull << lane) - 1));
            const int leader = __builtin_ctzll(mask);
            u32 sb = 0;
            if (lane == leader) sb = atomicAdd(&stage_n, cnt);
            sb = lane_u32(sb, (u32)leader);
            const u32 in_stage = sb >= (u32)STAGE ? 0u : min(cnt, (u32)STAGE - sb);
            u32 gb = 0;
            if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
            gb = lane_u32(gb, (u32)leader);
            if (!nw) return;
            const u32 pr = wave0 + par;  // parent rank
            if (below < in_stage) {
                const u32 kk = sb + below;
#pragma unroll
                for (int x = 0; x < W; ++x) stage[kk * W + x] = ns[x];
                stage_par[kk] = pr;
            } else {
                const u32 pos = gb + (below - in_stage);
                if (pos < next_cap) {
                    store_state<W>(next, pos, ns);
                    next_par[pos] = pr;
                    if (sw.naeb) sw.naeb[pos] = sw.peb[pr];
                } else {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                }
                eval_props(m, ns, pos, undiscovered, lc);
            }
        };
        for (u32 w0 = 0; w0 < total; w0 += MAPCAP) {
        const u32 wend = min(total, w0 + MAPCAP);
        if (MW <= 2 && ppw <= 8) {
            // Few parents per wave (small levels): the 64 lanes fill the map together, entry j
            // from parent p (the last whose exclusive offset is <= j) and its (j - offset)-th
            // enabled slot, instead of every parent lane writing its own successors one by one
            // (up to ~20 dependent iterations for a wave that is alone on its CU).
            const u32 excl = incl - cnt;
            for (u32 j0 = w0; j0 < wend; j0 += 64) {
                const u32 j = j0 + (u32)lane;
                u32 p = 0;
#pragma unroll
                for (int q = 1; q < 8; ++q) {
                    const u32 ex = lane_u32(excl, (u32)q);
                    if ((u32)q < ppw && ex <= j) p = (u32)q;
                }
                const u32 k = j - (u32)__shfl((int)excl, (int)p, 64);
                const u64 m0 = __shfl(mk[0], (int)p, 64);
                const u64 m1 = MW > 1 ? __shfl(mk[MW > 1 ? 1 : 0], (int)p, 64) : 0ull;
                const u32 c0 = (u32)__popcll(m0);
                const u32 a = k < c0 ? select_bit(m0, k) : 64u + select_bit(m1, k - c0);
                if (j < wend) smap[wid][j - w0] = (u16)(p | a << 6);
            }
        } else
        // this window's entries: each parent lane writes its successors with index in [w0, wend)
        while (nidx < wend && nidx < incl) {
            u32 a = 0;
#pragma unroll
            for (int w = MW - 1; w >= 0; --w)  // the lowest set bit over the mask words
                if (mk[w]) a = (u32)w * 64 + (u32)__builtin_ctzll(mk[w]);
            mk[a >> 6] &= mk[a >> 6] - 1;
            smap[wid][nidx - w0] = (u16)((u32)lane | a << 6);
            ++nidx;
        }
#if SR_TIMELINE
        if (tl_first_chunk) SR_TL(12);
#endif
        wave_lds_sync();  // pst and the map are the wave's own: no workgroup barrier
#if SR_TIMELINE
        if (tl_first_chunk) SR_TL(3);
        tl_first_chunk = false;
#endif

        if constexpr (PB < 0) {
            // Per-lane probe queue over R = -PB rounds of the window (DESIGN.md §3 "probe loops").
            // Phase A expands R rounds of successors with every lane busy (apply, fingerprint, the
            // LDS filter) and keeps each lane's probe keys in registers; phase B walks each lane's
            // keys one visited-set access per iteration (home load, linear-probe step or claim CAS),
            // a lane moving to its next key as soon as one resolves, so the wave's round trips are
            // not each as long as its slowest lane's chain. New states are appended after phase B
            // (their states recomputed from the map: only ~1 successor in 8 is new).
            constexpr int R = -PB;
            // without a packed key the table is always in fingerprint mode: home = tag & mask
            constexpr bool FP_ONLY = !has_qkey<M>::value;
            for (u32 s0 = w0; s0 < wend; s0 += 64u * R) {
                u64 kh[FP_ONLY ? 1 : R], kt[R];  // home slot and slot value of round r's successor
                u32 vmask = 0;     // bit r: round r's successor is probed
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (!FP_ONLY) kh[FP_ONLY ? 0 : r] = 0;
                    kt[r] = 0;
                    const u32 i = s0 + (u32)r * 64u + (u32)lane;
                    if (i < wend) {
                        const u32 e = smap[wid][i - w0];
                        const u32 p = e & 63, a = e >> 6;
                        u64 ps[W], q[W];
#pragma unroll
                        for (int x = 0; x < W; ++x) ps[x] = pst[wid][p * W + x];
                        bool ok = m.apply(ps, (int)a, q);
                        if (ok) {
                            ++succ;  // within boundary: counted once, whatever follows
                            ok = !same_state<W>(q, ps);  // self-loop: never probed
                        }
                        if (ok) {
                            const ProbeKey k = probe_key(m, t, q);
                            if (fmask)  // block-local duplicate filter (see the round loop below)
                                ok = !filter_seen(filt, fcompact, filt_log2, fmask, t, filter_key(t, k));
                            if (!FP_ONLY) kh[FP_ONLY ? 0 : r] = k.home;
                            kt[r] = k.tag;
                        }
                        if (ok) vmask |= 1u << r;
                    }
                }
#if SR_TIMELINE
                if (tl_first_round) SR_TL(4);
#endif
                u32 nmask = 0;  // bit r: round r's successor claimed a vacant slot (a new state)
                u32 st = 0, cr = 0, disp = 0;  // 0 idle, 1 load pending, 2 claim pending; its round
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
                    if (st == 1) v = slot_load<POL>(t, si);
                    if (st == 2) v = slot_cas(t, si, tag);
                    if constexpr (STATS) {
                        probes += st == 1;
                        cas += st == 2;
                    }
                    if (st != 0) {
                        if (v == tag) {
                            st = 0;  // visited already (or claimed by a concurrent duplicate)
                        } else if (v == 0) {
                            if (st == 2) nmask |= 1u << cr;  // our claim won
                            st = st == 1 ? 2u : 0u;
                        } else if (++disp >= t.plimit) {
                            atomicOr(&lc->err, (u32)ERR_TABLE_FULL);
                            st = 0;
                        } else {  // another key: the next slot
                            si = (si + 1) & t.mask;
                            tag += step;
                            st = 1;
                        }
                    }
                }
#if SR_TIMELINE
                if (tl_first_round) SR_TL(5);
                tl_first_round = false;
#endif
                // the new states, round by round (their states recomputed from the map)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool nw = nmask >> r & 1;
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
                    append_new(nw, q, p);
                }
            }
        } else
        for (u32 it = w0; it < wend; it += 64 * PB) {
            u64 ns[PB][W], cur[PB];
            ProbeKey pk[PB];
            u32 par[PB];
            bool ok[PB];
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
                    if (ok[j] && same_state<W>(ns[j], ps)) {  // self-loop: counted, never probed
                        ++succ;
                        ok[j] = false;
                    }
                }
                pk[j] = ok[j] ? probe_key(m, t, ns[j]) : ProbeKey{0, 0};
                // Block-local duplicate filter: a direct-mapped LDS cache of the fingerprints this
                // workgroup already sent to the visited set. Siblings' successors coincide often
                // (commuting actions), and a hit is a duplicate of a state whose probe another lane
                // of this block owns — counted, never probed again. A miss (or an eviction) only
                // costs the ordinary probe, so the filter never changes which states are new.
                // (Keyed on filter_key, injective on states; the host turns the filter off for
                // multi-word quotient-mode tables.)
                if (fmask && ok[j]) {
                    if (filter_seen(filt, fcompact, filt_log2, fmask, t, filter_key(t, pk[j]))) {
                        ++succ;
                        ok[j] = false;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                cur[j] = ok[j] ? slot_load<POL>(t, pk[j].home) : 0;
                if constexpr (STATS) probes += ok[j];
            }
#if SR_TIMELINE
            if (tl_first_round) SR_TL(4);
#endif
            bool nw[PB];
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                nw[j] = false;
                if (!ok[j]) continue;
                ++succ;
                if (cur[j] == pk[j].tag) continue;  // the common case: an already visited state
                find_or_claim_from<POL>(t, pk[j], cur[j], &nw[j], &lc->err, STATS ? &probes : nullptr,
                                        STATS ? &cas : nullptr);
            }
#if SR_TIMELINE
            if (tl_first_round) SR_TL(5);
            tl_first_round = false;
#endif
            // Append the new states of this round, aggregated per wave: one LDS atomic reserves the
            // wave's span of the stage; what does not fit goes straight to the next frontier with
            // ONE global atomic for the wave (never one per state).
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                const u64 mask = __ballot(nw[j]);
                if (!mask) continue;
                const u32 cnt = __popcll(mask);
                const u32 below = __popcll(mask & ((1ull << lane) - 1));
                const int leader = __builtin_ctzll(mask);
                u32 sb = 0;
                if (lane == leader) sb = atomicAdd(&stage_n, cnt);
                sb = lane_u32(sb, (u32)leader);
                const u32 in_stage = sb >= (u32)STAGE ? 0u : min(cnt, (u32)STAGE - sb);
                u32 gb = 0;
                if (cnt > in_stage && lane == leader) gb = atomicAdd(&lc->claims, cnt - in_stage);
                gb = lane_u32(gb, (u32)leader);
                if (!nw[j]) continue;
                const u32 pr = wave0 + par[j];  // parent rank
                if (below < in_stage) {
                    const u32 kk = sb + below;
#pragma unroll
                    for (int x = 0; x < W; ++x) stage[kk * W + x] = ns[j][x];
                    stage_par[kk] = pr;
                } else {
                    const u32 pos = gb + (below - in_stage);
                    if (pos < next_cap) {
                        store_state<W>(next, pos, ns[j]);
                        next_par[pos] = pr;
                        if (sw.naeb) sw.naeb[pos] = sw.peb[pr];
                    } else {
                        atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                    }
                    eval_props(m, ns[j], pos, undiscovered, lc);
                }
            }
        }
        wave_lds_sync();  // the window's map is read before the next window overwrites it
        }
        // A block that strides over several chunks (a grid capped below the frontier) flushes its
        // stage once it is half full: otherwise it stays full after the first chunks and every
        // later append becomes a per-wave atomic on the one claims counter (2pc N=11: 478 ms per
        // check instead of 80).
        if (dyn && threadIdx.x == 0) {
            u64 cn = hi;  // the chunk after c_next
            if (first_chunk) {
                cn = c_first + 2 * cstride;  // static
            } else if (pend) {
                const u64 k = 3ull * nblk + dshard + (u64)DYN_SHARDS * kpend;
                if (k < nchunks) cn = lo + k * chunk;
            }
            pend = cn < hi;
            if (pend) {  // used at the next chunk end
                // (an offset the compiler cannot prove uniform: the atomic optimizer would otherwise
                // turn the pull into a wave reduction whose result is waited for at once)
                u32 zoff;
                asm volatile("v_mov_b32 %0, 0" : "=v"(zoff));
                kpend = atomicAdd(&lc->chunk_next[dshard][0] + zoff, 1u);
            }
            s_cnext = cn;
        }
        first_chunk = false;
        __syncthreads();
        c0 = c_next;
        c_next = dyn ? s_cnext : c_next + cstride;  // (s_cnext is rewritten only after the next chunk-end barrier)
        if (stage_n >= (u32)STAGE / 2) {
            const u32 nst = min(stage_n, (u32)STAGE);
            if (threadIdx.x == 0) base = atomicAdd(&lc->claims, nst);
            __syncthreads();
            for (u32 i = threadIdx.x; i < nst; i += blockDim.x) {
                const u32 pos = base + i;
                u64 ns[W];
#pragma unroll
                for (int x = 0; x < W; ++x) ns[x] = stage[i * W + x];
                if (pos < next_cap) {
                    store_state<W>(next, pos, ns);
                    next_par[pos] = stage_par[i];
                    if (sw.naeb) sw.naeb[pos] = sw.peb[stage_par[i]];
                } else {
                    atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
                }
                eval_props(m, ns, pos, undiscovered, lc);
            }
            __syncthreads();
            if (threadIdx.x == 0) stage_n = 0;
        }
    }
    if (dyn && threadIdx.x == 0 && atomicAdd(&lc->chunk_done, 1u) == nblk - 1) {
        // every workgroup has pulled its last chunk: the counters back to zero for the slot's next launch
#pragma unroll
        for (u32 x = 0; x < DYN_SHARDS; ++x) atomicExch(&lc->chunk_next[x][0], 0u);
        atomicExch(&lc->chunk_done, 0u);
    }
    SR_TL(6);
    const bool repair = (sw.flags & SLOT_REPAIR) != 0;  // successors were counted by the first pass
    // The stage's span of the next frontier is reserved first; the round trip of that atomic
    // overlaps the block's reduction of its statistics (both sums in one pass).
    __syncthreads();  // the stage's fill is final
    const u32 n = min(stage_n, (u32)STAGE);
    u32 my_base = 0;
    if (threadIdx.x == 0 && n) my_base = atomicAdd(&lc->claims, n);
    u32 total_succ, total_enabled;
    block_sum2(repair ? 0u : succ, repair ? 0u : enabled, scratch, total_succ, total_enabled);
    u32 total_probes = STATS ? block_sum(probes, scratch) : 0u;
    u32 total_cas = STATS ? block_sum(cas, scratch) : 0u;
    if (threadIdx.x == 0) {
        base = my_base;
        add_stats(lc, total_succ, total_enabled, total_probes, total_cas);
    }
    SR_TL(7);
    __syncthreads();
    for (u32 i = threadIdx.x; i < n; i += blockDim.x) {
        u32 pos = base + i;
        u64 ns[W];
#pragma unroll
        for (int x = 0; x < W; ++x) ns[x] = stage[i * W + x];
        if (pos < next_cap) {
            store_state<W>(next, pos, ns);
            next_par[pos] = stage_par[i];
            if (sw.naeb) sw.naeb[pos] = sw.peb[stage_par[i]];
        } else {
            atomicOr(&lc->err, (u32)ERR_FRONTIER_OVERFLOW);
        }
        eval_props(m, ns, pos, undiscovered, lc);
    }
    };
    level(frontier, lo, hi, next, next_par, next_cap, lc, undiscovered);
    SR_TL(8);
    if (hc) publish<M::NPROPS>(lc, hc, seq, reset != 0, nullptr);  // a slotted launch is published by its successor
    SR_TL(9);
#if SR_TIMELINE
    tl_store();
#endif
}

// FIFO order, pass 1: insert-or-find every successor and record (level, parent rank, slot) in
// meta with atomicMin, so that the minimum — the generator the reference's single-threaded queue
// sees first (push_front/pop_back, bfs.rs:183,263) — owns each new state. The plain load of meta
// first skips the atomic whenever it cannot lower the value (meta only decreases within a level).
// Candidates go to cand[a * n + r] (action-major, so passes 2-3 read it coalesced).
template <class M>
__global__ void __launch_bounds__(256) expand_fifo(M m, const u64* __restrict__ frontier, u32 lo, u32 hi, u32 n,
                                                   TableView t, u32* __restrict__ cand, u32 A, u32 level,
                                                   LevelCounters* lc, HostCounters* hc, u32 seq, u32 count_succ) {
    __shared__ u32 scratch[4];
    const u32 r = lo + blockIdx.x * blockDim.x + threadIdx.x;
    u32 succ = 0, claims = 0;
    if (r < hi) {
        u64 s[M::W];
        load_state<M::W>(frontier, r, s);
        const u64 lvl = (u64)(level + 1) << META_SHIFT;
        for_each_successor(m, s, [&](int a, const u64* ns) {
            succ += count_succ;  // 0 in the repair pass of a chunk that overflowed the probe limit
            if (same_state<M::W>(ns, s)) return;  // self-loop: the parent is visited already
            bool is_new;
            u64 slot = find_or_claim(t, probe_key(m, t, ns), &is_new, &lc->err);
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
        add_stats(lc, ts, 0);
        if (tc) atomicAdd(&lc->claims, tc);
    }
    publish<M::NPROPS>(lc, hc, seq, false, nullptr);
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
__device__ __forceinline__ void scatter_fifo_body(M m, const u64* __restrict__ frontier, const u32* __restrict__ cand,
                                                  const u32* __restrict__ offs, u32 n, u32 A, u32 level,
                                                  TableView t, u64* __restrict__ next, u32* __restrict__ next_par,
                                                  LevelCounters* lc, u32 undiscovered,
                                                  const u32* __restrict__ peb = nullptr, u32* __restrict__ next_eb = nullptr) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u64 lvl = (u64)(level + 1) << META_SHIFT;
    const u32 eb = peb ? peb[r] : 0u;  // the parent's EventuallyBits after its pop (bfs.rs:263)
    u64 s[M::W];
    bool loaded = false;
    u32 j = offs[r];
    for (u32 a = 0; a < A; ++a) {
        u32 slot = cand[(u64)a * n + r];
        if (slot == CAND_NONE || t.meta[slot] != (lvl | ((u64)r * A + a))) continue;
        if (!loaded) {
            load_state<M::W>(frontier, r, s);
            loaded = true;
        }
        u64 ns[M::W];
        m.apply(s, (int)a, ns);
        store_state<M::W>(next, j, ns);
        next_par[j] = r;
        if (next_eb) next_eb[j] = eb;
        eval_props(m, ns, j, undiscovered, lc);
        ++j;
    }
}

template <class M>
__global__ void __launch_bounds__(256) scatter_fifo(M m, const u64* __restrict__ frontier, const u32* __restrict__ cand,
                                                    const u32* __restrict__ offs, u32 n, u32 A, u32 level,
                                                    TableView t, u64* __restrict__ next, u32* __restrict__ next_par,
                                                    LevelCounters* lc, u32 undiscovered, HostCounters* hc, u32 seq,
                                                    const u32* owners, const u32* peb, u32* next_eb) {
    scatter_fifo_body(m, frontier, cand, offs, n, A, level, t, next, next_par, lc, undiscovered, peb, next_eb);
    publish<M::NPROPS>(lc, hc, seq, true, owners);
}

// ---- `eventually` properties (src/checker/bfs.rs:52-60,212-222,265-272), FIFO order only ----
// Each frontier state carries EventuallyBits (one bit per eventually property still unmet on its
// BFS-tree path). At its pop a state clears the bits of undiscovered properties whose condition
// holds; a TERMINAL state (no successor within boundary) with a bit still set is a discovery, and
// `discoveries.insert` OVERWRITES, so the reported discovery is the last such terminal state in
// visit order. Pass 1 finds, per undiscovered property, the first terminal candidate of the level
// (which is where the property becomes discovered; from then on its bit is no longer cleared).
template <class M>
__global__ void __launch_bounds__(256) ev_scan(M m, const u64* __restrict__ frontier, const u32* __restrict__ eb_in,
                                               u32 n, u32 eund, u32 emask, u32* __restrict__ tsat, u32* evf) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    u64 s[M::W];
    load_state<M::W>(frontier, r, s);
    bool any = false;
    for_each_successor(m, s, [&](int, const u64*) { any = true; });
    u32 sat = 0;
    for (u32 e = emask; e; e &= e - 1) {
        const int p = __builtin_ctz(e);
        if (m.discovers(p, s)) sat |= 1u << p;
    }
    tsat[r] = sat | (any ? 0u : 0x80000000u);
    if (!any)
        for (u32 c = eb_in[r] & ~sat & eund; c; c &= c - 1) atomicMin(&evf[__builtin_ctz(c)], r);
}

// Pass 2 over the expanded ranks [0, limit): the bits each state passes to its children, and per
// property the LAST terminal state (rank + 1) whose bits still hold it.
template <int = 0> __global__ void __launch_bounds__(256) ev_resolve(const u32* __restrict__ tsat, const u32* __restrict__ eb_in, u32 limit,
                                                  u32 eund, const u32* __restrict__ evf, u32* __restrict__ peb,
                                                  u32* evl) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= limit) return;
    const u32 ts = tsat[r], sat = ts & 0x7fffffffu;
    u32 clear = 0;
    for (u32 c = sat & eund; c; c &= c - 1) {
        const int p = __builtin_ctz(c);
        if (r <= evf[p]) clear |= 1u << p;  // still undiscovered at this pop
    }
    const u32 eff = eb_in[r] & ~clear;
    peb[r] = eff;
    if (ts >> 31)
        for (u32 c = eff; c; c &= c - 1) atomicMax(&evl[__builtin_ctz(c)], r + 1);
}

template <int = 0> __global__ void fill_u32(u32* p, u32 n, u32 v) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
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

// The roots in ONE workgroup (n <= blockDim.x init states): insert_roots + eval_roots + the
// resetting publish, one launch instead of three at the start of every check.
template <class M>
__global__ void __launch_bounds__(256) roots_fused(M m, TableView t, const u64* states, u32 n, LevelCounters* lc,
                                                   u32 undiscovered, HostCounters* h, u32 seq) {
    const u32 r = threadIdx.x;
    if (r < n) {
        u64 s[M::W];
        load_state<M::W>(states, r, s);
        bool is_new;
        const u64 slot = find_or_claim(t, probe_key(m, t, s), &is_new, &lc->err);
        if (is_new) {
            if (t.meta) t.meta[slot] = 0;  // level 0
            atomicAdd(&lc->claims, 1u);
        }
        for (u32 und = undiscovered; und; und &= und - 1) {
            const int p = __builtin_ctz(und);
            if (m.discovers(p, s)) atomicMin(&lc->disc[p], r);
        }
    }
    publish<M::NPROPS>(lc, h, seq, true, nullptr);
}

// Device counters and the pipelined loop's counter slots to their level-start values (no host
// buffer, so no host wait at the start of a check).
__device__ __forceinline__ void init_counter_words(LevelCounters* lc, LevelCounters* slots, u32 nslots) {
    constexpr u32 WORDS = sizeof(LevelCounters) / 4;
    constexpr u32 D0 = offsetof(LevelCounters, disc) / 4;
    for (u32 i = threadIdx.x; i < WORDS * (1 + nslots); i += blockDim.x) {
        const u32 o = i % WORDS;
        u32* w = i < WORDS ? reinterpret_cast<u32*>(lc) + i : reinterpret_cast<u32*>(slots) + (i - WORDS);
        *w = o >= D0 && o < D0 + MAX_PROPS ? ~0u : 0u;
    }
}
template <int = 0> __global__ void init_level_counters(LevelCounters* lc, LevelCounters* slots, u32 nslots) {
    init_counter_words(lc, slots, nslots);
}

// The whole start of a check in ONE launch when the init states fit the kernel arguments (every
// model here has a handful): the counters and counter slots reset (init_level_counters), level 0
// written to the arena with no parents (and, for `eventually` models, every property pending),
// then roots_fused. Replaces a host-to-device copy, two fills and two launches per check.
constexpr u32 ROOTS_INLINE_WORDS = 32;
struct InlineStates {
    u64 w[ROOTS_INLINE_WORDS];
};
template <class M>
__global__ void __launch_bounds__(256) roots_start(M m, TableView t, InlineStates init, u32 n, u64* arena, u32* apar,
                                                   u32* aeb, u32 emask, LevelCounters* lc, LevelCounters* slots,
                                                   u32 nslots, u32 undiscovered, HostCounters* h, u32 seq) {
    constexpr int W = M::W;
    init_counter_words(lc, slots, nslots);
    for (u32 i = threadIdx.x; i < n * W; i += blockDim.x) arena[i] = init.w[i];
    for (u32 i = threadIdx.x; i < n; i += blockDim.x) {
        apar[i] = ~0u;
        if (aeb) aeb[i] = emask;
    }
    __syncthreads();  // the counters are reset before any thread claims or counts into them
    const u32 r = threadIdx.x;
    if (r < n) {
        u64 s[W];
#pragma unroll
        for (int i = 0; i < W; ++i) s[i] = init.w[r * W + i];
        bool is_new;
        const u64 slot = find_or_claim(t, probe_key(m, t, s), &is_new, &lc->err);
        if (is_new) {
            if (t.meta) t.meta[slot] = 0;  // level 0
            atomicAdd(&lc->claims, 1u);
        }
        for (u32 und = undiscovered; und; und &= und - 1) {
            const int p = __builtin_ctz(und);
            if (m.discovers(p, s)) atomicMin(&lc->disc[p], r);
        }
    }
    publish<M::NPROPS>(lc, h, seq, true, nullptr);
}

// Rehash into a larger table (keys and meta move together); an entry that does not fit the new
// table's probe limit sets ERR_TABLE_FULL in *err (the host then rehashes into a larger one).
template <int = 0> __global__ void rehash(TableView from, u64 from_cap, TableView to, u32* err) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    const u64 k = slot_load(from, i);
    if (!k) return;
    bool is_new;
    u64 slot = find_or_claim(to, reprobe(from, to, i, k), &is_new, err);
    if (slot == ~0ull) return;
    if (to.meta) to.meta[slot] = from.meta[i];
}

// Growth of a quotient-mode table (no meta) by g = 2^lg, built range by range with no clear of the
// new table before it: a key's home is the top bits of its permuted key, so new slots [r S, (r+1) S)
// receive exactly the entries whose OLD home is in [r S / g, (r+1) S / g), and those sit in the old
// table between that range's first home and the first vacant old slot past its last. Workgroup r
// inserts them by linear probing into S slots of LDS and writes the whole range, zeros included,
// with 16-byte stores: one pass over each table instead of a clear plus a CAS per entry into a
// table too large for any cache (increment_lock N=11 unhinted, 2^28 -> 2^31 slots: 2.8 ms of clear
// and 6.2 ms of rehash, profiles/r06_nohint_inclock11_trace.txt). Any order of insertion leaves a
// valid linear-probing table (every slot between a key's home and its slot is occupied). An entry
// whose probe runs past the range end goes to spill[1..] (spill[0] counts them) and is inserted by
// rehash_spill, with CAS, once every range is written. err: ERR_TABLE_FULL if a displacement
// reaches the new probe limit or the spill list overflows (the host then grows further).
// S: the slots of a range, 32 KB of LDS (8192 four-byte or 4096 eight-byte slots). The old slots
// are read REBUILD_ROWS rows of the workgroup at a time, all loads in flight together, over the
// range's homes plus one row at first (one barrier when that row holds a vacant slot, as it nearly
// always does), then one row more per round.
constexpr u32 REBUILD_BLOCK = 256;
constexpr u32 REBUILD_ROWS = 4;
constexpr u32 REBUILD_BYTES = 32768;
template <class T>
constexpr u32 rebuild_slots() { return REBUILD_BYTES / sizeof(T); }
template <class T>
__global__ void __launch_bounds__(REBUILD_BLOCK)
    rehash_ranges(TableView from, u64 from_cap, TableView to, u32 lg, u64* spill, u64 spill_cap, u32* err) {
    constexpr u32 S = rebuild_slots<T>();
    __shared__ uint4 lds4[REBUILD_BYTES / 16];
    T* lds = reinterpret_cast<T*>(lds4);
    for (u32 j = threadIdx.x; j < REBUILD_BYTES / 16; j += REBUILD_BLOCK) lds4[j] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const u64 r0 = (u64)blockIdx.x * S;
    const u64 a = r0 >> lg, span = S >> lg;  // old homes [a, a + span)
    const u64 omask = from_cap - 1, dmask = (1ull << from.dbits) - 1;
    // window [lo, hi) of offsets past a, never more than the old table (no slot is read twice)
    u64 lo = 0, hi = min<u64>(span + REBUILD_BLOCK, from_cap);
    for (;;) {
        bool done = false;
        for (u64 base = lo; base < hi; base += REBUILD_ROWS * REBUILD_BLOCK) {
            u64 v[REBUILD_ROWS];
#pragma unroll
            for (u32 r = 0; r < REBUILD_ROWS; ++r) {
                const u64 off = base + r * REBUILD_BLOCK + threadIdx.x;
                v[r] = off < hi ? slot_load(from, (a + off) & omask) : 1ull;  // (1: outside the window)
            }
#pragma unroll
            for (u32 r = 0; r < REBUILD_ROWS; ++r) {
                const u64 off = base + r * REBUILD_BLOCK + threadIdx.x, i = (a + off) & omask;
                if (off >= hi) continue;
                if (!v[r]) {
                    done |= off >= span;  // a vacant slot past the last home ends the range's entries
                    continue;
                }
                if (((i - ((v[r] & dmask) - 1) - a) & omask) >= span) continue;  // homed elsewhere
                const ProbeKey k = quot_probe(to, quot_decode(from, i, v[r]));
                u64 j = k.home - r0;
                if (j >= S) {
                    atomicOr(err, (u32)ERR_TABLE_FULL);  // (not homed in this range: cannot happen)
                    continue;
                }
                for (u64 d = 0;; ++d, ++j) {
                    if (d >= to.plimit) {
                        atomicOr(err, (u32)ERR_TABLE_FULL);
                        break;
                    }
                    if (j >= S) {
                        const u64 q = atomicAdd(reinterpret_cast<unsigned long long*>(spill), 1ull);
                        if (q < spill_cap) spill[1 + q] = i;
                        else atomicOr(err, (u32)ERR_TABLE_FULL);
                        break;
                    }
                    if (atomicCAS(&lds[j], (T)0, (T)(k.tag + d)) == (T)0) break;
                }
            }
        }
        if (__syncthreads_or(done) || hi >= from_cap) break;
        lo = hi;
        hi = min<u64>(hi + REBUILD_BLOCK, from_cap);
    }
    uint4* out = reinterpret_cast<uint4*>(reinterpret_cast<T*>(to.keys) + r0);
    for (u32 j = threadIdx.x; j < REBUILD_BYTES / 16; j += REBUILD_BLOCK) out[j] = lds4[j];
}
// The entries rehash_ranges spilled past their range's end, inserted into the finished table.
template <int = 0>
__global__ void rehash_spill(TableView from, TableView to, const u64* spill, u64 spill_cap, u32* err) {
    const u64 n = min(spill[0], spill_cap);
    for (u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (u64)gridDim.x * blockDim.x) {
        const u64 i = spill[1 + q];
        bool is_new;
        (void)find_or_claim(to, reprobe(from, to, i, slot_load(from, i)), &is_new, err);
    }
}

// Longest linear-probe displacement over the occupied slots (sr_stats.max_displacement): quotient
// mode stores 1 + the displacement in the low dbits; a fingerprint's home is fp & mask.
template <int = 0> __global__ void __launch_bounds__(256) table_max_disp(TableView t, u64 cap, u32* out) {
    u32 best = 0;
    const u64 dmask = t.qbits ? (1ull << t.dbits) - 1 : 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (u64)gridDim.x * blockDim.x) {
        const u64 v = slot_load(t, i);
        if (!v) continue;
        const u64 d = t.qbits ? (v & dmask) - 1 : (i - (v & t.mask)) & t.mask;
        best = max(best, (u32)min<u64>(d, 0xffffffffull));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) best = max(best, (u32)__shfl_xor((int)best, d, 64));
    if ((threadIdx.x & 63) == 0 && best) atomicMax(out, best);
}

// After a rehash: candidate slot indices of the old table -> slots of the new one.
template <int = 0> __global__ void remap_slots(u32* cand, u64 n, TableView from, TableView to) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 s = cand[i];
    if (s == CAND_NONE) return;
    cand[i] = (u32)find_slot(to, reprobe(from, to, s, slot_load(from, s)));
}

// ---- exclusive scan of u32 counts (3-phase: tile sums, scan of sums, tile scan + carry) ----
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ u32 block_exclusive_scan(u32 v, u32* total) {
    __shared__ u32 wsum[SCAN_BLOCK / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const u32 x = wave_incl_scan(v);
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

template <int = 0> __global__ void __launch_bounds__(SCAN_BLOCK) scan_tile_sums(const u32* in, u32 n, u32* sums) {
    u64 base = (u64)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i)
        if (base + i < n) acc += in[base + i];
    u32 tot;
    block_exclusive_scan(acc, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <int = 0> __global__ void __launch_bounds__(SCAN_BLOCK) scan_sums(u32* sums, u32 nt, u32* grand_total) {
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

template <int = 0> __global__ void __launch_bounds__(SCAN_BLOCK) scan_tiles(const u32* in, u32 n, const u32* sums, u32* out) {
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
