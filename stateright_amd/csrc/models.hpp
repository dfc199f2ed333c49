// GpuModel encodings: the device-side counterpart of `impl Model for X` (src/lib.rs:155-237).
//
// A GpuModel packs one state into W 64-bit words (equal states <=> equal words) and exposes the
// reference's `actions()` list as ACTION SLOTS 0..max_actions-1 in the reference's own order:
//   enabled(s, mask)   bit a of mask = slot a appears in `actions(s)`
//   apply(s, a, out)   `next_state(s, action)` is Some AND `within_boundary` holds -> out
//   discovers(p, s)    property p yields a discovery at s (always: !cond, sometimes: cond)
// Host-only helpers give init states, property names/expectations, the canonical description of a
// state (shared with the CPU oracle for set/order/path comparison) and canonical action ids.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace sr {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

#define SR_HD __host__ __device__ __forceinline__

enum Expect { ALWAYS = 0, EVENTUALLY = 1, SOMETIMES = 2 };

// Mask of a model's `eventually` properties (0 for models without an `emask()` member).
template <class M, class = void>
struct has_emask : std::false_type {};
template <class M>
struct has_emask<M, std::void_t<decltype(std::declval<const M&>().emask())>> : std::true_type {};
template <class M>
inline u32 model_emask(const M& m) {
    if constexpr (has_emask<M>::value) return m.emask();
    else return 0;
}

// Models whose states pack into a key of at most 120 bits (`qkey_bits()` and `qkey(s)`: an
// injective packing of the state into an integer below 2^qkey_bits) can use the exact quotient
// visited set (kernels.hpp TableView).
template <class M, class = void>
struct has_qkey : std::false_type {};
template <class M>
struct has_qkey<M, std::void_t<decltype(std::declval<const M&>().qkey_bits())>> : std::true_type {};

// Models that can rebuild a state from its canonical description (`undescribe`, the inverse of
// `describe`) expose their fingerprint to a host that holds the state (sr_model_fingerprint).
template <class M, class = void>
struct has_undescribe : std::false_type {};
template <class M>
struct has_undescribe<M, std::void_t<decltype(std::declval<const M&>().undescribe((const i64*)nullptr, (u64*)nullptr))>>
    : std::true_type {};

// Models with a canonical representative under their symmetry (`canonical(s, out)`).
template <class M, class = void>
struct has_canonical : std::false_type {};
template <class M>
struct has_canonical<M, std::void_t<decltype(std::declval<const M&>().canonical((const u64*)nullptr, (u64*)nullptr))>>
    : std::true_type {};

// Models that know which enabled actions return the state itself (`self_loops(s, enabled, out)`:
// out = the subset of `enabled` whose next_state is s). The FAST expansion counts those successors
// (they are state_count increments, bfs.rs:235, and never new) without generating them: on 2pc
// they are 37% of all successors. Exactness is tested against apply() over every reachable state
// (tests/test_gpu_parity.py, the oracle's state counts).
template <class M, class = void>
struct has_self_loops : std::false_type {};
template <class M>
struct has_self_loops<M, std::void_t<decltype(std::declval<const M&>().self_loops((const u64*)nullptr, (const u64*)nullptr,
                                                                                  (u64*)nullptr))>> : std::true_type {};

// Wide models whose enabled mask is a per-slot test (`enabled_slot(s, k)` = bit k of `enabled(s)`,
// `ESLOTS` = max_actions, a power of two <= 64, MW = 1). Small levels of such a model are chains of
// dependent instructions on a few lanes; the FAST expansion then evaluates the mask with one lane
// per (parent, slot) instead of one lane per parent walking all the slots (paxos: 16 slots, each a
// switch over the destination server's word), reading the parent from the wave's LDS copy.
template <class M, class = void>
struct has_enabled_slot : std::false_type {};
template <class M>
struct has_enabled_slot<M, std::void_t<decltype(std::declval<const M&>().enabled_slot((const u64*)nullptr, 0)),
                                       decltype(M::ESLOTS)>> : std::true_type {};

// Models with an OWNER KEY (`owner_key(s, &key)`: a projection of the state that most actions
// leave unchanged; returns false when this instance has none). The partitioned search then owns a
// state by its key instead of its fingerprint, so most successors stay in their parent's
// partition and are inserted there instead of crossing to another GPU. Any
// deterministic function of the state keeps the search exact (every state has exactly one
// owner); the projection only sets the share of successors that cross and the load balance.
template <class M, class = void>
struct has_owner_key : std::false_type {};
template <class M>
struct has_owner_key<M, std::void_t<decltype(std::declval<const M&>().owner_key((const u64*)nullptr, (u64*)nullptr))>>
    : std::true_type {};

// Init states (`Model::init_states`, src/lib.rs:163). A model writes its init states into a host
// buffer of W words each; the engine sizes that buffer from the model's optional `init_count()`,
// or for MAX_INIT_STATES states when the model has none (the documented bound of the GpuModel
// concept, include/stateright_gpu_model.hpp). Every host-side caller goes through init_states_of.
constexpr int MAX_INIT_STATES = 256;
template <class M, class = void>
struct has_init_count : std::false_type {};
template <class M>
struct has_init_count<M, std::void_t<decltype(std::declval<const M&>().init_count())>> : std::true_type {};
template <class M>
inline int init_capacity(const M& m) {
    if constexpr (has_init_count<M>::value) return m.init_count() > 0 ? m.init_count() : 1;
    else return MAX_INIT_STATES;
}

// The symmetry-reduced view of a model (the engine's opt-in canonical reduction): init states and
// successors are replaced by their canonical representatives, so the visited set, the frontier and
// the BFS tree hold one state per orbit. Everything else is the model's own.
template <class M>
struct Canon : M {
    Canon() = default;
    explicit Canon(const M& m) : M(m) {}
    const M& base() const { return *this; }
    SR_HD bool apply(const u64* s, int a, u64* o) const {
        u64 t[M::W];
        if (!M::apply(s, a, t)) return false;
        M::canonical(t, o);
        return true;
    }
    int init_states(u64* out) const {
        const int k = M::init_states(out);
        for (int i = 0; i < k; ++i) {
            u64 t[M::W];
            M::canonical(out + i * M::W, t);
            for (int w = 0; w < M::W; ++w) out[i * M::W + w] = t[w];
        }
        return k;
    }
};
template <class M>
struct is_canon : std::false_type {};
template <class M>
struct is_canon<Canon<M>> : std::true_type {};

// murmur3 fmix64: a bijection on u64 with fmix64(0) == 0.
SR_HD u64 fmix64(u64 k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// 64-bit state fingerprint (`fingerprint`, src/lib.rs:306-311). For W == 1 the packed state
// uses at most 63 bits, so XOR-ing bit 63 and mixing is a BIJECTION that is never zero: the
// visited set is then exact (no fingerprint collisions at all). For W > 1 it is a 64-bit hash
// like the reference's (collisions possible at ~n^2/2^65); zero is remapped to 1 where the
// reference would panic (src/lib.rs:310).
template <int W>
SR_HD u64 fingerprint(const u64* s) {
    if constexpr (W == 1) {
        return fmix64(s[0] ^ 0x8000000000000000ull);
    } else {
        // every word mixed on its own (position-keyed), then one mix of their sum: two mixes deep
        // instead of a chain of W (a lone wave of a small paxos level waits on that chain: C=3
        // 0.62 -> 0.61 ms, profiles/r05_paxos_lin.txt; round 4 had measured no gain, before the
        // linearizability test's chain was cut)
        u64 acc = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) acc += fmix64(s[i] ^ (0x632BE59BD9B4E019ull * (u64)(i + 1)));
        const u64 h = fmix64(acc ^ 0x9E3779B97F4A7C15ull);
        return h ? h : 1;
    }
}

// Words of a state that its fingerprint covers: M::FPW when the model declares it (EvBits<M>: the
// last word is bookkeeping that rides with the state but is not part of it), else all W. Every
// fingerprint the engines compute (visited set, partition owner, discovery chains) goes through
// state_fp, so an EvBits<M> state has the fingerprint of the M state it wraps.
template <class M, class = void>
struct fp_words_of : std::integral_constant<int, M::W> {};
template <class M>
struct fp_words_of<M, std::void_t<decltype(M::FPW)>> : std::integral_constant<int, M::FPW> {};
template <class M>
SR_HD u64 state_fp(const u64* s) {
    return fingerprint<fp_words_of<M>::value>(s);
}

// `eventually` properties for the PARTITIONED search (src/checker/bfs.rs:52-60,212-222,265-272):
// the EventuallyBits of a pending state ride in one extra word of it, so the records the ranks
// exchange carry them and the owner's claim keeps the claiming generator's bits (the FAST order's
// rule of the one-GPU engine, kernels.hpp expand_fast naeb). A successor gets its parent's bits
// minus the eventually properties whose condition holds at the parent (the parent's pop), and an
// eventually property is discovered at a state that still carries its bit, where its condition
// does not hold and that has no successor within boundary (a terminal state, bfs.rs:265-272).
// The engine sees no `eventually` property (emask() == 0): such a discovery is an ordinary
// discovery of the new state, with its path.  The visited set and every fingerprint cover the
// wrapped state only (FPW), so a state reached with two different bit words is ONE state, as in
// the reference (bfs.rs:235-246: the first generator's bits win).
template <class M>
struct EvBits : M {
    static constexpr int W = M::W + 1, FPW = M::W;
    u32 ev_props_ = 0;  // the wrapped model's eventually properties
    EvBits() = default;
    explicit EvBits(const M& m) : M(m), ev_props_(model_emask(m)) {}
    const M& base() const { return *this; }
    u32 emask() const { return 0; }
    SR_HD u32 holds(const u64* s) const {
        u32 h = 0;
        for (u32 e = ev_props_; e; e &= e - 1)
            if (M::discovers(__builtin_ctz(e), s)) h |= 1u << __builtin_ctz(e);
        return h;
    }
    SR_HD bool apply(const u64* s, int a, u64* o) const {
        if (!M::apply(s, a, o)) return false;
        o[M::W] = s[M::W] & ~(u64)holds(s);
        return true;
    }
    SR_HD bool discovers(int p, const u64* s) const {
        if (!(ev_props_ >> p & 1)) return M::discovers(p, s);
        if (!(s[M::W] >> p & 1) || M::discovers(p, s)) return false;
        u64 mask[M::MW];
        M::enabled(s, mask);
        for (int w = 0; w < M::MW; ++w)
            for (u64 bits = mask[w]; bits; bits &= bits - 1) {
                u64 t[M::W];
                if (M::apply(s, w * 64 + __builtin_ctzll(bits), t)) return false;
            }
        return true;
    }
    int init_states(u64* out) const {
        const int k = M::init_states(out);
        for (int i = k - 1; i >= 0; --i) {
            for (int w = M::W - 1; w >= 0; --w) out[i * W + w] = out[i * M::W + w];
            out[i * W + M::W] = ev_props_;
        }
        return k;
    }
};
template <class M>
struct is_evbits : std::false_type {};
template <class M>
struct is_evbits<EvBits<M>> : std::true_type {};

SR_HD u64 getb(const u64* s, int off, int width) {
    // bit field [off, off+width) of a little-endian multi-word state; width <= 8, no word crossing
    return (s[off >> 6] >> (off & 63)) & ((1ull << width) - 1);
}
SR_HD void setb(u64* s, int off, int width, u64 v) {
    u64 m = ((1ull << width) - 1) << (off & 63);
    s[off >> 6] = (s[off >> 6] & ~m) | ((v << (off & 63)) & m);
}

// -----------------------------------------------------------------------------------------------
// LinearEquation (src/test_util.rs:140-188): state (x: u8, y: u8); actions IncreaseX, IncreaseY.
// -----------------------------------------------------------------------------------------------
struct LinearEquation {
    static constexpr int W = 1, MW = 1, NPROPS = 1;
    u32 a, b, c;
    int max_actions() const { return 2; }
    int max_out_degree() const { return 2; }
    SR_HD void enabled(const u64*, u64* m) const { m[0] = 3; }
    SR_HD bool apply(const u64* s, int a_, u64* o) const {
        u64 x = s[0] & 0xff, y = (s[0] >> 8) & 0xff;
        if (a_ == 0) x = (x + 1) & 0xff; else y = (y + 1) & 0xff;
        o[0] = x | (y << 8);
        return true;
    }
    SR_HD bool discovers(int, const u64* s) const {  // sometimes "solvable": a*x + b*y == c (u8)
        u64 x = s[0] & 0xff, y = (s[0] >> 8) & 0xff;
        return ((a * x + b * y) & 0xff) == c;
    }
    int init_states(u64* out) const { out[0] = 0; return 1; }
    int expectation(int) const { return SOMETIMES; }
    const char* prop_name(int) const { return "solvable"; }
    int describe_width() const { return 2; }
    void describe(const u64* s, i64* d) const { d[0] = (i64)(s[0] & 0xff); d[1] = (i64)((s[0] >> 8) & 0xff); }
    void undescribe(const i64* d, u64* s) const { s[0] = ((u64)d[0] & 0xff) | ((u64)d[1] & 0xff) << 8; }
    i64 action_id(const u64*, int a_) const { return a_; }
    std::string action_name(i64 id) const { return id == 0 ? "IncreaseX" : "IncreaseY"; }
    i64 action_id_bound() const { return 2; }
};

// -----------------------------------------------------------------------------------------------
// BinaryClock (src/test_util.rs:4-45): i8 state in {0, 1}; one action (GoHigh at 0, GoLow at 1).
// -----------------------------------------------------------------------------------------------
struct BinaryClock {
    static constexpr int W = 1, MW = 1, NPROPS = 1;
    int max_actions() const { return 1; }
    int max_out_degree() const { return 1; }
    SR_HD void enabled(const u64*, u64* m) const { m[0] = 1; }
    SR_HD bool apply(const u64* s, int, u64* o) const { o[0] = (s[0] & 0xff) == 0 ? 1 : 0; return true; }
    SR_HD bool discovers(int, const u64* s) const {  // always "in [0, 1]"
        int8_t v = (int8_t)(s[0] & 0xff);
        return !(0 <= v && v <= 1);
    }
    int init_states(u64* out) const { out[0] = 0; out[1] = 1; return 2; }
    int expectation(int) const { return ALWAYS; }
    const char* prop_name(int) const { return "in [0, 1]"; }
    int describe_width() const { return 1; }
    void describe(const u64* s, i64* d) const { d[0] = (int8_t)(s[0] & 0xff); }
    void undescribe(const i64* d, u64* s) const { s[0] = (u64)(u8)d[0]; }
    i64 action_id(const u64* s, int) const { return (s[0] & 0xff) == 0 ? 1 : 0; }  // GoLow=0, GoHigh=1
    std::string action_name(i64 id) const { return id == 0 ? "GoLow" : "GoHigh"; }
    i64 action_id_bound() const { return 2; }
};

// -----------------------------------------------------------------------------------------------
// Two-phase commit (examples/2pc.rs:10-121), n <= 14 resource managers, 4n+4 bits:
//   [0,2n)      rm_state[rm]   (Working 0, Prepared 1, Committed 2, Aborted 3)
//   [2n,2n+2)   tm_state       (Init 0, Committed 1, Aborted 2)
//   [2n+2,3n+2) tm_prepared[rm]
//   [3n+2,4n+2) msgs ∋ Prepared{rm}
//   4n+2        msgs ∋ Commit;  4n+3  msgs ∋ Abort
// Slots follow `actions()` (examples/2pc.rs:56-81): 0 TmCommit, 1 TmAbort, then for each rm
// 2+5rm+{0 TmRcvPrepared, 1 RmPrepare, 2 RmChooseToAbort, 3 RmRcvCommitMsg, 4 RmRcvAbortMsg}.
// Every action returns Some (examples/2pc.rs:83-104), self-loops included.
// -----------------------------------------------------------------------------------------------
// NC > 0: the rm count as a compile-time constant (the engine's specialization of the bench
// configurations, reg_two_phase.hip); the device functions read it through N(), so their per-rm
// loops unroll with constant shifts. NC = 0 reads the runtime n.
template <int NC = 0>
struct TwoPhaseT {
    static constexpr int W = 1, MW = 2, NPROPS = 3;
    int n;
    SR_HD int N() const {
        if constexpr (NC > 0) return NC;
        else return n;
    }
    // Owner key of the partitioned search: the per-RM tuples (rm_state, tm_prepared,
    // Prepared{rm} in msgs) of the first okey_rms resource managers (0: no key, own by
    // fingerprint). Only the five actions of those RMs change it; TmCommit/TmAbort and the other
    // RMs' actions keep a successor in its parent's partition.
    int okey_rms = 0;
    SR_HD bool owner_key(const u64* sp, u64* key) const {
        const int n = N();
        const int k = okey_rms;
        const u64 s = sp[0], m = (1ull << k) - 1;
        *key = (s & ((1ull << (2 * k)) - 1)) | ((s >> (2 * n + 2)) & m) << (2 * k) | ((s >> (3 * n + 2)) & m) << (3 * k);
        return k > 0;
    }
    int max_actions() const { return 2 + 5 * n; }
    // Per rm at most three of its five slots (a Working rm after TmAbort: Prepare, ChooseToAbort,
    // RcvAbort); TmCommit/TmAbort only while the TM is Init (then at most two per rm).
    int max_out_degree() const { return 2 + 3 * n; }
    SR_HD u64 rmask() const { return (1ull << N()) - 1; }
    // per-rm bit vectors
    SR_HD u64 working(u64 s) const {  // rm_state == 0, one bit per rm
        const int n = N();
        const u64 ev = 0x5555555555555555ull & ((1ull << (2 * n)) - 1);
        u64 w = ~(s | (s >> 1)) & ev;  // bit 2rm: field rm == 0
        // compress the even bits to bits 0..n-1
        w = (w | (w >> 1)) & 0x3333333333333333ull;
        w = (w | (w >> 2)) & 0x0f0f0f0f0f0f0f0full;
        w = (w | (w >> 4)) & 0x00ff00ff00ff00ffull;
        w = (w | (w >> 8)) & 0x0000ffff0000ffffull;
        w = (w | (w >> 16)) & 0x00000000ffffffffull;
        return w;
    }
    // One 5-bit group per rm at slot 2 + 5rm (TmRcvPrepared, RmPrepare, RmChooseToAbort,
    // RmRcvCommitMsg, RmRcvAbortMsg), placed without per-action branches.
    SR_HD void enabled(const u64* sp, u64* m) const {
        const int n = N();
        const u64 s = sp[0];
        const u64 tm = (s >> (2 * n)) & 3;
        const u64 prepared = (s >> (2 * n + 2)) & rmask();
        const u64 msgp = (s >> (3 * n + 2)) & rmask();
        const u64 commit = (s >> (4 * n + 2)) & 1, abort = (s >> (4 * n + 3)) & 1;
        const u64 work = working(s);
        const u64 rcv = tm == 0 ? msgp : 0;
        const u64 tail = commit << 3 | abort << 4;
        u64 lo = (u64)(tm == 0 && prepared == rmask()) | (u64)(tm == 0) << 1, hi = 0;
        for (int rm = 0; rm < n; ++rm) {
            const int b = 2 + 5 * rm;
            const u64 bits = ((rcv >> rm) & 1) | ((work >> rm) & 1) * 6ull | tail;
            if (b < 64) lo |= bits << b;
            if (b + 4 >= 64) hi |= b >= 64 ? bits << (b - 64) : bits >> (64 - b);
        }
        m[0] = lo;
        m[1] = hi;
    }
    // The enabled actions that return s itself: TmRcvPrepared(rm) with tm_prepared[rm] already set,
    // RmRcvCommitMsg(rm) with rm already Committed, RmRcvAbortMsg(rm) with rm already Aborted. No
    // other action can (RmPrepare and RmChooseToAbort need a Working rm and change it, TmCommit and
    // TmAbort need tm_state Init and change it).
    SR_HD void self_loops(const u64* sp, const u64* mk, u64* sl) const {
        const int n = N();
        const u64 s = sp[0];
        const u64 tm = (s >> (2 * n)) & 3;
        const u64 prepared = (s >> (2 * n + 2)) & rmask();
        const u64 msgp = (s >> (3 * n + 2)) & rmask();
        const bool commit = (s >> (4 * n + 2)) & 1, abort = (s >> (4 * n + 3)) & 1;
        u64 lo = 0, hi = 0;
        for (int rm = 0; rm < n; ++rm) {
            const u64 r = (s >> (2 * rm)) & 3;
            const int b = 2 + 5 * rm;
            const u64 bits = (u64)(tm == 0 && ((msgp & prepared) >> rm & 1)) | (u64)(commit && r == 2) << 3 |
                             (u64)(abort && r == 3) << 4;
            if (b < 64) lo |= bits << b;
            if (b + 4 >= 64) hi |= b >= 64 ? bits << (b - 64) : bits >> (64 - b);
        }
        sl[0] = lo & mk[0];
        sl[1] = hi & mk[1];
    }
    // Branch-free: the lanes of a wave apply different actions, and a switch over them ran every
    // taken arm for the whole wave. Every action writes at most one 2-bit field (rm_state[rm] or
    // tm_state) and sets at most one bit:
    //   a = 0 TmCommit         tm_state <- 1, bit 4n+2 (Commit)
    //   a = 1 TmAbort          tm_state <- 2, bit 4n+3 (Abort)
    //   k = 0 TmRcvPrepared    bit 2n+2+rm (tm_prepared)
    //   k = 1 RmPrepare        rm_state <- 1, bit 3n+2+rm (Prepared{rm})
    //   k = 2 RmChooseToAbort  rm_state <- 3
    //   k = 3 RmRcvCommitMsg   rm_state <- 2
    //   k = 4 RmRcvAbortMsg    rm_state <- 3
    SR_HD bool apply(const u64* sp, int a, u64* o) const {
        const int n = N();
        const u64 s = sp[0];
        const bool tm = a < 2;
        const u32 b = tm ? 0u : (u32)(a - 2), rm = b / 5, k = b - 5 * rm;
        const u32 fpos = tm ? 2u * n : 2u * rm;
        const u64 fval = tm ? (u64)(a + 1) : k == 1 ? 1ull : k == 3 ? 2ull : 3ull;
        const u64 fmask = (tm || k != 0) ? 3ull << fpos : 0ull;
        const u32 epos = tm ? 4u * n + 2 + (u32)a : (k == 0 ? 2u * n + 2 : 3u * n + 2) + rm;
        const u64 ebit = (tm || k <= 1) ? 1ull << epos : 0ull;
        o[0] = ((s & ~fmask) | ((fval << fpos) & fmask)) | ebit;
        return true;
    }
    // rm_state fields, bit-parallel: bit 2rm of `ab` is set iff rm is Aborted (3), of `cm` iff
    // Committed (2) (the loop over the rms ran once per property for every new state).
    SR_HD u64 even_mask() const { return 0x5555555555555555ull & ((1ull << (2 * N())) - 1); }
    SR_HD bool discovers(int p, const u64* sp) const {
        const u64 s = sp[0], ev = even_mask();
        const u64 lo = s & ev, hi = (s >> 1) & ev;
        const u64 ab = hi & lo, cm = hi & ~lo;
        if (p == 0) return ab == ev;           // sometimes "abort agreement"
        if (p == 1) return cm == ev;           // sometimes "commit agreement"
        return ab != 0 && cm != 0;             // always "consistent" violated
    }
    int init_states(u64* out) const { out[0] = 0; return 1; }
    // Exact key (quotient visited set): the packed word itself, 4N+4 bits. At N=9 a 2^25-slot
    // table keeps a 15-bit remainder and 17 displacement bits in a 32-bit slot (kernels.hpp).
    int qkey_bits() const { return 4 * N() + 4; }
    SR_HD unsigned __int128 qkey(const u64* s) const { return s[0]; }
    int expectation(int p) const { return p == 2 ? ALWAYS : SOMETIMES; }
    const char* prop_name(int p) const {
        return p == 0 ? "abort agreement" : p == 1 ? "commit agreement" : "consistent";
    }
    int describe_width() const { return 3 * n + 3; }
    void describe(const u64* sp, i64* d) const {
        u64 s = sp[0];
        int k = 0;
        for (int rm = 0; rm < n; ++rm) d[k++] = (i64)((s >> (2 * rm)) & 3);
        d[k++] = (i64)((s >> (2 * n)) & 3);
        for (int rm = 0; rm < n; ++rm) d[k++] = (i64)((s >> (2 * n + 2 + rm)) & 1);
        for (int rm = 0; rm < n; ++rm) d[k++] = (i64)((s >> (3 * n + 2 + rm)) & 1);
        d[k++] = (i64)((s >> (4 * n + 2)) & 1);
        d[k++] = (i64)((s >> (4 * n + 3)) & 1);
    }
    void undescribe(const i64* d, u64* sp) const {
        u64 s = 0;
        int k = 0;
        for (int rm = 0; rm < n; ++rm) s |= ((u64)d[k++] & 3) << (2 * rm);
        s |= ((u64)d[k++] & 3) << (2 * n);
        for (int rm = 0; rm < n; ++rm) s |= ((u64)d[k++] & 1) << (2 * n + 2 + rm);
        for (int rm = 0; rm < n; ++rm) s |= ((u64)d[k++] & 1) << (3 * n + 2 + rm);
        s |= ((u64)d[k++] & 1) << (4 * n + 2);
        s |= ((u64)d[k++] & 1) << (4 * n + 3);
        sp[0] = s;
    }
    // Canonical representative under permutations of the resource managers (the symmetry the
    // reference's `representative` exploits, examples/2pc.rs:156-187): the per-RM tuples
    // (rm_state, tm_prepared, Prepared{rm} in msgs) sorted ascending by that 4-bit key. Unlike the
    // reference's sort by rm_state alone (ties kept in index order), equal orbits always give equal
    // words, so the reduced state count does not depend on the visit order.
    SR_HD void canonical(const u64* sp, u64* o) const {
        const int n = N();
        const u64 s = sp[0];
        u32 cnt[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) cnt[k] = 0;
        for (int rm = 0; rm < n; ++rm) {
            const u32 key = (u32)((s >> (2 * rm)) & 3) | (u32)((s >> (2 * n + 2 + rm)) & 1) << 2 |
                            (u32)((s >> (3 * n + 2 + rm)) & 1) << 3;
            ++cnt[key];
        }
        u64 r = s & (3ull << (2 * n) | 3ull << (4 * n + 2));  // tm_state, Commit, Abort
        int rm = 0;
        for (u32 key = 0; key < 16; ++key)
            for (u32 c = 0; c < cnt[key]; ++c, ++rm)
                r |= (u64)(key & 3) << (2 * rm) | (u64)(key >> 2 & 1) << (2 * n + 2 + rm) | (u64)(key >> 3 & 1) << (3 * n + 2 + rm);
        o[0] = r;
    }
    i64 action_id(const u64*, int a) const { return a; }
    i64 action_id_bound() const { return 2 + 5 * n; }
    std::string action_name(i64 id) const {
        if (id == 0) return "TmCommit";
        if (id == 1) return "TmAbort";
        const char* names[] = {"TmRcvPrepared", "RmPrepare", "RmChooseToAbort", "RmRcvCommitMsg", "RmRcvAbortMsg"};
        return std::string(names[(id - 2) % 5]) + "(" + std::to_string((id - 2) / 5) + ")";
    }
};
using TwoPhase = TwoPhaseT<0>;

// -----------------------------------------------------------------------------------------------
// Increment (examples/increment.rs:109-197), n <= 15 threads: i (4 bits) then per thread
// t (4 bits) + pc (2 bits, values 1..3). 4+6n bits; W = 1 for n <= 9, else 2.
// Slot = thread id (each thread has at most one enabled action: Read at pc 1, Write at pc 2).
// -----------------------------------------------------------------------------------------------
template <int W_>
struct Increment {
    static constexpr int W = W_, MW = 1, NPROPS = 1;
    int n;
    int max_actions() const { return n; }
    int max_out_degree() const { return n; }
    SR_HD static int toff(int t) { return 4 + 6 * t; }
    SR_HD void enabled(const u64* s, u64* m) const {
        u64 r = 0;
        for (int t = 0; t < n; ++t) {
            u64 pc = getb(s, toff(t) + 4, 2);
            r |= (u64)(pc == 1 || pc == 2) << t;
        }
        m[0] = r;
    }
    SR_HD bool apply(const u64* s, int t, u64* o) const {
#pragma unroll
        for (int i = 0; i < W; ++i) o[i] = s[i];
        u64 pc = getb(s, toff(t) + 4, 2);
        if (pc == 1) {  // Read: s[t] = {t: i, pc: 2}
            setb(o, toff(t), 4, getb(s, 0, 4));
            setb(o, toff(t) + 4, 2, 2);
        } else {  // Write: pc = 3; i = t + 1
            setb(o, toff(t) + 4, 2, 3);
            setb(o, 0, 4, getb(s, toff(t), 4) + 1);
        }
        return true;
    }
    SR_HD bool discovers(int, const u64* s) const {  // always "fin": #(pc == 3) == i
        u64 c = 0;
        for (int t = 0; t < n; ++t) c += getb(s, toff(t) + 4, 2) == 3;
        return c != getb(s, 0, 4);
    }
    int init_states(u64* out) const {
        for (int i = 0; i < W; ++i) out[i] = 0;
        for (int t = 0; t < n; ++t) setb(out, toff(t) + 4, 2, 1);
        return 1;
    }
    int expectation(int) const { return ALWAYS; }
    const char* prop_name(int) const { return "fin"; }
    // Exact key (quotient visited set) of the two-word layout: word 0 is full (4 + 6*10 = 64 bits),
    // word 1 holds threads 10.. : the state is an integer below 2^(4 + 6n).
    int qkey_bits() const { return 4 + 6 * n; }
    SR_HD unsigned __int128 qkey(const u64* s) const {
        if constexpr (W_ == 1) return s[0];
        else return (unsigned __int128)s[0] | ((unsigned __int128)s[W_ - 1] << 64);
    }
    int describe_width() const { return 1 + 2 * n; }
    void describe(const u64* s, i64* d) const {
        d[0] = (i64)getb(s, 0, 4);
        for (int t = 0; t < n; ++t) {
            d[1 + 2 * t] = (i64)getb(s, toff(t), 4);
            d[2 + 2 * t] = (i64)getb(s, toff(t) + 4, 2);
        }
    }
    void undescribe(const i64* d, u64* s) const {
        for (int i = 0; i < W; ++i) s[i] = 0;
        setb(s, 0, 4, (u64)d[0]);
        for (int t = 0; t < n; ++t) {
            setb(s, toff(t), 4, (u64)d[1 + 2 * t]);
            setb(s, toff(t) + 4, 2, (u64)d[2 + 2 * t]);
        }
    }
    i64 action_id(const u64* s, int t) const { return 2 * t + (getb(s, toff(t) + 4, 2) == 2 ? 1 : 0); }
    i64 action_id_bound() const { return 2 * n; }
    std::string action_name(i64 id) const {
        return std::string(id % 2 ? "Write(" : "Read(") + std::to_string(id / 2) + ")";
    }
};

// -----------------------------------------------------------------------------------------------
// IncrementLock (examples/increment_lock.rs:3-107), n <= 12 threads: i (4 bits), lock (1 bit),
// then per thread t (4 bits) + pc (3 bits, 0..4); 5+7n bits, W = 1 for n <= 8, else 2.
// Per-thread fields are placed so that none crosses a word boundary.
// -----------------------------------------------------------------------------------------------
template <int W_>
struct IncrementLock {
    static constexpr int W = W_, MW = 1, NPROPS = 2;
    int n;
    int max_actions() const { return n; }
    int max_out_degree() const { return n; }
    // threads 0..7 live in word 0 (bits 5..60), threads 8.. in word 1 (bits 0..)
    SR_HD static int toff(int t) { return t < 8 ? 5 + 7 * t : 64 + 7 * (t - 8); }
    // Bit-parallel over the threads: bit 0 of thread t's pc field sits at pc_pos(t); pc_mask(w) has
    // those bits of word w, so b0/b1/b2 of every pc are three masked shifts of the word.
    SR_HD static int pc_pos(int t) { return t < 8 ? 9 + 7 * t : 4 + 7 * (t - 8); }
    SR_HD u64 pc_mask(int w) const {
        u64 m = 0;
        for (int t = w == 0 ? 0 : 8; t < (w == 0 ? (n < 8 ? n : 8) : n); ++t) m |= 1ull << pc_pos(t);
        return m;
    }
    SR_HD void enabled(const u64* s, u64* m) const {
        const bool lock = (s[0] >> 4) & 1;
        u64 r = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const u64 M = pc_mask(w), x = s[w];
            const u64 b0 = x & M, b1 = (x >> 1) & M, b2 = (x >> 2) & M;
            // Lock at pc 0 (lock free), Read at 1, Write at 2, Release at 3 (lock held)
            const u64 en = ~b2 & ((b1 ^ b0) | (~(b1 | b0) & (lock ? 0 : M)) | (b1 & b0 & (lock ? M : 0))) & M;
            for (int t = w == 0 ? 0 : 8; t < (w == 0 ? (n < 8 ? n : 8) : n); ++t) r |= ((en >> pc_pos(t)) & 1) << t;
        }
        m[0] = r;
    }
    // Every action advances pc by one (Lock 0->1, Read 1->2, Write 2->3, Release 3->4); the other
    // field it writes is selected without branches (the lanes of a wave run different threads).
    SR_HD bool apply(const u64* s, int t, u64* o) const {
#pragma unroll
        for (int i = 0; i < W; ++i) o[i] = s[i];
        const u64 pc = getb(s, toff(t) + 4, 3), iv = getb(s, 0, 4), tv = getb(s, toff(t), 4);
        const u64 lock = getb(s, 4, 1);
        setb(o, toff(t) + 4, 3, pc + 1);
        setb(o, 4, 1, pc == 0 ? 1 : pc == 3 ? 0 : lock);  // Lock / Release
        setb(o, toff(t), 4, pc == 1 ? iv : tv);           // Read: t = i
        setb(o, 0, 4, pc == 2 ? tv + 1 : iv);             // Write: i = t + 1
        return true;
    }
    SR_HD bool discovers(int p, const u64* s) const {
        u64 fin = 0, crit = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const u64 M = pc_mask(w), x = s[w];
            const u64 b0 = x & M, b1 = (x >> 1) & M, b2 = (x >> 2) & M;
            fin += __builtin_popcountll(b2 | (b1 & b0));   // pc >= 3
            crit += __builtin_popcountll(~b2 & (b1 | b0) & M);  // 1 <= pc < 4
        }
        if (p == 0) return fin != getb(s, 0, 4);  // always "fin"
        return crit > 1;                          // always "mutex"
    }
    int init_states(u64* out) const {
        for (int i = 0; i < W; ++i) out[i] = 0;
        return 1;
    }
    int expectation(int) const { return ALWAYS; }
    const char* prop_name(int p) const { return p == 0 ? "fin" : "mutex"; }
    // Exact key (quotient visited set), 5 + 6n bits: i and lock, then one 6-bit code per thread for
    // its (t, pc) pair: pc while pc < 2 (t is still 0 there: it is set by Read, pc 1 -> 2), else
    // 2 + 3t + (pc - 2) <= 49. Injective on every state whose threads hold t = 0 before their Read
    // and pc <= 4, i.e. on every reachable state. Two bits per thread shorter than the packed
    // words (5 + 7n): at N = 12 the key is 77 bits, so a table of 2^33 slots keeps 20 displacement
    // bits per slot (a probe limit far beyond any run) where the packed words left 8 (254 slots).
    int qkey_bits() const { return 5 + 6 * n; }
    SR_HD unsigned __int128 qkey(const u64* s) const {
        u64 lo = s[0] & 31, hi = 0;  // threads 0..8 in lo bits 5..58, threads 9.. in hi
        for (int t = 0; t < n; ++t) {
            const u64 f = getb(s, toff(t), 7);  // t | pc << 4
            const u64 tv = f & 15, pc = f >> 4;
            const u64 code = pc < 2 ? pc : 2 + 3 * tv + (pc - 2);
            if (t < 9) lo |= code << (5 + 6 * t);
            else hi |= code << (6 * (t - 9));
        }
        return (unsigned __int128)lo | ((unsigned __int128)hi << 59);
    }
    int describe_width() const { return 2 + 2 * n; }
    void describe(const u64* s, i64* d) const {
        d[0] = (i64)getb(s, 0, 4);
        d[1] = (i64)getb(s, 4, 1);
        for (int t = 0; t < n; ++t) {
            d[2 + 2 * t] = (i64)getb(s, toff(t), 4);
            d[3 + 2 * t] = (i64)getb(s, toff(t) + 4, 3);
        }
    }
    void undescribe(const i64* d, u64* s) const {
        for (int i = 0; i < W; ++i) s[i] = 0;
        setb(s, 0, 4, (u64)d[0]);
        setb(s, 4, 1, (u64)d[1]);
        for (int t = 0; t < n; ++t) {
            setb(s, toff(t), 4, (u64)d[2 + 2 * t]);
            setb(s, toff(t) + 4, 3, (u64)d[3 + 2 * t]);
        }
    }
    i64 action_id(const u64* s, int t) const { return 4 * t + (i64)getb(s, toff(t) + 4, 3); }
    i64 action_id_bound() const { return 4 * n; }
    std::string action_name(i64 id) const {
        const char* names[] = {"Lock", "Read", "Write", "Release"};
        return std::string(names[id % 4]) + "(" + std::to_string(id / 4) + ")";
    }
};

}  // namespace sr
