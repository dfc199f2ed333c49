// MI355X breadth-first model-checking engine: the host level loop over the HIP kernels, as a
// header of templates over a GpuModel M (models.hpp), so that the engine library (engine.hip: the
// compiled-in registry + the C ABI) and a user's own plugin build (include/stateright_gpu_model.hpp)
// instantiate the same code.
//
// Replaces `BfsChecker` (src/checker/bfs.rs). The reference's T worker threads, job market and
// 1500-state blocks (bfs.rs:75-152) become one host driver thread per GPU that runs the search
// level by level; each level is one pass of HIP kernels over the frontier held in HBM (kernels.hpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <immintrin.h>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/stateright_gpu.h"
#include "device.hpp"
#include "kernels.hpp"

namespace sr {


using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static inline u32 blocks_for(u64 n, u32 bs) { return (u32)((n + bs - 1) / bs); }

using Ctx = DeviceContext<LevelCounters, HostCounters>;
using CtxPool = ContextPool<Ctx>;

// Holds a pooled device context for the duration of a scope.
struct CtxLease {
    Ctx* c;
    explicit CtxLease(int dev) : c(CtxPool::get().acquire(dev)) {}
    ~CtxLease() { CtxPool::get().release(c); }
};

struct DiscoveryRec {
    bool found = false;
    u32 level = 0, rank = 0;  // the discovering state: rank in the visit order of its level
};

class EngineBase {
  public:
    virtual ~EngineBase() = default;
    virtual void run() = 0;
    virtual int nprops() const = 0;
    virtual const char* prop_name(int p) const = 0;
    virtual int expectation(int p) const = 0;
    virtual int width() const = 0;
    virtual std::string action_name(i64 id) const = 0;
    virtual int chain(int p, std::vector<u64>& out) = 0;
    virtual int path(int p, std::vector<i64>& actions, std::vector<i64>& states) = 0;
    virtual std::vector<i64> visits() const = 0;
    // Per visit (visit order): the visit index of its BFS-tree parent (-1 for an init state) and
    // the canonical id of the first action leading there (-1 for an init state). Returns false if
    // the engine keeps no visit record.
    virtual bool visit_tree(std::vector<i64>&, std::vector<i64>&) const { return false; }
    virtual i64 action_id_bound() const = 0;
    virtual int init_count() const = 0;
    // `Path::from_actions` (src/checker/path.rs:90-112) from init state `init`: the states, each
    // property's CONDITION on the last state, optionally on every state ((n + 1) x nprops), and
    // whether the last state is terminal (`actions()` lists nothing). -1: an action is not enabled.
    virtual int replay(int init, const i64* ids, int n, std::vector<i64>& states, std::vector<int>& conds,
                       std::vector<int>* all_conds = nullptr, int* terminal = nullptr) const = 0;
    virtual int explore(const u64* fps, int n, std::vector<i64>& action, std::vector<int>& has, std::vector<u64>& fp,
                        std::vector<i64>& states) const = 0;

    std::atomic<u64> state_count{0}, unique{0};
    std::atomic<u32> max_depth{0};
    std::atomic<bool> finished{false};
    bool reference_done = false;  // `is_done` (bfs.rs:307-311): explored all or discovered all
    int status = SR_OK;
    std::string error;
    sr_stats stats{};
    std::vector<DiscoveryRec> disc;
    std::vector<double> launch_ms;    // per timed launch (profile=1), in launch order
    std::vector<u64> launch_frontier; // the frontier each launch expanded (0 if unknown)
    std::vector<u64> launch_probes;   // visited-set probes / CAS claims of each launch (the pipelined
    std::vector<u64> launch_cas;      // FAST loop with sr_opts.counters; 0 otherwise)
};

// The model's init states (k * W words), in a buffer sized by init_capacity; a model that reports
// more states than fit is refused (every host-side caller goes through here, and the engines call
// it once when they are created, so a bad plugin fails at spawn).
template <class M>
std::vector<u64> init_states_of(const M& m) {
    const int cap = init_capacity(m);
    std::vector<u64> v((size_t)cap * M::W + M::W);  // one spare state: a model off by one is caught, not silent
    const int k = m.init_states(v.data());
    if (k < 0 || k > cap)
        throw Error(SR_ERR_ARG, "init_states returned " + std::to_string(k) + " states; at most " + std::to_string(cap) +
                                    " fit (a model with more than " + std::to_string(MAX_INIT_STATES) +
                                    " init states must report init_count())");
    v.resize((size_t)k * M::W);
    return v;
}

template <class M>
int replay_model(const M& m, int init, const i64* ids, int n, std::vector<i64>& states, std::vector<int>& conds,
                 std::vector<int>* all_conds, int* terminal) {
    constexpr int W = M::W;
    const std::vector<u64> inits = init_states_of(m);
    const int k = (int)(inits.size() / W);
    if (init < 0 || init >= k) return -1;
    const int wd = m.describe_width();
    std::vector<u64> cur(&inits[init * W], &inits[init * W] + W);
    // the property's condition (discovers() is !condition for `always`, the condition otherwise)
    auto cond = [&](int p, const u64* s) { return m.expectation(p) == ALWAYS ? !m.discovers(p, s) : m.discovers(p, s); };
    auto emit = [&](const u64* s) {
        size_t o = states.size();
        states.resize(o + wd);
        m.describe(s, &states[o]);
        if (all_conds)
            for (int p = 0; p < M::NPROPS; ++p) all_conds->push_back(cond(p, s) ? 1 : 0);
    };
    if (all_conds) all_conds->clear();
    for (int i = 0; i < n; ++i) {
        u64 mask[M::MW];
        m.enabled(cur.data(), mask);
        bool found = false;
        for (int w = 0; w < M::MW && !found; ++w)
            for (u64 bits = mask[w]; bits && !found; bits &= bits - 1) {
                int a = w * 64 + __builtin_ctzll(bits);
                if (m.action_id(cur.data(), a) != ids[i]) continue;
                u64 ns[W];
                if (!m.apply(cur.data(), a, ns)) continue;
                emit(cur.data());
                cur.assign(ns, ns + W);
                found = true;
            }
        if (!found) return -1;
    }
    emit(cur.data());
    conds.assign(M::NPROPS, 0);
    for (int p = 0; p < M::NPROPS; ++p) conds[p] = cond(p, cur.data()) ? 1 : 0;
    if (terminal) {
        u64 mask[M::MW];
        m.enabled(cur.data(), mask);
        u64 any = 0;
        for (int w = 0; w < M::MW; ++w) any |= mask[w];
        *terminal = any == 0;
    }
    return n;
}

// Explorer's `states` route (src/checker/explorer.rs:159-240) on the host copy of the encoding:
// with no fingerprints, the init states; otherwise `Path::final_state` (src/checker/path.rs:115-136:
// the init state with the first fingerprint, then the first matching step per fingerprint) and,
// for every action `actions()` lists there in order, the next state (has = 0: `next_state` is
// None, the reference's "Action ignored" view). Returns the number of views, or -1 if no state
// follows the fingerprints.
template <class M>
int explore_model(const M& m, const u64* fps, int n, std::vector<i64>& action, std::vector<int>& has,
                  std::vector<u64>& fp_out, std::vector<i64>& states) {
    constexpr int W = M::W;
    const int wd = m.describe_width();
    auto emit = [&](i64 a, const u64* s) {
        action.push_back(a);
        has.push_back(s ? 1 : 0);
        fp_out.push_back(s ? state_fp<M>(s) : 0);
        const size_t o = states.size();
        states.resize(o + wd, 0);
        if (s) m.describe(s, &states[o]);
    };
    const std::vector<u64> inits = init_states_of(m);
    const int k = (int)(inits.size() / W);
    if (n == 0) {
        for (int i = 0; i < k; ++i) emit(-1, &inits[i * W]);
        return k;
    }
    std::vector<u64> cur;
    for (int i = 0; i < k && cur.empty(); ++i)
        if (state_fp<M>(&inits[i * W]) == fps[0]) cur.assign(&inits[i * W], &inits[i * W] + W);
    if (cur.empty()) return -1;
    for (int j = 1; j < n; ++j) {
        u64 mask[M::MW];
        m.enabled(cur.data(), mask);
        bool found = false;
        for (int w = 0; w < M::MW && !found; ++w)
            for (u64 bits = mask[w]; bits && !found; bits &= bits - 1) {
                const int a = w * 64 + __builtin_ctzll(bits);
                u64 ns[W];
                if (m.apply(cur.data(), a, ns) && state_fp<M>(ns) == fps[j]) {
                    cur.assign(ns, ns + W);
                    found = true;
                }
            }
        if (!found) return -1;
    }
    u64 mask[M::MW];
    m.enabled(cur.data(), mask);
    int views = 0;
    for (int w = 0; w < M::MW; ++w)
        for (u64 bits = mask[w]; bits; bits &= bits - 1) {
            const int a = w * 64 + __builtin_ctzll(bits);
            u64 ns[W];
            const bool ok = m.apply(cur.data(), a, ns);
            emit(m.action_id(cur.data(), a), ok ? ns : nullptr);
            ++views;
        }
    return views;
}

// The model a host-side walk runs on: the original model under the canonical symmetry reduction
// (Canon<M> steps through orbit representatives; replay, the Explorer and discovery paths speak of
// concrete states of the original model) and under EvBits<M> (whose extra word is the search's
// bookkeeping), the model itself otherwise.
template <class M>
decltype(auto) base_model(const M& m) {
    if constexpr (is_canon<M>::value || is_evbits<M>::value) return m.base();
    else return (m);
}

// `Path::from_fingerprints` (src/checker/path.rs:20-86) over the states of a BFS-tree path (W words
// each): from the init state, each step is the FIRST action in `actions()` order whose successor is
// the next state. Under the canonical symmetry reduction (Canon<M>) the tree holds orbit
// representatives; the path is then made concrete in the original model: an init state whose
// representative is the first state, and at each step the first action whose successor's
// representative is the next one. Returns the number of actions; `raw` (optional) receives the
// concrete states (W words each), whose fingerprints are the discovery's chain.
template <class M>
int concrete_path(const M& m, const std::vector<u64>& st, std::vector<i64>& actions, std::vector<i64>& states,
                  std::vector<u64>* raw = nullptr) {
    constexpr int W = M::W;
    const size_t len = st.size() / W;
    if (!len) return -1;
    const int wd = m.describe_width();
    std::vector<u64> cur(st.begin(), st.begin() + W);
    if constexpr (is_canon<M>::value) {
        const std::vector<u64> inits = init_states_of(m.base());
        const int k = (int)(inits.size() / W);
        cur.clear();
        for (int i = 0; i < k && cur.empty(); ++i) {
            u64 c[W];
            m.base().canonical(&inits[i * W], c);
            if (std::equal(c, c + W, st.begin())) cur.assign(&inits[i * W], &inits[i * W] + W);
        }
        if (cur.empty()) throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path`: no init state has the expected representative");
    }
    auto emit = [&](const u64* s) {
        const size_t o = states.size();
        states.resize(o + wd);
        m.describe(s, &states[o]);
        if (raw) raw->insert(raw->end(), s, s + W);
    };
    for (size_t i = 1; i < len; ++i) {
        const u64* target = &st[i * W];
        u64 mask[M::MW];
        m.enabled(cur.data(), mask);
        bool found = false;
        for (int w = 0; w < M::MW && !found; ++w)
            for (u64 bits = mask[w]; bits && !found; bits &= bits - 1) {
                const int a = w * 64 + __builtin_ctzll(bits);
                u64 ns[W];
                if (!m.apply(cur.data(), a, ns) || !std::equal(ns, ns + W, target)) continue;
                u64 next[W];
                if constexpr (is_canon<M>::value) m.base().apply(cur.data(), a, next);
                else std::copy(ns, ns + W, next);
                emit(cur.data());
                actions.push_back(m.action_id(cur.data(), a));
                cur.assign(next, next + W);
                found = true;
            }
        if (!found)
            throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path`: " + std::to_string(i) +
                                                   " previous state(s) reconstructed but no successor is the next state");
    }
    emit(cur.data());
    return (int)actions.size();
}

// `reconstruct_path`'s fingerprint chain (src/checker/bfs.rs:314-342) of a BFS-tree path: the
// fingerprints of its states, or under Canon<M> of the concrete states of the original model that
// concrete_path walks (the ones `discovery_path`, `replay` and the Explorer speak of).
template <class M>
int fingerprint_chain(const M& m, const std::vector<u64>& st, std::vector<u64>& out) {
    constexpr int W = M::W;
    out.clear();
    std::vector<u64> raw;
    if constexpr (is_canon<M>::value) {
        std::vector<i64> actions, described;
        concrete_path(m, st, actions, described, &raw);
    } else {
        raw = st;
    }
    for (size_t i = 0; i < raw.size() / W; ++i) out.push_back(state_fp<M>(&raw[i * W]));
    return (int)out.size();
}

template <class M>
class Engine final : public EngineBase {
    static constexpr int W = M::W;
    static constexpr u32 WPB = (u32)expand_wpb<M>();  // expand_fast's waves per workgroup

  public:
    Engine(M m, const sr_opts& o)
        : m_(m), o_(o), A_((u32)m.max_actions()), D_((u32)m.max_out_degree()), emask_(model_emask(m)) {
        disc.resize(M::NPROPS);
        (void)init_states_of(m_);  // a model with more init states than it declares fails at spawn
        // Internal tuning knobs (not part of the ABI): successors per lane per probe round and
        // the visited-set load factor the capacity hint is sized for.
        if (const char* e = std::getenv("SR_PROBE_BATCH")) probe_batch_ = std::atoi(e);
        if (const char* e = std::getenv("SR_TABLE_LOAD")) table_load_ = std::atof(e), load_env_ = true;
        if (const char* e = std::getenv("SR_PPW_LOG2")) ppw_env_ = std::atoi(e);
        if (const char* e = std::getenv("SR_FILTER_LOG2")) filt_log2_ = (u32)std::atoi(e);
        // The LDS duplicate filter must be injective on states (kernels.hpp filter_key): one-word
        // states in either mode; a multi-word quotient-mode table runs without it.
        if (!filter_exact(m_)) filt_log2_ = 0;
        // 4-byte entries where they are exact: twice the entries in the same LDS (SR_FILTER_COMPACT=0: off)
        if (filt_log2_ && (!std::getenv("SR_FILTER_COMPACT") || std::atoi(std::getenv("SR_FILTER_COMPACT"))) &&
            filter_compact_ok(m_, filt_log2_ + 1))
            filt_log2_ += 1, filt_compact_ = true;
        // residencies per expand grid (expand_grid_cap): one for one-word states, two otherwise
        // (profiles/r06_grid_cap.txt). SR_GRID_RES (measurement knob) overrides.
        grid_res_ = W == 1 ? 1u : 2u;
        if (const char* e = std::getenv("SR_GRID_RES"))
            if (std::atoi(e) > 0) grid_res_ = (u32)std::atoi(e);
        if (const char* e = std::getenv("SR_PIPELINE")) pipeline_ = std::atoi(e) != 0;
        if (const char* e = std::getenv("SR_QUERY_LOG2")) query_mask_ = (1ull << std::atoi(e)) - 1;
        if (const char* e = std::getenv("SR_GRID_MAX")) grid_env_ = (u32)std::max(0, std::atoi(e));  // <= 0: unset
        if (const char* e = std::getenv("SR_WIDE_NOPF")) wide_nopf_ = std::atoi(e) ? 1 : 0;
        if (const char* e = std::getenv("SR_CHAIN_MAX")) chain_max_ = (u64)std::max(0ll, std::atoll(e));
        if (const char* e = std::getenv("SR_TABLE_KIND")) table_kind_ = std::atoi(e);
        if (const char* e = std::getenv("SR_TABLE_RECYCLE")) table_recycle_ = std::atoi(e) != 0;
    }
    ~Engine() override = default;

    int nprops() const override { return M::NPROPS; }
    const char* prop_name(int p) const override { return m_.prop_name(p); }
    int expectation(int p) const override { return m_.expectation(p); }
    int width() const override { return m_.describe_width(); }
    std::string action_name(i64 id) const override { return m_.action_name(id); }

    void run() override {
        SR_HIP(hipSetDevice(o_.device));
        CtxLease lease(o_.device);
        bind(lease.c);
        int order = o_.order;
        if (order == SR_ORDER_AUTO) order = o_.target_state_count ? SR_ORDER_FIFO : SR_ORDER_FAST;
        // `eventually` discoveries depend on the visit order (which generator passes its bits on,
        // which terminal state overwrites), so by default such models run in the reference's
        // single-threaded FIFO order. An explicit FAST order is honoured: each state takes the
        // bits of the generator that claims it, as in one of the reference's multi-threaded
        // orders (`threads(n)`, src/checker/bfs.rs:75-152), and the discoveries are valid
        // counterexamples of that order (the reference's false negatives may differ).
        if (emask_ && o_.order != SR_ORDER_FAST) order = SR_ORDER_FIFO;
        bool order_dependent = run_with_restart(order);
        if (order_dependent && o_.order == SR_ORDER_AUTO && order == SR_ORDER_FAST) {
            // An early exit inside a level makes counts depend on the visit order: redo the
            // check in the reference's exact FIFO order.
            if (o_.verbose) std::fprintf(stderr, "[sr] early exit in FAST order; re-running in FIFO order\n");
            run_with_restart(SR_ORDER_FIFO);
        }
        bind(nullptr);
    }

    // Capacity planning is optimistic (a chunk is sized for twice the previous level's growth, not
    // for every successor being new). If a level ever outgrows it, the device reports a full table
    // or arena and the check restarts from scratch in the pessimistic mode with larger buffers.
    bool run_with_restart(int order) {
        for (int attempt = 0;; ++attempt) {
            try {
                return run_order(order);
            } catch (const Error& e) {
                if (e.code != SR_ERR_CAPACITY || attempt >= 3) throw;
                if (o_.verbose) std::fprintf(stderr, "[sr] %s; restarting with larger buffers\n", e.what());
                pessimistic_ = true;
                grow_factor_ *= 4;
                (void)stream_sync(stream_);
                rehash_pending_ = false;  // (a failed enqueued rehash is this restart's cause, or moot)
                retired_keys_.clear();
                retired_arena_.clear();
                retired_u32_.clear();
                init_counters();
            }
        }
    }

    // `reconstruct_path` (src/checker/bfs.rs:314-342): the discovery's fingerprint chain, found by
    // walking parent ranks back through the BFS-tree arena.
    int chain(int p, std::vector<u64>& out) override {
        out.clear();
        if (p < 0 || p >= M::NPROPS || !disc[p].found) return 0;
        SR_HIP(hipSetDevice(o_.device));
        std::vector<u64> st;
        tree_path(disc[p].level, disc[p].rank, st);
        return fingerprint_chain(m_, st, out);
    }

    // States (W words each) from the init state down to (level, rank).
    void tree_path(u32 level, u32 rank, std::vector<u64>& st) {
        std::vector<u64> idx;
        u64 r = rank;
        for (int d = (int)level;; --d) {
            u64 a = lstart_[d] + r;
            idx.push_back(a);
            if (d == 0) break;
            u32 pr = 0;
            SR_HIP(hipMemcpy(&pr, apar_.p + a, sizeof(u32), hipMemcpyDeviceToHost));
            r = pr;
        }
        std::reverse(idx.begin(), idx.end());
        st.resize(idx.size() * W);
        for (size_t i = 0; i < idx.size(); ++i)
            SR_HIP(hipMemcpy(&st[i * W], arena_.p + idx[i] * W, W * sizeof(u64), hipMemcpyDeviceToHost));
    }

    // `Path::from_fingerprints` (src/checker/path.rs:20-86) on the host copy of the GpuModel.
    int path(int p, std::vector<i64>& actions, std::vector<i64>& states) override {
        if (p < 0 || p >= M::NPROPS || !disc[p].found) return -1;
        SR_HIP(hipSetDevice(o_.device));
        std::vector<u64> st;
        tree_path(disc[p].level, disc[p].rank, st);
        return concrete_path(m_, st, actions, states);
    }

    i64 action_id_bound() const override { return m_.action_id_bound(); }
    int init_count() const override { return (int)(init_states_of(base_model(m_)).size() / std::decay_t<decltype(base_model(m_))>::W); }
    // replay and the Explorer walk concrete states of the original model (under Canon<M> too)
    int replay(int init, const i64* ids, int n, std::vector<i64>& states, std::vector<int>& conds,
               std::vector<int>* all_conds, int* terminal) const override {
        return replay_model(base_model(m_), init, ids, n, states, conds, all_conds, terminal);
    }
    int explore(const u64* fps, int n, std::vector<i64>& action, std::vector<int>& has, std::vector<u64>& fp,
                std::vector<i64>& states) const override {
        return explore_model(base_model(m_), fps, n, action, has, fp, states);
    }

    // The visitor's paths (src/checker/bfs.rs:187-189 builds `Path::from_fingerprints` of every
    // popped state): each visited state's BFS-tree parent and the FIRST action, in `actions()`
    // order, that leads from the parent to it (src/checker/path.rs:55-79).
    bool visit_tree(std::vector<i64>& parent, std::vector<i64>& action) const override {
        parent.clear();
        action.clear();
        std::vector<u64> prev_states;
        i64 prev_base = 0;  // visit index of the previous level's first state
        for (size_t d = 0; d < lvisited_.size(); ++d) {
            const u64 nv = lvisited_[d];
            std::vector<u64> st(nv * W);
            std::vector<u32> par(nv);
            if (nv) {
                SR_HIP(hipMemcpy(st.data(), arena_.p + lstart_[d] * W, nv * W * sizeof(u64), hipMemcpyDeviceToHost));
                SR_HIP(hipMemcpy(par.data(), apar_.p + lstart_[d], nv * sizeof(u32), hipMemcpyDeviceToHost));
            }
            const i64 base = (i64)parent.size();
            for (u64 i = 0; i < nv; ++i) {
                if (d == 0) {
                    parent.push_back(-1);
                    action.push_back(-1);
                    continue;
                }
                const u64 pr = par[i];
                if (pr >= prev_states.size() / W) throw Error(SR_ERR_NONDETERMINISM, "visit parent outside the visited prefix");
                const u64* ps = &prev_states[pr * W];
                const u64 want = state_fp<M>(&st[i * W]);
                u64 mask[M::MW];
                m_.enabled(ps, mask);
                i64 id = -1;
                for (int w = 0; w < M::MW && id < 0; ++w)
                    for (u64 bits = mask[w]; bits && id < 0; bits &= bits - 1) {
                        const int a = w * 64 + __builtin_ctzll(bits);
                        u64 ns[W];
                        if (m_.apply(ps, a, ns) && state_fp<M>(ns) == want) id = m_.action_id(ps, a);
                    }
                if (id < 0) throw Error(SR_ERR_NONDETERMINISM, "Unable to reconstruct a `Path` for a visited state");
                parent.push_back(prev_base + (i64)pr);
                action.push_back(id);
            }
            prev_states.swap(st);
            prev_base = base;
        }
        return true;
    }

    std::vector<i64> visits() const override {
        const int wd = m_.describe_width();
        std::vector<u64> st;
        for (size_t d = 0; d < lvisited_.size(); ++d) {
            size_t o = st.size();
            st.resize(o + lvisited_[d] * W);
            if (lvisited_[d])
                SR_HIP(hipMemcpy(&st[o], arena_.p + lstart_[d] * W, lvisited_[d] * W * sizeof(u64), hipMemcpyDeviceToHost));
        }
        std::vector<i64> out(st.size() / W * wd);
        for (size_t i = 0; i < st.size() / W; ++i) m_.describe(&st[i * W], &out[i * wd]);
        return out;
    }

  private:
    TableView view() const { return make_table_view(m_, keys_.p, fifo_ ? meta_.p : nullptr, cap_); }

    // zero = false: the caller writes every slot (rehash_ranges), so no clear is enqueued.
    void alloc_table(u64 cap, bool zero = true) {
        cap_ = cap;
        lmax_ = max_load(cap);
        const u64 words = table_words(make_table_view(m_, nullptr, nullptr, cap), cap);
        table_unzeroed_ = false;
        if (zero) keys_.alloc_zero(o_.device, words, stream_, table_kind_);
        else keys_.alloc(o_.device, words, table_kind_);
        if (fifo_) {
            meta_.alloc(o_.device, cap);
            SR_HIP(hipMemsetAsync(meta_.p, 0xff, cap * sizeof(u64), stream_));
        }
    }

    // Doubles the visited set (quotient mode: one more displacement bit per slot, so twice the
    // probe limit). If an entry does not fit the new table's probe limit, the rehash starts over
    // from the old table into one twice as large again. In FIFO order the level's candidate slots
    // (cand) are remapped to the new table, since the rehash moves every entry.
    // min_slots: grow to at least this many slots (one rehash, however many doublings that is).
    void grow_table(u32* cand = nullptr, u64 cand_n = 0, u64 min_slots = 0) {
        check_async_growth();  // an earlier asynchronous rehash's outcome first (aux_ is reused)
        const auto tg = Clock::now();
        DBuf<u64> ok, om;
        ok.swap(keys_);
        if (fifo_) om.swap(meta_);
        const TableView from = make_table_view(m_, ok.p, fifo_ ? om.p : nullptr, cap_);
        const u64 old_cap = cap_;
        if (!aux_.p) aux_.alloc(o_.device, 2);
        u64 f0 = 2;
        while (old_cap * f0 < min_slots) f0 *= 2;
        for (u64 f = f0;; f *= 2) {
            launch_rehash(from, old_cap, f);
            u32 err = 0;
            SR_HIP(hipMemcpyAsync(&err, aux_.p, sizeof(u32), hipMemcpyDeviceToHost, stream_));
            SR_HIP(stream_sync(stream_));
            if (!err) break;
            if (f >= 64) throw Error(SR_ERR_CAPACITY, "rehash: probe limit exceeded at 64x the capacity");
        }
        if (cand && cand_n) {
            remap_slots<<<blocks_for(cand_n, 256), 256, 0, stream_>>>(cand, cand_n, from, view());
            SR_HIP(hipGetLastError());
        }
        SR_HIP(stream_sync(stream_));
        stats.rehashes++;
        if (o_.verbose)
            std::fprintf(stderr, "[sr] visited set %llu -> %llu slots in %.3f ms\n", (unsigned long long)old_cap,
                         (unsigned long long)cap_, secs(tg, Clock::now()) * 1e3);
    }

    // The same growth ENQUEUED behind the level in flight, without waiting for it (the early growth
    // of the pipelined loop, FAST order): the rehash reads the whole old table, so it needs nothing
    // from the host, and the next level is launched on the new table right behind it. The old table
    // is retired until the stream has passed the rehash (retire / release_retired), and the rehash's
    // error word is read at the next synchronous point (check_async_growth): an entry that did not
    // fit the new table fails the check with a capacity error, and the check restarts.
    void grow_table_async(u64 min_slots) {
        check_async_growth_pending_first();
        retired_keys_.emplace_back();
        retired_keys_.back().swap(keys_);
        const TableView from = make_table_view(m_, retired_keys_.back().p, nullptr, cap_);
        const u64 old_cap = cap_;
        if (!aux_.p) aux_.alloc(o_.device, 2);
        u64 f = 2;
        while (old_cap * f < min_slots) f *= 2;
        launch_rehash(from, old_cap, f);
        rehash_pending_ = true;
        stats.rehashes++;
        if (o_.verbose)
            std::fprintf(stderr, "[sr] visited set %llu -> %llu slots enqueued\n", (unsigned long long)old_cap,
                         (unsigned long long)cap_);
    }
    // Allocates the table of old_cap * f slots and enqueues the rehash of `from` into it (error bits
    // in aux_[0]): range by range without a clear (rehash_ranges + rehash_spill) when the new homes
    // of a range of old homes are a range (quotient mode, f = 2^(from.qbits - to.qbits)) and no meta
    // moves along (FAST order), else a clear plus one CAS insertion per entry (rehash).
    // SR_REHASH_RANGES=0 (measurement knob) always takes the latter.
    void launch_rehash(const TableView& from, u64 old_cap, u64 f) {
        const u64 cap = old_cap * f;
        const TableView to0 = make_table_view(m_, nullptr, nullptr, cap);
        u32 lg = 0;
        while ((1ull << lg) < f) ++lg;
        const u64 S = to0.s32 ? rebuild_slots<u32>() : rebuild_slots<u64>();
        const bool ranges = rehash_ranges_ && !from.meta && from.qbits && to0.qbits &&
                            from.qbits == to0.qbits + lg && f <= S && cap % S == 0;
        alloc_table(cap, !ranges);
        table_unzeroed_ = ranges;
        SR_HIP(hipMemsetAsync(aux_.p, 0, sizeof(u32), stream_));
        if (ranges) {
            const u64 nranges = cap / S, spill_cap = nranges + 65536;
            if (spill_.n < spill_cap + 1) spill_.alloc(o_.device, spill_cap + 1);
            SR_HIP(hipMemsetAsync(spill_.p, 0, sizeof(u64), stream_));
            if (to0.s32)
                rehash_ranges<u32><<<(u32)nranges, REBUILD_BLOCK, 0, stream_>>>(from, old_cap, view(), lg, spill_.p,
                                                                               spill_cap, aux_.p);
            else
                rehash_ranges<u64><<<(u32)nranges, REBUILD_BLOCK, 0, stream_>>>(from, old_cap, view(), lg, spill_.p,
                                                                               spill_cap, aux_.p);
            SR_HIP(hipGetLastError());
            rehash_spill<<<256, 256, 0, stream_>>>(from, view(), spill_.p, spill_cap, aux_.p);
        } else {
            rehash<<<blocks_for(old_cap, 256), 256, 0, stream_>>>(from, old_cap, view(), aux_.p);
        }
        SR_HIP(hipGetLastError());
    }
    bool rehash_ranges_ = !std::getenv("SR_REHASH_RANGES") || std::atoi(std::getenv("SR_REHASH_RANGES")) != 0;
    DBuf<u64> spill_;  // rehash_ranges' spill list: [0] count, then old slot indices
    // The visited set was built by rehash_ranges (allocated without a clear): released without one
    // too, since the next unhinted check grows into its tables the same way (a hinted check clears
    // what it takes).
    bool table_unzeroed_ = false;

    // (an asynchronous growth is enqueued only while none is pending)
    void check_async_growth_pending_first() {
        if (rehash_pending_) check_async_growth();
    }
    // The outcome of an enqueued rehash (waits for the stream) and the retired buffers released.
    void check_async_growth() {
        if (!rehash_pending_ && retired_keys_.empty() && retired_arena_.empty()) return;
        SR_HIP(stream_sync(stream_));
        retired_keys_.clear();
        retired_arena_.clear();
        retired_u32_.clear();
        if (!rehash_pending_) return;
        rehash_pending_ = false;
        u32 err = 0;
        SR_HIP(hipMemcpy(&err, aux_.p, sizeof(u32), hipMemcpyDeviceToHost));
        if (err) throw Error(SR_ERR_CAPACITY, "an enqueued rehash exceeded the new table's probe limit");
    }
    bool rehash_pending_ = false;
    std::vector<DBuf<u64>> retired_keys_, retired_arena_;
    std::vector<DBuf<u32>> retired_u32_;

    // Growth during a check (no capacity hint, or one too small: the path a user of the reference
    // gets, whose DashMap grows as it goes, src/checker/bfs.rs:26) takes a few large steps rather
    // than doublings: every growth stops the level pipeline, and a table growth rehashes every
    // entry. A step multiplies the size by SR_GROW_STEP (default 8), within a share of the free
    // device memory (never below what the level needs).
    u64 growth_slots(u64 need_slots) const {
        // the first growth of a check that started without a hint (the model has outgrown the
        // default table) takes a larger step, SR_GROW_FIRST (measurement knob; 0: grow_step_)
        const u64 step = !o_.capacity_hint && stats.rehashes == 0 && grow_first_ ? grow_first_ : grow_step_;
        u64 target = std::max<u64>(need_slots, cap_ * step);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b) target = std::min<u64>(target, std::max<u64>(need_slots, free_b / 4 / 8));
        return target;
    }
    u64 grow_step_ = std::getenv("SR_GROW_STEP") && std::atoi(std::getenv("SR_GROW_STEP")) >= 2
                         ? (u64)std::atoi(std::getenv("SR_GROW_STEP")) : 8u;
    u64 grow_first_ = std::getenv("SR_GROW_FIRST") ? (u64)std::atoi(std::getenv("SR_GROW_FIRST")) : 0u;

    // The growth threshold of the visited set: 0.8 load, or lower for a quotient-mode table whose
    // probe limit (set by its displacement bits) would otherwise be reached by the longest
    // linear-probe run to be expected at that load (kernels.hpp max_load_for).
    double max_load(u64 cap) const {
        const TableView v = make_table_view(m_, nullptr, nullptr, cap, true);
        return max_load_for(v.plimit, (double)cap, 0.8);
    }

    // sr_stats.max_displacement / displacement_limit of the final table (the scan runs only in a
    // measurement pass, sr_opts.counters: it reads the whole table).
    void displacement_stats() {
        const TableView v = view();
        stats.displacement_limit = v.plimit;
        if (!o_.counters || !cap_) return;
        if (!aux_.p) aux_.alloc(o_.device, 2);
        SR_HIP(hipMemsetAsync(aux_.p + 1, 0, sizeof(u32), stream_));
        const u32 grid = (u32)std::min<u64>(blocks_for(cap_, 256), 8192);
        table_max_disp<<<grid, 256, 0, stream_>>>(v, cap_, aux_.p + 1);
        SR_HIP(hipGetLastError());
        u32 d = 0;
        SR_HIP(hipMemcpyAsync(&d, aux_.p + 1, sizeof(u32), hipMemcpyDeviceToHost, stream_));
        SR_HIP(stream_sync(stream_));
        stats.max_displacement = d;
    }

    // The BFS-tree arena holds every level's states (visit order) and their parent ranks; grows
    // by copying the used prefix.
    // async: the copy is enqueued behind the work in flight and the old buffers retired until the
    // stream has passed it (check_async_growth), instead of waiting here.
    // The arena's growth step (SR_ARENA_STEP; default 8 for states of <= 2 words, 4 for wider ones, as
    // every model until round 6): unhinted 2pc N=10 8.17-8.24 -> 7.93-8.00 ms, increment_lock N=11
    // 33.9-35.0 -> 32.5-33.3; paxos C=6 (W = 12) 3.02-3.04 -> 3.20-3.21 with 8, so it keeps 4
    // (profiles/r06_arena_step.txt).
    u64 arena_step_ = std::getenv("SR_ARENA_STEP") && std::atoi(std::getenv("SR_ARENA_STEP")) >= 2
                          ? (u64)std::atoi(std::getenv("SR_ARENA_STEP")) : W <= 2 ? 8u : 4u;
    void ensure_arena(u64 states, u64 used, bool async = false) {
        if (arena_cap_ >= states) return;
        const auto ta = Clock::now();
        // (each growth step copies the arena so far and stops the level pipeline; a step never takes
        // more than half the device's free memory, nor less than `states`)
        u64 cap = std::max<u64>(states, arena_cap_ * (arena_cap_ ? arena_step_ : 1));
        if (cap > states) {
            size_t fr = 0, tot = 0;
            const u64 per = W * sizeof(u64) + sizeof(u32) + (emask_ ? sizeof(u32) : 0);
            if (hipMemGetInfo(&fr, &tot) == hipSuccess) cap = std::max<u64>(states, std::min<u64>(cap, fr / 2 / per));
            else (void)hipGetLastError();
        }
        DBuf<u64> na;
        DBuf<u32> np, ne;
        na.alloc(o_.device, cap * W);
        np.alloc(o_.device, cap);
        if (emask_) ne.alloc(o_.device, cap);
        const double alloc_ms = secs(ta, Clock::now()) * 1e3;
        if (used) {
            SR_HIP(hipMemcpyAsync(na.p, arena_.p, used * W * sizeof(u64), hipMemcpyDeviceToDevice, stream_));
            SR_HIP(hipMemcpyAsync(np.p, apar_.p, used * sizeof(u32), hipMemcpyDeviceToDevice, stream_));
            if (emask_) SR_HIP(hipMemcpyAsync(ne.p, aeb_.p, used * sizeof(u32), hipMemcpyDeviceToDevice, stream_));
        }
        const bool had = arena_.p != nullptr;
        arena_.swap(na);
        apar_.swap(np);
        if (emask_) aeb_.swap(ne);
        arena_cap_ = cap;
        // the old buffers go back to the pool when na/np/ne leave scope: wait until no enqueued work
        // reads them (a first allocation has none, and the start of a check does not wait here)
        if (had && async) {
            retired_arena_.emplace_back();
            retired_arena_.back().swap(na);
            retired_u32_.emplace_back();
            retired_u32_.back().swap(np);
            retired_u32_.emplace_back();
            retired_u32_.back().swap(ne);
        } else if (had) {
            SR_HIP(stream_sync(stream_));
        }
        if (o_.verbose && had)
            std::fprintf(stderr, "[sr] arena -> %llu states (%llu copied) in %.3f ms (allocation %.3f ms)\n",
                         (unsigned long long)cap, (unsigned long long)used, secs(ta, Clock::now()) * 1e3, alloc_ms);
    }

    void bind(Ctx* c) {
        ctx_ = c;
        stream_ = c ? c->stream : nullptr;
        lc_d_ = c ? c->lc : nullptr;
    }

    // Device counters to their level-start values (once per run; afterwards the publishing
    // workgroup of each level resets them).
    void init_counters() {
        if (!slots_.p) slots_.alloc(o_.device, (SLOTS * sizeof(LevelCounters) + 7) / 8);
        init_level_counters<<<1, 256, 0, stream_>>>(lc_d_, reinterpret_cast<LevelCounters*>(slots_.p), SLOTS);
        SR_HIP(hipGetLastError());
        slot_k_ = 0;
        slot_published_ = true;
    }

    // Per-level counter slots of the pipelined loop (SlotWork, kernels.hpp).
    LevelCounters* slot(u32 k) const { return reinterpret_cast<LevelCounters*>(slots_.p) + (k % SLOTS); }
    // The slot duties of the next slotted launch: its frontier size from the previous slot (dev_n),
    // the previous slot's publish unless it is already done, and the reset of slot K-2.
    SlotWork slot_work(bool dev_n) {
        SlotWork sw{};
        if (dev_n) sw.prev_n = slot_k_ ? &slot(slot_k_ - 1)->claims : &lc_d_->prev_claims;
        if (slot_k_ && !slot_published_) {
            sw.pub = slot(slot_k_ - 1);
            sw.hc = hcd(slot_seq_);
            sw.seq = slot_seq_;
            slot_published_ = true;
        }
        if (slot_k_ >= 2) sw.zero = slot(slot_k_ - 2);
        return sw;
    }
    // The last slotted level's publish, when no launch that would carry it is enqueued before the
    // host waits for it.
    void publish_pending_slot() {
        if (slot_published_) return;
        SlotWork sw{};
        sw.pub = slot(slot_k_ - 1);
        sw.hc = hcd(slot_seq_);
        sw.seq = slot_seq_;
        slot_publish_kernel<M::NPROPS><<<1, 64, 0, stream_>>>(sw);
        SR_HIP(hipGetLastError());
        slot_published_ = true;
    }
    u32 next_seq() { return ++ctx_->seq; }
    HostCounters* hcd(u32 seq) const { return ctx_->hc_dev + (seq & 1); }  // device view of seq's mirror

    // Waits until the launch tagged `seq` has published its counters to pinned host memory: a
    // spin on one host word (no stream synchronisation, no copy), with a periodic stream query
    // so that a failed launch cannot hang the host.
    // recoverable: a level that overflowed the visited set's probe limit (and nothing else) returns
    // false instead of throwing; the caller doubles the table and repairs the level.
    bool wait_publish(u32 seq, bool recoverable = false) {
        volatile u32* flag = &ctx_->hc[seq & 1].seq;
        for (u64 spin = 1;; ++spin) {
            if (*flag == seq) break;
            if ((spin & query_mask_) == 0) {
                hipError_t e = hipStreamQuery(stream_);
                if (e != hipSuccess && e != hipErrorNotReady) SR_HIP(e);
                if (e == hipSuccess && *flag != seq) {
                    if (*flag == seq) break;
                    throw Error(SR_ERR_HIP, "launch finished without publishing its counters");
                }
            }
            _mm_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        std::memcpy(&lc_, (const void*)&ctx_->hc[seq & 1], sizeof(lc_));
        if (recoverable && (lc_.err == ERR_TABLE_FULL || lc_.err == ERR_DEFERRED)) return false;
        if (lc_.err & ERR_TABLE_FULL) throw Error(SR_ERR_CAPACITY, "visited set probe limit exceeded");
        if (lc_.err & ERR_DEFERRED) throw Error(SR_ERR_CAPACITY, "deferred level");
        if (lc_.err & ERR_FRONTIER_OVERFLOW) throw Error(SR_ERR_CAPACITY, "frontier overflow");
        return true;
    }

    // A level (frontier of n states at arena offset fbase) whose expansion overflowed the visited
    // set's probe limit: its successors were all counted, but some were neither found nor claimed.
    // The table is doubled (quotient mode: one more displacement bit, twice the probe limit) and
    // the level is expanded again in repair mode on the larger table: every successor is probed
    // again, the states still missing are claimed and appended after the ones the first pass
    // appended, and no successor is counted twice. A launch enqueued behind the failed level saw
    // its err word and expanded nothing. lc_ holds the failed pass's counters on entry and the
    // level's complete counters on return (the slot ring starts over).
    void repair_level(u64 fbase, u64 n, u32 undiscovered) {
        const HostCounters first = lc_;
        u32 dmin[MAX_PROPS];  // discoveries among the states appended by every pass, failed ones too
        std::copy(first.disc, first.disc + MAX_PROPS, dmin);
        for (int attempt = 0;; ++attempt) {
            if (attempt >= 8) throw Error(SR_ERR_CAPACITY, "visited set probe limit exceeded after 8 doublings");
            SR_HIP(stream_sync(stream_));
            if (o_.verbose)
                std::fprintf(stderr, "[sr] level of %llu states overflowed the probe limit %u at %llu slots: doubling\n",
                             (unsigned long long)n, view().plimit, (unsigned long long)cap_);
            grow_table();
            stats.table_doublings++;
            const u32 partial = lc_.claims;
            init_counters();  // the slot ring starts over: slot 0 continues the level's frontier cursor
            SR_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&slot(0)->claims), (int)partial, 1, stream_));
            const u32 sq = launch_expand(fbase, (u32)n, false, n, undiscovered, SLOT_REPAIR);
            publish_pending_slot();
            const bool ok = wait_publish(sq, true);
            for (int p = 0; p < MAX_PROPS; ++p) dmin[p] = std::min(dmin[p], lc_.disc[p]);
            if (ok) break;
        }
        // successors and enabled slots: the first pass counted them all; claims: the repair's cursor
        lc_.successors = first.successors;
        lc_.enabled = first.enabled;
        lc_.probes += first.probes;
        lc_.cas += first.cas;
        std::copy(dmin, dmin + MAX_PROPS, lc_.disc);
    }

    // Launch bracketed by pooled events (profile=1); durations are summed once at the end of the
    // run, so timing adds no synchronisation to the level loop.
    template <class F>
    void timed(F&& launch, u64 frontier = 0) {
        size_t i = 2 * stats.expand_launches;
        if (o_.profile) SR_HIP(hipEventRecord(ctx_->event(i), stream_));
        launch();
        SR_HIP(hipGetLastError());
        if (o_.profile) SR_HIP(hipEventRecord(ctx_->event(i + 1), stream_));
        stats.expand_launches++;
        launch_frontier.push_back(frontier);
        launch_probes.push_back(0);
        launch_cas.push_back(0);
    }
    void collect_timing() {
        if (!o_.profile || !stats.expand_launches) return;
        SR_HIP(hipEventSynchronize(ctx_->event(2 * stats.expand_launches - 1)));
        double ms = 0;
        launch_ms.assign(stats.expand_launches, 0.0);
        for (u64 i = 0; i < stats.expand_launches; ++i) {
            float t = 0;
            SR_HIP(hipEventElapsedTime(&t, ctx_->event(2 * i), ctx_->event(2 * i + 1)));
            ms += t;
            launch_ms[i] = t;
        }
        stats.expand_kernel_ms = ms;
    }

    // Returns true when the run stopped early inside a level in an order-dependent way.
    bool run_order(int order) {
        auto t_start = Clock::now();
        fifo_ = order == SR_ORDER_FIFO;
        state_count = 0;
        unique = 0;
        max_depth = 0;
        for (auto& d : disc) d = DiscoveryRec{};
        stats = sr_stats{};
        stats.words_per_state = W;
        stats.order_used = (u32)order;
        launch_ms.clear();
        launch_frontier.clear();
        launch_probes.clear();
        launch_cas.clear();
        seq_launch_.clear();

        // Visited set sized for <= table_load_ load at the hinted unique count.
        // (without a hint: 2^22 slots, 32 MiB, a few us to clear and recycled between checks; the
        // table then grows in steps of SR_GROW_STEP)
        u64 cap = std::max<u64>((u64)(1u << 22) * grow_factor_, min_table_cap(m_));
        // Hints beyond 2^31 states (increment_lock N=12: 5.2e9) size the table for <= 0.75 load and
        // the arena with 30% slack, so that table + arena fit one MI355X's 288 GB.
        const bool huge = o_.capacity_hint > (1ull << 31);
        const double load = huge && !load_env_ ? 0.75 : table_load_;
        // (a quotient-mode table also stays under the load its probe limit allows, max_load)
        if (o_.capacity_hint)
            while ((double)cap * std::min(load, max_load(cap)) < (double)o_.capacity_hint * grow_factor_) cap <<= 1;
        ratio_ = (double)D_;
        nratio_ = 0;
        en_ratio_ = std::max(1.0, (double)D_ / 2.0);
        alloc_table(cap);

        // Init states (bfs.rs:43-66): all of them are counted and queued (duplicates too), the
        // visited set keeps distinct ones; `pending` pops from the back, so level 0 is visited in
        // REVERSE init order.
        const std::vector<u64> f0 = init_states_of(m_);
        const int k = (int)(f0.size() / W);
        std::vector<u64> rev(k * W);
        for (int i = 0; i < k; ++i) std::copy(&f0[i * W], &f0[i * W] + W, &rev[(k - 1 - i) * W]);
        arena_cap_ = 0;
        // hinted: room for every state plus one level's worth of planning slack (a regrowth copies
        // the whole arena mid-run)
        const u64 slack = huge ? o_.capacity_hint / 10 * 3 : o_.capacity_hint / 2;
        // (without a hint: 2^24 words, 128 MiB + its parent ranks, never cleared and pooled across
        // checks, so that the early table growth needs no arena copy behind it: 2pc N=9 fits)
        const u64 arena0 = o_.capacity_hint ? (1u << 22) / W : (1u << 24) / W;
        ensure_arena(std::max<u64>(std::max<u64>(1u << 16, arena0), (o_.capacity_hint + slack + 1024) * grow_factor_), 0);
        lstart_.assign({0, (u64)k});
        lvisited_.clear();
        const u32 und0 = ((1u << M::NPROPS) - 1) & ~emask_;
        u32 sq = 0;
        if ((u64)k * W <= ROOTS_INLINE_WORDS) {
            // one launch: counters reset, level 0 into the arena (no parents; `eventually` bits
            // pending, bfs.rs:52-60), roots inserted and evaluated, published
            InlineStates init{};
            std::copy(rev.begin(), rev.end(), init.w);
            if (!slots_.p) slots_.alloc(o_.device, (SLOTS * sizeof(LevelCounters) + 7) / 8);
            slot_k_ = 0;
            slot_published_ = true;
            sq = next_seq();
            roots_start<M><<<1, 256, 0, stream_>>>(m_, view(), init, (u32)k, arena_.p, apar_.p, emask_ ? aeb_.p : nullptr,
                                                   emask_, lc_d_, reinterpret_cast<LevelCounters*>(slots_.p), SLOTS,
                                                   und0, hcd(sq), sq);
        } else {
            SR_HIP(hipMemcpyAsync(arena_.p, rev.data(), rev.size() * sizeof(u64), hipMemcpyHostToDevice, stream_));
            SR_HIP(hipMemsetAsync(apar_.p, 0xff, (size_t)k * sizeof(u32), stream_));
            init_counters();
            if (emask_) fill_u32<<<blocks_for(k, 64), 64, 0, stream_>>>(aeb_.p, (u32)k, emask_);  // bfs.rs:52-60
            sq = next_seq();
            if (k <= 256) {
                roots_fused<M><<<1, 256, 0, stream_>>>(m_, view(), arena_.p, (u32)k, lc_d_, und0, hcd(sq), sq);
            } else {
                insert_roots<M><<<blocks_for(k, 64), 64, 0, stream_>>>(m_, view(), arena_.p, (u32)k, lc_d_);
                eval_roots<M><<<blocks_for(k, 64), 64, 0, stream_>>>(m_, arena_.p, (u32)k, lc_d_, und0);
                publish_kernel<<<1, 64, 0, stream_>>>(lc_d_, hcd(sq), sq, 1, nullptr);
            }
        }
        SR_HIP(hipGetLastError());
        // FAST pipelined order: level 0 is enqueued before the host reads the roots' outcome (it is
        // ignored if the roots already discover every property)
        const bool pipelined = !fifo_ && !emask_ && !o_.target_state_count && M::NPROPS > 0 && pipeline_;
        const u32 sq_level0 = pipelined ? launch_sync((u64)k, (1u << M::NPROPS) - 1) : 0u;
        wait_publish(sq);
        state_count = (u64)k;
        unique = lc_.claims;

        u32 undiscovered = (1u << M::NPROPS) - 1;
        u64 n = (u64)k, popped_before = 0;
        u32 level = 0;
        bool order_dependent = false;
        auto t_loop = Clock::now();
        if (pipelined) order_dependent = pipeline_levels(n, sq_level0);
        else for (;;) {
            // 1. Discoveries among this level's states (evaluated when they were produced).
            u32 newly = 0, max_rank = 0;
            for (int p = 0; p < M::NPROPS; ++p)
                if ((undiscovered >> p & 1) && lc_.disc[p] != ~0u) {
                    newly |= 1u << p;
                    max_rank = std::max(max_rank, lc_.disc[p]);
                    disc[p].found = true;
                    disc[p].level = level;
                    disc[p].rank = lc_.disc[p];
                }
            // `eventually` properties: the first terminal candidate of each undiscovered one.
            const u32 eund = undiscovered & emask_;
            std::vector<u32> evf(M::NPROPS, ~0u);
            DBuf<u32> tsat, evd;
            if (emask_ && n) {
                tsat.alloc(o_.device, n);
                evd.alloc(o_.device, 2 * M::NPROPS);  // [first terminal candidate | last terminal + 1]
                SR_HIP(hipMemsetAsync(evd.p, 0xff, M::NPROPS * sizeof(u32), stream_));
                SR_HIP(hipMemsetAsync(evd.p + M::NPROPS, 0, M::NPROPS * sizeof(u32), stream_));
                ev_scan<M><<<blocks_for(n, 256), 256, 0, stream_>>>(m_, cur(), aeb_.p + lstart_[level], (u32)n, eund,
                                                                    emask_, tsat.p, evd.p);
                SR_HIP(hipGetLastError());
                SR_HIP(hipMemcpyAsync(evf.data(), evd.p, M::NPROPS * sizeof(u32), hipMemcpyDeviceToHost, stream_));
                SR_HIP(stream_sync(stream_));
            }
            u64 limit = n, visited = n;
            bool stop = false;
            if (M::NPROPS == 0) {
                limit = 0;
                visited = std::min<u64>(1, n);
                stop = true;
            } else if (undiscovered == 0) {
                // Every property was discovered at a terminal state of the previous level: the next
                // pop finds nothing to await and returns (bfs.rs:226).
                limit = 0;
                visited = std::min<u64>(1, n);
                stop = true;
                order_dependent = true;
            } else {
                // The first pop at which every property is discovered: always/sometimes ones at the
                // pop of their discovering state, eventually ones right after their terminal state.
                const u32 pop_und = undiscovered & ~emask_;
                bool all = (newly & pop_und) == pop_und;
                u64 at = newly ? (u64)max_rank : 0;
                for (u32 e = eund; e; e &= e - 1) {
                    const int p = __builtin_ctz(e);
                    if (evf[p] == ~0u) all = false;
                    else at = std::max<u64>(at, (u64)evf[p] + 1);
                }
                if (all && at < n) {
                    // The pop of rank `at` finds every property discovered: check_block returns
                    // without expanding it (bfs.rs:226) and the worker shuts down (bfs.rs:121-128).
                    limit = at;
                    visited = at + 1;
                    stop = true;
                    order_dependent = true;
                }
            }
            undiscovered &= ~newly;

            // 2. target_state_count: the reference checks it after each 1500-pop block (bfs.rs:113-135).
            bool target_stop = false;
            if (o_.target_state_count && state_count + limit * D_ >= o_.target_state_count) {
                u64 lt = target_limit(n, popped_before, limit);
                if (lt != ~0ull) {
                    limit = lt;
                    visited = lt;
                    target_stop = true;
                    stop = true;
                    order_dependent = true;
                }
            }

            lvisited_.push_back(visited);

            // 3. Expand ranks [0, limit) (eventually: the bits passed on, terminal discoveries).
            u64 produced = 0;
            DBuf<u32> peb;
            std::vector<u32> evl(M::NPROPS, 0);
            if (emask_ && limit) {
                peb.alloc(o_.device, limit);
                ev_resolve<<<blocks_for(limit, 256), 256, 0, stream_>>>(tsat.p, aeb_.p + lstart_[level], (u32)limit, eund,
                                                                       evd.p, peb.p, evd.p + M::NPROPS);
                SR_HIP(hipGetLastError());
                SR_HIP(hipMemcpyAsync(evl.data(), evd.p + M::NPROPS, M::NPROPS * sizeof(u32), hipMemcpyDeviceToHost, stream_));
                SR_HIP(stream_sync(stream_));
            }
            if (limit) {
                produced = expand_level(level, n, limit, undiscovered & ~emask_, peb.p);
            } else {
                std::memset(&lc_, 0, sizeof(lc_));
            }
            for (int p = 0; p < M::NPROPS; ++p) {
                if (!evl[p]) continue;  // discoveries.insert at a terminal state (bfs.rs:265-272)
                disc[p].found = true;
                disc[p].level = level;
                disc[p].rank = evl[p] - 1;
                undiscovered &= ~(1u << p);
            }
            state_count += lc_.successors;
            unique += lc_.claims;
            stats.successors += lc_.successors;
            stats.probes += lc_.probes;
            stats.cas += lc_.cas;
            stats.algorithmic_bytes += limit * 8 * W + lc_.successors * 8 + (u64)lc_.claims * (16 + 8 * W);
            stats.levels++;
            if (produced) max_depth = level + 1;
            if (o_.verbose)
                std::fprintf(stderr, "[sr] level %u: frontier %llu expanded %llu succ %llu new %llu unique %llu cap %llu\n",
                             level, (unsigned long long)n, (unsigned long long)limit,
                             (unsigned long long)lc_.successors, (unsigned long long)produced,
                             (unsigned long long)unique.load(), (unsigned long long)cap_);
            popped_before += visited;
            if (stop || produced == 0) {
                if (target_stop) reference_done = false;  // the worker returns without waiting
                else if (stop) reference_done = true;     // all properties discovered
                else  // exhausted: the last (partial) block still checks the target (bfs.rs:129-135)
                    reference_done = !(o_.target_state_count && state_count >= o_.target_state_count);
                break;
            }
            lstart_.push_back(lstart_.back() + produced);
            n = produced;
            ++level;
        }
        auto t_end = Clock::now();
        collect_timing();
        displacement_stats();
        stats.level_loop_sec = secs(t_loop, t_end);
        stats.total_sec = secs(t_start, t_end);
        stats.table_capacity = cap_;
        release_table();  // (the pipelined loop released it already)
        free_unzeroed_table();
        return order_dependent && !fifo_;
    }

    // FAST order without `eventually` properties or a target count: the expansion of level L+1 is
    // enqueued while level L still runs (its frontier size is read on the device: the claims of the
    // last resetting publish), so the GPU does not idle while the host digests a level. The host
    // keeps one level in flight beyond the one it waits for. A speculative launch is skipped when
    // the visited set or the arena might not hold it (that level is then launched after the wait,
    // sized exactly). A speculative level launched past the end (an exhausted frontier or an early
    // exit) is ignored. Returns whether the run stopped early inside a level.
    bool pipeline_levels(u64 n, u32 sq_level0) {
        u32 undiscovered = (1u << M::NPROPS) - 1;
        u32 level = 0;
        bool order_dependent = false;
        auto discoveries_of = [&](u32 lvl, const HostCounters& c, u32& max_rank) {
            u32 newly = 0;
            for (int p = 0; p < M::NPROPS; ++p)
                if ((undiscovered >> p & 1) && c.disc[p] != ~0u) {
                    newly |= 1u << p;
                    max_rank = std::max(max_rank, c.disc[p]);
                    disc[p].found = true;
                    disc[p].level = lvl;
                    disc[p].rank = c.disc[p];
                }
            return newly;
        };
        u32 max_rank = 0;
        u32 newly = discoveries_of(0, lc_, max_rank);  // among the init states (roots publish)
        undiscovered &= ~newly;
        if (newly && undiscovered == 0) {
            lvisited_.push_back(max_rank + 1);
            reference_done = true;
            drain();  // the level-0 launch is not counted
            return true;
        }
        // One level's outcome (counters c); false when the check is over.
        auto account = [&](const HostCounters& c, const char* how) -> bool {
            const u64 produced = c.claims;
            state_count += c.successors;
            unique += produced;
            stats.successors += c.successors;
            stats.probes += c.probes;
            stats.cas += c.cas;
            stats.algorithmic_bytes += n * 8 * W + c.successors * 8 + produced * (16 + 8 * W);
            stats.levels++;
            ratio_ = (double)produced / (double)n;
            note_ratio(ratio_);
            en_ratio_ = std::max(1.0, (double)c.enabled / (double)n);
            lvisited_.push_back(n);
            if (o_.verbose)
                std::fprintf(stderr, "[sr] level %u: frontier %llu succ %llu new %llu unique %llu cap %llu%s at %.3f ms\n", level,
                             (unsigned long long)n, (unsigned long long)c.successors, (unsigned long long)produced,
                             (unsigned long long)unique.load(), (unsigned long long)cap_, how, secs(vt0_, Clock::now()) * 1e3);
            if (produced == 0) {  // exhausted (a speculative launch saw an empty frontier)
                reference_done = true;
                return false;
            }
            max_depth = level + 1;
            lstart_.push_back(lstart_.back() + produced);
            n = produced;
            ++level;
            max_rank = 0;
            newly = discoveries_of(level, c, max_rank);
            undiscovered &= ~newly;
            if (newly && undiscovered == 0) {
                // every property discovered inside this level: the reference stops at that pop
                // (order-dependent in FAST order; AUTO re-runs FIFO). A speculative expansion of
                // this level is not counted.
                lvisited_.push_back(max_rank + 1);
                reference_done = true;
                order_dependent = true;
                return false;
            }
            return true;
        };
        u32 sq = sq_level0;  // enqueued before the roots' outcome was read
        // Launches enqueued beyond the one waited for, in level order: one (the next level, its
        // frontier size read on the device), or two while the levels are small (the second CHAINED:
        // its frontier's offset is read on the device too). A level the host has to read before the
        // next is enqueued costs the host's turnaround (its publish seen, the launch issued: ~10-15
        // us) whenever the level in flight is shorter than that, which small levels are.
        std::deque<u32> ahead;
        vt0_ = Clock::now();
        for (;;) {
            const double g = std::max(ratio_, 1.0) * 1.5;
            const u64 est1 = (u64)((double)n * g) + 1024;     // the next frontier
            const u64 est2 = (u64)((double)est1 * g) + 1024;  // the states it will claim (= the frontier after)
            const u64 est3 = (u64)((double)est2 * g) + 1024;  // ... and those that one will claim
            const u64 nb_next = lstart_.back();
            // launch shape: a tight estimate (the grid strides over any excess)
            const u64 shape = (u64)((double)n * std::max(ratio_, 0.05) * 1.1) + 64;
            // Early growth (no capacity hint): a visited set that the next three levels
            // are projected to outgrow is grown now, while the level in flight is small. The rehash
            // then moves few entries and the stop costs one small level's latency, instead of both
            // at the first level that no longer fits (2pc N=9: ~1 M entries and a pipeline stop at
            // level 9, 0.1 ms per check).
            if (ahead.empty() && !pessimistic_ && !o_.capacity_hint && n <= early_grow_max_ &&
                (double)(unique + est1 + est2 + est3) >= lmax_ * (double)cap_) {
                // (enqueued behind the level in flight: no host wait; the whole old arena is copied,
                // since the host does not know yet how much of it that level fills)
                const u64 want = unique + est1 + est2 + est3;
                grow_table_async(growth_slots((u64)((double)want / lmax_) + 1));
                // (the arena only as far as the projection needs: it starts at 2^24 words)
                if (nb_next + est1 + est2 + est3 > arena_cap_) ensure_arena(nb_next + est1 + est2 + est3, arena_cap_, true);
                if (o_.verbose) std::fprintf(stderr, "[sr] early growth at a frontier of %llu states\n", (unsigned long long)n);
            }
            // enqueue the next level before waiting for this one
            if (ahead.empty()) {
                const bool spec = !pessimistic_ && (double)(unique + est1 + est2) < lmax_ * (double)cap_ &&
                                  nb_next + est1 + est2 <= arena_cap_;
                if (spec) ahead.push_back(launch_expand(nb_next, 0, true, shape, undiscovered));
            }
            // ... and the one after it while the next is small (a launch shorter than the host's turnaround)
            if (ahead.size() == 1 && chain_max_ && est1 <= chain_max_ && !pessimistic_ &&
                (double)(unique + est1 + est2 + est3) < lmax_ * (double)cap_ && nb_next + est1 + est2 + est3 <= arena_cap_) {
                const u64 shape2 = (u64)((double)shape * std::max(ratio_, 0.05) * 1.1) + 64;
                ahead.push_back(launch_expand(0, 0, true, shape2, undiscovered, 0, true));
            }
            if (ahead.empty()) publish_pending_slot();  // otherwise the enqueued level publishes this one

            bool spec_ok = !ahead.empty();
            if (!wait_publish(sq, true)) {  // lc_ = this level's counters
                if (lc_.err == ERR_DEFERRED) {
                    // a speculative launch whose frontier outgrew the room planned for it expanded
                    // nothing: the table and the arena are grown for it and it runs again
                    SR_HIP(stream_sync(stream_));
                    init_counters();
                    if (o_.verbose)
                        std::fprintf(stderr, "[sr] level of %llu states outgrew the room planned for it: deferred\n",
                                     (unsigned long long)n);
                    const u32 s2 = launch_sync(n, undiscovered);
                    publish_pending_slot();
                    if (!wait_publish(s2, true)) repair_level(lstart_[lstart_.size() - 2], n, undiscovered);
                } else {
                    // the level overflowed the probe limit: double the table, finish the level on it
                    repair_level(lstart_[lstart_.size() - 2], n, undiscovered);
                }
                // the enqueued next level saw the error and expanded nothing
                spec_ok = false;
            }
            auto it = seq_launch_.find(sq);
            if (it != seq_launch_.end() && it->second < launch_frontier.size()) {
                launch_frontier[it->second] = n;
                launch_probes[it->second] = lc_.probes;
                launch_cas[it->second] = lc_.cas;
            }
            if (!spec_ok) ahead.clear();  // (launches behind a failed level expanded nothing)
            if (!account(lc_, ahead.size() == 2 ? " (next two enqueued)" : spec_ok ? " (next enqueued)" : "")) break;
            if (!ahead.empty()) {
                sq = ahead.front();
                ahead.pop_front();
            } else {
                sq = launch_sync(n, undiscovered);
            }
        }
        // A speculative level past the end may still be in flight: the host waits for it, but the
        // visited set's clear for the next check is enqueued behind it first (release_table), so
        // that the clear runs while this check returns and the next one is set up.
        SR_HIP(hipEventRecord(ctx_->done, stream_));
        release_table();
        drain(ctx_->done);
        check_async_growth();
        free_unzeroed_table();
        return order_dependent;
    }

    // Until the stream has passed event `ev` (or every launch enqueued on it, ev = nullptr): a
    // spin on the query. (A blocking hipStreamSynchronize returned ~30 us after a check's last
    // kernel had ended.)
    void drain(hipEvent_t ev = nullptr) {
        if (!ev) {
            SR_HIP(stream_sync(stream_));
            return;
        }
        for (;;) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return clear_not_ready();
            if (e != hipErrorNotReady) SR_HIP(e);
            _mm_pause();
        }
    }

    // Nothing reads the visited set after the search (paths, replay and the Explorer use the arena
    // and the model): it goes back to the pool, zeroed on this stream behind the work enqueued so
    // far (a full table write: ~34 us for 2pc N=9's 256 MiB), and the next check takes it without
    // a clear at its start. Kept for the displacement scan of a counting run (sr_opts.counters),
    // and in FIFO order. SR_TABLE_RECYCLE=0: an ordinary free, each check clears its own table.
    void release_table() {
        if (table_recycle_ && !fifo_ && !o_.counters && !table_unzeroed_) keys_.release_zero(stream_);
    }
    // A table built by rehash_ranges goes back to the pool as it is, once the stream is idle.
    void free_unzeroed_table() {
        if (!table_recycle_ || fifo_ || o_.counters || !table_unzeroed_ || !keys_.p) return;
        SR_HIP(stream_sync(stream_));
        keys_.reset();
    }

    // Launch of the level whose frontier (n states) ends the arena, after the previous one is done:
    // the visited set and the arena are grown first if the level might not fit.
    u32 launch_sync(u64 n, u32 undiscovered) {
        const u64 d_eff = pessimistic_ ? D_ : std::min<u64>(D_, (u64)std::ceil(2.0 * recent_ratio() + 1.0));
        const double need = (double)(unique + n * d_eff);
        const u64 fbase = lstart_[lstart_.size() - 2];
        if (need > lmax_ * (double)cap_) {
            grow_table(nullptr, 0, growth_slots((u64)(need / lmax_) + 1));
            // The arena takes its next step (x8 / x4) with the table: a table that had to grow holds nearly
            // as many states as the arena (both start at 2^22), and the arena's own step, a copy and
            // a second stop of the level pipeline, would follow a level later (2pc N=9 without a
            // hint: levels 9 and 10).
            if ((double)arena_cap_ < lmax_ * (double)cap_) ensure_arena(arena_cap_ + 1, fbase + n);
        }
        ensure_arena(fbase + n + n * d_eff, fbase + n);
        return launch_expand(fbase, (u32)n, false, n, undiscovered);
    }

    // expand_fast's grid is capped at whole residencies of the device (resident blocks per CU at
    // its LDS footprint x CUs, grid_res_ of them); the kernel strides over any further parents.
    // Whole residencies avoid a partial last wave of workgroups. For 2pc one residency (every block
    // starting at once and striding with its prefetch) beats two: N=9 1.556 -> 1.520 ms, N=10 7.93
    // -> 7.76, N=11 50.7 -> 50.5 (1.17 / 0.83 residencies were slower); increment_lock (36.8 ms with
    // one against 33.3) and paxos stay at two (round 6, `profiles/r06_grid_cap.txt`). The cap is
    // printed with verbose=1. SR_GRID_MAX > 0 overrides it (<= 0 or unparsable: the default).
    // The cap is cached per kernel form (the probe loop switches to the queue form once
    // the table grows past 2^27 slots, whose occupancy differs from the rounds form's).
    u32 expand_grid_cap(bool nopf = false) {
        const int form = nopf ? 2 : probe_loop() < 0 ? 1 : 0;
        u32& cap = grid_max_[form];
        if (cap) return cap;
        if (grid_env_) return cap = grid_env_;
        int per_cu = 0, cus = 0;
        const size_t dyn = filt_bytes();
        const void* k = form == 1 ? (const void*)expand_fast<M, -4, 0> : (const void*)expand_fast<M, 1, 0>;
        if constexpr (W >= 4)
            if (nopf) k = (const void*)expand_fast<M, 1, 0, false, true>;
        SR_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64 * WPB, dyn));
        SR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, o_.device));
        cap = per_cu > 0 && cus > 0 ? (u32)(grid_res_ * per_cu * cus) : ~0u;
        if (o_.verbose) std::fprintf(stderr, "[sr] expand grid cap %u blocks (%d per CU x %d CUs x %u)%s\n", cap, per_cu, cus, grid_res_, nopf ? " [no prefetch]" : "");
        return cap;
    }
    // A level of more than DYN_MIN_RATIO chunks per workgroup takes the kernel with dynamic chunks
    // (kernels.hpp SR_DYN_CHUNKS; the kernel checks the real frontier again). Narrow states only: the
    // wide kernels' registers set their residency.
    bool deep_level(u64 chunks, u32 grid) const {
        return SR_DYN_CHUNKS && W < 4 && dyn_env_ && grid >= DYN_SHARDS && chunks > (u64)DYN_MIN_RATIO * grid;
    }
    bool dyn_env_ = !std::getenv("SR_DYN") || std::atoi(std::getenv("SR_DYN")) != 0;  // SR_DYN=0: measurement knob
    // Wide states: the kernel without the register prefetch of the next chunk's parents when every
    // chunk of the level has its own workgroup within that kernel's grid cap (DESIGN.md §3 "Wide
    // states"); the prefetching kernel when workgroups stride over chunks. SR_WIDE_NOPF=0/1 forces.
    bool use_nopf(u64 chunks) {
        if constexpr (W < 4) return false;
        if (o_.counters || wide_nopf_ == 0) return false;
        if (wide_nopf_ == 1) return true;
        return chunks <= expand_grid_cap(true);
    }

    // One expand_fast launch over a whole level whose frontier starts at arena offset `fbase`:
    // n states (dev_n = 0), or the previous level's claims read on the device (dev_n = 1, `shape`
    // is then an estimate used only for the launch shape; the grid strides over any excess).
    // chained (dev_n only): enqueued two levels ahead, the frontier's arena offset is not known to
    // the host either: the launch reads it, and the unique count, from the previous slot (SlotWork.chain).
    u32 launch_expand(u64 fbase, u32 n, bool dev_n, u64 shape, u32 undiscovered, u32 flags = 0, bool chained = false) {
        const u32 sq = next_seq();
        if (chained) fbase = 0;  // (read on the device)
        const u64 nbase = fbase + (dev_n ? 0 : n);  // start of the next level (dev_n: + n on the device)
        const u32 ncap = (u32)std::min<u64>(arena_cap_ - nbase, 0xffffffffu);
        const u32 ppw_log2 = ppw_env_ >= 0 ? (u32)ppw_env_ : ppw_for(shape);
        const u32 chunks = std::max<u32>(1, blocks_for((shape + (1u << ppw_log2) - 1) >> ppw_log2, WPB));
        const bool nopf = use_nopf(chunks);
        const u32 grid = std::min(expand_grid_cap(nopf), chunks);
        const bool deep = deep_level(chunks, grid);
        seq_launch_[sq] = launch_frontier.size();
        // a slotted launch: it counts into its own slot and is published by its successor
        SlotWork sw = slot_work(dev_n);
        sw.flags = flags;
        sw.arena = arena_.p;
        sw.apar = apar_.p;
        sw.arena_cap = arena_cap_;
        sw.fbase = fbase;
        // unique states before the frontier (level 0 is launched before the roots' claims are read: 0)
        const u64 u = unique.load();
        sw.ubase = dev_n ? u : u >= n ? u - n : 0ull;
        if (chained) sw.chain = slot(slot_k_ - 1);
        if (dev_n) {  // speculative: the device checks its frontier against the room left (ERR_DEFERRED)
            sw.room = (u64)(lmax_ * (double)cap_);  // (the device adds the unique states before the level)
            sw.gmul = (u32)std::min(64.0 * 256.0, std::ceil(std::max(recent_ratio(), 1.0) * 1.5 * 256.0));
        }
        LevelCounters* lc = slot(slot_k_);
        const u32 svc = sw.pub || sw.zero ? 1u : 0u;  // the extra service workgroup (SlotWork)
        timed([&] {
            auto launch = [&](auto kern) {
                kern<<<grid + svc, 64 * WPB, filt_bytes(), stream_>>>(
                    m_, arena_.p + fbase * W, 0u, n, view(), arena_.p + nbase * W, apar_.p + nbase, ncap, lc,
                    undiscovered, nullptr, sq, 0u, ppw_log2, filt_arg(), sw);
            };
            if (o_.counters) launch(expand_fast<M, 1, 0, true>);
            else if (nopf) launch_nopf(launch);
            else if (deep) probe_loop() < 0 ? launch(expand_fast<M, -4, 0, false, false, true>) : launch(expand_fast<M, 1, 0, false, false, true>);
            else if (probe_loop() < 0) launch(expand_fast<M, -4, 0>);
            else launch(expand_fast<M, 1, 0>);
        }, n);
        slot_seq_ = sq;
        slot_published_ = false;
        ++slot_k_;
        return sq;
    }

    // Smallest 1500-pop block boundary inside this level at which state_count >= target.
    u64 target_limit(u64 n, u64 popped_before, u64 limit) {
        DBuf<u32> counts;
        counts.alloc(o_.device, n);
        count_successors<M><<<blocks_for(n, 256), 256, 0, stream_>>>(m_, cur(), (u32)n, counts.p);
        SR_HIP(hipGetLastError());
        std::vector<u32> h(n);
        SR_HIP(hipMemcpyAsync(h.data(), counts.p, n * sizeof(u32), hipMemcpyDeviceToHost, stream_));
        SR_HIP(stream_sync(stream_));
        u64 sc = state_count;
        u64 r = 0;
        for (u64 k = popped_before / 1500 + 1;; ++k) {
            u64 b = k * 1500 - popped_before;  // pops of this level at the block boundary
            if (b > n || b > limit) return ~0ull;
            for (; r < b; ++r) sc += h[r];
            if (sc >= o_.target_state_count) return b;
        }
    }

    // Expands frontier ranks [0, limit) of `level` into next_; returns the next frontier size.
    u64 expand_level(u32 level, u64 n, u64 limit, u32 undiscovered, const u32* peb = nullptr) {
        const u32 A = A_;  // action slots (FIFO candidate layout)
        u64 claims = 0;
        DBuf<u32> cand;
        if (fifo_) {
            cand.alloc(o_.device, limit * A);
            SR_HIP(hipMemsetAsync(cand.p, 0xff, limit * A * sizeof(u32), stream_));
        }
        const u64 nbase = lstart_.back();  // arena offset of the next level
        // New states per parent assumed when sizing a chunk: twice the last level's growth (the
        // model's max out-degree D in pessimistic mode); see run_with_restart.
        const u64 d_eff = pessimistic_ ? D_ : std::min<u64>(D_, (u64)std::ceil(2.0 * ratio_ + 1.0));
        for (u64 lo = 0; lo < limit;) {
            // Chunk so the visited set stays under 80% load.
            u64 head = (u64)(lmax_ * (double)cap_) - std::min<u64>((u64)(lmax_ * (double)cap_), unique + claims);
            u64 c = std::min<u64>(limit - lo, head / std::max<u64>(d_eff, 1));
            if (c < std::min<u64>(limit - lo, 1u << 16)) {
                grow_table(fifo_ ? cand.p : nullptr, fifo_ ? limit * A : 0);
                continue;
            }
            if (!fifo_) ensure_arena(nbase + claims + c * d_eff, nbase + claims);
            const u32 ulo = (u32)lo, uhi = (u32)(lo + c);
            const bool last = lo + c == limit;
            // repair: the chunk's first pass overflowed the probe limit (see repair_level)
            auto launch_chunk = [&](bool repair) {
                const u32 sq = next_seq();
                if (fifo_) {
                    timed([&] {
                        expand_fifo<M><<<blocks_for(c, 256), 256, 0, stream_>>>(m_, cur(), ulo, uhi, (u32)limit, view(), cand.p,
                                                                                A, level, lc_d_, hcd(sq), sq, repair ? 0u : 1u);
                    });
                } else {
                    const u32 ncap = (u32)std::min<u64>(arena_cap_ - nbase, 0xffffffffu);
                    u64* next = arena_.p + nbase * W;
                    u32* npar = apar_.p + nbase;
                    const u32 ppw_log2 = ppw_env_ >= 0 ? (u32)ppw_env_ : ppw_for(c);
                    const u32 chunks = std::max<u32>(1, blocks_for((c + (1u << ppw_log2) - 1) >> ppw_log2, WPB));
                    const bool nopf = use_nopf(chunks);
                    const u32 grid = std::min(expand_grid_cap(nopf), chunks);
                    SlotWork sw{};
                    sw.flags = repair ? SLOT_REPAIR : 0u;
                    if (emask_ && peb) {
                        sw.peb = peb;
                        sw.naeb = aeb_.p + nbase;
                    }
                    timed([&] {
                        auto launch = [&](auto kern) {
                            kern<<<grid, 64 * WPB, filt_bytes(), stream_>>>(
                                m_, cur(), ulo, uhi, view(), next, npar, ncap, lc_d_, undiscovered, hcd(sq), sq,
                                last ? 1u : 0u, ppw_log2, filt_arg(), sw);
                        };
                        if (o_.counters) launch(expand_fast<M, 1, 0, true>);
                        else if (nopf) launch_nopf(launch);
                        else if (deep_level(chunks, grid))
                            probe_loop() < 0 ? launch(expand_fast<M, -4, 0, false, false, true>) : launch(expand_fast<M, 1, 0, false, false, true>);
                        else if (probe_loop() < 0) launch(expand_fast<M, -4, 0>);
                        else launch(expand_fast<M, 1, 0>);
                    });
                }
                return sq;
            };
            if (!wait_publish(launch_chunk(false), true)) {
                // Double the table (FIFO: the level's candidate slots move with it) and probe the
                // chunk again: the missing states are claimed, nothing is counted twice. The
                // counters continue from the failed pass (a last FAST chunk's publish reset them).
                const HostCounters first = lc_;
                u32 dmin[MAX_PROPS];
                std::copy(first.disc, first.disc + MAX_PROPS, dmin);
                for (int attempt = 0;; ++attempt) {
                    if (attempt >= 8) throw Error(SR_ERR_CAPACITY, "visited set probe limit exceeded after 8 doublings");
                    grow_table(fifo_ ? cand.p : nullptr, fifo_ ? limit * A : 0);
                    stats.table_doublings++;
                    SR_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&lc_d_->claims), (int)lc_.claims, 1, stream_));
                    SR_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&lc_d_->err), 0, 1, stream_));
                    const bool ok = wait_publish(launch_chunk(true), true);
                    for (int p = 0; p < MAX_PROPS; ++p) dmin[p] = std::min(dmin[p], lc_.disc[p]);
                    if (ok) break;
                }
                lc_.successors = std::max(lc_.successors, first.successors);
                lc_.enabled = std::max(lc_.enabled, first.enabled);
                std::copy(dmin, dmin + MAX_PROPS, lc_.disc);
            }
            claims = lc_.claims;
            lo += c;
        }
        ratio_ = (double)claims / (double)limit;
        if (!fifo_) {
            en_ratio_ = std::max(1.0, (double)lc_.enabled / (double)limit);
            return claims;
        }

        // FIFO passes 2-3: owners per parent, exclusive scan, ordered scatter.
        ensure_arena(nbase + claims, nbase);
        DBuf<u32> counts, offs, sums, total;
        counts.alloc(o_.device, limit);
        offs.alloc(o_.device, limit);
        u32 tiles = blocks_for(limit, SCAN_TILE);
        sums.alloc(o_.device, tiles);
        total.alloc(o_.device, 1);
        timed([&] { own_count<M><<<blocks_for(limit, 256), 256, 0, stream_>>>(cand.p, (u32)limit, A, level, view(), counts.p); });
        scan_tile_sums<<<tiles, SCAN_BLOCK, 0, stream_>>>(counts.p, (u32)limit, sums.p);
        scan_sums<<<1, SCAN_BLOCK, 0, stream_>>>(sums.p, tiles, total.p);
        scan_tiles<<<tiles, SCAN_BLOCK, 0, stream_>>>(counts.p, (u32)limit, sums.p, offs.p);
        SR_HIP(hipGetLastError());
        const u32 sq = next_seq();
        timed([&] {
            scatter_fifo<M><<<blocks_for(limit, 256), 256, 0, stream_>>>(m_, cur(), cand.p, offs.p, (u32)limit, A, level,
                                                                         view(), arena_.p + nbase * W, apar_.p + nbase, lc_d_,
                                                                         undiscovered, hcd(sq), sq, total.p, peb,
                                                                         emask_ ? aeb_.p + nbase : nullptr);
        });
        wait_publish(sq);
        const u32 owners = lc_.aux;
        if (owners != claims) throw Error(SR_ERR_CAPACITY, "FIFO ownership mismatch: owners " + std::to_string(owners) + " claims " + std::to_string(claims));
        return owners;
    }

    // Parents per wave (log2) of the FAST kernel for a chunk of c parents. A wave walks the
    // enabled action slots of its parents 64 at a time. Light models (a few ALU ops per successor)
    // amortise the wave's setup over ~16 such rounds; heavy ones (paxos: ~1.3K VALU ops per
    // successor) want ~4 rounds per wave and more waves to hide the probe latency. Small levels
    // use fewer parents per wave until ~2K waves are in flight (minimum 4 parents per wave).
    // Measured per level with SR_PPW_LOG2 sweeps (profiles/r01_ppw_levels.txt).
    u32 ppw_for(u64 c) const {
        const double rounds = W >= 4 ? 4.0 : 16.0;
        const double ppw = 64.0 * rounds / en_ratio_;
        const u32 lmax = W >= 4 ? SR_WIDE_PPW_LOG2_MAX : 6;  // expand_fast's PPW_LOG2_MAX
        u32 l = 2;
        while (l < lmax && (double)(2u << l) <= ppw) ++l;
        while (l > 2 && ((c + (1u << l) - 1) >> l) < ppw_waves_) --l;
        return l;
    }
    u64 ppw_waves_ = std::getenv("SR_PPW_WAVES") && std::atoll(std::getenv("SR_PPW_WAVES")) > 0
                         ? (u64)std::atoll(std::getenv("SR_PPW_WAVES")) : 2048;

    // The frontier being expanded: the arena's second-to-last level.
    const u64* cur() const { return arena_.p + lstart_[lstart_.size() - 2] * W; }

    M m_;
    sr_opts o_;
    u32 A_;  // action slots
    u32 D_;  // max successors of one state (bounds the new states a chunk can create)
    u32 emask_;  // the model's `eventually` properties
    bool fifo_ = false;
    int probe_batch_ = 0;  // SR_PROBE_BATCH: 1 forces the probe rounds, -4 the per-lane probe queues (0: probe_loop)
    // expand_fast's probe loop (DESIGN.md §3 "Probe loops"): rounds of one successor per lane, or
    // per-lane queues over 4 rounds (-4) once the visited set is far beyond the 256 MB Infinity
    // Cache (>= 2^27 slots), where each probe is a longer round trip: 2pc N=10 -7 %, N=11 -6 %,
    // N=9 (2^25 slots) +6 % (profiles/r05_probe_loops.txt). Fingerprint-mode narrow states only.
    int probe_loop() const {
        if (probe_batch_) return probe_batch_ < 0 ? -4 : 1;
        constexpr bool queue_ok = W == 1 || !has_qkey<M>::value;  // not multi-word quotient tables
        if (queue_ok && W < 4 && queue_ratio_ > 0 && ratio_ >= queue_ratio_) return -4;  // (measurement knob)
        return queue_ok && W < 4 && cap_ >= (1ull << 27) ? -4 : 1;
    }
    // SR_QUEUE_RATIO: the per-lane queues also for levels after one that made at least this many new
    // states per parent (the claim-heavy ascending levels; 0: off)
    double queue_ratio_ = std::getenv("SR_QUEUE_RATIO") ? std::atof(std::getenv("SR_QUEUE_RATIO")) : 0.0;
    int ppw_env_ = -1;
    bool table_recycle_ = true;  // the visited set is returned zeroed (~Engine)
    u32 grid_res_ = 2;  // residencies per expand grid (set in the constructor)
    u32 grid_max_[3] = {0, 0, 0};  // cap on expand_fast's grid per form (rounds, queue, wide no-prefetch);
                                   // 0 = not computed yet (two device residencies, or SR_GRID_MAX)
    u32 grid_env_ = 0;       // SR_GRID_MAX
    int wide_nopf_ = -1;     // SR_WIDE_NOPF: -1 chosen per level (use_nopf), 0 never, 1 always
    // The pipelined loop enqueues a second level ahead (chained) while the next frontier is
    // estimated at <= this many states (SR_CHAIN_MAX; 0: never).
    u64 chain_max_ = 16384;
    // Early growth of an unhinted visited set happens while the frontier is at most this large
    // (SR_EARLY_GROW_MAX; 0: never).
    u64 early_grow_max_ = std::getenv("SR_EARLY_GROW_MAX") ? std::strtoull(std::getenv("SR_EARLY_GROW_MAX"), nullptr, 10)
                                                           : (u64)1 << 17;
    int table_kind_ = 0;  // DevicePool memory kind of the visited set (SR_TABLE_KIND, measurement knob)
    // the no-prefetch form exists for wide states only (it is the prefetching kernel otherwise)
    template <class L>
    void launch_nopf(L& launch) {
        if constexpr (W >= 4) launch(expand_fast<M, 1, 0, false, true>);
    }
    u64 query_mask_ = 4095;  // spins between hipStreamQuery calls in wait_publish (SR_QUERY_LOG2)
    bool pipeline_ = true;  // FAST-order level pipelining (SR_PIPELINE=0 disables, for A/B runs)
    DBuf<u64> slots_;                 // SLOTS per-level counter slots (the pipelined loop)
    u32 slot_k_ = 0;                  // slotted launches in this run
    u32 slot_seq_ = 0;                // sequence number of the last one
    bool slot_published_ = true;      // its publish is done or enqueued
    std::map<u32, size_t> seq_launch_;  // launch sequence number -> index in launch_frontier
    u32 filt_log2_ = W >= 4 ? 10 : 9;  // block-local duplicate filter (SR_FILTER_LOG2 sweep in profiles/)
    bool filt_compact_ = false;         // ... in 4-byte entries (kernels.hpp FILT_COMPACT)
    size_t filt_bytes() const { return filt_log2_ ? (size_t)(filt_compact_ ? 4u : 8u) << filt_log2_ : 0u; }
    u32 filt_arg() const { return filt_log2_ | (filt_compact_ ? FILT_COMPACT : 0u); }
    bool pessimistic_ = false;  // size chunks for max out-degree new states per parent
    u64 grow_factor_ = 1;       // initial-capacity multiplier after a capacity restart
    double ratio_ = 1.0;        // new states per expanded parent in the last level
    double ratios_[4] = {};     // ... in the last four levels (a model's growth can be periodic:
    u32 nratio_ = 0;            // increment_lock grows x5 every fourth level)
    void note_ratio(double r) { ratios_[nratio_++ & 3] = r; }
    double recent_ratio() const {
        double m = ratio_;
        for (u32 i = 0; i < std::min<u32>(nratio_, 4); ++i) m = std::max(m, ratios_[i]);
        return m;
    }
    double en_ratio_ = 8.0;     // enabled action slots per expanded parent in the last level
    // planned load of the visited set at the capacity hint (SR_TABLE_LOAD): 0.3 with 4-byte slots (2pc
    // N=9: 2^26 slots, 256 MiB, 1.615 -> 1.565 ms; N=10 8.64 -> 7.89 ms; profiles/r06_table_load.txt)
    double table_load_ = 0.3;
    bool load_env_ = false;
    Ctx* ctx_ = nullptr;
    hipStream_t stream_ = nullptr;
    HostCounters lc_{};  // host copy of the last published counters
    LevelCounters* lc_d_ = nullptr;
    u64 cap_ = 0;
    DBuf<u64> keys_, meta_;      // visited set
    double lmax_ = 0.8;          // growth threshold of the current table (max_load)
    Clock::time_point vt0_{};    // verbose log: start of the level loop
    DBuf<u32> aux_;              // [0] rehash error bits, [1] max displacement (displacement_stats)
    DBuf<u64> arena_;            // BFS tree: every level's states in visit order
    DBuf<u32> apar_;             // parent rank (in the previous level) of each arena state
    DBuf<u32> aeb_;              // EventuallyBits of each arena state (models with eventually properties)
    u64 arena_cap_ = 0;          // states
    std::vector<u64> lstart_;    // arena offset of each level (+ one past the newest)
    std::vector<u64> lvisited_;  // states of each level that the reference would pop
};

}  // namespace sr

#include "dist.hpp"

namespace sr {

// The fingerprint of a state given by its canonical description (the integers of
// sr_gpu_bfs_discovery_path / `describe`): what a host that holds the state compares with a
// discovery's fingerprint chain (`Path::from_fingerprints`, src/checker/path.rs:20-86).
// The description must be canonical: undescribe masks its fields, so a malformed or contradictory
// description (a paxos Get return value for a client still in phase 1, a field out of range) would
// otherwise map to some state and a plausible fingerprint. It is described again and compared.
template <class M>
int described_fingerprint(const M& m, const i64* d, int width, u64* fp, std::string* why = nullptr) {
    if constexpr (has_undescribe<M>::value) {
        if (!d || !fp || width != m.describe_width()) {
            if (why) *why = "bad description width";
            return SR_ERR_ARG;
        }
        u64 s[M::W];
        m.undescribe(d, s);
        std::vector<i64> back((size_t)width);
        m.describe(s, back.data());
        for (int i = 0; i < width; ++i)
            if (back[i] != d[i]) {
                if (why)
                    *why = "not a canonical state description (element " + std::to_string(i) + ": " + std::to_string(d[i]) +
                           " describes back as " + std::to_string(back[i]) + ")";
                return SR_ERR_ARG;
            }
        *fp = state_fp<M>(s);
        return SR_OK;
    } else {
        (void)m, (void)d, (void)width, (void)fp;
        if (why) *why = "model has no state description inverse";
        return SR_ERR_UNSUPPORTED;
    }
}

// ---- plugins: a GpuModel compiled into its own shared library (include/stateright_gpu_model.hpp) ----
// MAKE(params, nparams, device) builds the model (device < 0: host-only use); it may throw Error.
inline sr_opts normalized_opts(const sr_opts* opts) {
    sr_opts o;
    std::memset(&o, 0, sizeof(o));
    o.struct_size = sizeof(sr_opts);
    if (opts) std::memcpy(&o, opts, std::min<size_t>(sizeof(o), opts->struct_size ? opts->struct_size : sizeof(o)));
    return o;
}

template <class M, class Make>
void* plugin_create(Make make, const int64_t* p, int32_t np, const sr_opts* opts, void* comm, int32_t vparts, char* err,
                    int32_t errcap) {
    try {
        const sr_opts o = normalized_opts(opts);
        M m = make(p, np, o.device);
        EngineBase* e = nullptr;
        if (o.symmetry) {
            if constexpr (has_canonical<M>::value) {
                if (comm || vparts > 1) e = new DistEngine<Canon<M>>(Canon<M>(m), o, static_cast<Comm*>(comm), (int)vparts);
                else e = new Engine<Canon<M>>(Canon<M>(m), o);
            } else {
                throw Error(SR_ERR_UNSUPPORTED, "symmetry reduction: the plugin model has no `canonical`");
            }
        } else if (comm || vparts > 1) {
            if constexpr (has_emask<M>::value) {
                if (model_emask(m)) e = new DistEngine<EvBits<M>>(EvBits<M>(m), o, static_cast<Comm*>(comm), (int)vparts);
            }
            if (!e) e = new DistEngine<M>(m, o, static_cast<Comm*>(comm), (int)vparts);
        } else {
            e = new Engine<M>(m, o);
        }
        return e;
    } catch (const std::exception& x) {
        if (err && errcap > 0) std::snprintf(err, (size_t)errcap, "%s", x.what());
        return nullptr;
    }
}

template <class M, class Make>
int32_t plugin_fingerprint(Make make, const int64_t* p, int32_t np, const int64_t* d, int32_t width, uint64_t* fp) {
    try {
        return described_fingerprint(make(p, np, -1), d, width, fp);
    } catch (const Error& x) {
        return x.code;
    } catch (const std::exception&) {
        return SR_ERR_ARG;
    }
}

}  // namespace sr
