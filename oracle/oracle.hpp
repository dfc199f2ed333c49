// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement of Stateright's breadth-first checker (`src/checker/bfs.rs`, crate 0.28.0,
// snapshot 2025-02-09) used to CHECK the MI355X engine. Nothing in `stateright_amd/` links,
// loads or calls this code: only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
// `cpu_baseline` leg use it.
//
// Parity pinning: the reference is Rust and no Rust toolchain exists in this image, so the
// reference itself cannot be built or run. This restatement is pinned by the reference's own
// test goldens, asserted in tests/test_oracle_golden.py.
//
// Fingerprints: the reference hashes with ahash 0.3.8 (`src/lib.rs:306-344`), a crate that is not
// vendored under /root/reference. Its output for primitives is pinned by
// `src/checker/explorer.rs:260-268`, but a restatement of its fallback algorithm from memory did
// not reproduce those two values, so the oracle uses its own 64-bit fold-multiply stream hasher
// over the same `Hash` byte/word stream shape. Fingerprint VALUES are therefore "parity unpinned";
// nothing in BFS order or counts depends on them (only on equality), see DESIGN.md.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <shared_mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace oracle {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

// ---------------------------------------------------------------------------------------------
// Stable hashing (stand-in for `stable::hasher()`, src/lib.rs:331-344).
// ---------------------------------------------------------------------------------------------
struct Hasher {
    u64 buffer = 123456789987654321ull;  // KEY1, src/lib.rs:334
    u64 pad = 98765432123456789ull;      // KEY2, src/lib.rs:335
    static u64 folded_multiply(u64 s, u64 by) {
        unsigned __int128 r = (unsigned __int128)s * by;
        return (u64)r ^ (u64)(r >> 64);
    }
    void write_u64(u64 x) { buffer = folded_multiply(x ^ buffer, 6364136223846793005ull); }
    void write_u8(u8 x) { write_u64(x); }
    void write_bool(bool b) { write_u64(b ? 1 : 0); }
    void write_usize(size_t x) { write_u64((u64)x); }
    u64 finish() const {
        unsigned rot = (unsigned)(pad & 63);
        u64 v = folded_multiply(buffer, pad);
        return rot ? (v << rot) | (v >> (64 - rot)) : v;
    }
};

// ---------------------------------------------------------------------------------------------
// Model API (src/lib.rs:155-300).
// ---------------------------------------------------------------------------------------------
enum class Expectation { Always, Eventually, Sometimes };

template <class M>
struct Property {
    Expectation expectation;
    const char* name;
    std::function<bool(const M&, const typename M::State&)> condition;

    static Property always(const char* n, std::function<bool(const M&, const typename M::State&)> c) {
        return Property{Expectation::Always, n, std::move(c)};
    }
    static Property sometimes(const char* n, std::function<bool(const M&, const typename M::State&)> c) {
        return Property{Expectation::Sometimes, n, std::move(c)};
    }
    static Property eventually(const char* n, std::function<bool(const M&, const typename M::State&)> c) {
        return Property{Expectation::Eventually, n, std::move(c)};
    }
};

// `fingerprint` (src/lib.rs:306-311): hash the state, panic on zero.
template <class M>
u64 fingerprint(const M& m, const typename M::State& s) {
    Hasher h;
    m.hash_state(s, h);
    u64 fp = h.finish();
    if (fp == 0) throw std::runtime_error("hasher returned zero, an invalid fingerprint");
    return fp;
}

// `Model::next_steps` (src/lib.rs:192-202): (action, state) pairs whose next_state is Some.
template <class M>
std::vector<std::pair<typename M::Action, typename M::State>> next_steps(const M& m,
                                                                        const typename M::State& s) {
    std::vector<typename M::Action> actions;
    m.actions(s, actions);
    std::vector<std::pair<typename M::Action, typename M::State>> out;
    for (auto& a : actions) {
        auto ns = m.next_state(s, a);
        if (ns) out.emplace_back(a, std::move(*ns));
    }
    return out;
}

// ---------------------------------------------------------------------------------------------
// Path (src/checker/path.rs).
// ---------------------------------------------------------------------------------------------
template <class M>
struct Path {
    std::vector<std::pair<typename M::State, std::optional<typename M::Action>>> steps;

    // `Path::from_fingerprints` (src/checker/path.rs:20-86): pick the init state with the first
    // fingerprint, then for each next fingerprint the FIRST step whose successor matches.
    static Path from_fingerprints(const M& m, std::deque<u64> fps) {
        if (fps.empty()) throw std::runtime_error("empty path is invalid");
        u64 init_print = fps.front();
        fps.pop_front();
        std::optional<typename M::State> last;
        for (auto& s : m.init_states())
            if (fingerprint(m, s) == init_print) { last = s; break; }
        if (!last) throw std::runtime_error("Unable to reconstruct a `Path`: no init state has the expected fingerprint");
        Path p;
        while (!fps.empty()) {
            u64 next_fp = fps.front();
            fps.pop_front();
            bool found = false;
            for (auto& [a, ns] : next_steps(m, *last)) {
                if (fingerprint(m, ns) == next_fp) {
                    p.steps.emplace_back(*last, a);
                    last = ns;
                    found = true;
                    break;
                }
            }
            if (!found)
                throw std::runtime_error("Unable to reconstruct a `Path`: " +
                                         std::to_string(1 + p.steps.size()) +
                                         " previous state(s) reconstructed but no subsequent state has the next fingerprint");
        }
        p.steps.emplace_back(*last, std::nullopt);
        return p;
    }

    // `Path::from_actions` (src/checker/path.rs:90-112), matching actions by canonical id.
    static std::optional<Path> from_actions(const M& m, const typename M::State& init,
                                            const std::vector<i64>& action_ids) {
        bool ok = false;
        for (auto& s : m.init_states())
            if (m.describe(s) == m.describe(init)) ok = true;
        if (!ok) return std::nullopt;
        Path p;
        typename M::State prev = init;
        for (i64 id : action_ids) {
            bool found = false;
            for (auto& [a, ns] : next_steps(m, prev)) {
                if (m.action_id(a) == id) {
                    p.steps.emplace_back(prev, a);
                    prev = ns;
                    found = true;
                    break;
                }
            }
            if (!found) return std::nullopt;
        }
        p.steps.emplace_back(prev, std::nullopt);
        return p;
    }

    const typename M::State& last_state() const { return steps.back().first; }
    std::vector<i64> action_ids(const M& m) const {
        std::vector<i64> out;
        for (auto& [s, a] : steps)
            if (a) out.push_back(m.action_id(*a));
        return out;
    }
    // `impl Display for Path` (src/checker/path.rs:174-187).
    std::string display(const M& m) const {
        std::ostringstream os;
        os << "Path[" << steps.size() - 1 << "]:\n";
        for (auto& [s, a] : steps)
            if (a) os << "- " << m.format_action(*a) << "\n";
        return os.str();
    }
};

// ---------------------------------------------------------------------------------------------
// BFS checker (src/checker/bfs.rs).
// ---------------------------------------------------------------------------------------------
struct CheckerOptions {
    size_t thread_count = 1;          // `CheckerBuilder::threads`, src/checker.rs:170-172
    u64 target_state_count = 0;       // `target_state_count` (0 = None), src/checker.rs:164-166
    bool record_visits = false;       // a `StateRecorder` visitor, src/checker/visitor.rs:70-99
};

// `DashMap<Fingerprint, Option<Fingerprint>>` with per-shard RwLocks (dashmap 3.11.10): the
// shard count follows dashmap's `(num_cpus * 4).next_power_of_two()` default.
// A word-sized reader/writer spin lock: the same fast path as `parking_lot::RwLock` (one atomic
// RMW per acquire), which backs both DashMap shards and the reference's discoveries map.
class RwLock {
  public:
    void lock_shared() {
        for (unsigned spins = 0;; ++spins) {
            u32 s = state_.load(std::memory_order_relaxed);
            if (!(s & kWriter) && state_.compare_exchange_weak(s, s + 1, std::memory_order_acquire)) return;
            backoff(spins);
        }
    }
    void unlock_shared() { state_.fetch_sub(1, std::memory_order_release); }
    void lock() {
        for (unsigned spins = 0;; ++spins) {
            u32 s = 0;
            if (state_.compare_exchange_weak(s, kWriter, std::memory_order_acquire)) return;
            backoff(spins);
        }
    }
    void unlock() { state_.store(0, std::memory_order_release); }

  private:
    static void backoff(unsigned spins) {
        if (spins > 64) std::this_thread::yield();
    }
    static constexpr u32 kWriter = 1u << 31;
    std::atomic<u32> state_{0};
};

class Generated {
  public:
    explicit Generated(size_t shard_hint) {
        size_t n = 1;
        while (n < shard_hint) n <<= 1;
        shards_ = std::vector<Shard>(n);
        mask_ = n - 1;
    }
    // Returns true when `fp` was vacant (and inserts fp -> parent); `bfs.rs:246-247`.
    bool insert_if_vacant(u64 fp, u64 parent, u32 depth) {
        Shard& s = shard(fp);
        std::unique_lock<RwLock> g(s.lock);
        return s.map.insert(fp, parent, depth);
    }
    std::optional<std::pair<u64, u32>> get(u64 fp) const {
        const Shard& s = shard(fp);
        std::shared_lock<RwLock> g(s.lock);
        const Slot* e = s.map.find(fp);
        if (!e) return std::nullopt;
        return std::make_pair(e->parent, e->depth);
    }
    size_t len() const {
        size_t n = 0;
        for (auto& s : shards_) {
            std::shared_lock<RwLock> g(s.lock);
            n += s.map.len;
        }
        return n;
    }
    u32 max_depth() const {
        u32 d = 0;
        for (auto& s : shards_) {
            std::shared_lock<RwLock> g(s.lock);
            for (auto& e : s.map.slots)
                if (e.key) d = std::max(d, e.depth);
        }
        return d;
    }

  private:
    // One shard = an open-addressing table (hashbrown stand-in); key 0 = vacant (fingerprints
    // are non-zero); parent 0 == None.
    struct Slot { u64 key; u64 parent; u32 depth; };
    struct Table {
        std::vector<Slot> slots = std::vector<Slot>(16, Slot{0, 0, 0});
        size_t len = 0;
        const Slot* find(u64 k) const {
            size_t m = slots.size() - 1;
            for (size_t i = (size_t)(k * 0x9E3779B97F4A7C15ull >> 20) & m;; i = (i + 1) & m) {
                if (slots[i].key == k) return &slots[i];
                if (slots[i].key == 0) return nullptr;
            }
        }
        bool insert(u64 k, u64 parent, u32 depth) {
            if ((len + 1) * 8 > slots.size() * 7) grow();
            size_t m = slots.size() - 1;
            for (size_t i = (size_t)(k * 0x9E3779B97F4A7C15ull >> 20) & m;; i = (i + 1) & m) {
                if (slots[i].key == k) return false;
                if (slots[i].key == 0) {
                    slots[i] = Slot{k, parent, depth};
                    ++len;
                    return true;
                }
            }
        }
        void grow() {
            std::vector<Slot> old(slots.size() * 2, Slot{0, 0, 0});
            old.swap(slots);
            len = 0;
            for (auto& e : old)
                if (e.key) insert(e.key, e.parent, e.depth);
        }
    };
    struct Shard {
        mutable RwLock lock;
        Table map;
    };
    // nohash-hasher: the key is its own hash; the shard comes from high bits.
    Shard& shard(u64 fp) { return shards_[(fp >> 40) & mask_]; }
    const Shard& shard(u64 fp) const { return shards_[(fp >> 40) & mask_]; }
    std::vector<Shard> shards_;
    size_t mask_;
};

template <class M>
class BfsChecker {
  public:
    using State = typename M::State;
    using EventuallyBits = u64;  // `id_set::IdSet` (src/checker.rs:347), <= 64 properties
    struct Job {
        State state;
        u64 fp;
        EventuallyBits ebits;
        u32 depth;  // not in the reference; carried to report the BFS depth metric
    };

    // `BfsChecker::spawn` (src/checker/bfs.rs:36-163).
    BfsChecker(M model, CheckerOptions opt)
        : model_(std::move(model)), opt_(opt),
          generated_(std::max<size_t>(4 * std::max<unsigned>(1, std::thread::hardware_concurrency()), 4)) {
        properties_ = model_.properties();
        const size_t property_count = properties_.size();
        std::vector<State> init_states;
        for (auto& s : model_.init_states())
            if (model_.within_boundary(s)) init_states.push_back(s);
        state_count_ = init_states.size();
        for (auto& s : init_states) generated_.insert_if_vacant(fingerprint(model_, s), 0, 0);
        EventuallyBits ebits = 0;
        for (size_t i = 0; i < property_count; ++i)
            if (properties_[i].expectation == Expectation::Eventually) ebits |= (1ull << i);
        std::deque<Job> pending;
        for (auto& s : init_states) pending.push_back(Job{s, fingerprint(model_, s), ebits, 0});
        market_.wait_count = opt_.thread_count;
        market_.jobs.push_back(std::move(pending));
        start_ = std::chrono::steady_clock::now();
        for (size_t t = 0; t < opt_.thread_count; ++t)
            handles_.emplace_back([this, t] { worker(t); });
    }
    ~BfsChecker() { join(); }

    // `Checker` impl (src/checker/bfs.rs:277-312).
    u64 state_count() const { return state_count_.load(std::memory_order_relaxed); }
    u64 unique_state_count() const { return generated_.len(); }
    u32 max_depth() const { return generated_.max_depth(); }
    BfsChecker& join() {
        for (auto& h : handles_)
            if (h.joinable()) h.join();
        if (!elapsed_set_) {
            elapsed_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - start_).count();
            elapsed_set_ = true;
        }
        if (worker_error_) std::rethrow_exception(worker_error_);
        return *this;
    }
    bool is_done() const {
        std::lock_guard<std::mutex> g(market_mu_);
        return (market_.jobs.empty() && market_.wait_count == opt_.thread_count) ||
               discoveries_len() == properties_.size();
    }
    double elapsed_sec() const { return elapsed_; }

    // `discoveries` (src/checker/bfs.rs:289-298): property name -> reconstructed path.
    std::map<std::string, Path<M>> discoveries() const {
        std::map<std::string, Path<M>> out;
        std::shared_lock<RwLock> g(disc_mu_);
        for (auto& [name, fp] : discoveries_) out.emplace(name, reconstruct_path(fp));
        return out;
    }
    std::vector<std::string> discovery_names() const {
        std::shared_lock<RwLock> g(disc_mu_);
        std::vector<std::string> out;
        for (auto& kv : discoveries_) out.push_back(kv.first);
        return out;
    }
    std::optional<u64> discovery_fp(const std::string& name) const {
        std::shared_lock<RwLock> g(disc_mu_);
        auto it = discoveries_.find(name);
        if (it == discoveries_.end()) return std::nullopt;
        return it->second;
    }
    const M& model() const { return model_; }
    const std::vector<State>& visits() const { return visits_; }
    const std::vector<u64>& visit_fps() const { return visit_fps_; }

    // `reconstruct_path` (src/checker/bfs.rs:314-342).
    Path<M> reconstruct_path(u64 fp) const {
        std::deque<u64> fps;
        u64 next = fp;
        while (auto src = generated_.get(next)) {
            fps.push_front(next);
            if (src->first == 0) break;
            next = src->first;
        }
        return Path<M>::from_fingerprints(model_, fps);
    }

    // `Checker::report` tail (src/checker.rs:229-238), without the polling loop.
    std::string report_done() const {
        std::ostringstream os;
        os << "Done. states=" << state_count() << ", unique=" << unique_state_count()
           << ", sec=" << (u64)elapsed_ << "\n";
        for (auto& [name, path] : discoveries()) {
            const char* cls = "counterexample";
            for (auto& p : properties_)
                if (name == p.name && p.expectation == Expectation::Sometimes) cls = "example";
            os << "Discovered \"" << name << "\" " << cls << " " << path.display(model_);
        }
        return os.str();
    }

  private:
    size_t discoveries_len() const {
        std::shared_lock<RwLock> g(disc_mu_);
        return discoveries_.size();
    }
    bool has_discovery(const char* name) const {
        std::shared_lock<RwLock> g(disc_mu_);
        return discoveries_.count(name) != 0;
    }
    void insert_discovery(const char* name, u64 fp) {
        // `discoveries.insert` (bfs.rs:199,207,268): later writers overwrite ("races, fine").
        std::unique_lock<RwLock> g(disc_mu_);
        discoveries_[name] = fp;
    }

    // Worker loop + job market (src/checker/bfs.rs:75-152).
    void worker(size_t t) {
        (void)t;
        try {
            const size_t property_count = properties_.size();
            std::deque<Job> pending;
            for (;;) {
                if (pending.empty()) {
                    std::unique_lock<std::mutex> g(market_mu_);
                    if (market_.jobs.empty()) {
                        if (market_.wait_count == opt_.thread_count) {
                            has_new_job_.notify_all();
                            return;
                        }
                        has_new_job_.wait(g);
                        continue;
                    }
                    pending = std::move(market_.jobs.back());
                    market_.jobs.pop_back();
                    market_.wait_count -= 1;
                }
                check_block(pending, 1500);
                if (discoveries_len() == property_count) {
                    {
                        std::lock_guard<std::mutex> g(market_mu_);
                        market_.wait_count += 1;
                    }
                    has_new_job_.notify_all();
                    return;
                }
                if (opt_.target_state_count != 0 &&
                    opt_.target_state_count <= state_count_.load(std::memory_order_relaxed))
                    return;
                if (pending.size() > 1 && opt_.thread_count > 1) {
                    std::lock_guard<std::mutex> g(market_mu_);
                    size_t pieces = 1 + std::min<size_t>(market_.wait_count, pending.size());
                    size_t size = pending.size() / pieces;
                    for (size_t i = 1; i < pieces; ++i) {
                        // `pending.split_off(pending.len() - size)`: the back (oldest) part.
                        std::deque<Job> piece(std::make_move_iterator(pending.end() - size), std::make_move_iterator(pending.end()));
                        pending.erase(pending.end() - size, pending.end());
                        market_.jobs.push_back(std::move(piece));
                        has_new_job_.notify_one();
                    }
                } else if (pending.empty()) {
                    std::lock_guard<std::mutex> g(market_mu_);
                    market_.wait_count += 1;
                }
            }
        } catch (...) {
            std::lock_guard<std::mutex> g(market_mu_);
            if (!worker_error_) worker_error_ = std::current_exception();
            market_.wait_count += 1;
            has_new_job_.notify_all();
        }
    }

    // `check_block` (src/checker/bfs.rs:165-274).
    void check_block(std::deque<Job>& pending, size_t max_count) {
        std::vector<typename M::Action> actions;
        for (;;) {
            if (max_count == 0) return;
            max_count -= 1;
            if (pending.empty()) return;
            Job job = std::move(pending.back());
            pending.pop_back();
            if (opt_.record_visits) {
                std::lock_guard<std::mutex> g(visit_mu_);
                visits_.push_back(job.state);
                visit_fps_.push_back(job.fp);  // the visitor gets reconstruct_path(fp), bfs.rs:187-189
            }
            bool is_awaiting_discoveries = false;
            for (size_t i = 0; i < properties_.size(); ++i) {
                const auto& p = properties_[i];
                if (has_discovery(p.name)) continue;
                switch (p.expectation) {
                    case Expectation::Always:
                        if (!p.condition(model_, job.state)) insert_discovery(p.name, job.fp);
                        else is_awaiting_discoveries = true;
                        break;
                    case Expectation::Sometimes:
                        if (p.condition(model_, job.state)) insert_discovery(p.name, job.fp);
                        else is_awaiting_discoveries = true;
                        break;
                    case Expectation::Eventually:
                        is_awaiting_discoveries = true;
                        if (p.condition(model_, job.state)) job.ebits &= ~(1ull << i);
                        break;
                }
            }
            if (!is_awaiting_discoveries) return;

            bool is_terminal = true;
            actions.clear();
            model_.actions(job.state, actions);
            for (auto& a : actions) {
                auto next = model_.next_state(job.state, a);
                if (!next) continue;
                if (!model_.within_boundary(*next)) continue;
                state_count_.fetch_add(1, std::memory_order_relaxed);
                u64 nfp = fingerprint(model_, *next);
                is_terminal = false;
                if (!generated_.insert_if_vacant(nfp, job.fp, job.depth + 1)) continue;
                pending.push_front(Job{std::move(*next), nfp, job.ebits, job.depth + 1});
            }
            if (is_terminal) {
                for (size_t i = 0; i < properties_.size(); ++i)
                    if (job.ebits & (1ull << i)) insert_discovery(properties_[i].name, job.fp);
            }
        }
    }

    M model_;
    CheckerOptions opt_;
    std::vector<Property<M>> properties_;
    std::atomic<u64> state_count_{0};
    Generated generated_;
    mutable RwLock disc_mu_;
    std::map<std::string, u64> discoveries_;
    struct JobMarket {
        size_t wait_count = 0;
        std::vector<std::deque<Job>> jobs;
    };
    mutable std::mutex market_mu_;
    std::condition_variable has_new_job_;
    JobMarket market_;
    std::vector<std::thread> handles_;
    std::exception_ptr worker_error_;
    std::mutex visit_mu_;
    std::vector<State> visits_;
    std::vector<u64> visit_fps_;
    std::chrono::steady_clock::time_point start_;
    double elapsed_ = 0;
    bool elapsed_set_ = false;
};

}  // namespace oracle
