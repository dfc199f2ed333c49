// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp's header).
//
// A CPU restatement of Stateright's depth-first checker (`src/checker/dfs.rs`), including its
// symmetry reduction (`CheckerBuilder::symmetry`, src/checker.rs:145-160): the visited set holds
// the fingerprint of `representative(next_state)`, while the ORIGINAL state and its fingerprint
// continue the path (dfs.rs:258-267). Used to pin what the GPU engine's `spawn_dfs` reproduces
// (full-exploration counts are traversal-independent) and to show what it cannot (see
// tests/test_oracle_dfs.py: with a non-canonical representative the symmetry-reduced count
// depends on the visit order).
#pragma once

#include "oracle.hpp"

namespace oracle {

template <class M>
class DfsChecker {
  public:
    using State = typename M::State;
    using EventuallyBits = u64;
    struct Job {
        State state;
        std::vector<u64> fps;  // fingerprints init..state (the path so far)
        EventuallyBits ebits;
    };
    using Representative = std::function<State(const State&)>;

    // `DfsChecker::spawn` (src/checker/dfs.rs:35-170).
    DfsChecker(M model, CheckerOptions opt, Representative symmetry = nullptr)
        : model_(std::move(model)), opt_(opt), symmetry_(std::move(symmetry)),
          generated_(std::max<size_t>(4 * std::max<unsigned>(1, std::thread::hardware_concurrency()), 4)) {
        properties_ = model_.properties();
        std::vector<State> init_states;
        for (auto& s : model_.init_states())
            if (model_.within_boundary(s)) init_states.push_back(s);
        state_count_ = init_states.size();
        for (auto& s : init_states) generated_.insert_if_vacant(key(s), 0, 0);
        EventuallyBits ebits = 0;
        for (size_t i = 0; i < properties_.size(); ++i)
            if (properties_[i].expectation == Expectation::Eventually) ebits |= (1ull << i);
        std::vector<Job> pending;
        for (auto& s : init_states) pending.push_back(Job{s, {fingerprint(model_, s)}, ebits});
        market_.wait_count = opt_.thread_count;
        market_.jobs.push_back(std::move(pending));
        start_ = std::chrono::steady_clock::now();
        for (size_t t = 0; t < opt_.thread_count; ++t) handles_.emplace_back([this] { worker(); });
    }
    ~DfsChecker() { join(); }

    // `Checker` impl (src/checker/dfs.rs:304-341).
    u64 state_count() const { return state_count_.load(std::memory_order_relaxed); }
    u64 unique_state_count() const { return generated_.len(); }
    u32 max_depth() const { return 0; }  // DFS has no depth metric
    DfsChecker& join() {
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
    const M& model() const { return model_; }
    std::vector<std::string> discovery_names() const {
        std::lock_guard<std::mutex> g(disc_mu_);
        std::vector<std::string> out;
        for (auto& kv : discoveries_) out.push_back(kv.first);
        return out;
    }
    std::optional<Path<M>> discovery(const std::string& name) const {
        std::lock_guard<std::mutex> g(disc_mu_);
        auto it = discoveries_.find(name);
        if (it == discoveries_.end()) return std::nullopt;
        return Path<M>::from_fingerprints(model_, std::deque<u64>(it->second.begin(), it->second.end()));
    }
    const std::vector<State>& visits() const { return visits_; }
    // The visitor's path at visit i (`Path::from_fingerprints(fingerprints)`, dfs.rs:195-199).
    Path<M> visit_path(size_t i) const {
        return Path<M>::from_fingerprints(model_, std::deque<u64>(visit_fps_[i].begin(), visit_fps_[i].end()));
    }
    size_t visit_count() const { return visit_fps_.size(); }

  private:
    u64 key(const State& s) const { return symmetry_ ? fingerprint(model_, symmetry_(s)) : fingerprint(model_, s); }
    size_t discoveries_len() const {
        std::lock_guard<std::mutex> g(disc_mu_);
        return discoveries_.size();
    }
    bool has_discovery(const char* n) const {
        std::lock_guard<std::mutex> g(disc_mu_);
        return discoveries_.count(n) != 0;
    }
    void insert_discovery(const char* n, const std::vector<u64>& fps) {
        std::lock_guard<std::mutex> g(disc_mu_);
        discoveries_[n] = fps;
    }

    // Worker loop + job market (src/checker/dfs.rs:89-159).
    void worker() {
        try {
            std::vector<Job> pending;
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
                if (discoveries_len() == properties_.size()) {
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
                        // `pending.split_off(pending.len() - size)`: the top of the stack
                        std::vector<Job> piece(std::make_move_iterator(pending.end() - size),
                                               std::make_move_iterator(pending.end()));
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

    // `check_block` (src/checker/dfs.rs:172-301).
    void check_block(std::vector<Job>& pending, size_t max_count) {
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
                visit_fps_.push_back(job.fps);
            }
            bool is_awaiting_discoveries = false;
            for (size_t i = 0; i < properties_.size(); ++i) {
                const auto& p = properties_[i];
                if (has_discovery(p.name)) continue;
                switch (p.expectation) {
                    case Expectation::Always:
                        if (!p.condition(model_, job.state)) insert_discovery(p.name, job.fps);
                        else is_awaiting_discoveries = true;
                        break;
                    case Expectation::Sometimes:
                        if (p.condition(model_, job.state)) insert_discovery(p.name, job.fps);
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
                if (!generated_.insert_if_vacant(key(*next), 0, 0)) {
                    is_terminal = false;
                    continue;
                }
                is_terminal = false;
                std::vector<u64> fps = job.fps;
                fps.push_back(fingerprint(model_, *next));  // the original, not the representative
                pending.push_back(Job{std::move(*next), std::move(fps), job.ebits});
            }
            if (is_terminal) {
                for (size_t i = 0; i < properties_.size(); ++i)
                    if (job.ebits & (1ull << i)) insert_discovery(properties_[i].name, job.fps);
            }
        }
    }

    M model_;
    CheckerOptions opt_;
    Representative symmetry_;
    std::vector<Property<M>> properties_;
    std::atomic<u64> state_count_{0};
    Generated generated_;
    mutable std::mutex disc_mu_;
    std::map<std::string, std::vector<u64>> discoveries_;
    struct JobMarket {
        size_t wait_count = 0;
        std::vector<std::vector<Job>> jobs;
    };
    mutable std::mutex market_mu_;
    std::condition_variable has_new_job_;
    JobMarket market_;
    std::vector<std::thread> handles_;
    std::exception_ptr worker_error_;
    std::mutex visit_mu_;
    std::vector<State> visits_;
    std::vector<std::vector<u64>> visit_fps_;
    std::chrono::steady_clock::time_point start_;
    double elapsed_ = 0;
    bool elapsed_set_ = false;
};

}  // namespace oracle
