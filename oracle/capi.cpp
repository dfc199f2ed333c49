// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp). extern "C" surface for tests/ and bench.py.
#include <cstring>

#include "models.hpp"
#include "paxos.hpp"
#include "actor.hpp"
#include "dfs.hpp"

using namespace oracle;

namespace {

thread_local std::string g_last_error;

// Model ids are shared with include/stateright_gpu.h (SR_MODEL_*).
enum ModelId { LINEAR_EQUATION = 1, BINARY_CLOCK = 2, TWO_PHASE = 3, INCREMENT = 4, INCREMENT_LOCK = 5, DGRAPH = 6, PAXOS = 7, SYM_TOY = 8,
               PINGPONG = 9, ACTOR_FIXTURE = 10, ABD = 11, SINGLE_COPY = 12 };

struct HandleBase {
    virtual ~HandleBase() = default;
    virtual void join() = 0;
    virtual u64 state_count() const = 0;
    virtual u64 unique_state_count() const = 0;
    virtual u32 max_depth() const = 0;
    virtual bool is_done() const = 0;
    virtual double elapsed() const = 0;
    virtual std::vector<std::string> discovery_names() const = 0;
    virtual std::optional<std::vector<i64>> discovery_actions(const std::string& n) const = 0;
    virtual std::optional<std::vector<i64>> discovery_states(const std::string& n) const = 0;
    virtual std::vector<i64> visits() const = 0;
    // The path a visitor receives for visit i (`Path::from_fingerprints(reconstruct_path(fp))`).
    virtual std::optional<std::vector<i64>> visit_path(i64 i) const = 0;
    virtual int width() const = 0;
    virtual std::string report() const = 0;
};

template <class M>
struct Handle : HandleBase {
    BfsChecker<M> c;
    Handle(M m, CheckerOptions o) : c(std::move(m), o) {}
    void join() override { c.join(); }
    u64 state_count() const override { return c.state_count(); }
    u64 unique_state_count() const override { return c.unique_state_count(); }
    u32 max_depth() const override { return c.max_depth(); }
    bool is_done() const override { return c.is_done(); }
    double elapsed() const override { return c.elapsed_sec(); }
    std::vector<std::string> discovery_names() const override { return c.discovery_names(); }
    std::optional<std::vector<i64>> visit_path(i64 i) const override {
        const auto& f = c.visit_fps();
        if (i < 0 || i >= (i64)f.size()) return std::nullopt;
        return c.reconstruct_path(f[(size_t)i]).action_ids(c.model());
    }
    std::optional<std::vector<i64>> discovery_actions(const std::string& n) const override {
        auto fp = c.discovery_fp(n);
        if (!fp) return std::nullopt;
        return c.reconstruct_path(*fp).action_ids(c.model());
    }
    std::optional<std::vector<i64>> discovery_states(const std::string& n) const override {
        auto fp = c.discovery_fp(n);
        if (!fp) return std::nullopt;
        std::vector<i64> out;
        for (auto& [s, a] : c.reconstruct_path(*fp).steps) {
            auto d = c.model().describe(s);
            out.insert(out.end(), d.begin(), d.end());
        }
        return out;
    }
    std::vector<i64> visits() const override {
        std::vector<i64> out;
        for (auto& s : c.visits()) {
            auto d = c.model().describe(s);
            out.insert(out.end(), d.begin(), d.end());
        }
        return out;
    }
    int width() const override { return (int)c.model().describe(c.model().init_states().front()).size(); }
    std::string report() const override { return c.report_done(); }
};

template <class M, class = void>
struct has_representative : std::false_type {};
template <class M>
struct has_representative<M, std::void_t<decltype(std::declval<const M&>().representative(
                                 std::declval<const typename M::State&>()))>> : std::true_type {};

// `spawn_dfs` (src/checker/dfs.rs), optionally with `symmetry()`.
template <class M>
struct DfsHandle : HandleBase {
    DfsChecker<M> c;
    DfsHandle(M m, CheckerOptions o, typename DfsChecker<M>::Representative rep) : c(std::move(m), o, std::move(rep)) {}
    void join() override { c.join(); }
    u64 state_count() const override { return c.state_count(); }
    u64 unique_state_count() const override { return c.unique_state_count(); }
    u32 max_depth() const override { return 0; }
    bool is_done() const override { return c.is_done(); }
    double elapsed() const override { return c.elapsed_sec(); }
    std::vector<std::string> discovery_names() const override { return c.discovery_names(); }
    std::optional<std::vector<i64>> visit_path(i64 i) const override {
        if (i < 0 || i >= (i64)c.visit_count()) return std::nullopt;
        return c.visit_path((size_t)i).action_ids(c.model());
    }
    std::optional<std::vector<i64>> discovery_actions(const std::string& n) const override {
        auto p = c.discovery(n);
        if (!p) return std::nullopt;
        return p->action_ids(c.model());
    }
    std::optional<std::vector<i64>> discovery_states(const std::string& n) const override {
        auto p = c.discovery(n);
        if (!p) return std::nullopt;
        std::vector<i64> out;
        for (auto& [s, a] : p->steps) {
            auto d = c.model().describe(s);
            out.insert(out.end(), d.begin(), d.end());
        }
        return out;
    }
    std::vector<i64> visits() const override {
        std::vector<i64> out;
        for (auto& s : c.visits()) {
            auto d = c.model().describe(s);
            out.insert(out.end(), d.begin(), d.end());
        }
        return out;
    }
    int width() const override { return (int)c.model().describe(c.model().init_states().front()).size(); }
    std::string report() const override { return ""; }
};

DGraph make_dgraph(const i64* p, int np) {
    // params: [expectation(0 always,1 eventually,2 sometimes), len0, v..., len1, v..., ...]
    DGraph g;
    g.expectation = p[0] == 0 ? Expectation::Always : p[0] == 1 ? Expectation::Eventually : Expectation::Sometimes;
    int i = 1;
    while (i < np) {
        int len = (int)p[i++];
        std::vector<u8> path;
        for (int k = 0; k < len && i < np; ++k) path.push_back((u8)p[i++]);
        if (!path.empty()) g = g.with_path(path);
    }
    return g;
}

template <class F>
auto with_model(int model, const i64* p, int np, F&& f) {
    switch (model) {
        case LINEAR_EQUATION: return f(LinearEquation{(u8)p[0], (u8)p[1], (u8)p[2]});
        case BINARY_CLOCK: return f(BinaryClock{});
        case TWO_PHASE: return f(TwoPhaseSys{(size_t)p[0]});
        case INCREMENT: return f(Increment{(size_t)p[0]});
        case INCREMENT_LOCK: return f(IncrementLock{(size_t)p[0]});
        case DGRAPH: return f(make_dgraph(p, np));
        case PAXOS: return f(paxos::PaxosModel{(size_t)p[0], 3});
        case SYM_TOY: return f(SymToy{});
        case PINGPONG: {  // (max_nat, lossy, duplicating, maintains_history)
            actor::PingPongModel m;
            m.sys.max_nat = (u32)p[0];
            m.sys.lossy = np > 1 && p[1];
            m.sys.duplicating = np > 2 ? p[2] != 0 : true;
            m.sys.maintains_history = np > 3 && p[3];
            return f(m);
        }
        case ACTOR_FIXTURE: {  // (kind: 0 undeliverable, 1 timer)
            actor::FixtureModel m;
            m.sys.kind = (int)p[0];
            return f(m);
        }
        case ABD: {  // (client_count, server_count)
            actor::AbdModel m;
            m.sys.client_count = (size_t)p[0];
            m.sys.server_count = np > 1 ? (size_t)p[1] : 2;
            return f(m);
        }
        case SINGLE_COPY: {  // (client_count, server_count)
            actor::SingleCopyModel m;
            m.sys.client_count = (size_t)p[0];
            m.sys.server_count = np > 1 ? (size_t)p[1] : 1;
            return f(m);
        }
    }
    throw std::runtime_error("unknown model id " + std::to_string(model));
}

int copy_out(const std::vector<i64>& v, i64* out, i64 cap) {
    if (out) std::memcpy(out, v.data(), sizeof(i64) * (size_t)std::min<i64>(cap, (i64)v.size()));
    return (int)v.size();
}

}  // namespace

extern "C" {

const char* oracle_last_error() { return g_last_error.c_str(); }

void* oracle_spawn_bfs(int model, const i64* params, int nparams, int threads, u64 target, int record_visits) {
    try {
        CheckerOptions o;
        o.thread_count = threads > 0 ? (size_t)threads : 1;
        o.target_state_count = target;
        o.record_visits = record_visits != 0;
        return with_model(model, params, nparams, [&](auto m) -> HandleBase* {
            return new Handle<decltype(m)>(std::move(m), o);
        });
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return nullptr;
    }
}

void* oracle_spawn_dfs(int model, const i64* params, int nparams, int threads, u64 target, int record_visits,
                       int symmetry) {
    try {
        CheckerOptions o;
        o.thread_count = threads > 0 ? (size_t)threads : 1;
        o.target_state_count = target;
        o.record_visits = record_visits != 0;
        return with_model(model, params, nparams, [&](auto m) -> HandleBase* {
            using Mt = decltype(m);
            typename DfsChecker<Mt>::Representative rep = nullptr;
            if (symmetry) {
                if constexpr (has_representative<Mt>::value) {
                    Mt copy = m;
                    rep = [copy](const typename Mt::State& s) { return copy.representative(s); };
                } else {
                    throw std::runtime_error("model has no Representative implementation");
                }
            }
            return new DfsHandle<Mt>(std::move(m), o, std::move(rep));
        });
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return nullptr;
    }
}

int oracle_join(void* h) {
    try {
        static_cast<HandleBase*>(h)->join();
        return 0;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -1;
    }
}
u64 oracle_state_count(void* h) { return static_cast<HandleBase*>(h)->state_count(); }
u64 oracle_unique_state_count(void* h) { return static_cast<HandleBase*>(h)->unique_state_count(); }
u32 oracle_max_depth(void* h) { return static_cast<HandleBase*>(h)->max_depth(); }
int oracle_is_done(void* h) { return static_cast<HandleBase*>(h)->is_done() ? 1 : 0; }
double oracle_elapsed_sec(void* h) { return static_cast<HandleBase*>(h)->elapsed(); }
int oracle_width(void* h) { return static_cast<HandleBase*>(h)->width(); }

int oracle_discovery_count(void* h) { return (int)static_cast<HandleBase*>(h)->discovery_names().size(); }
int oracle_discovery_name(void* h, int i, char* buf, int cap) {
    auto names = static_cast<HandleBase*>(h)->discovery_names();
    if (i < 0 || i >= (int)names.size()) return -1;
    std::snprintf(buf, (size_t)cap, "%s", names[(size_t)i].c_str());
    return (int)names[(size_t)i].size();
}
// Returns the number of actions on the discovery path (-1 if none / error).
int oracle_discovery_actions(void* h, const char* name, i64* out, i64 cap) {
    try {
        auto v = static_cast<HandleBase*>(h)->discovery_actions(name);
        if (!v) return -1;
        return copy_out(*v, out, cap);
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -2;
    }
}
// Returns the number of i64 written: (path length + 1) * width.
int oracle_discovery_states(void* h, const char* name, i64* out, i64 cap) {
    try {
        auto v = static_cast<HandleBase*>(h)->discovery_states(name);
        if (!v) return -1;
        return copy_out(*v, out, cap);
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -2;
    }
}
i64 oracle_visits(void* h, i64* out, i64 cap) {
    auto v = static_cast<HandleBase*>(h)->visits();
    if (out) std::memcpy(out, v.data(), sizeof(i64) * (size_t)std::min<i64>(cap, (i64)v.size()));
    return (i64)v.size();
}
// Action ids of the path the visitor receives for visit i; -1 if out of range.
int oracle_visit_path(void* h, i64 i, i64* out, i64 cap) {
    try {
        auto v = static_cast<HandleBase*>(h)->visit_path(i);
        if (!v) return -1;
        return copy_out(*v, out, cap);
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -2;
    }
}
int oracle_report(void* h, char* buf, int cap) {
    auto s = static_cast<HandleBase*>(h)->report();
    std::snprintf(buf, (size_t)cap, "%s", s.c_str());
    return (int)s.size();
}
void oracle_free(void* h) { delete static_cast<HandleBase*>(h); }

// Replays `actions` (canonical ids) from the first init state on the CPU model
// (`Path::from_actions`, src/checker/path.rs:90-112). Writes the states' descriptions to
// `states_out` and, per property, whether its condition holds on the final state to `holds_out`.
// Returns the number of i64 written to states_out, or -1 if some action is not enabled.
int oracle_replay(int model, const i64* params, int nparams, const i64* actions, int n_actions,
                  i64* states_out, i64 cap, int* holds_out, int holds_cap) {
    try {
        return with_model(model, params, nparams, [&](auto m) -> int {
            using M = decltype(m);
            auto init = m.init_states().front();
            auto p = Path<M>::from_actions(m, init, std::vector<i64>(actions, actions + n_actions));
            if (!p) return -1;
            std::vector<i64> out;
            for (auto& [s, a] : p->steps) {
                auto d = m.describe(s);
                out.insert(out.end(), d.begin(), d.end());
            }
            auto props = m.properties();
            for (int i = 0; i < (int)props.size() && i < holds_cap; ++i)
                holds_out[i] = props[(size_t)i].condition(m, p->last_state()) ? 1 : 0;
            return copy_out(out, states_out, cap);
        });
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -2;
    }
}

// Fingerprint of a primitive i8 with the oracle hasher (explorer.rs:260-268 golden shape).
u64 oracle_fingerprint_i8(int8_t v) {
    Hasher h;
    h.write_u8((u8)v);
    return h.finish();
}

}  // extern "C"
