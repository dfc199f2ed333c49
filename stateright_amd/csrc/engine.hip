// MI355X breadth-first model-checking engine library: the compiled-in GpuModel registry and the
// C ABI (include/stateright_gpu.h). The engine itself is engine.hpp.
#include <unordered_set>
#include "registry.hpp"
#include "dgraph.hpp"
#include "paxos.hpp"
#include "actor.hpp"
#include "dist_host.hpp"

namespace sr {

static thread_local std::string g_last_error;
static void set_error(const std::string& e) { g_last_error = e; }

}  // namespace sr

namespace sr {

// The registry (registry.hpp): each family of models compiles in its own translation unit.
static std::unique_ptr<EngineBase> make_model_engine(const EngineArgs& a) {
    if (a.o->symmetry && a.model != SR_MODEL_2PC)
        throw Error(SR_ERR_UNSUPPORTED, "symmetry reduction: model " + std::to_string(a.model) + " has no canonical form");
    switch (a.model) {
        case SR_MODEL_LINEAR_EQUATION:
        case SR_MODEL_BINARY_CLOCK:
        case SR_MODEL_DGRAPH:
        case SR_MODEL_ACTOR_FIXTURE:
            return reg_basic(a);
        case SR_MODEL_2PC: return reg_two_phase(a);
        case SR_MODEL_INCREMENT: return reg_increment(a);
        case SR_MODEL_INCREMENT_LOCK: return reg_increment_lock(a);
        case SR_MODEL_PAXOS:
            a.need(1);
            if (a.p[0] < 1 || a.p[0] > px::MAX_CLIENTS) throw Error(SR_ERR_UNSUPPORTED, "paxos: client_count must be in 1..=6");
            return a.p[0] <= Paxos::max_clients() ? reg_paxos(a) : reg_paxos_wide(a);
        case SR_MODEL_PINGPONG: return reg_ping_pong(a);
        case SR_MODEL_ABD:
        case SR_MODEL_SINGLE_COPY:
            return reg_registers(a);
    }
    throw Error(SR_ERR_ARG, "unknown model id " + std::to_string(a.model));
}

static std::unique_ptr<EngineBase> make_engine(int model, const i64* p, int np, const sr_opts& o) {
    return make_model_engine(EngineArgs{model, p, np, &o, false, nullptr, 0});
}

}  // namespace sr

using namespace sr;

struct sr_bfs {
    std::unique_ptr<EngineBase> e;
    bool joined = false;
};

namespace sr {
// Driver threads of the checks, pooled: a check runs on an idle pooled thread, which after its
// job spins for up to ~2 ms for the next one before it sleeps, so back-to-back checks pay neither
// thread creation nor a wake-up (~20-50 us per check on a 2 ms check). Threads are never joined:
// the pool lives for the process.
class DriverPool {
    struct Worker {
        std::mutex mu;
        std::condition_variable cv;
        std::function<void()> job;
        std::atomic<bool> has_job{false};
        std::atomic<bool> idle{false};
    };

  public:
    static DriverPool& get() {
        static DriverPool* p = new DriverPool();  // never destroyed (its threads outlive main)
        return *p;
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            for (Worker* w : workers_) {
                bool t = true;
                if (w->idle.compare_exchange_strong(t, false)) {
                    hand(w, std::move(f));
                    return;
                }
            }
        }
        Worker* w = new Worker();
        hand(w, std::move(f));
        std::thread([w] { loop(w); }).detach();
        std::lock_guard<std::mutex> g(mu_);
        workers_.push_back(w);
    }

  private:
    static void hand(Worker* w, std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(w->mu);
            w->job = std::move(f);
            w->has_job.store(true, std::memory_order_release);
        }
        w->cv.notify_one();
    }
    static void loop(Worker* w) {
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            for (u32 spin = 1; !w->has_job.load(std::memory_order_acquire); ++spin) {
                _mm_pause();
                if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                    std::unique_lock<std::mutex> g(w->mu);
                    w->cv.wait(g, [w] { return w->has_job.load(std::memory_order_acquire); });
                    break;
                }
            }
            std::function<void()> job;
            {
                std::lock_guard<std::mutex> g(w->mu);
                job.swap(w->job);
                w->has_job.store(false, std::memory_order_relaxed);
            }
            job();
            job = nullptr;
            w->idle.store(true, std::memory_order_release);
        }
    }
    std::mutex mu_;
    std::vector<Worker*> workers_;
};
}  // namespace sr

namespace sr {
// Host BFS over the reachable states of m: every slot self_loops() reports must be enabled and
// must return the state itself (the FAST expansion counts those slots without generating them).
template <class M>
static bool check_self_loops(const M& m, std::string& why) {
    constexpr int W = M::W, MW = M::MW;
    struct H {
        size_t operator()(const std::vector<u64>& v) const {
            u64 h = 0;
            for (u64 x : v) h = fmix64(h ^ x) + 0x9E3779B97F4A7C15ull;
            return (size_t)h;
        }
    };
    std::unordered_set<std::vector<u64>, H> seen;
    const std::vector<u64> inits = init_states_of(m);
    const int k = (int)(inits.size() / W);
    std::vector<std::vector<u64>> queue;
    for (int i = 0; i < k; ++i) {
        std::vector<u64> st(inits.begin() + i * W, inits.begin() + (i + 1) * W);
        if (seen.insert(st).second) queue.push_back(st);
    }
    for (size_t q = 0; q < queue.size(); ++q) {
        const std::vector<u64> st = queue[q];
        u64 mk[MW], sl[MW], o[W];
        m.enabled(st.data(), mk);
        m.self_loops(st.data(), mk, sl);
        for (int w = 0; w < MW; ++w) {
            if (sl[w] & ~mk[w]) {
                why = "self_loops reports a slot that is not enabled";
                return false;
            }
            for (u64 bits = sl[w]; bits; bits &= bits - 1) {
                const int a = w * 64 + __builtin_ctzll(bits);
                if (!m.apply(st.data(), a, o) || !std::equal(o, o + W, st.data())) {
                    why = "self_loops reports slot " + std::to_string(a) + ", whose next state differs";
                    return false;
                }
            }
            for (u64 bits = mk[w]; bits; bits &= bits - 1) {
                const int a = w * 64 + __builtin_ctzll(bits);
                if (!m.apply(st.data(), a, o)) continue;
                std::vector<u64> nx(o, o + W);
                if (seen.insert(nx).second) queue.push_back(std::move(nx));
            }
        }
    }
    return true;
}

}  // namespace sr

extern "C" {

void sr_opts_init(sr_opts* o) {
    std::memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(sr_opts);
}

void sr_opts_init_sized(sr_opts* o, uint32_t size) {
    // a caller built against an older (shorter) sr_opts: only its own bytes are written, and the
    // engine reads only struct_size bytes back (normalized_opts), defaulting the rest
    const uint32_t n = size < (uint32_t)sizeof(sr_opts) ? size : (uint32_t)sizeof(sr_opts);
    if (!o || n < sizeof(uint32_t)) return;
    std::memset(o, 0, n);
    o->struct_size = n;
}

const char* sr_last_error(void) { return g_last_error.c_str(); }

int sr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

struct sr_dist {
    std::unique_ptr<Comm> c;
    hipStream_t stream = nullptr;  // for sr_dist_barrier / sr_dist_allreduce_f64
    hipStream_t get_stream() {
        if (!stream) {
            SR_HIP(hipSetDevice(c->device));
            SR_HIP(create_stream(&stream, c->device));
        }
        return stream;
    }
};

// Starts the driver thread of an engine (spawn returns at once, like the reference's spawn_bfs).
static sr_bfs* start(std::unique_ptr<EngineBase> engine) {
    auto b = std::make_unique<sr_bfs>();
    b->e = std::move(engine);
    EngineBase* e = b->e.get();
    DriverPool::get().submit([e] {
        try {
            e->run();
        } catch (const Error& x) {
            e->status = x.code;
            e->error = x.what();
        } catch (const std::exception& x) {
            e->status = SR_ERR_HIP;
            e->error = x.what();
        }
        e->finished.store(true, std::memory_order_release);  // the last access to the engine
    });
    return b.release();
}

sr_bfs* sr_gpu_bfs_spawn(int32_t model_id, const int64_t* params, int32_t nparams, const sr_opts* opts) {
    try {
        const sr_opts o = normalized_opts(opts);
        if (sr_device_count() <= 0) throw Error(SR_ERR_NO_DEVICE, "no HIP device visible");
        return start(make_engine(model_id, params, nparams, o));
    } catch (const std::exception& x) {
        set_error(x.what());
        return nullptr;
    }
}

static sr_bfs* spawn_plugin(const sr_plugin* pl, sr_dist* comm, int32_t vparts, const int64_t* params, int32_t nparams,
                            const sr_opts* opts) {
    try {
        if (!pl || !pl->create) throw Error(SR_ERR_ARG, "null plugin");
        if (pl->abi != SR_PLUGIN_ABI || pl->opts_size != sizeof(sr_opts))
            throw Error(SR_ERR_ARG, std::string("plugin ") + (pl->name ? pl->name : "?") + " was built against other headers (abi " +
                                        std::to_string(pl->abi) + ", engine " + std::to_string(SR_PLUGIN_ABI) + ")");
        sr_opts o = normalized_opts(opts);
        if (comm) o.device = comm->c->device;
        if (sr_device_count() <= 0) throw Error(SR_ERR_NO_DEVICE, "no HIP device visible");
        char err[512] = {0};
        void* e = pl->create(params, nparams, &o, comm ? comm->c.get() : nullptr, vparts, err, sizeof(err));
        if (!e) throw Error(SR_ERR_ARG, std::string("plugin ") + (pl->name ? pl->name : "?") + ": " + err);
        return start(std::unique_ptr<EngineBase>(static_cast<EngineBase*>(e)));
    } catch (const std::exception& x) {
        set_error(x.what());
        return nullptr;
    }
}

sr_bfs* sr_gpu_bfs_spawn_plugin(const sr_plugin* pl, const int64_t* params, int32_t nparams, const sr_opts* opts) {
    return spawn_plugin(pl, nullptr, 0, params, nparams, opts);
}

sr_bfs* sr_gpu_bfs_spawn_plugin_partitioned(const sr_plugin* pl, sr_dist* comm, int32_t vparts, const int64_t* params,
                                            int32_t nparams, const sr_opts* opts) {
    if (!comm && vparts < 1) {
        set_error("partitioned plugin spawn: a communicator or virtual_partitions >= 1");
        return nullptr;
    }
    return spawn_plugin(pl, comm, comm ? 0 : std::max(vparts, 2), params, nparams, opts);
}

}  // extern "C"

namespace sr {
// A registered model built for host use only (no device tables), handed to f: the models whose
// description determines the state (`undescribe`), for sr_model_fingerprint and the self-test.
template <class F>
static i64 with_host_model(int model, const i64* p, int np, F&& f) {
    auto need = [&](int k) {
        if (np < k) throw Error(SR_ERR_ARG, "model " + std::to_string(model) + " needs " + std::to_string(k) + " params");
    };
    switch (model) {
        case SR_MODEL_LINEAR_EQUATION:
            need(3);
            return f(LinearEquation{(u32)(p[0] & 0xff), (u32)(p[1] & 0xff), (u32)(p[2] & 0xff)});
        case SR_MODEL_BINARY_CLOCK: return f(BinaryClock{});
        case SR_MODEL_2PC:
            need(1);
            if (p[0] < 1 || p[0] > 14) throw Error(SR_ERR_UNSUPPORTED, "2pc: rm_count must be in 1..=14");
            return f(TwoPhase{(int)p[0]});
        case SR_MODEL_INCREMENT:
            need(1);
            if (p[0] < 1 || p[0] > 15) throw Error(SR_ERR_UNSUPPORTED, "increment: threads must be in 1..=15");
            return p[0] <= 9 ? f(Increment<1>{(int)p[0]}) : f(Increment<2>{(int)p[0]});
        case SR_MODEL_INCREMENT_LOCK:
            need(1);
            if (p[0] < 1 || p[0] > 12) throw Error(SR_ERR_UNSUPPORTED, "increment_lock: threads must be in 1..=12");
            return p[0] <= 8 ? f(IncrementLock<1>{(int)p[0]}) : f(IncrementLock<2>{(int)p[0]});
        case SR_MODEL_PAXOS:
            need(1);
            if (p[0] < 1 || p[0] > px::MAX_CLIENTS) throw Error(SR_ERR_UNSUPPORTED, "paxos: client_count must be in 1..=6");
            return p[0] <= Paxos::max_clients() ? f(Paxos::make((int)p[0])) : f(PaxosWide::make((int)p[0]));
        case SR_MODEL_PINGPONG: {
            need(1);
            if (p[0] < 0 || p[0] > (i64)PingPongWide::MAX_NAT) throw Error(SR_ERR_UNSUPPORTED, "ping-pong: max_nat must be in 0..=14");
            auto fill = [&](auto& m) {
                m.max_nat = (u32)p[0];
                m.lossy = np > 1 && p[1] != 0;
                m.duplicating = np > 2 ? p[2] != 0 : true;
                m.maintains_history = np > 3 && p[3] != 0;
            };
            if (p[0] <= (i64)PingPong::MAX_NAT) {
                PingPong m;
                fill(m);
                return f(m);
            }
            PingPongWide m;
            fill(m);
            return f(m);
        }
        case SR_MODEL_ACTOR_FIXTURE: {
            need(1);
            ActorFixture m;
            m.kind = (int)p[0];
            return f(m);
        }
        case SR_MODEL_ABD: {
            need(1);
            AbdRegister m;
            static_cast<act::AbdSys&>(m) = act::AbdSys::make((int)p[0], np > 1 ? (int)p[1] : 2, -1);
            return f(m);
        }
        case SR_MODEL_SINGLE_COPY: {
            need(1);
            SingleCopyRegister m;
            static_cast<act::SingleCopySys&>(m) = act::SingleCopySys::make((int)p[0], np > 1 ? (int)p[1] : 1);
            return f(m);
        }
        default:
            return SR_ERR_UNSUPPORTED;
    }
}

// Host BFS over up to max_states reachable states of m: every state's description must give the
// state back (undescribe) and so the engine's fingerprint of it. Returns the states checked.
template <class M>
static i64 describe_roundtrip(const M& m, i64 max_states, std::string& why) {
    if constexpr (!has_undescribe<M>::value) {
        why = "model has no state description inverse";
        return SR_ERR_UNSUPPORTED;
    } else {
        constexpr int W = M::W, MW = M::MW;
        struct H {
            size_t operator()(const std::vector<u64>& v) const {
                u64 h = 0;
                for (u64 x : v) h = fmix64(h ^ x) + 0x9E3779B97F4A7C15ull;
                return (size_t)h;
            }
        };
        std::unordered_set<std::vector<u64>, H> seen;
        std::vector<std::vector<u64>> queue;
        const std::vector<u64> inits = init_states_of(m);
        for (size_t i = 0; i + W <= inits.size(); i += W) {
            std::vector<u64> st(inits.begin() + (i64)i, inits.begin() + (i64)(i + W));
            if (seen.insert(st).second) queue.push_back(st);
        }
        std::vector<i64> d((size_t)m.describe_width());
        for (size_t q = 0; q < queue.size() && (i64)q < max_states; ++q) {
            const std::vector<u64> st = queue[q];
            m.describe(st.data(), d.data());
            u64 back[W];
            m.undescribe(d.data(), back);
            if (!std::equal(back, back + W, st.data())) {
                why = "state " + std::to_string(q) + " does not survive describe -> undescribe";
                return SR_ERR_ARG;
            }
            u64 fp = 0;
            if (described_fingerprint(m, d.data(), (int)d.size(), &fp) != SR_OK || fp != state_fp<M>(st.data())) {
                why = "state " + std::to_string(q) + ": sr_model_fingerprint differs from the engine's fingerprint";
                return SR_ERR_ARG;
            }
            u64 mk[MW], o[W];
            m.enabled(st.data(), mk);
            for (int w = 0; w < MW; ++w)
                for (u64 bits = mk[w]; bits; bits &= bits - 1) {
                    const int a = w * 64 + __builtin_ctzll(bits);
                    if (!m.apply(st.data(), a, o)) continue;
                    std::vector<u64> nx(o, o + W);
                    if (seen.insert(nx).second) queue.push_back(std::move(nx));
                }
        }
        return (i64)std::min<size_t>(queue.size(), (size_t)max_states);
    }
}
}  // namespace sr

extern "C" {

int32_t sr_model_fingerprint(int32_t model, const int64_t* p, int32_t np, const int64_t* d, int32_t width, uint64_t* fp) {
    try {
        std::string why;
        const int r = (int)with_host_model(model, p, np, [&](const auto& m) { return (i64)described_fingerprint(m, d, width, fp, &why); });
        if (r != SR_OK) set_error(why);
        return r;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int64_t sr_selftest_describe(int32_t model, const int64_t* p, int32_t np, int64_t max_states) {
    try {
        std::string why;
        const i64 r = with_host_model(model, p, np, [&](const auto& m) { return (i64)describe_roundtrip(m, max_states, why); });
        if (r < 0) set_error(why);
        return r;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

// Until the check's driver job has finished: a spin for the first ~20 ms (a short check's end is
// seen at once), then polls every 50 us.
static void wait_finished(sr_bfs* b) {
    const auto t0 = std::chrono::steady_clock::now();
    for (u32 spin = 1; !b->e->finished.load(std::memory_order_acquire); ++spin) {
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20))
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        else
            _mm_pause();
    }
}

int32_t sr_gpu_bfs_join(sr_bfs* b) {
    if (!b) return SR_ERR_ARG;
    if (!b->joined) {
        wait_finished(b);
        b->joined = true;
    }
    if (b->e->status != SR_OK) set_error(b->e->error);
    return b->e->status;
}

int32_t sr_gpu_bfs_is_done(const sr_bfs* b) { return b && b->e->finished && b->e->reference_done ? 1 : 0; }
int32_t sr_gpu_bfs_is_running(const sr_bfs* b) { return b && !b->e->finished ? 1 : 0; }
uint64_t sr_gpu_bfs_state_count(const sr_bfs* b) { return b ? b->e->state_count.load() : 0; }
uint64_t sr_gpu_bfs_unique_state_count(const sr_bfs* b) { return b ? b->e->unique.load() : 0; }
uint32_t sr_gpu_bfs_max_depth(const sr_bfs* b) { return b ? b->e->max_depth.load() : 0; }

int32_t sr_gpu_bfs_stats(const sr_bfs* b, sr_stats* out) {
    if (!b || !out) return SR_ERR_ARG;
    *out = b->e->stats;
    return SR_OK;
}

int32_t sr_gpu_bfs_stats_sized(const sr_bfs* b, sr_stats* out, uint32_t size) {
    if (!b || (!out && size)) return SR_ERR_ARG;
    if (out) std::memcpy(out, &b->e->stats, std::min<size_t>(size, sizeof(sr_stats)));
    return (int32_t)sizeof(sr_stats);
}

int64_t sr_gpu_bfs_launch_profile(const sr_bfs* b, double* kernel_ms, uint64_t* frontier, int64_t cap) {
    if (!b) return SR_ERR_ARG;
    const auto& ms = b->e->launch_ms;
    const auto& fr = b->e->launch_frontier;
    const int64_t n = (int64_t)ms.size();
    for (int64_t i = 0; i < std::min(n, cap); ++i) {
        if (kernel_ms) kernel_ms[i] = ms[i];
        if (frontier) frontier[i] = i < (int64_t)fr.size() ? fr[i] : 0;
    }
    return n;
}

int64_t sr_gpu_bfs_launch_counters(const sr_bfs* b, uint64_t* probes, uint64_t* cas, int64_t cap) {
    if (!b) return SR_ERR_ARG;
    const auto& pr = b->e->launch_probes;
    const auto& cs = b->e->launch_cas;
    const int64_t n = (int64_t)pr.size();
    for (int64_t i = 0; i < std::min(n, cap); ++i) {
        if (probes) probes[i] = pr[i];
        if (cas) cas[i] = i < (int64_t)cs.size() ? cs[i] : 0;
    }
    return n;
}

int32_t sr_gpu_bfs_property_count(const sr_bfs* b) { return b ? b->e->nprops() : 0; }

int32_t sr_gpu_bfs_property(const sr_bfs* b, int32_t p, char* name, int32_t cap, int32_t* expectation) {
    if (!b || p < 0 || p >= b->e->nprops()) return SR_ERR_ARG;
    const char* n = b->e->prop_name(p);
    if (name && cap > 0) std::snprintf(name, (size_t)cap, "%s", n);
    if (expectation) *expectation = b->e->expectation(p);
    return (int32_t)std::strlen(n);
}

int32_t sr_gpu_bfs_discovery(const sr_bfs* b, int32_t p, uint64_t* fp_chain, uint32_t cap) {
    try {
        if (!b) return SR_ERR_ARG;
        std::vector<u64> c;
        b->e->chain(p, c);
        if (fp_chain) std::memcpy(fp_chain, c.data(), std::min<size_t>(cap, c.size()) * sizeof(u64));
        return (int32_t)c.size();
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int32_t sr_gpu_bfs_discovery_path(const sr_bfs* b, int32_t p, int64_t* action_ids, int32_t cap_actions,
                                  int64_t* states, int64_t cap_states) {
    try {
        if (!b) return SR_ERR_ARG;
        std::vector<i64> a, s;
        int n = b->e->path(p, a, s);
        if (n < 0) return -1;
        if (action_ids) std::memcpy(action_ids, a.data(), std::min<size_t>((size_t)cap_actions, a.size()) * sizeof(i64));
        if (states) std::memcpy(states, s.data(), std::min<size_t>((size_t)cap_states, s.size()) * sizeof(i64));
        return n;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int32_t sr_gpu_bfs_describe_width(const sr_bfs* b) { return b ? b->e->width() : 0; }

int32_t sr_gpu_bfs_action_name(const sr_bfs* b, int64_t id, char* buf, int32_t cap) {
    if (!b) return SR_ERR_ARG;
    std::string s = b->e->action_name(id);
    if (buf && cap > 0) std::snprintf(buf, (size_t)cap, "%s", s.c_str());
    return (int32_t)s.size();
}

int64_t sr_gpu_bfs_visits(const sr_bfs* b, int64_t* out, int64_t cap) {
    if (!b) return SR_ERR_ARG;
    auto v = b->e->visits();
    if (out) std::memcpy(out, v.data(), (size_t)std::min<int64_t>(cap, (int64_t)v.size()) * sizeof(int64_t));
    return (int64_t)v.size();
}

int64_t sr_gpu_bfs_visit_tree(const sr_bfs* b, int64_t* parent, int64_t* action, int64_t cap) {
    try {
        if (!b) return SR_ERR_ARG;
        std::vector<i64> p, a;
        if (!b->e->visit_tree(p, a)) {
            set_error("this check kept no visit record (sr_opts.record_visits = 0)");
            return SR_ERR_UNSUPPORTED;
        }
        const size_t n = std::min<size_t>((size_t)std::max<int64_t>(cap, 0), p.size());
        if (parent) std::memcpy(parent, p.data(), n * sizeof(i64));
        if (action) std::memcpy(action, a.data(), n * sizeof(i64));
        return (int64_t)p.size();
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int64_t sr_gpu_bfs_action_id_bound(const sr_bfs* b) { return b ? b->e->action_id_bound() : 0; }
int32_t sr_gpu_bfs_init_count(const sr_bfs* b) { return b ? b->e->init_count() : 0; }

int32_t sr_gpu_bfs_replay_trace(const sr_bfs* b, int32_t init, const int64_t* ids, int32_t n, int32_t* conditions,
                                int64_t cap, int32_t* terminal) {
    if (!b) return SR_ERR_ARG;
    std::vector<i64> s;
    std::vector<int> c, all;
    int term = 0;
    int r = b->e->replay(init, ids, n, s, c, &all, &term);
    if (r < 0) return -1;
    for (int64_t i = 0; i < (int64_t)all.size() && i < cap; ++i) conditions[i] = all[i];
    if (terminal) *terminal = term;
    return r;
}

int32_t sr_gpu_bfs_explore(const sr_bfs* b, const uint64_t* fps, int32_t n, int64_t* action_ids, int32_t* has_state,
                           uint64_t* fp_out, int64_t* states, int32_t cap) {
    try {
        if (!b || (n > 0 && !fps)) return SR_ERR_ARG;
        std::vector<i64> a, st;
        std::vector<int> h;
        std::vector<u64> f;
        const int v = b->e->explore(fps, n, a, h, f, st);
        if (v < 0) {
            set_error("Unable to find state following fingerprints");
            return -1;
        }
        const int wd = b->e->width();
        for (int i = 0; i < v && i < cap; ++i) {
            if (action_ids) action_ids[i] = a[i];
            if (has_state) has_state[i] = h[i];
            if (fp_out) fp_out[i] = f[i];
            if (states) std::memcpy(states + (size_t)i * wd, st.data() + (size_t)i * wd, wd * sizeof(i64));
        }
        return v;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int32_t sr_gpu_bfs_replay(const sr_bfs* b, int32_t init, const int64_t* ids, int32_t n, int64_t* states, int64_t cap_states,
                          int32_t* conds, int32_t cap_conds) {
    if (!b) return SR_ERR_ARG;
    std::vector<i64> s;
    std::vector<int> c;
    int r = b->e->replay(init, ids, n, s, c);
    if (r < 0) return -1;
    if (states) std::memcpy(states, s.data(), (size_t)std::min<int64_t>(cap_states, (int64_t)s.size()) * sizeof(int64_t));
    for (int i = 0; i < (int)c.size() && i < cap_conds; ++i) conds[i] = c[i];
    return r;
}


int32_t sr_dist_unique_id(uint8_t* out) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) {
        set_error("ncclGetUniqueId failed");
        return SR_ERR_HIP;
    }
    static_assert(sizeof(ncclUniqueId) == SR_DIST_ID_BYTES, "RCCL unique id size");
    std::memcpy(out, &id, sizeof(id));
    return SR_OK;
}

sr_dist* sr_dist_init(int32_t rank, int32_t world, const uint8_t* idb, int32_t device) {
    try {
        if (world < 1 || rank < 0 || rank >= world) throw Error(SR_ERR_ARG, "bad rank/world");
        SR_HIP(hipSetDevice(device));
        auto c = std::make_unique<RcclComm>();
        c->rank = rank;
        c->world = world;
        c->device = device;
        ncclUniqueId id;
        std::memcpy(&id, idb, sizeof(id));
        SR_NCCL(ncclCommInitRank(&c->nccl, world, id, rank));
        auto d = std::make_unique<sr_dist>();
        d->c = std::move(c);
        return d.release();
    } catch (const std::exception& x) {
        set_error(x.what());
        return nullptr;
    }
}

int32_t sr_dist_local_group(int32_t world, const int32_t* devices, sr_dist** out) {
    try {
        if (world < 1 || !out) throw Error(SR_ERR_ARG, "bad world/out");
        auto g = std::make_shared<LocalGroup>(world);
        for (int r = 0; r < world; ++r) {
            auto c = std::make_unique<LocalComm>();
            c->rank = r;
            c->world = world;
            c->device = devices ? devices[r] : 0;
            c->g = g;
            g->devices[r] = c->device;
            auto d = std::make_unique<sr_dist>();
            d->c = std::move(c);
            out[r] = d.release();
        }
        return SR_OK;
    } catch (const std::exception& x) {
        set_error(x.what());
        return SR_ERR_ARG;
    }
}

sr_dist* sr_dist_shm_init(int32_t rank, int32_t world, const char* name, int32_t device, int64_t slot_bytes,
                          int32_t devices_distinct) {
    try {
        if (world < 1 || rank < 0 || rank >= world || !name || slot_bytes < 4096) throw Error(SR_ERR_ARG, "bad shm communicator");
        SR_HIP(hipSetDevice(device));
        auto d = std::make_unique<sr_dist>();
        d->c = std::make_unique<ShmComm>(rank, world, std::string(name), device, (size_t)slot_bytes, devices_distinct != 0);
        return d.release();
    } catch (const std::exception& x) {
        set_error(x.what());
        return nullptr;
    }
}

int32_t sr_dist_host_protocol(const char* name, int32_t rank, int32_t world, const sr_dist_host_opts* opts,
                              sr_dist_host_result* out) {
    try {
        if (world < 1 || rank < 0 || rank >= world || !name || !opts || !out) throw Error(SR_ERR_ARG, "bad host protocol run");
        sr_dist_host_opts o;
        std::memset(&o, 0, sizeof(o));
        std::memcpy(&o, opts, std::min<size_t>(sizeof(o), opts->struct_size ? opts->struct_size : sizeof(o)));
        if (o.rm_count < 1 || o.rm_count > 7) throw Error(SR_ERR_UNSUPPORTED, "host protocol run: rm_count must be in 1..=7");
        ShmComm c(rank, world, std::string(name), -1, (size_t)1 << 24, false);
        c.host_only = true;
        DistHostRun run(c, o);
        const int r = run.run();
        *out = run.r;
        return r;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    } catch (const std::exception& x) {
        set_error(x.what());
        return SR_ERR_ARG;
    }
}

int32_t sr_dist_rank(const sr_dist* d) { return d ? d->c->rank : SR_ERR_ARG; }
int32_t sr_dist_world(const sr_dist* d) { return d ? d->c->world : SR_ERR_ARG; }
int32_t sr_dist_nranks(const sr_dist* d) { return d ? d->c->nranks() : SR_ERR_ARG; }
int32_t sr_dist_kind(const sr_dist* d, char* buf, int32_t cap) {
    if (!d) return SR_ERR_ARG;
    const char* k = d->c->kind();
    if (buf && cap > 0) std::snprintf(buf, (size_t)cap, "%s", k);
    return (int32_t)std::strlen(k);
}

int32_t sr_dist_barrier(sr_dist* d) {
    try {
        if (!d) return SR_ERR_ARG;
        SR_HIP(hipSetDevice(d->c->device));
        SR_HIP(hipDeviceSynchronize());
        d->c->barrier(d->get_stream());
        return SR_OK;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

int32_t sr_dist_allreduce_f64(sr_dist* d, double* values, int32_t n, int32_t op) {
    try {
        if (!d || !values || n < 1 || op < 0 || op > 2) return SR_ERR_ARG;
        // doubles travel as order-preserving u64 keys, so min and max are exact (no sum)
        if (op == 2) throw Error(SR_ERR_ARG, "sr_dist_allreduce_f64: only min (0) and max (1)");
        std::vector<u64> k(n);
        for (int i = 0; i < n; ++i) {
            u64 b;
            std::memcpy(&b, &values[i], 8);
            k[i] = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
        }
        SR_HIP(hipSetDevice(d->c->device));
        hipStream_t s = d->get_stream();
        DBuf<u64> buf;
        buf.alloc(d->c->device, n);
        SR_HIP(hipMemcpyAsync(buf.p, k.data(), n * 8, hipMemcpyHostToDevice, s));
        d->c->all_reduce(buf.p, n, op == 0 ? RedOp::Min : RedOp::Max, s);
        SR_HIP(hipMemcpyAsync(k.data(), buf.p, n * 8, hipMemcpyDeviceToHost, s));
        SR_HIP(hipStreamSynchronize(s));
        for (int i = 0; i < n; ++i) {
            const u64 b = (k[i] >> 63) ? (k[i] & 0x7fffffffffffffffull) : ~k[i];
            std::memcpy(&values[i], &b, 8);
        }
        return SR_OK;
    } catch (const Error& x) {
        set_error(x.what());
        return x.code;
    }
}

void sr_dist_free(sr_dist* d) {
    if (!d) return;
    if (d->stream && hipStreamDestroy(d->stream) == hipSuccess) StreamCensus::get().destroyed(d->c->device);
    delete d;
}

int32_t sr_rccl_version(int32_t* runtime, int32_t* compiled) {
    int v = 0;
    if (ncclGetVersion(&v) != ncclSuccess) return SR_ERR_HIP;
    if (runtime) *runtime = v;
    if (compiled) *compiled = NCCL_VERSION_CODE;
    return SR_OK;
}

#ifndef SR_BUILD_DIGEST
#define SR_BUILD_DIGEST "unstamped"
#endif
const char* sr_build_digest(void) { return SR_BUILD_DIGEST; }

int32_t sr_hip_runtime_version(int32_t* runtime, int32_t* compiled) {
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return SR_ERR_HIP;
    if (runtime) *runtime = v;
    if (compiled) *compiled = HIP_VERSION;
    return SR_OK;
}

int32_t sr_selftest_tables(void) {
    // qperm is a bijection on B bits (exhaustive for small B)
    for (u32 B = 1; B <= 18; ++B) {
        std::vector<u8> seen(1u << B, 0);
        for (u64 x = 0; x < (1ull << B); ++x) {
            const u64 y = (u64)qperm(x, B);
            if (y >> B || seen[y]) {
                set_error("qperm is not a bijection on " + std::to_string(B) + " bits");
                return SR_ERR_ARG;
            }
            seen[y] = 1;
        }
    }
    // qmix (one-word keys) is a bijection on B bits
    for (u32 B = 2; B <= 20; ++B) {
        std::vector<u8> seen(1u << B, 0);
        for (u64 x = 0; x < (1ull << B); ++x) {
            const u64 y = qmix(x, B);
            if (y >> B || seen[y]) {
                set_error("qmix is not a bijection on " + std::to_string(B) + " bits");
                return SR_ERR_ARG;
            }
            seen[y] = 1;
        }
    }
    // narrow (32-bit) quotient slots: 2pc N=9..12 keys in their tables, and a table larger than
    // the key space (remainder 1 bit); the filter key gives the permuted key back
    const u32 ncases[][2] = {{40, 25}, {40, 22}, {44, 27}, {48, 29}, {52, 31}, {16, 22}, {62, 40}};
    u64 rn = 0x452821E638D01377ull;
    for (auto& c : ncases) {
        const u32 q = c[0] > c[1] ? c[0] - c[1] : 1u;
        TableView t{nullptr, nullptr, (1ull << c[1]) - 1, q, 32 - q, c[0]};
        t.s32 = 1;
        if (q + SLOT32_DMIN > 32) {
            t.s32 = 0;
            t.dbits = 64 - q;
        }
        for (int i = 0; i < 100000; ++i) {
            rn = fmix64(rn + 0x9E3779B97F4A7C15ull);
            const u64 key = rn & ((1ull << c[0]) - 1);
            const u64 h = qmix(key, c[0]);
            const ProbeKey pk = quot_probe(t, h);
            const u64 d = (rn >> 40) % 500;
            const u64 slotv = pk.tag + d;
            if ((t.s32 && slotv >> 32) || quot_decode(t, (pk.home + d) & t.mask, slotv) != h || pk.home > t.mask ||
                filter_key(t, pk) != h + 1) {
                set_error("narrow quotient slot encode/decode mismatch at B=" + std::to_string(c[0]));
                return SR_ERR_ARG;
            }
        }
    }
    // quotient slot values decode to the key at every displacement (B = 89, k = 33: increment_lock
    // N=12's table; B = 68, k = 20)
    const u32 cases[][2] = {{89, 33}, {68, 20}, {82, 26}, {120, 64}};
    u64 r = 0x243F6A8885A308D3ull;
    for (auto& c : cases) {
        TableView t{nullptr, nullptr, (c[1] >= 64 ? ~0ull : (1ull << c[1]) - 1), c[0] - c[1], 64 - (c[0] - c[1]), c[0]};
        for (int i = 0; i < 100000; ++i) {
            r = fmix64(r + 0x9E3779B97F4A7C15ull);
            const u64 r2 = fmix64(r ^ 0xABCDEFull);
            const u128 key = ((u128)r2 << 64 | r) & (((u128)1 << c[0]) - 1);
            const u128 h = qperm(key, c[0]);
            const ProbeKey pk = quot_probe(t, h);
            const u64 d = r2 % 200;
            if (quot_decode(t, (pk.home + d) & t.mask, pk.tag + d) != h || pk.home > t.mask || (pk.tag & ((1ull << t.dbits) - 1)) != 1) {
                set_error("quotient slot encode/decode mismatch at B=" + std::to_string(c[0]));
                return SR_ERR_ARG;
            }
        }
    }
    return SR_OK;
}

// PaxosHist::linearizable (the cluster-graph test) against PaxosHist::linearizable_search (the
// tester's serialization search) on random histories of the register clients' protocol (every
// client: Write invoked at init; on its completion the Read is invoked, recording how many ops every
// other client had completed; the Read completes with any value): all client counts 1..6.
static bool check_linearizability(std::string& why) {
    u64 x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { return x = fmix64(x + 0x632BE59BD9B4E019ull); };
    for (u32 C = 1; C <= px::MAX_CLIENTS; ++C) {
        PaxosHist h;
        h.C = C;
        u32 nonlin = 0;
        for (int it = 0; it < 40000; ++it) {
            u64 lo = 0, hi = 0;
            const u32 steps = (u32)(rnd() % (2 * C + 1));
            for (u32 k = 0; k < steps; ++k) {
                const u32 t = (u32)(rnd() % C), ph = h.phase(lo, hi, t);
                if (ph == 0) {
                    for (u32 u = 0; u < C; ++u)
                        if (u != t) PaxosHist::put(lo, hi, h.last_off(t, u), 2, h.phase(lo, hi, u));
                } else if (ph == 1) {
                    PaxosHist::put(lo, hi, h.ret_off(t), 3, rnd() % (C + 1));
                } else {
                    continue;
                }
                PaxosHist::put(lo, hi, 2 * t, 2, ph + 1);
            }
            const bool a = h.linearizable(lo, hi), b = h.linearizable_search(lo, hi);
            nonlin += !b;
            if (a != b) {
                why = "linearizability: C=" + std::to_string(C) + " history " + std::to_string(lo) + "/" + std::to_string(hi) +
                      ": cluster test " + std::to_string(a) + ", search " + std::to_string(b);
                return false;
            }
        }
        if (C >= 2 && nonlin == 0) {
            why = "linearizability: no non-linearizable history drawn at C=" + std::to_string(C);
            return false;
        }
    }
    return true;
}

int32_t sr_selftest_models(void) {
    std::string why;
    if (!check_linearizability(why)) {
        set_error(why);
        return SR_ERR_ARG;
    }
    for (int n = 1; n <= 7; ++n) {
        TwoPhase m;
        m.n = n;
        if (!sr::check_self_loops(m, why)) {
            set_error("2pc n=" + std::to_string(n) + ": " + why);
            return SR_ERR_ARG;
        }
        if (n <= 6 && !sr::check_self_loops(Canon<TwoPhase>(m), why)) {
            set_error("2pc n=" + std::to_string(n) + " (canonical): " + why);
            return SR_ERR_ARG;
        }
    }
    return SR_OK;
}

int32_t sr_device_synchronize(int32_t device) {
    if (hipSetDevice(device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        set_error("hipDeviceSynchronize failed");
        return SR_ERR_HIP;
    }
    return SR_OK;
}

sr_bfs* sr_gpu_bfs_spawn_partitioned(sr_dist* comm, int32_t virtual_parts, int32_t model_id, const int64_t* params,
                                     int32_t nparams, const sr_opts* opts) {
    try {
        sr_opts o = normalized_opts(opts);
        if (comm) o.device = comm->c->device;
        if (sr_device_count() <= 0) throw Error(SR_ERR_NO_DEVICE, "no HIP device visible");
        return start(make_model_engine(EngineArgs{model_id, params, nparams, &o, true, comm ? comm->c.get() : nullptr, (int)virtual_parts}));
    } catch (const std::exception& x) {
        set_error(x.what());
        return nullptr;
    }
}

void sr_gpu_bfs_free(sr_bfs* b) {
    if (!b) return;
    if (!b->joined) wait_finished(b);  // the pooled driver thread must be done with the engine
    delete b;
}

}  // extern "C"

#if SR_TIMELINE
// ---- diagnostic build only (SR_TIMELINE=1): expand_fast's per-workgroup timeline ----
static u64* g_timeline_host_ptr = nullptr;
extern "C" int64_t sr_timeline_reset(int32_t device) {
    const size_t words = (size_t)TL_LAUNCHES * TL_BLOCKS * TL_STAMPS;
    if (hipSetDevice(device) != hipSuccess) return SR_ERR_HIP;
    if (!g_timeline_host_ptr) {
        if (hipMalloc(&g_timeline_host_ptr, words * 8) != hipSuccess) return SR_ERR_HIP;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), &g_timeline_host_ptr, sizeof(u64*)) != hipSuccess) return SR_ERR_HIP;
    }
    if (hipMemset(g_timeline_host_ptr, 0, words * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SR_ERR_HIP;
    return (int64_t)words;
}
extern "C" int64_t sr_timeline_fetch(int32_t device, uint64_t* out, int64_t cap) {
    const size_t words = (size_t)TL_LAUNCHES * TL_BLOCKS * TL_STAMPS;
    if (!g_timeline_host_ptr || hipSetDevice(device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SR_ERR_HIP;
    if (out && hipMemcpy(out, g_timeline_host_ptr, std::min<size_t>(words, (size_t)cap) * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return SR_ERR_HIP;
    return (int64_t)words;
}
#endif

#ifdef SR_ONE_TU
// One translation unit (diagnostic builds, scripts/build_timeline.sh): the registry families too.
#include "reg_basic.hip"
#include "reg_two_phase.hip"
#include "reg_increment.hip"
#include "reg_increment_lock.hip"
#include "reg_paxos.hip"
#include "reg_paxos_wide.hip"
#include "reg_ping_pong.hip"
#include "reg_registers.hip"
#endif
