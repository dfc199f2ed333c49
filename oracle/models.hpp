// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp).
//
// CPU restatements of the reference models with the reference's own data structures (Vec,
// BTreeSet, enums), so that the oracle pays the same per-successor costs as the Rust code it
// stands in for (clone of heap-allocated vectors/sets, stream hashing) when timed as the CPU
// baseline. Each model also exposes:
//   describe(state)  -> canonical integer vector (shared with the GPU engine's describe), and
//   action_id(action) -> canonical action id (shared with the GPU engine's action slots),
// so tests can compare state SETS, visit ORDER and PATHS between the oracle and the GPU engine.
#pragma once
#include "oracle.hpp"

namespace oracle {

inline void hash_vec_u8(const std::vector<u8>& v, Hasher& h) {
    h.write_usize(v.size());
    for (u8 x : v) h.write_u8(x);
}

// ---------------------------------------------------------------------------------------------
// LinearEquation (src/test_util.rs:140-188).
// ---------------------------------------------------------------------------------------------
struct LinearEquation {
    u8 a, b, c;
    using State = std::pair<u8, u8>;
    enum class Action { IncreaseX, IncreaseY };
    std::vector<State> init_states() const { return {State{0, 0}}; }
    void actions(const State&, std::vector<Action>& out) const {
        out.push_back(Action::IncreaseX);
        out.push_back(Action::IncreaseY);
    }
    std::optional<State> next_state(const State& s, Action a) const {
        if (a == Action::IncreaseX) return State{(u8)(s.first + 1), s.second};
        return State{s.first, (u8)(s.second + 1)};
    }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<LinearEquation>> properties() const {
        return {Property<LinearEquation>::sometimes("solvable", [](const LinearEquation& m, const State& s) {
            return (u8)(m.a * s.first + m.b * s.second) == m.c;
        })};
    }
    void hash_state(const State& s, Hasher& h) const { h.write_u8(s.first); h.write_u8(s.second); }
    std::vector<i64> describe(const State& s) const { return {s.first, s.second}; }
    i64 action_id(Action a) const { return a == Action::IncreaseX ? 0 : 1; }
    std::string format_action(Action a) const { return a == Action::IncreaseX ? "IncreaseX" : "IncreaseY"; }
};

// ---------------------------------------------------------------------------------------------
// BinaryClock (src/test_util.rs:4-45).
// ---------------------------------------------------------------------------------------------
struct BinaryClock {
    using State = int8_t;
    enum class Action { GoLow, GoHigh };
    std::vector<State> init_states() const { return {0, 1}; }
    void actions(const State& s, std::vector<Action>& out) const {
        out.push_back(s == 0 ? Action::GoHigh : Action::GoLow);
    }
    std::optional<State> next_state(const State&, Action a) const { return a == Action::GoLow ? 0 : 1; }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<BinaryClock>> properties() const {
        return {Property<BinaryClock>::always("in [0, 1]", [](const BinaryClock&, const State& s) {
            return 0 <= s && s <= 1;
        })};
    }
    void hash_state(const State& s, Hasher& h) const { h.write_u8((u8)s); }
    std::vector<i64> describe(const State& s) const { return {s}; }
    i64 action_id(Action a) const { return a == Action::GoLow ? 0 : 1; }
    std::string format_action(Action a) const { return a == Action::GoLow ? "GoLow" : "GoHigh"; }
};

// ---------------------------------------------------------------------------------------------
// DGraph (src/test_util.rs:47-116): a graph given by paths; one property.
// ---------------------------------------------------------------------------------------------
struct DGraph {
    std::set<u8> inits;
    std::map<u8, std::set<u8>> edges;
    Expectation expectation = Expectation::Eventually;
    int predicate = 0;  // 0: odd (s % 2 == 1), the only predicate the reference tests use
    using State = u8;
    using Action = u8;

    DGraph with_path(const std::vector<u8>& path) const {
        DGraph g = *this;
        u8 src = path.front();
        g.inits.insert(src);
        for (size_t i = 1; i < path.size(); ++i) {
            g.edges[src].insert(path[i]);
            src = path[i];
        }
        return g;
    }
    std::vector<State> init_states() const { return std::vector<State>(inits.begin(), inits.end()); }
    void actions(const State& s, std::vector<Action>& out) const {
        auto it = edges.find(s);
        if (it != edges.end())
            for (u8 d : it->second) out.push_back(d);
    }
    std::optional<State> next_state(const State&, Action a) const { return a; }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<DGraph>> properties() const {
        auto odd = [](const DGraph&, const State& s) { return s % 2 == 1; };
        return {Property<DGraph>{expectation, "odd", odd}};
    }
    void hash_state(const State& s, Hasher& h) const { h.write_u8(s); }
    std::vector<i64> describe(const State& s) const { return {s}; }
    i64 action_id(Action a) const { return a; }
    std::string format_action(Action a) const { return std::to_string(a); }
};

// ---------------------------------------------------------------------------------------------
// Two-phase commit (examples/2pc.rs:10-121).
// ---------------------------------------------------------------------------------------------
struct TwoPhaseSys {
    size_t rm_count;
    enum class RmState : u8 { Working, Prepared, Committed, Aborted };
    enum class TmState : u8 { Init, Committed, Aborted };
    // `enum Message { Prepared { rm }, Commit, Abort }` with derived Ord: by variant, then rm.
    struct Message {
        u8 kind;  // 0 Prepared, 1 Commit, 2 Abort
        size_t rm;
        bool operator<(const Message& o) const { return kind != o.kind ? kind < o.kind : rm < o.rm; }
        bool operator==(const Message& o) const { return kind == o.kind && rm == o.rm; }
    };
    struct State {
        std::vector<RmState> rm_state;
        TmState tm_state;
        std::vector<bool> tm_prepared;
        // `BTreeSet<Message>`: for <= 11 elements a B-tree is one leaf node, so a sorted vector
        // has the same clone cost (one allocation) and the same iteration order.
        std::vector<Message> msgs;
        bool contains(const Message& m) const { return std::binary_search(msgs.begin(), msgs.end(), m); }
        void insert(const Message& m) {
            auto it = std::lower_bound(msgs.begin(), msgs.end(), m);
            if (it == msgs.end() || !(*it == m)) msgs.insert(it, m);
        }
    };
    enum class Kind : u8 { TmRcvPrepared, TmCommit, TmAbort, RmPrepare, RmChooseToAbort, RmRcvCommitMsg, RmRcvAbortMsg };
    struct Action { Kind kind; size_t rm; };

    std::vector<State> init_states() const {
        return {State{std::vector<RmState>(rm_count, RmState::Working), TmState::Init,
                      std::vector<bool>(rm_count, false), {}}};
    }
    void actions(const State& s, std::vector<Action>& out) const {
        bool all_prepared = std::all_of(s.tm_prepared.begin(), s.tm_prepared.end(), [](bool p) { return p; });
        if (s.tm_state == TmState::Init && all_prepared) out.push_back({Kind::TmCommit, 0});
        if (s.tm_state == TmState::Init) out.push_back({Kind::TmAbort, 0});
        bool has_commit = s.contains(Message{1, 0});
        bool has_abort = s.contains(Message{2, 0});
        for (size_t rm = 0; rm < rm_count; ++rm) {
            if (s.tm_state == TmState::Init && s.contains(Message{0, rm})) out.push_back({Kind::TmRcvPrepared, rm});
            if (s.rm_state[rm] == RmState::Working) out.push_back({Kind::RmPrepare, rm});
            if (s.rm_state[rm] == RmState::Working) out.push_back({Kind::RmChooseToAbort, rm});
            if (has_commit) out.push_back({Kind::RmRcvCommitMsg, rm});
            if (has_abort) out.push_back({Kind::RmRcvAbortMsg, rm});
        }
    }
    std::optional<State> next_state(const State& last, Action a) const {
        State s = last;  // `last_state.clone()`, examples/2pc.rs:84
        switch (a.kind) {
            case Kind::TmRcvPrepared: s.tm_prepared[a.rm] = true; break;
            case Kind::TmCommit: s.tm_state = TmState::Committed; s.insert(Message{1, 0}); break;
            case Kind::TmAbort: s.tm_state = TmState::Aborted; s.insert(Message{2, 0}); break;
            case Kind::RmPrepare: s.rm_state[a.rm] = RmState::Prepared; s.insert(Message{0, a.rm}); break;
            case Kind::RmChooseToAbort: s.rm_state[a.rm] = RmState::Aborted; break;
            case Kind::RmRcvCommitMsg: s.rm_state[a.rm] = RmState::Committed; break;
            case Kind::RmRcvAbortMsg: s.rm_state[a.rm] = RmState::Aborted; break;
        }
        return s;
    }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<TwoPhaseSys>> properties() const {
        using P = Property<TwoPhaseSys>;
        return {
            P::sometimes("abort agreement", [](const TwoPhaseSys&, const State& s) {
                return std::all_of(s.rm_state.begin(), s.rm_state.end(), [](RmState r) { return r == RmState::Aborted; });
            }),
            P::sometimes("commit agreement", [](const TwoPhaseSys&, const State& s) {
                return std::all_of(s.rm_state.begin(), s.rm_state.end(), [](RmState r) { return r == RmState::Committed; });
            }),
            P::always("consistent", [](const TwoPhaseSys&, const State& s) {
                bool any_abort = false, any_commit = false;
                for (auto r : s.rm_state) {
                    any_abort |= r == RmState::Aborted;
                    any_commit |= r == RmState::Committed;
                }
                return !(any_abort && any_commit);
            }),
        };
    }
    // derive(Hash): Vec len + element discriminants, enum discriminant, Vec<bool>, BTreeSet len + elements.
    void hash_state(const State& s, Hasher& h) const {
        h.write_usize(s.rm_state.size());
        for (auto r : s.rm_state) h.write_u64((u64)r);
        h.write_u64((u64)s.tm_state);
        h.write_usize(s.tm_prepared.size());
        for (bool p : s.tm_prepared) h.write_bool(p);
        h.write_usize(s.msgs.size());
        for (auto& m : s.msgs) {
            h.write_u64(m.kind);
            if (m.kind == 0) h.write_usize(m.rm);
        }
    }
    // `impl Representative for TwoPhaseState` (examples/2pc.rs:164-182): RewritePlan sorts the
    // (rm_state, index) pairs (src/checker/rewrite_plan.rs:36-49), so RMs with EQUAL rm_state keep
    // their index order — not a canonical form of the RM permutation group.
    State representative(const State& s) const {
        std::vector<std::pair<RmState, size_t>> combined;
        for (size_t i = 0; i < s.rm_state.size(); ++i) combined.emplace_back(s.rm_state[i], i);
        std::sort(combined.begin(), combined.end());
        std::vector<size_t> reindex, rewrite(s.rm_state.size());
        for (auto& c : combined) reindex.push_back(c.second);
        for (size_t dst = 0; dst < reindex.size(); ++dst) rewrite[reindex[dst]] = dst;
        State r;
        r.tm_state = s.tm_state;
        for (size_t i : reindex) {
            r.rm_state.push_back(s.rm_state[i]);
            r.tm_prepared.push_back(s.tm_prepared[i]);
        }
        for (auto& m : s.msgs) r.insert(m.kind == 0 ? Message{0, rewrite[m.rm]} : m);
        return r;
    }
    // [rm_state x N, tm_state, tm_prepared x N, msg Prepared(rm) x N, msg Commit, msg Abort]
    std::vector<i64> describe(const State& s) const {
        std::vector<i64> d;
        for (auto r : s.rm_state) d.push_back((i64)r);
        d.push_back((i64)s.tm_state);
        for (bool p : s.tm_prepared) d.push_back(p);
        for (size_t rm = 0; rm < rm_count; ++rm) d.push_back(s.contains(Message{0, rm}) ? 1 : 0);
        d.push_back(s.contains(Message{1, 0}) ? 1 : 0);
        d.push_back(s.contains(Message{2, 0}) ? 1 : 0);
        return d;
    }
    // Action slots in `actions()` order: TmCommit=0, TmAbort=1, then per rm 5 slots.
    i64 action_id(Action a) const {
        switch (a.kind) {
            case Kind::TmCommit: return 0;
            case Kind::TmAbort: return 1;
            case Kind::TmRcvPrepared: return 2 + 5 * (i64)a.rm + 0;
            case Kind::RmPrepare: return 2 + 5 * (i64)a.rm + 1;
            case Kind::RmChooseToAbort: return 2 + 5 * (i64)a.rm + 2;
            case Kind::RmRcvCommitMsg: return 2 + 5 * (i64)a.rm + 3;
            case Kind::RmRcvAbortMsg: return 2 + 5 * (i64)a.rm + 4;
        }
        return -1;
    }
    std::string format_action(Action a) const {
        const char* names[] = {"TmRcvPrepared", "TmCommit", "TmAbort", "RmPrepare", "RmChooseToAbort", "RmRcvCommitMsg", "RmRcvAbortMsg"};
        std::string n = names[(int)a.kind];
        if (a.kind == Kind::TmCommit || a.kind == Kind::TmAbort) return n;
        return n + "(" + std::to_string(a.rm) + ")";
    }
};

// ---------------------------------------------------------------------------------------------
// Increment (examples/increment.rs:109-197): racy read/write of a shared u8.
// ---------------------------------------------------------------------------------------------
struct ProcState {
    u8 t, pc;
};

struct Increment {
    size_t n;
    struct State {
        u8 i;
        std::vector<ProcState> s;
    };
    struct Action { bool write; size_t thread; };
    std::vector<State> init_states() const { return {State{0, std::vector<ProcState>(n, ProcState{0, 1})}}; }
    void actions(const State& s, std::vector<Action>& out) const {
        for (size_t t = 0; t < n; ++t) {
            if (s.s[t].pc == 1) out.push_back({false, t});
            else if (s.s[t].pc == 2) out.push_back({true, t});
        }
    }
    std::optional<State> next_state(const State& last, Action a) const {
        State s = last;
        if (!a.write) {
            s.s[a.thread] = ProcState{last.i, 2};
        } else {
            s.s[a.thread].pc = 3;
            s.i = (u8)(last.s[a.thread].t + 1);
        }
        return s;
    }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<Increment>> properties() const {
        return {Property<Increment>::always("fin", [](const Increment&, const State& s) {
            u8 c = 0;
            for (auto& p : s.s) c += p.pc == 3;
            return c == s.i;
        })};
    }
    void hash_state(const State& s, Hasher& h) const {
        h.write_u8(s.i);
        h.write_usize(s.s.size());
        for (auto& p : s.s) { h.write_u8(p.t); h.write_u8(p.pc); }
    }
    std::vector<i64> describe(const State& s) const {
        std::vector<i64> d{s.i};
        for (auto& p : s.s) { d.push_back(p.t); d.push_back(p.pc); }
        return d;
    }
    i64 action_id(Action a) const { return 2 * (i64)a.thread + (a.write ? 1 : 0); }
    std::string format_action(Action a) const {
        return std::string(a.write ? "Write(" : "Read(") + std::to_string(a.thread) + ")";
    }
};

// ---------------------------------------------------------------------------------------------
// IncrementLock (examples/increment_lock.rs:3-107).
// ---------------------------------------------------------------------------------------------
struct IncrementLock {
    size_t n;
    struct State {
        u8 i;
        bool lock;
        std::vector<ProcState> s;
    };
    enum class Kind : u8 { Lock, Read, Write, Release };
    struct Action { Kind kind; size_t thread; };
    std::vector<State> init_states() const { return {State{0, false, std::vector<ProcState>(n, ProcState{0, 0})}}; }
    void actions(const State& s, std::vector<Action>& out) const {
        for (size_t t = 0; t < n; ++t) {
            switch (s.s[t].pc) {
                case 0: if (!s.lock) out.push_back({Kind::Lock, t}); break;
                case 1: out.push_back({Kind::Read, t}); break;
                case 2: out.push_back({Kind::Write, t}); break;
                case 3: if (s.lock) out.push_back({Kind::Release, t}); break;
                default: break;
            }
        }
    }
    std::optional<State> next_state(const State& last, Action a) const {
        State s = last;
        switch (a.kind) {
            case Kind::Lock: s.s[a.thread].pc = 1; s.lock = true; break;
            case Kind::Read: s.s[a.thread].pc = 2; s.s[a.thread].t = last.i; break;
            case Kind::Write: s.s[a.thread].pc = 3; s.i = (u8)(last.s[a.thread].t + 1); break;
            case Kind::Release: s.s[a.thread].pc = 4; s.lock = false; break;
        }
        return s;
    }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<IncrementLock>> properties() const {
        using P = Property<IncrementLock>;
        return {
            P::always("fin", [](const IncrementLock&, const State& s) {
                u8 c = 0;
                for (auto& p : s.s) c += p.pc >= 3;
                return c == s.i;
            }),
            P::always("mutex", [](const IncrementLock&, const State& s) {
                size_t c = 0;
                for (auto& p : s.s) c += (p.pc >= 1 && p.pc < 4);
                return c <= 1;
            }),
        };
    }
    void hash_state(const State& s, Hasher& h) const {
        h.write_u8(s.i);
        h.write_bool(s.lock);
        h.write_usize(s.s.size());
        for (auto& p : s.s) { h.write_u8(p.t); h.write_u8(p.pc); }
    }
    std::vector<i64> describe(const State& s) const {
        std::vector<i64> d{s.i, s.lock ? 1 : 0};
        for (auto& p : s.s) { d.push_back(p.t); d.push_back(p.pc); }
        return d;
    }
    i64 action_id(Action a) const { return 4 * (i64)a.thread + (i64)a.kind; }
    std::string format_action(Action a) const {
        const char* names[] = {"Lock", "Read", "Write", "Release"};
        return std::string(names[(int)a.kind]) + "(" + std::to_string(a.thread) + ")";
    }
};

// ---------------------------------------------------------------------------------------------
// The symmetry fixture of src/checker/dfs.rs:393-476 (`Sys`): two processes, each
// Loading -> Running <-> Paused; either process can step. Its representative sorts the process
// states (derived Ord: Paused < Loading < Running).
// ---------------------------------------------------------------------------------------------
struct SymToy {
    enum class Proc : u8 { Paused, Loading, Running };
    using State = std::vector<Proc>;
    using Action = size_t;  // `Id`
    std::vector<State> init_states() const { return {State{Proc::Loading, Proc::Loading}}; }
    void actions(const State&, std::vector<Action>& out) const {
        out.push_back(0);
        out.push_back(1);
    }
    std::optional<State> next_state(const State& last, Action i) const {
        State s = last;
        s[i] = s[i] == Proc::Loading ? Proc::Running : s[i] == Proc::Running ? Proc::Paused : Proc::Running;
        return s;
    }
    bool within_boundary(const State&) const { return true; }
    std::vector<Property<SymToy>> properties() const {
        using P = Property<SymToy>;
        return {
            P::always("visit all states", [](const SymToy&, const State&) { return true; }),
            P::sometimes("a process pauses", [](const SymToy&, const State& s) {
                return s[0] == Proc::Paused || s[1] == Proc::Paused;
            }),
        };
    }
    State representative(const State& s) const {
        State r = s;
        std::stable_sort(r.begin(), r.end());
        return r;
    }
    void hash_state(const State& s, Hasher& h) const {
        h.write_usize(s.size());
        for (auto p : s) h.write_u64((u64)p);
    }
    std::vector<i64> describe(const State& s) const { return {(i64)s[0], (i64)s[1]}; }
    i64 action_id(Action a) const { return (i64)a; }
    std::string format_action(Action a) const { return "Id(" + std::to_string(a) + ")"; }
};

}  // namespace oracle
