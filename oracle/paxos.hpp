// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp).
//
// Restatement of the paxos example as the reference composes it:
//   ActorModel (src/actor/model.rs:176-327) over RegisterActor (src/actor/register.rs:119-217)
//   wrapping PaxosActor (examples/paxos.rs:93-221), with a LinearizabilityTester<Id,
//   Register<char>> history (src/semantics/linearizability.rs:57-241,
//   src/semantics/register.rs:10-48) recorded by RegisterMsg::record_{invocations,returns}
//   (src/actor/register.rs:37-87), a non-duplicating lossless network (a SET of envelopes,
//   src/actor/model.rs:69) and the properties of examples/paxos.rs:251-261.
//
// The network is iterated in sorted order. The reference iterates a HashSet seeded by ahash, so
// its action ORDER (and thus which of several shortest discovery paths it reports) is not
// reproducible here; counts of full explorations do not depend on it.
#pragma once
#include "oracle.hpp"

namespace oracle {
namespace paxos {

using Id = u64;
struct Ballot {
    u32 round = 0;
    Id id = 0;
    auto key() const { return std::make_tuple(round, id); }
    bool operator<(const Ballot& o) const { return key() < o.key(); }
    bool operator<=(const Ballot& o) const { return key() <= o.key(); }
    bool operator==(const Ballot& o) const { return key() == o.key(); }
};
struct Proposal {  // (RequestId, Id, Value)
    u64 req = 0;
    Id requester = 0;
    char value = 0;
    auto key() const { return std::make_tuple(req, requester, value); }
    bool operator<(const Proposal& o) const { return key() < o.key(); }
    bool operator==(const Proposal& o) const { return key() == o.key(); }
};
using Acc = std::optional<std::pair<Ballot, Proposal>>;  // Option<(Ballot, Proposal)>

enum Kind : u8 { PREPARE, PREPARED, ACCEPT, ACCEPTED, DECIDED, PUT, GET, PUTOK, GETOK };
struct Msg {
    Kind kind = PREPARE;
    Ballot ballot;
    Acc last_accepted;  // Prepared
    Proposal proposal;  // Accept / Decided
    u64 req = 0;        // Put / Get / PutOk / GetOk
    char value = 0;     // Put / GetOk
    auto key() const {
        return std::make_tuple(kind, ballot.key(), last_accepted.has_value(),
                               last_accepted ? last_accepted->first.key() : std::make_tuple(0u, (u64)0),
                               last_accepted ? last_accepted->second.key() : std::make_tuple((u64)0, (u64)0, (char)0),
                               proposal.key(), req, value);
    }
    bool operator<(const Msg& o) const { return key() < o.key(); }
    bool operator==(const Msg& o) const { return key() == o.key(); }
};
struct Envelope {
    Id src = 0, dst = 0;
    Msg msg;
    bool operator<(const Envelope& o) const {
        return std::tie(src, dst) != std::tie(o.src, o.dst) ? std::tie(src, dst) < std::tie(o.src, o.dst) : msg < o.msg;
    }
    bool operator==(const Envelope& o) const { return src == o.src && dst == o.dst && msg == o.msg; }
};

struct PaxosState {  // examples/paxos.rs:78-91
    Ballot ballot;
    std::optional<Proposal> proposal;
    std::map<Id, Acc> prepares;
    std::set<Id> accepts;
    Acc accepted;
    bool is_decided = false;
    bool operator==(const PaxosState& o) const {
        return ballot == o.ballot && proposal == o.proposal && prepares == o.prepares && accepts == o.accepts &&
               accepted == o.accepted && is_decided == o.is_decided;
    }
};
struct ClientState {  // RegisterActorState::Client
    std::optional<u64> awaiting;
    u64 op_count = 0;
    bool operator==(const ClientState& o) const { return awaiting == o.awaiting && op_count == o.op_count; }
};
struct ActorState {
    bool is_server = true;
    PaxosState server;
    ClientState client;
    bool operator==(const ActorState& o) const {
        return is_server == o.is_server && (is_server ? server == o.server : client == o.client);
    }
};

// LinearizabilityTester<Id, Register<char>> (src/semantics/linearizability.rs:57-241).
struct Op {
    bool write = false;
    char value = 0;
    bool operator==(const Op& o) const { return write == o.write && value == o.value; }
};
struct Ret {
    bool write_ok = false;
    char value = 0;
    bool operator==(const Ret& o) const { return write_ok == o.write_ok && value == o.value; }
};
using LastCompleted = std::map<Id, size_t>;
struct Complete {
    LastCompleted last;
    Op op;
    Ret ret;
    bool operator==(const Complete& o) const { return last == o.last && op == o.op && ret == o.ret; }
};
struct InFlight {
    LastCompleted last;
    Op op;
    bool operator==(const InFlight& o) const { return last == o.last && op == o.op; }
};
struct History {
    char init = 0;  // Register(Value::default())
    std::map<Id, std::deque<Complete>> by_thread;
    std::map<Id, InFlight> in_flight;
    bool valid = true;
    bool operator==(const History& o) const {
        return by_thread == o.by_thread && in_flight == o.in_flight && valid == o.valid;
    }

    void on_invoke(Id t, Op op) {  // linearizability.rs:102-125
        if (!valid) return;
        if (in_flight.count(t)) {
            valid = false;
            return;
        }
        LastCompleted last;
        for (auto& [id, cs] : by_thread)
            if (id != t && !cs.empty()) last[id] = cs.size() - 1;
        in_flight[t] = InFlight{last, op};
        by_thread[t];  // `serialize` requires the entry
    }
    void on_return(Id t, Ret ret) {  // linearizability.rs:131-147
        if (!valid) return;
        auto it = in_flight.find(t);
        if (it == in_flight.end()) {
            valid = false;
            by_thread[t];
            return;
        }
        InFlight f = it->second;
        in_flight.erase(it);
        by_thread[t].push_back(Complete{f.last, f.op, ret});
    }

    // `serialized_history().is_some()` (linearizability.rs:159-240): backtracking search over the
    // interleavings consistent with real-time order and the register's semantics.
    bool linearizable() const {
        if (!valid) return false;
        std::map<Id, std::deque<std::pair<size_t, Complete>>> rem;
        for (auto& [t, cs] : by_thread) {
            auto& d = rem[t];
            for (size_t i = 0; i < cs.size(); ++i) d.emplace_back(i, cs[i]);
        }
        return serialize(init, rem, in_flight);
    }
    static bool violates(const LastCompleted& last, const std::map<Id, std::deque<std::pair<size_t, Complete>>>& rem) {
        for (auto& [peer, min_t] : last) {
            auto it = rem.find(peer);
            if (it != rem.end() && !it->second.empty() && it->second.front().first <= min_t) return true;
        }
        return false;
    }
    static bool serialize(char reg, const std::map<Id, std::deque<std::pair<size_t, Complete>>>& rem,
                          const std::map<Id, InFlight>& inflight) {
        bool done = true;
        for (auto& [t, h] : rem)
            if (!h.empty()) done = false;
        if (done) return true;
        for (auto& [t, h] : rem) {
            if (h.empty()) {
                auto f = inflight.find(t);
                if (f == inflight.end()) continue;
                if (violates(f->second.last, rem)) continue;
                char r2 = reg;
                if (f->second.op.write) r2 = f->second.op.value;  // invoke: Write sets, Read returns
                auto inflight2 = inflight;
                inflight2.erase(t);
                if (serialize(r2, rem, inflight2)) return true;
            } else {
                auto rem2 = rem;
                auto [idx, c] = rem2[t].front();
                rem2[t].pop_front();
                if (violates(c.last, rem2)) continue;
                char r2 = reg;
                // Register::is_valid_step (src/semantics/register.rs:34-47)
                if (c.op.write && c.ret.write_ok) r2 = c.op.value;
                else if (!c.op.write && !c.ret.write_ok) {
                    if (c.ret.value != reg) continue;
                } else continue;
                if (serialize(r2, rem2, inflight)) return true;
            }
        }
        return false;
    }
};

// The register history in canonical form (shared with the GPU encodings' `describe`, so that a
// description determines the state and the engine can fingerprint it: sr_model_fingerprint). Per
// client c (actor id first_id + c), c = 0..C-1: its Get's returned value (value code: '\0' 0,
// the k-th client's letter k + 1; -1 while the Get has not returned), then for every other client
// u in ascending order how many of u's ops had completed when c invoked its Get (-1 before it).
// Every client runs put_count 1 (a Put invoked at init, then one Get).
inline void describe_register_history(const History& H, size_t first_id, size_t C, std::vector<i64>& d) {
    for (size_t c = 0; c < C; ++c) {
        const Id id = first_id + c;
        auto bt = H.by_thread.find(id);
        const size_t ndone = bt == H.by_thread.end() ? 0 : bt->second.size();
        const LastCompleted* last = nullptr;  // the Get's real-time predecessors
        if (ndone >= 2) last = &bt->second[1].last;
        else if (ndone == 1 && H.in_flight.count(id)) last = &H.in_flight.at(id).last;
        const char v = ndone >= 2 ? bt->second[1].ret.value : 0;
        d.push_back(ndone >= 2 ? (v ? (i64)(v - 'A' + 1) : 0) : -1);
        for (size_t u = 0; u < C; ++u) {
            if (u == c) continue;
            if (!last) {
                d.push_back(-1);
                continue;
            }
            auto it = last->find(first_id + u);
            d.push_back(it == last->end() ? 0 : (i64)it->second + 1);
        }
    }
}
inline int register_history_width(size_t C) { return (int)(C * C); }

struct State {
    std::vector<ActorState> actors;
    History history;
    std::set<Envelope> network;  // is_timer_set is always empty: no actor sets timers
};

struct Action {
    Envelope env;  // ActorModelAction::Deliver { src, dst, msg }
};

inline size_t majority(size_t n) { return n / 2 + 1; }  // src/actor.rs:437-439

struct PaxosModel {
    size_t client_count = 2, server_count = 3;
    using State = paxos::State;
    using Action = paxos::Action;

    std::vector<Id> peers(Id i) const {  // model_peers (src/actor/model.rs:79-84)
        std::vector<Id> p;
        for (Id j = 0; j < server_count; ++j)
            if (j != i) p.push_back(j);
        return p;
    }

    // record_msg_out = RegisterMsg::record_invocations (src/actor/register.rs:37-58)
    static void record_out(History& h, const Envelope& e) {
        if (e.msg.kind == GET) h.on_invoke(e.src, Op{false, 0});
        else if (e.msg.kind == PUT) h.on_invoke(e.src, Op{true, e.msg.value});
    }
    // record_msg_in = RegisterMsg::record_returns (src/actor/register.rs:64-87)
    static bool record_in(History& h, const Envelope& e) {
        if (e.msg.kind == GETOK) {
            h.on_return(e.dst, Ret{false, e.msg.value});
            return true;
        }
        if (e.msg.kind == PUTOK) {
            h.on_return(e.dst, Ret{true, 0});
            return true;
        }
        return false;
    }
    // process_commands (src/actor/model.rs:176-202): record, then insert into the set network.
    static void send_all(State& s, const std::vector<Envelope>& out) {
        for (auto& e : out) {
            record_out(s.history, e);
            s.network.insert(e);
        }
    }

    std::vector<State> init_states() const {  // src/actor/model.rs:215-242
        State s;
        std::vector<Envelope> out;
        for (Id i = 0; i < server_count + client_count; ++i) {
            ActorState a;
            if (i < server_count) {
                a.is_server = true;  // PaxosActor::on_start: ballot (0, Id(0)), nothing sent
            } else {
                // RegisterActor::Client::on_start with put_count = 1 (src/actor/register.rs:130-160)
                a.is_server = false;
                u64 req = 1 * i;
                char value = (char)('A' + (i - server_count));
                std::vector<Envelope> o{Envelope{i, (i + 0) % server_count, Msg{PUT, {}, {}, {}, req, value}}};
                a.client = ClientState{req, 1};
                s.actors.push_back(a);
                send_all(s, o);
                continue;
            }
            s.actors.push_back(a);
        }
        return {s};
    }

    void actions(const State& s, std::vector<Action>& out) const {  // src/actor/model.rs:238-257
        for (auto& e : s.network)
            if (e.dst < s.actors.size()) out.push_back(Action{e});
    }

    // PaxosActor::on_msg (examples/paxos.rs:116-221). Returns true when the actor "touched" its
    // state (Cow::Owned); outputs go to `o`.
    bool server_on_msg(Id id, PaxosState& st, Id src, const Msg& msg, std::vector<Envelope>& o) const {
        if (st.is_decided) {
            if (msg.kind == GET) {
                o.push_back(Envelope{id, src, Msg{GETOK, {}, {}, {}, msg.req, st.accepted->second.value}});
            }
            return false;
        }
        auto bcast = [&](const Msg& m) {
            for (Id p : peers(id)) o.push_back(Envelope{id, p, m});
        };
        switch (msg.kind) {
            case PUT:
                if (st.proposal) return false;
                st.proposal = Proposal{msg.req, src, msg.value};
                st.prepares.clear();
                st.accepts.clear();
                st.ballot = Ballot{st.ballot.round + 1, id};
                st.prepares[id] = st.accepted;
                bcast(Msg{PREPARE, st.ballot, {}, {}, 0, 0});
                return true;
            case PREPARE:
                if (!(st.ballot < msg.ballot)) return false;
                st.ballot = msg.ballot;
                o.push_back(Envelope{id, src, Msg{PREPARED, msg.ballot, st.accepted, {}, 0, 0}});
                return true;
            case PREPARED:
                if (!(msg.ballot == st.ballot)) return false;
                st.prepares[src] = msg.last_accepted;
                if (st.prepares.size() == majority(server_count)) {
                    // max over Option<(Ballot, Proposal)> values (None < Some)
                    Acc best;
                    for (auto& [k, v] : st.prepares)
                        if (v && (!best || best->first < v->first || (best->first == v->first && best->second < v->second))) best = v;
                    Proposal p = best ? best->second : *st.proposal;
                    st.proposal = p;
                    st.accepted = std::make_pair(msg.ballot, p);
                    st.accepts.insert(id);
                    bcast(Msg{ACCEPT, msg.ballot, {}, p, 0, 0});
                }
                return true;
            case ACCEPT:
                if (!(st.ballot <= msg.ballot)) return false;
                st.ballot = msg.ballot;
                st.accepted = std::make_pair(msg.ballot, msg.proposal);
                o.push_back(Envelope{id, src, Msg{ACCEPTED, msg.ballot, {}, {}, 0, 0}});
                return true;
            case ACCEPTED:
                if (!(msg.ballot == st.ballot)) return false;
                st.accepts.insert(src);
                if (st.accepts.size() == majority(server_count)) {
                    st.is_decided = true;
                    Proposal p = *st.proposal;
                    bcast(Msg{DECIDED, msg.ballot, {}, p, 0, 0});
                    o.push_back(Envelope{id, p.requester, Msg{PUTOK, {}, {}, {}, p.req, 0}});
                }
                return true;
            case DECIDED:
                st.ballot = msg.ballot;
                st.accepted = std::make_pair(msg.ballot, msg.proposal);
                st.is_decided = true;
                return true;
            default:
                return false;
        }
    }

    // RegisterActor::Client::on_msg (src/actor/register.rs:170-200), put_count = 1.
    bool client_on_msg(Id id, ClientState& st, const Msg& msg, std::vector<Envelope>& o) const {
        if (!st.awaiting) return false;
        if (msg.kind == PUTOK && msg.req == *st.awaiting) {
            u64 req = (st.op_count + 1) * id;
            if (st.op_count < 1) {
                o.push_back(Envelope{id, (id + st.op_count) % server_count,
                                     Msg{PUT, {}, {}, {}, req, (char)('Z' - (id - server_count))}});
            } else {
                o.push_back(Envelope{id, (id + st.op_count) % server_count, Msg{GET, {}, {}, {}, req, 0}});
            }
            st = ClientState{req, st.op_count + 1};
            return true;
        }
        if (msg.kind == GETOK && msg.req == *st.awaiting) {
            st = ClientState{std::nullopt, st.op_count + 1};
            return true;
        }
        return false;
    }

    std::optional<State> next_state(const State& last, const Action& a) const {  // model.rs:259-327
        const Envelope& e = a.env;
        ActorState as = last.actors[e.dst];
        std::vector<Envelope> out;
        bool owned = as.is_server ? server_on_msg(e.dst, as.server, e.src, e.msg, out)
                                  : client_on_msg(e.dst, as.client, e.msg, out);
        if (!owned && out.empty()) return std::nullopt;  // is_no_op
        State s = last;
        record_in(s.history, e);
        s.network.erase(e);  // DuplicatingNetwork::No
        if (owned) s.actors[e.dst] = as;
        send_all(s, out);
        return s;
    }

    bool within_boundary(const State&) const { return true; }

    std::vector<Property<PaxosModel>> properties() const {  // examples/paxos.rs:251-261
        using P = Property<PaxosModel>;
        return {
            P::always("linearizable", [](const PaxosModel&, const State& s) { return s.history.linearizable(); }),
            P::sometimes("value chosen", [](const PaxosModel&, const State& s) {
                for (auto& e : s.network)
                    if (e.msg.kind == GETOK && e.msg.value != 0) return true;
                return false;
            }),
        };
    }

    // ---- hashing / canonical forms ----
    static void hash_acc(const Acc& a, Hasher& h) {
        h.write_bool(a.has_value());
        if (a) {
            h.write_u64(a->first.round);
            h.write_u64(a->first.id);
            h.write_u64(a->second.req);
            h.write_u64(a->second.requester);
            h.write_u64((u8)a->second.value);
        }
    }
    static void hash_msg(const Msg& m, Hasher& h) {
        h.write_u64(m.kind);
        h.write_u64(m.ballot.round);
        h.write_u64(m.ballot.id);
        hash_acc(m.last_accepted, h);
        h.write_u64(m.proposal.req);
        h.write_u64(m.proposal.requester);
        h.write_u64((u8)m.proposal.value);
        h.write_u64(m.req);
        h.write_u64((u8)m.value);
    }
    void hash_state(const State& s, Hasher& h) const {
        for (auto& a : s.actors) {
            h.write_bool(a.is_server);
            if (a.is_server) {
                auto& p = a.server;
                h.write_u64(p.ballot.round);
                h.write_u64(p.ballot.id);
                h.write_bool(p.proposal.has_value());
                if (p.proposal) {
                    h.write_u64(p.proposal->req);
                    h.write_u64(p.proposal->requester);
                    h.write_u64((u8)p.proposal->value);
                }
                h.write_usize(p.prepares.size());
                for (auto& [k, v] : p.prepares) {
                    h.write_u64(k);
                    hash_acc(v, h);
                }
                h.write_usize(p.accepts.size());
                for (auto k : p.accepts) h.write_u64(k);
                hash_acc(p.accepted, h);
                h.write_bool(p.is_decided);
            } else {
                h.write_bool(a.client.awaiting.has_value());
                h.write_u64(a.client.awaiting.value_or(0));
                h.write_u64(a.client.op_count);
            }
        }
        auto& H = s.history;
        h.write_bool(H.valid);
        for (auto& [t, cs] : H.by_thread) {
            h.write_u64(t);
            h.write_usize(cs.size());
            for (auto& c : cs) {
                h.write_usize(c.last.size());
                for (auto& [k, v] : c.last) { h.write_u64(k); h.write_u64(v); }
                h.write_bool(c.op.write);
                h.write_u64((u8)c.op.value);
                h.write_bool(c.ret.write_ok);
                h.write_u64((u8)c.ret.value);
            }
        }
        h.write_u64(0xFFFF);
        for (auto& [t, f] : H.in_flight) {
            h.write_u64(t);
            h.write_usize(f.last.size());
            for (auto& [k, v] : f.last) { h.write_u64(k); h.write_u64(v); }
            h.write_bool(f.op.write);
            h.write_u64((u8)f.op.value);
        }
        h.write_usize(s.network.size());
        for (auto& e : s.network) {
            h.write_u64(e.src);
            h.write_u64(e.dst);
            hash_msg(e.msg, h);
        }
    }

    // Canonical envelope code, shared with the GPU encoding (action id of Deliver).
    static i64 acc_code(const Acc& a) {  // 0 = None, else 1 + round*4*4 + id*4 + client index
        if (!a) return 0;
        return 1 + (i64)a->first.round * 64 + (i64)a->first.id * 8 + (i64)(a->second.requester);
    }
    i64 envelope_code(const Envelope& e) const {
        const Msg& m = e.msg;
        i64 f = 0;
        switch (m.kind) {
            case PREPARE: case ACCEPTED: f = (i64)m.ballot.round * 8 + (i64)m.ballot.id; break;
            case PREPARED: f = ((i64)m.ballot.round * 8 + (i64)m.ballot.id) * 4096 + acc_code(m.last_accepted); break;
            case ACCEPT: case DECIDED: f = ((i64)m.ballot.round * 8 + (i64)m.ballot.id) * 16 + (i64)m.proposal.requester; break;
            case PUT: case GET: case PUTOK: f = (i64)m.req; break;
            case GETOK: f = (i64)m.req * 256 + (u8)m.value; break;
        }
        return (((f * 16) + m.kind) * 16 + (i64)e.dst) * 16 + (i64)e.src;
    }
    i64 action_id(const Action& a) const { return envelope_code(a.env); }
    std::string format_action(const Action& a) const {
        static const char* names[] = {"Prepare", "Prepared", "Accept", "Accepted", "Decided", "Put", "Get", "PutOk", "GetOk"};
        return "Deliver { src: Id(" + std::to_string(a.env.src) + "), dst: Id(" + std::to_string(a.env.dst) +
               "), msg: " + names[a.env.msg.kind] + " }";
    }

    // Canonical description (shared with the GPU encoding): per server [round, ballot id,
    // proposal client (-1 none), prepares per server (-1 absent, else acc code), accepts mask,
    // accepted acc code, decided], per client [op_count], then the network as 16 sorted
    // envelope codes padded with -1, then the register history (describe_register_history).
    std::vector<i64> describe(const State& s) const {
        std::vector<i64> d;
        for (Id i = 0; i < server_count; ++i) {
            auto& p = s.actors[i].server;
            d.push_back(p.ballot.round);
            d.push_back((i64)p.ballot.id);
            d.push_back(p.proposal ? (i64)p.proposal->requester : -1);
            for (Id j = 0; j < server_count; ++j) {
                auto it = p.prepares.find(j);
                d.push_back(it == p.prepares.end() ? -1 : acc_code(it->second));
            }
            i64 mask = 0;
            for (auto k : p.accepts) mask |= 1ll << k;
            d.push_back(mask);
            d.push_back(acc_code(p.accepted));
            d.push_back(p.is_decided);
        }
        for (Id c = 0; c < client_count; ++c) d.push_back((i64)s.actors[server_count + c].client.op_count);
        std::vector<i64> net;
        for (auto& e : s.network) net.push_back(envelope_code(e));
        std::sort(net.begin(), net.end());
        net.resize(16, -1);
        d.insert(d.end(), net.begin(), net.end());
        describe_register_history(s.history, server_count, client_count, d);
        return d;
    }
};

}  // namespace paxos
}  // namespace oracle
