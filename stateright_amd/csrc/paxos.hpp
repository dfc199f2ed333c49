// GpuModel for the paxos example (BASELINE.json config 5).
//
// The reference composes ActorModel (src/actor/model.rs:176-327) + RegisterActor
// (src/actor/register.rs:119-217) + PaxosActor (examples/paxos.rs:93-221) + a
// LinearizabilityTester<Id, Register<char>> history (src/semantics/linearizability.rs:57-241).
// Its per-state heap objects (Arc'd actor states, a HashSet network, BTreeMap histories) become
// W = 11 words:
//
//   word 0   server 0 (42 bits) | 3 client phases (2 bits each) | history index (16 bits)
//   word 1   server 1           word 2   server 2
//   words 3+ the network: 16 envelope codes (u32, ascending, unused = 0xffffffff)
//
// A server is PaxosState (examples/paxos.rs:78-91) in bit fields:
//   [0,4) ballot (round << 2 | id)   [4,7) proposal (requester id 3..5, 0 = None)
//   [7,31) prepares[j] (present << 7 | acc)   [31,34) accepts mask   [34,41) accepted acc
//   [41] is_decided
// with acc = Option<(Ballot, Proposal)> as some << 6 | ballot << 2 | (requester - 3). Every
// field is ORDER-PRESERVING, so comparing codes compares the reference's values. Ballot rounds
// fit 2 bits: a round is raised only when a server takes a Put (examples/paxos.rs:128-140), each
// server takes at most one (its proposal is never reset) and there are C <= 3 Puts.
//
// An envelope code is src | dst | kind | ballot | last_accepted | proposal | request | value
// (MSB first, 30 bits) — the lexicographic order of the reference's Envelope fields — so the
// sorted code list is the network SET (src/actor/model.rs:69, non-duplicating) and action slot k
// (deliver the k-th envelope) enumerates `actions()` in the same order as the CPU oracle's
// ordered set.
//
// Histories change only on client deliveries (record_returns / record_invocations,
// src/actor/register.rs:37-87); the reachable ones are interned on the host by a closure over
// per-client events, and `linearizable` is precomputed per history with the reference's
// backtracking search (linearizability.rs:159-240).
#pragma once
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/stateright_gpu.h"
#include "device.hpp"
#include "models.hpp"

namespace sr {
namespace px {

enum Kind : u32 { PREPARE, PREPARED, ACCEPT, ACCEPTED, DECIDED, PUT, GET, PUTOK, GETOK };
constexpr int SLOTS = 16;          // network capacity (the reachable maximum is 13 at C = 3)
constexpr u32 EMPTY = 0xffffffffu;
constexpr int SBITS = 42;          // bits per server
constexpr int NEV_PER_CLIENT = 5;  // PutOk, GetOk('\0'), GetOk('A'..'C')

SR_HD u32 env(u32 src, u32 dst, u32 kind, u32 bal, u32 acc, u32 pcl, u32 req, u32 val) {
    return src << 27 | dst << 24 | kind << 20 | bal << 16 | acc << 9 | pcl << 6 | req << 2 | val;
}
SR_HD u32 e_src(u32 e) { return e >> 27 & 7; }
SR_HD u32 e_dst(u32 e) { return e >> 24 & 7; }
SR_HD u32 e_kind(u32 e) { return e >> 20 & 15; }
SR_HD u32 e_bal(u32 e) { return e >> 16 & 15; }
SR_HD u32 e_acc(u32 e) { return e >> 9 & 127; }
SR_HD u32 e_pcl(u32 e) { return e >> 6 & 7; }
SR_HD u32 e_req(u32 e) { return e >> 2 & 15; }
SR_HD u32 e_val(u32 e) { return e & 3; }

struct Srv {
    u32 bal, prop, prep[3], accepts, accepted, decided;
    SR_HD static Srv load(u64 w) {
        Srv s;
        s.bal = (u32)(w & 15);
        s.prop = (u32)(w >> 4 & 7);
#pragma unroll
        for (int j = 0; j < 3; ++j) s.prep[j] = (u32)(w >> (7 + 8 * j) & 255);
        s.accepts = (u32)(w >> 31 & 7);
        s.accepted = (u32)(w >> 34 & 127);
        s.decided = (u32)(w >> 41 & 1);
        return s;
    }
    SR_HD u64 store() const {
        u64 w = bal | (u64)prop << 4 | (u64)accepts << 31 | (u64)accepted << 34 | (u64)decided << 41;
#pragma unroll
        for (int j = 0; j < 3; ++j) w |= (u64)prep[j] << (7 + 8 * j);
        return w;
    }
};

// PaxosActor::on_msg (examples/paxos.rs:116-221). Returns "state touched" (Cow::Owned); the
// messages it sends go to out[0..n).
SR_HD bool server_on_msg(u32 id, Srv& s, u32 e, u32* out, int& n) {
    const u32 src = e_src(e), kind = e_kind(e), bal = e_bal(e);
    const u32 p0 = id == 0 ? 1 : 0, p1 = id == 2 ? 1 : 2;  // peers, ascending
    if (s.decided) {
        if (kind == GET) out[n++] = env(id, src, GETOK, 0, 0, 0, e_req(e), (s.accepted & 3) + 1);
        return false;
    }
    switch (kind) {
        case PUT:
            if (s.prop) return false;
            s.prop = src;
            s.accepts = 0;
            s.bal = ((s.bal >> 2) + 1) << 2 | id;
#pragma unroll
            for (int j = 0; j < 3; ++j) s.prep[j] = (u32)j == id ? (128u | s.accepted) : 0u;
            out[n++] = env(id, p0, PREPARE, s.bal, 0, 0, 0, 0);
            out[n++] = env(id, p1, PREPARE, s.bal, 0, 0, 0, 0);
            return true;
        case PREPARE:
            if (!(s.bal < bal)) return false;
            s.bal = bal;
            out[n++] = env(id, src, PREPARED, bal, s.accepted, 0, 0, 0);
            return true;
        case PREPARED: {
            if (bal != s.bal) return false;
            u32 cnt = 0, best = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                if ((u32)j == src) s.prep[j] = 128u | e_acc(e);
                cnt += s.prep[j] >> 7;
                if ((s.prep[j] >> 7) && (s.prep[j] & 127) > best) best = s.prep[j] & 127;
            }
            if (cnt == 2) {  // majority(3) (src/actor.rs:437-439)
                const u32 p = best ? (best & 3) + 3 : s.prop;
                s.prop = p;
                s.accepted = 64u | bal << 2 | (p - 3);
                s.accepts |= 1u << id;
                out[n++] = env(id, p0, ACCEPT, bal, 0, p, 0, 0);
                out[n++] = env(id, p1, ACCEPT, bal, 0, p, 0, 0);
            }
            return true;
        }
        case ACCEPT:
            if (bal < s.bal) return false;
            s.bal = bal;
            s.accepted = 64u | bal << 2 | (e_pcl(e) - 3);
            out[n++] = env(id, src, ACCEPTED, bal, 0, 0, 0, 0);
            return true;
        case ACCEPTED:
            if (bal != s.bal) return false;
            s.accepts |= 1u << src;
            if (__builtin_popcount(s.accepts) == 2) {
                s.decided = 1;
                out[n++] = env(id, p0, DECIDED, bal, 0, s.prop, 0, 0);
                out[n++] = env(id, p1, DECIDED, bal, 0, s.prop, 0, 0);
                out[n++] = env(id, s.prop, PUTOK, 0, 0, 0, s.prop, 0);  // request id = requester (put_count 1)
            }
            return true;
        case DECIDED:
            s.bal = bal;
            s.accepted = 64u | bal << 2 | (e_pcl(e) - 3);
            s.decided = 1;
            return true;
        default:
            return false;
    }
}

// Canonical forms shared with the CPU oracle (oracle/paxos.hpp acc_code / envelope_code).
inline i64 acc_code(u32 acc) {
    if (!(acc & 64)) return 0;
    return 1 + (i64)(acc >> 4 & 3) * 64 + (i64)(acc >> 2 & 3) * 8 + (i64)(acc & 3) + 3;
}
inline i64 env_code(u32 e) {
    const u32 kind = e_kind(e);
    const i64 bal = (i64)(e_bal(e) >> 2) * 8 + (e_bal(e) & 3);
    i64 f = 0;
    switch (kind) {
        case PREPARE: case ACCEPTED: f = bal; break;
        case PREPARED: f = bal * 4096 + acc_code(e_acc(e)); break;
        case ACCEPT: case DECIDED: f = bal * 16 + e_pcl(e); break;
        case PUT: case GET: case PUTOK: f = e_req(e); break;
        case GETOK: f = (i64)e_req(e) * 256 + (e_val(e) ? 'A' + e_val(e) - 1 : 0); break;
    }
    return (((f * 16) + kind) * 16 + e_dst(e)) * 16 + e_src(e);
}

// LinearizabilityTester<Id, Register<char>> over the C client threads (host only).
struct Hist {
    struct Op { bool write = false; int value = 0; };
    struct Complete { std::vector<int> last; Op op; bool ret_write = false; int ret_value = 0; };
    struct InFlight { bool some = false; std::vector<int> last; Op op; };
    std::vector<bool> entry;  // thread has a `history_by_thread` entry
    std::vector<std::vector<Complete>> done;
    std::vector<InFlight> inflight;
    bool valid = true;
    explicit Hist(int C = 0) : entry(C), done(C), inflight(C) {}
    std::vector<long> key() const {
        std::vector<long> k{valid};
        for (size_t t = 0; t < done.size(); ++t) {
            k.push_back(entry[t]);
            k.push_back((long)done[t].size());
            for (auto& c : done[t]) {
                for (int x : c.last) k.push_back(x);
                k.push_back(c.op.write); k.push_back(c.op.value); k.push_back(c.ret_write); k.push_back(c.ret_value);
            }
            k.push_back(inflight[t].some);
            if (inflight[t].some) {
                for (int x : inflight[t].last) k.push_back(x);
                k.push_back(inflight[t].op.write); k.push_back(inflight[t].op.value);
            }
        }
        return k;
    }
    void invoke(int t, Op op) {  // linearizability.rs:102-125
        if (!valid) return;
        if (inflight[t].some) { valid = false; return; }
        std::vector<int> last(done.size(), -1);
        for (size_t u = 0; u < done.size(); ++u)
            if ((int)u != t && !done[u].empty()) last[u] = (int)done[u].size() - 1;
        inflight[t] = InFlight{true, last, op};
        entry[t] = true;
    }
    void ret(int t, bool write_ok, int value) {  // linearizability.rs:131-147
        if (!valid) return;
        entry[t] = true;
        if (!inflight[t].some) { valid = false; return; }
        InFlight f = inflight[t];
        inflight[t] = InFlight{};
        done[t].push_back(Complete{f.last, f.op, write_ok, value});
    }
    bool linearizable() const {  // serialized_history().is_some()
        if (!valid) return false;
        std::vector<size_t> next(done.size(), 0);
        std::vector<bool> used(done.size(), false);
        return serialize(0, next, used);
    }
    bool violates(const std::vector<int>& last, const std::vector<size_t>& next) const {
        for (size_t p = 0; p < last.size(); ++p)
            if (last[p] >= 0 && next[p] < done[p].size() && (int)next[p] <= last[p]) return true;
        return false;
    }
    // Depth-first over the next op of each thread: a completed op must respect real-time order
    // and Register::is_valid_step (src/semantics/register.rs:34-47); an in-flight op may be
    // linearized once its thread's completed ops are placed (a Write takes effect, a Read
    // returns anything).
    bool serialize(int reg, std::vector<size_t>& next, std::vector<bool>& used) const {
        bool all = true;
        for (size_t t = 0; t < done.size(); ++t)
            if (next[t] < done[t].size()) all = false;
        if (all) return true;
        for (size_t t = 0; t < done.size(); ++t) {
            if (!entry[t]) continue;
            if (next[t] == done[t].size()) {
                if (!inflight[t].some || used[t] || violates(inflight[t].last, next)) continue;
                used[t] = true;
                bool ok = serialize(inflight[t].op.write ? inflight[t].op.value : reg, next, used);
                used[t] = false;
                if (ok) return true;
            } else {
                const Complete& c = done[t][next[t]];
                next[t]++;
                bool ok = false;
                if (!violates(c.last, next)) {
                    if (c.op.write && c.ret_write) ok = serialize(c.op.value, next, used);
                    else if (!c.op.write && !c.ret_write && c.ret_value == reg) ok = serialize(reg, next, used);
                }
                next[t]--;
                if (ok) return true;
            }
        }
        return false;
    }
};

// Host-compiled history tables, one copy per (process, C) plus one device copy per GPU.
struct Tables {
    int C = 0, nh = 0, nev = 0;
    u32 init_hist = 0;
    std::vector<u16> h_next;  // [h * nev + event], 0xffff = never occurs
    std::vector<u8> h_lin;    // linearizable per history
    std::map<int, std::pair<u16*, u8*>> dev;  // device copies (process lifetime)
};

inline Tables compile(int C) {
    if (C < 1 || C > 3) throw Error(SR_ERR_UNSUPPORTED, "paxos: client_count must be in 1..=3");
    Tables T;
    T.C = C;
    T.nev = C * NEV_PER_CLIENT;
    std::map<std::vector<long>, int> idx;
    std::vector<Hist> H;
    auto add = [&](const Hist& h) {
        auto k = h.key();
        auto it = idx.find(k);
        if (it != idx.end()) return it->second;
        idx[k] = (int)H.size();
        H.push_back(h);
        return (int)H.size() - 1;
    };
    Hist h0(C);  // init: every client invokes its Put (src/actor/model.rs:215-242 via record_out)
    for (int c = 0; c < C; ++c) h0.invoke(c, Hist::Op{true, 'A' + c});
    T.init_hist = (u32)add(h0);
    std::vector<std::vector<int>> rows;
    for (size_t k = 0; k < H.size(); ++k) {
        std::vector<int> row(T.nev, -1);
        for (int ev = 0; ev < T.nev; ++ev) {
            const int c = ev / NEV_PER_CLIENT, kind = ev % NEV_PER_CLIENT;
            // a client's completed-op count is its phase: PutOk is delivered in phase 0 only,
            // GetOk in phase 1 only (RegisterActor client, src/actor/register.rs:170-200)
            if ((int)H[k].done[c].size() != (kind == 0 ? 0 : 1)) continue;
            Hist h = H[k];
            if (kind == 0) {
                h.ret(c, true, 0);                // PutOk: return WriteOk ...
                h.invoke(c, Hist::Op{false, 0});  // ... then the client's Get is recorded
            } else {
                h.ret(c, false, kind == 1 ? 0 : 'A' + kind - 2);
            }
            row[ev] = add(h);
        }
        rows.push_back(row);
        if (H.size() > 65000) throw Error(SR_ERR_UNSUPPORTED, "paxos: history closure too large");
    }
    T.nh = (int)H.size();
    T.h_next.assign((size_t)T.nh * T.nev, 0xffff);
    T.h_lin.assign(T.nh, 0);
    for (int k = 0; k < T.nh; ++k) {
        for (int ev = 0; ev < T.nev; ++ev)
            if (rows[k][ev] >= 0) T.h_next[(size_t)k * T.nev + ev] = (u16)rows[k][ev];
        T.h_lin[k] = H[k].linearizable() ? 1 : 0;
    }
    return T;
}

// Process-lifetime table cache (tables are a few KB; device copies are made once per GPU).
inline Tables& tables(int C, int device) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<Tables>> cache;
    std::lock_guard<std::mutex> g(mu);
    auto& t = cache[C];
    if (!t) t = std::make_unique<Tables>(compile(C));
    if (device >= 0 && !t->dev.count(device)) {
        int prev = 0;
        SR_HIP(hipGetDevice(&prev));
        SR_HIP(hipSetDevice(device));
        u16* hn = nullptr;
        u8* hl = nullptr;
        SR_HIP(hipMalloc(&hn, t->h_next.size() * sizeof(u16)));
        SR_HIP(hipMalloc(&hl, t->h_lin.size()));
        SR_HIP(hipMemcpy(hn, t->h_next.data(), t->h_next.size() * sizeof(u16), hipMemcpyHostToDevice));
        SR_HIP(hipMemcpy(hl, t->h_lin.data(), t->h_lin.size(), hipMemcpyHostToDevice));
        SR_HIP(hipSetDevice(prev));
        t->dev[device] = {hn, hl};
    }
    return *t;
}

}  // namespace px

struct Paxos {
    static constexpr int W = 3 + px::SLOTS / 2, MW = 1, NPROPS = 2;
    int C = 2;
    int nev = 0;
    u32 init_hist = 0;
    const u16* h_next_d = nullptr;  // device tables
    const u8* h_lin_d = nullptr;
    const u16* h_next_h = nullptr;  // host tables (paths, replay)
    const u8* h_lin_h = nullptr;

    // device < 0: host-only (no device copy of the tables)
    static Paxos make(int C, int device) {
        px::Tables& t = px::tables(C, device);
        Paxos m;
        m.C = C;
        m.nev = t.nev;
        m.init_hist = t.init_hist;
        if (device >= 0) {
            m.h_next_d = t.dev.at(device).first;
            m.h_lin_d = t.dev.at(device).second;
        }
        m.h_next_h = t.h_next.data();
        m.h_lin_h = t.h_lin.data();
        return m;
    }
    SR_HD const u16* h_next() const {
#if defined(__HIP_DEVICE_COMPILE__)
        return h_next_d;
#else
        return h_next_h;
#endif
    }
    SR_HD const u8* h_lin() const {
#if defined(__HIP_DEVICE_COMPILE__)
        return h_lin_d;
#else
        return h_lin_h;
#endif
    }

    int max_actions() const { return px::SLOTS; }
    int max_out_degree() const { return px::SLOTS; }
    SR_HD static u32 slot(const u64* s, int k) { return (u32)(s[3 + k / 2] >> (32 * (k & 1))); }
    SR_HD static u32 hist(const u64* s) { return (u32)(s[0] >> 48); }
    SR_HD static u32 phase(const u64* s, int c) { return (u32)(s[0] >> (px::SBITS + 2 * c) & 3); }

    // Every envelope is deliverable (model.rs:238-257), but most deliveries are no-ops
    // (`next_state` = None, src/actor/model.rs:299-301: the actor ignores the message). The mask
    // keeps the slots whose delivery changes the state: the exact complement of apply's `false`
    // returns below, so the successors and their slot order are unchanged, and the load-balanced
    // expansion spends its lanes on real successors only.
    SR_HD bool delivers(const u64* s, u32 e) const {
        const u32 dst = px::e_dst(e), kind = px::e_kind(e), bal = px::e_bal(e);
        if (dst >= 3) {
            const u32 ph = phase(s, (int)(dst - 3)), req = px::e_req(e);
            return (ph == 0 && kind == px::PUTOK && req == dst) || (ph == 1 && kind == px::GETOK && req == 2 * dst);
        }
        const u64 sw = s[dst] & (dst == 0 ? ((1ull << px::SBITS) - 1) : ~0ull);
        const u32 sbal = (u32)(sw & 15), sprop = (u32)(sw >> 4 & 7), decided = (u32)(sw >> 41 & 1);
        if (decided) return kind == px::GET;  // answered with GetOk, the state untouched
        switch (kind) {
            case px::PUT: return sprop == 0;
            case px::PREPARE: return sbal < bal;
            case px::PREPARED: return bal == sbal;
            case px::ACCEPT: return !(bal < sbal);
            case px::ACCEPTED: return bal == sbal;
            case px::DECIDED: return true;
            default: return false;
        }
    }
    SR_HD void enabled(const u64* s, u64* m) const {
        u64 mk = 0;
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) {
            const u32 e = slot(s, k);
            if (e != px::EMPTY && delivers(s, e)) mk |= 1ull << k;
        }
        m[0] = mk;
    }

    // Deliver the a-th envelope (src/actor/model.rs:259-327); false = no-op (None).
    SR_HD bool apply(const u64* s, int a, u64* o) const {
        u32 net[px::SLOTS], e = 0;
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) {
            net[k] = slot(s, k);
            if (k == a) e = net[k];
        }
        const u32 dst = px::e_dst(e);
        u32 out[3] = {0, 0, 0};
        int nout = 0;
        u64 w0 = s[0], w1 = s[1], w2 = s[2];
        if (dst < 3) {
            const u64 sw = dst == 0 ? (w0 & ((1ull << px::SBITS) - 1)) : dst == 1 ? w1 : w2;
            px::Srv sv = px::Srv::load(sw);
            const bool owned = px::server_on_msg(dst, sv, e, out, nout);
            if (!owned && nout == 0) return false;  // is_no_op (src/actor.rs:232-234)
            const u64 nw = sv.store();
            if (dst == 0) w0 = (w0 & ~((1ull << px::SBITS) - 1)) | nw;
            else if (dst == 1) w1 = nw;
            else w2 = nw;
        } else {  // RegisterActor::Client::on_msg (src/actor/register.rs:170-200), put_count = 1
            const u32 c = dst - 3, ph = phase(s, (int)c), kind = px::e_kind(e), req = px::e_req(e);
            u32 ev;
            if (ph == 0 && kind == px::PUTOK && req == dst) {
                out[nout++] = px::env(dst, (dst + 1) % 3, px::GET, 0, 0, 0, 2 * dst, 0);
                ev = c * px::NEV_PER_CLIENT;
            } else if (ph == 1 && kind == px::GETOK && req == 2 * dst) {
                ev = c * px::NEV_PER_CLIENT + 1 + px::e_val(e);
            } else {
                return false;
            }
            const int off = px::SBITS + 2 * (int)c;
            w0 = (w0 & ~(3ull << off)) | ((u64)(ph + 1) << off);
            const u64 h = h_next()[(size_t)hist(s) * nev + ev];  // record_returns, record_invocations
            w0 = (w0 & ((1ull << 48) - 1)) | h << 48;
        }
        // remove the delivered envelope (DuplicatingNetwork::No), then insert what was sent
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) net[k] = k < a ? net[k] : (k + 1 < px::SLOTS ? net[k + 1] : px::EMPTY);
        for (int j = 0; j < nout; ++j) {
            const u32 x = out[j];
            bool dup = false;
#pragma unroll
            for (int k = 0; k < px::SLOTS; ++k) dup |= net[k] == x;
            if (dup) continue;
            u32 prev = 0;  // sorted insert: new[k] = old[k] < x ? old[k] : (old[k-1] < x ? x : old[k-1])
#pragma unroll
            for (int k = 0; k < px::SLOTS; ++k) {
                const u32 cur = net[k];
                net[k] = cur < x ? cur : ((k == 0 || prev < x) ? x : prev);
                prev = cur;
            }
        }
        o[0] = w0;
        o[1] = w1;
        o[2] = w2;
#pragma unroll
        for (int k = 0; k < px::SLOTS / 2; ++k) o[3 + k] = (u64)net[2 * k] | (u64)net[2 * k + 1] << 32;
        return true;
    }

    SR_HD bool discovers(int p, const u64* s) const {
        if (p == 0) return !h_lin()[hist(s)];  // always "linearizable" (examples/paxos.rs:251-254)
        bool any = false;                      // sometimes "value chosen" (examples/paxos.rs:255-261)
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) {
            const u32 e = slot(s, k);
            any |= e != px::EMPTY && px::e_kind(e) == px::GETOK && px::e_val(e) != 0;
        }
        return any;
    }

    int init_states(u64* out) const {  // src/actor/model.rs:215-242
        u32 net[px::SLOTS];
        for (int k = 0; k < px::SLOTS; ++k) net[k] = px::EMPTY;
        for (int c = 0; c < C; ++c) {
            const u32 id = 3 + (u32)c;
            net[c] = px::env(id, id % 3, px::PUT, 0, 0, 0, id, (u32)c + 1);
        }
        std::sort(net, net + C);
        out[0] = (u64)init_hist << 48;
        out[1] = out[2] = 0;
        for (int k = 0; k < px::SLOTS / 2; ++k) out[3 + k] = (u64)net[2 * k] | (u64)net[2 * k + 1] << 32;
        return 1;
    }
    int expectation(int p) const { return p == 0 ? ALWAYS : SOMETIMES; }
    const char* prop_name(int p) const { return p == 0 ? "linearizable" : "value chosen"; }
    // The oracle's canonical description (oracle/paxos.hpp describe).
    int describe_width() const { return 3 * 9 + C + 16; }
    void describe(const u64* s, i64* d) const {
        int k = 0;
        for (int i = 0; i < 3; ++i) {
            const px::Srv v = px::Srv::load(i == 0 ? s[0] & ((1ull << px::SBITS) - 1) : s[i]);
            d[k++] = v.bal >> 2;
            d[k++] = v.bal & 3;
            d[k++] = v.prop ? (i64)v.prop : -1;
            for (int j = 0; j < 3; ++j) d[k++] = (v.prep[j] >> 7) ? px::acc_code(v.prep[j] & 127) : -1;
            d[k++] = v.accepts;
            d[k++] = px::acc_code(v.accepted);
            d[k++] = v.decided;
        }
        for (int c = 0; c < C; ++c) d[k++] = (i64)phase(s, c) + 1;  // op_count
        std::vector<i64> net;
        for (int j = 0; j < px::SLOTS; ++j)
            if (slot(s, j) != px::EMPTY) net.push_back(px::env_code(slot(s, j)));
        std::sort(net.begin(), net.end());
        net.resize(16, -1);
        for (i64 v : net) d[k++] = v;
    }
    i64 action_id(const u64* s, int a) const { return px::env_code(slot(s, a)); }
    i64 action_id_bound() const { return 0; }  // ids are sparse envelope codes
    std::string action_name(i64 code) const {
        static const char* names[] = {"Prepare", "Prepared", "Accept", "Accepted", "Decided", "Put", "Get", "PutOk", "GetOk"};
        const long src = code % 16, dst = (code / 16) % 16, kind = (code / 256) % 16;
        return "Deliver { src: Id(" + std::to_string(src) + "), dst: Id(" + std::to_string(dst) + "), msg: " +
               (kind < 9 ? names[kind] : "?") + " }";
    }
};

}  // namespace sr
