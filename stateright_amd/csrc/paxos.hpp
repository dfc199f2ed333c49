// GpuModel for the paxos example (BASELINE.json config 5).
//
// The reference composes ActorModel (src/actor/model.rs:176-327) + RegisterActor
// (src/actor/register.rs:119-217) + PaxosActor (examples/paxos.rs:93-221) + a
// LinearizabilityTester<Id, Register<char>> history (src/semantics/linearizability.rs:57-241).
// Its per-state heap objects (Arc'd actor states, a HashSet network, BTreeMap histories) become
// W = 11 words, for any client count C <= 6 (the reference's bench.sh runs `paxos check 6`):
//
//   word 0   server 0 (47 bits) | history index (16 bits, from bit 48)
//   word 1   server 1 (47 bits) | C client phases (2 bits each, from bit 48)
//   word 2   server 2
//   words 3+ the network: 16 envelope codes (u32, ascending, unused = 0xffffffff); at most 13,
//            14 and 16 envelopes are ever in flight at C = 3, 4 and 6
//
// A server is PaxosState (examples/paxos.rs:78-91) in bit fields:
//   [0,4) ballot (round << 2 | id)   [4,8) proposal (requester id 3..8, 0 = None)
//   [8,35) prepares[j] (present << 8 | acc)   [35,38) accepts mask   [38,46) accepted acc
//   [46] is_decided
// with acc = Option<(Ballot, Proposal)> as some << 7 | ballot << 3 | (requester - 3). Every
// field is ORDER-PRESERVING, so comparing codes compares the reference's values. Ballot rounds
// fit 2 bits: a round is raised only when a server takes a Put (examples/paxos.rs:128-140), and
// each of the 3 servers takes at most one (its proposal is never reset).
//
// An envelope code is src | dst | kind | ballot | payload (MSB first, 24 bits) — the
// lexicographic order of the reference's Envelope fields: the payload is the one message field
// that varies for a given (src, dst, kind, ballot): last_accepted (Prepared), the proposal's
// requester (Accept, Decided: its request id and value are the requester's) or the value
// (GetOk); a request id is always the client's own (Put/PutOk: its id, Get/GetOk: twice its id,
// src/actor/register.rs:130-200), and a Put's value is the client's letter. So the sorted code
// list is the network SET (src/actor/model.rs:69, non-duplicating) and action slot k (deliver the
// k-th envelope) enumerates `actions()` in the same order as the CPU oracle's ordered set.
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
constexpr int SLOTS = 16;          // network capacity (the reachable maximum is 16 at C = 6)
constexpr int MAX_CLIENTS = 6;
constexpr u32 EMPTY = 0xffffffffu;
constexpr int SBITS = 47;          // bits per server
constexpr u64 SMASK = (1ull << SBITS) - 1;
constexpr int HIST_SHIFT = 48;     // word 0: history index
constexpr int PHASE_SHIFT = 48;    // word 1: client phases
// History events per client: PutOk, GetOk('\0'), GetOk('A' + v - 1) for v = 1..MAX_CLIENTS.
constexpr int NEV_PER_CLIENT = 2 + MAX_CLIENTS;

// payload: acc (Prepared), requester id (Accept, Decided), value (GetOk), else 0
SR_HD u32 env(u32 src, u32 dst, u32 kind, u32 bal, u32 payload) {
    return src << 20 | dst << 16 | kind << 12 | bal << 8 | payload;
}
SR_HD u32 e_src(u32 e) { return e >> 20 & 15; }
SR_HD u32 e_dst(u32 e) { return e >> 16 & 15; }
SR_HD u32 e_kind(u32 e) { return e >> 12 & 15; }
SR_HD u32 e_bal(u32 e) { return e >> 8 & 15; }
SR_HD u32 e_acc(u32 e) { return e & 255; }
SR_HD u32 e_pcl(u32 e) { return e & 15; }
SR_HD u32 e_val(u32 e) { return e & 7; }
// request ids are the client's: Put/PutOk carry its id, Get/GetOk twice its id
SR_HD u32 e_req(u32 e) {
    const u32 k = e_kind(e), client = k == PUT || k == GET ? e_src(e) : e_dst(e);  // Put, Get: from the client
    return k == GET || k == GETOK ? 2 * client : client;
}

struct Srv {
    u32 bal, prop, prep[3], accepts, accepted, decided;
    SR_HD static Srv load(u64 w) {
        Srv s;
        s.bal = (u32)(w & 15);
        s.prop = (u32)(w >> 4 & 15);
#pragma unroll
        for (int j = 0; j < 3; ++j) s.prep[j] = (u32)(w >> (8 + 9 * j) & 511);
        s.accepts = (u32)(w >> 35 & 7);
        s.accepted = (u32)(w >> 38 & 255);
        s.decided = (u32)(w >> 46 & 1);
        return s;
    }
    SR_HD u64 store() const {
        u64 w = bal | (u64)prop << 4 | (u64)accepts << 35 | (u64)accepted << 38 | (u64)decided << 46;
#pragma unroll
        for (int j = 0; j < 3; ++j) w |= (u64)prep[j] << (8 + 9 * j);
        return w;
    }
};

// PaxosActor::on_msg (examples/paxos.rs:116-221). Returns "state touched" (Cow::Owned); the
// messages it sends go to out[0..n).
SR_HD bool server_on_msg(u32 id, Srv& s, u32 e, u32* out, int& n) {
    const u32 src = e_src(e), kind = e_kind(e), bal = e_bal(e);
    const u32 p0 = id == 0 ? 1 : 0, p1 = id == 2 ? 1 : 2;  // peers, ascending
    if (s.decided) {
        if (kind == GET) out[n++] = env(id, src, GETOK, 0, (s.accepted & 7) + 1);
        return false;
    }
    switch (kind) {
        case PUT:
            if (s.prop) return false;
            s.prop = src;
            s.accepts = 0;
            s.bal = ((s.bal >> 2) + 1) << 2 | id;
#pragma unroll
            for (int j = 0; j < 3; ++j) s.prep[j] = (u32)j == id ? (256u | s.accepted) : 0u;
            out[n++] = env(id, p0, PREPARE, s.bal, 0);
            out[n++] = env(id, p1, PREPARE, s.bal, 0);
            return true;
        case PREPARE:
            if (!(s.bal < bal)) return false;
            s.bal = bal;
            out[n++] = env(id, src, PREPARED, bal, s.accepted);
            return true;
        case PREPARED: {
            if (bal != s.bal) return false;
            u32 cnt = 0, best = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                if ((u32)j == src) s.prep[j] = 256u | e_acc(e);
                cnt += s.prep[j] >> 8;
                if ((s.prep[j] >> 8) && (s.prep[j] & 255) > best) best = s.prep[j] & 255;
            }
            if (cnt == 2) {  // majority(3) (src/actor.rs:437-439)
                const u32 p = best ? (best & 7) + 3 : s.prop;
                s.prop = p;
                s.accepted = 128u | bal << 3 | (p - 3);
                s.accepts |= 1u << id;
                out[n++] = env(id, p0, ACCEPT, bal, p);
                out[n++] = env(id, p1, ACCEPT, bal, p);
            }
            return true;
        }
        case ACCEPT:
            if (bal < s.bal) return false;
            s.bal = bal;
            s.accepted = 128u | bal << 3 | (e_pcl(e) - 3);
            out[n++] = env(id, src, ACCEPTED, bal, 0);
            return true;
        case ACCEPTED:
            if (bal != s.bal) return false;
            s.accepts |= 1u << src;
            if (__builtin_popcount(s.accepts) == 2) {
                s.decided = 1;
                out[n++] = env(id, p0, DECIDED, bal, s.prop);
                out[n++] = env(id, p1, DECIDED, bal, s.prop);
                out[n++] = env(id, s.prop, PUTOK, 0, 0);  // request id = requester (put_count 1)
            }
            return true;
        case DECIDED:
            s.bal = bal;
            s.accepted = 128u | bal << 3 | (e_pcl(e) - 3);
            s.decided = 1;
            return true;
        default:
            return false;
    }
}

// Canonical forms shared with the CPU oracle (oracle/paxos.hpp acc_code / envelope_code).
inline i64 acc_code(u32 acc) {
    if (!(acc & 128)) return 0;
    return 1 + (i64)(acc >> 5 & 3) * 64 + (i64)(acc >> 3 & 3) * 8 + (i64)(acc & 7) + 3;
}
// Inverses (sr_model_fingerprint: a described state back to its words).
inline u32 acc_decode(i64 code) {
    if (code <= 0) return 0;
    const i64 c = code - 1, round = c / 64, id = c / 8 % 8, req = c % 8;
    return 128u | (u32)((round << 2 | id) << 3) | (u32)(req - 3);
}
inline u32 env_decode(i64 code) {
    const u32 src = (u32)(code % 16), dst = (u32)(code / 16 % 16), kind = (u32)(code / 256 % 16);
    const i64 f = code / 4096;
    auto bal = [](i64 b) { return (u32)((b / 8) << 2 | (b % 8)); };
    switch (kind) {
        case PREPARE: case ACCEPTED: return env(src, dst, kind, bal(f), 0);
        case PREPARED: return env(src, dst, kind, bal(f / 4096), acc_decode(f % 4096));
        case ACCEPT: case DECIDED: return env(src, dst, kind, bal(f / 16), (u32)(f % 16));
        case GETOK: {
            const i64 v = f % 256;
            return env(src, dst, kind, 0, v ? (u32)(v - 'A' + 1) : 0u);
        }
        default: return env(src, dst, kind, 0, 0);
    }
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

// The canonical description of a history (oracle/paxos.hpp describe_register_history): per
// client c its Get's returned value (-1 before it returned), then per other client u the number of
// u's ops completed when c invoked its Get (-1 before the Get). C * C values.
inline void describe_hist(const Hist& h, int C, i64* d) {
    int k = 0;
    for (int c = 0; c < C; ++c) {
        const size_t nd = h.done[c].size();
        const std::vector<int>* last = nd >= 2 ? &h.done[c][1].last : nd == 1 && h.inflight[c].some ? &h.inflight[c].last : nullptr;
        const int v = nd >= 2 ? h.done[c][1].ret_value : 0;
        d[k++] = nd >= 2 ? (v ? (i64)(v - 'A' + 1) : 0) : -1;
        for (int u = 0; u < C; ++u)
            if (u != c) d[k++] = last ? (i64)(*last)[u] + 1 : -1;
    }
}

// Host-compiled history tables, one copy per (process, C) plus one device copy per GPU.
struct Tables {
    int C = 0, nh = 0, nev = 0;
    u32 init_hist = 0;
    std::vector<u16> h_next;  // [h * nev + event], 0xffff = never occurs
    std::vector<u8> h_lin;    // linearizable per history
    std::vector<Hist> hists;  // the interned histories (describe)
    std::map<int, std::pair<u16*, u8*>> dev;  // device copies (process lifetime)
    // The index of a described history (undescribe); throws if no reachable history has it.
    u32 hist_index(const i64* d) {
        static std::mutex mu;
        std::lock_guard<std::mutex> g(mu);
        if (by_desc_.empty()) {
            std::vector<i64> k((size_t)(C * C));
            for (size_t h = 0; h < hists.size(); ++h) {
                describe_hist(hists[h], C, k.data());
                by_desc_.emplace(k, (u32)h);
            }
        }
        auto it = by_desc_.find(std::vector<i64>(d, d + C * C));
        if (it == by_desc_.end()) throw Error(SR_ERR_ARG, "register history: no reachable history has this description");
        return it->second;
    }
    std::map<std::vector<i64>, u32> by_desc_;
};

inline Tables compile(int C) {
    if (C < 1 || C > MAX_CLIENTS) throw Error(SR_ERR_UNSUPPORTED, "paxos: client_count must be in 1..=6");
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
            // GetOk in phase 1 only (RegisterActor client, src/actor/register.rs:170-200); a
            // GetOk carries no value or one of the C clients' letters
            if ((int)H[k].done[c].size() != (kind == 0 ? 0 : 1) || kind > 1 + C) continue;
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
    T.hists = std::move(H);
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

// The history of LinearizabilityTester<Id, Register<char>> (src/semantics/linearizability.rs:
// 57-241) under this protocol, stored in the state: client t invokes its Put at init (its `last`
// vector all -1: nothing has completed), receives PutOk (phase 0 -> 1) and at once invokes its Get,
// whose `last` vector records how many ops of every other client had completed then (that
// client's phase: 0, 1 or 2), and receives GetOk(v) (phase 1 -> 2). Per client: phase (2 bits) |
// Get's returned value (3 bits: 0 = '\0', v = the v-th client's letter) | the Get's `last` entries
// for the other clients in ascending id (2 bits each). The field is a FUNCTION of the reference's
// tester state (equal states <=> equal words still holds), so nothing is precomputed per history
// and any client count fits; `linearizable` runs the tester's serialization search on it.
template <int CC = 0>
struct PaxosHistT {
    u32 C = 2;
    // CC > 0: the client count as a compile-time constant (PaxosT<W, CC>): the per-client loops of
    // the tester and of `apply` unroll. The methods read it through NC().
    SR_HD u32 NC() const {
        if constexpr (CC > 0) return (u32)CC;
        else return C;
    }
    // Layout: every client's phase first (2 bits each: they sit in word 0's spare bits, where
    // `enabled` reads them with one shift), then the returned values (3 bits each), then each
    // client's Get `last` entries (2 bits per other client).
    SR_HD u32 ret_off(u32 c) const { return 2 * NC() + 3 * c; }
    SR_HD u32 last_off(u32 t, u32 u) const { return 5 * NC() + 2 * (NC() - 1) * t + 2 * (u < t ? u : u - 1); }
    SR_HD static u32 get(u64 lo, u64 hi, u32 off, u32 w) {
        const u64 v = off >= 64 ? hi >> (off - 64) : (lo >> off) | (off + w > 64 && off ? hi << (64 - off) : 0);
        return (u32)(v & ((1ull << w) - 1));
    }
    SR_HD static void put(u64& lo, u64& hi, u32 off, u32 w, u64 v) {
        const u64 m = (1ull << w) - 1;
        if (off >= 64) {
            hi = (hi & ~(m << (off - 64))) | (v & m) << (off - 64);
            return;
        }
        lo = (lo & ~(m << off)) | (v & m) << off;
        if (off + w > 64) {
            const u32 k = 64 - off;  // bits in lo
            hi = (hi & ~(m >> k)) | (v & m) >> k;
        }
    }
    SR_HD u32 phase(u64 lo, u64, u32 c) const { return (u32)(lo >> (2 * c)) & 3u; }  // 2C <= 12 bits
    // record_invocations of client c's Get: its `last` entries = every other client's phase, in
    // ascending id — the phase field without c's own two bits, stored with one put.
    SR_HD void record_get(u64& lo, u64& hi, u32 c) const {
        const u32 ph = (u32)lo & ((1u << (2 * NC())) - 1);
        put(lo, hi, 5 * NC() + 2 * (NC() - 1) * c, 2 * (NC() - 1), (ph & ((1u << (2 * c)) - 1)) | (ph >> (2 * c + 2)) << (2 * c));
    }
    SR_HD u32 ret(u64 lo, u64 hi, u32 c) const { return get(lo, hi, ret_off(c), 3); }
    // completed-op count of client u when client t invoked its Get
    SR_HD u32 last(u64 lo, u64 hi, u32 t, u32 u) const { return get(lo, hi, last_off(t, u), 2); }

    // LinearizabilityTester::serialized_history().is_some() (linearizability.rs:159-240; the host
    // restatement is px::Hist::serialize): a depth-first search for an order of every completed
    // op (and any subset of the in-flight ones) that respects real time and the register. Ops of
    // client t: 0 = Write(t's letter) (completed from phase 1, with no real-time predecessor),
    // 1 = Read (in flight in phase 1 with predecessors from `last`, completed in phase 2). Threads
    // are tried in id order, completed ops before an in-flight one, as the reference does.
    // `linearizable` without a search. Every Write has its own value (client t writes t + 1), so a
    // serialization is a sequence of CLUSTERS: first the Reads of the initial value (cluster 0),
    // then, per written value v, Write(v) directly followed by the Reads that returned v (no other
    // Write can come between them, and no Read of another value either), Writes nobody read being
    // clusters of their own and pending ops left out (a pending Read changes nothing, a pending
    // Write nobody read only overwrites). Real-time order only runs INTO Reads (every Write is
    // invoked at init): Write(u) precedes Read(t) when u's Write had completed at t's invocation
    // (t's own Write always), Read(u) precedes Read(t) when both of u's ops had. A serialization
    // exists iff no such edge enters cluster 0 from another cluster and the edges between the
    // value clusters have no cycle (a topological order of the clusters, each cluster in real-time
    // order inside, is one). O(C^2) bit operations instead of a search whose interleavings grow
    // factorially (a single-copy register with 4 clients: 4.6 ms for one history on a host core).
    // Checked against the search (`linearizable_search`) on every history of the paxos and
    // single-copy state spaces and on random histories (sr_selftest_models).
    // The fields are unpacked once (phases, the returned values and every Get's `last` entries, each
    // a contiguous run of the 128-bit field), and every loop runs its maximal trip count unrolled
    // with the clients past C masked out: the per-client rows are independent chains the wave
    // issues interleaved, and no branch depends on the history. The loop form was a dependent chain
    // of ~1 000 instructions on every workgroup's last flush (2.4-3.6 us per level of paxos C=6, 11 %
    // of its check: profiles/r05_paxos_lin.txt).
    SR_HD bool linearizable(u64 lo, u64 hi) const {
        constexpr u32 MC = px::MAX_CLIENTS;
        const u32 C = NC();
        const u32 phases = (u32)lo & ((1u << (2 * C)) - 1);  // 2 bits per client (2C <= 12)
        const u32 rets = get(lo, hi, 2 * C, 3 * C);           // 3 bits per client (3C <= 18)
        const u32 lb = 5 * C, lw = 2 * C * (C - 1);             // the `last` runs: lw <= 60 bits from bit lb <= 30
        const u64 lasts = lw ? ((lo >> lb) | (hi << (64 - lb))) & ((1ull << lw) - 1) : 0ull;
        u64 in = 0;  // byte b: the clusters that must precede cluster b (bit a)
#pragma unroll
        for (u32 t = 0; t < MC; ++t) {
            const u32 r = rets >> (3 * t) & 7;
            const u32 sh = 2 * (C - 1) * t;
            const u64 lt = sh < 64 ? lasts >> sh : 0ull;  // t's `last` entries, ascending other client
            u32 row = 1u << (t + 1);                       // t's own Write
#pragma unroll
            for (u32 k = 0; k + 1 < MC; ++k) {
                const u32 u = k < t ? k : k + 1, l = (u32)(lt >> (2 * k)) & 3u;
                const u32 e = (l >= 1 ? 1u << (u + 1) : 0u) | (l >= 2 ? 1u << (rets >> (3 * u) & 7) : 0u);
                row |= k + 1 < C ? e : 0u;
            }
            row &= ~(1u << r);  // (an op of the Read's own cluster is no constraint)
            const bool read_done = t < C && (phases >> (2 * t) & 3u) == 2u;  // completed Reads only
            in |= read_done ? (u64)(row & 0xffu) << (8 * r) : 0ull;
        }
        // An op of a value cluster before a Read of the initial value, or a cycle among the value
        // clusters: each round removes the clusters nothing alive precedes, and C rounds empty an
        // acyclic graph.
        u32 alive = ((1u << (C + 1)) - 1) & ~1u;
#pragma unroll
        for (u32 round = 0; round < MC; ++round) {
            u32 rm = 0;
#pragma unroll
            for (u32 b = 1; b <= MC; ++b)
                rm |= (alive >> b & 1) && !((u32)(in >> (8 * b)) & alive & 0xffu) ? 1u << b : 0u;
            alive &= ~rm;
        }
        return !(in & 0xffull) && alive == 0;
    }
    SR_HD bool linearizable_search(u64 lo, u64 hi) const {
        const u32 C = NC();
        // No completed Read: the completed ops are Writes invoked together at init, unordered in
        // real time, and any order of them (in-flight ops left out) is a valid serialization.
        // Packed scalars only (2-bit fields per client, 8-bit frames): an array indexed by client
        // would live in scratch memory and raise the registers of every kernel this inlines into.
        u32 done = 0, any_read = 0;  // phase of client t at bits 2t
        for (u32 t = 0; t < C; ++t) {
            const u32 p = phase(lo, hi, t);
            done |= p << (2 * t);
            any_read |= p == 2;
        }
        if (!any_read) return true;
        // In-flight ops worth placing: a pending Read never helps (it changes nothing and may
        // return anything), and a pending Write only helps if some completed Read returned its
        // value. Leaving the others out keeps the existence of a serialization (the tester's
        // `is_some()`) and removes their interleavings from the search.
        u32 wanted = 0;  // bit t: some completed Read returned client t's value
        for (u32 t = 0; t < C; ++t)
            if (phase(lo, hi, t) == 2 && ret(lo, hi, t)) wanted |= 1u << (ret(lo, hi, t) - 1);
        auto f2 = [](u32 v, u32 t) { return v >> (2 * t) & 3u; };
        u32 next = 0, used = 0;  // next op of client t at bits 2t; in-flight op used: bit t
        u64 fl = 0, fh = 0;      // frames (8 bits each): thread | kind << 3 | register before << 4
        u32 depth = 0, reg = 0, t0 = 0;
        // op (t, i) may be placed once every op that completed before its invocation is placed
        auto violates = [&](u32 t, u32 i) {
            if (i == 0) return false;  // a Put: invoked before anything completed
            for (u32 u = 0; u < C; ++u)
                if (u != t && f2(next, u) < f2(done, u) && f2(next, u) < last(lo, hi, t, u)) return true;
            return false;
        };
        auto push = [&](u32 t, u32 kind) {
            const u64 f = (u64)(t | kind << 3 | reg << 4);
            if (depth < 8) fl |= f << (8 * depth);
            else fh |= f << (8 * (depth - 8));
            ++depth;
        };
        for (int guard = 0; guard < 1 << 20; ++guard) {
            if (next == done) return true;  // every completed op placed
            bool found = false;
            for (u32 t = t0; t < C && !found; ++t) {
                const u32 n = f2(next, t), d = f2(done, t);
                if (n == d) {
                    // in-flight op: index d (a Write only when wanted, never a Read)
                    if (d != 0 || !(wanted >> t & 1) || (used >> t & 1)) continue;
                    push(t, 1);
                    used |= 1u << t;
                    if (d == 0) reg = t + 1;  // a Write takes effect; a Read returns anything
                    found = true;
                } else {
                    next += 1u << (2 * t);
                    if (violates(t, n) || (n == 1 && ret(lo, hi, t) != reg)) {
                        next -= 1u << (2 * t);
                        continue;
                    }
                    push(t, 0);
                    if (n == 0) reg = t + 1;
                    found = true;
                }
            }
            if (found) {
                t0 = 0;
                continue;
            }
            if (depth == 0) return false;
            --depth;
            const u32 f = (u32)((depth < 8 ? fl >> (8 * depth) : fh >> (8 * (depth - 8))) & 0xff);
            if (depth < 8) fl &= ~(0xffull << (8 * depth));
            else fh &= ~(0xffull << (8 * (depth - 8)));
            const u32 t = f & 7;
            if (f >> 3 & 1) used &= ~(1u << t);
            else next -= 1u << (2 * t);
            reg = f >> 4;
            t0 = t + 1;
        }
        return false;
    }
    static constexpr u32 MAXC = px::MAX_CLIENTS;

    // Canonical description of the history (oracle/paxos.hpp describe_register_history): per
    // client c its Get's returned value (-1 before the Get returned), then per other client u how
    // many of u's ops had completed when c invoked its Get (-1 before the Get). C * C values.
    int width() const { return (int)(C * C); }
    void describe(u64 lo, u64 hi, i64* d) const {
        int k = 0;
        for (u32 c = 0; c < C; ++c) {
            const u32 ph = phase(lo, hi, c);
            d[k++] = ph == 2 ? (i64)ret(lo, hi, c) : -1;
            for (u32 u = 0; u < C; ++u)
                if (u != c) d[k++] = ph >= 1 ? (i64)last(lo, hi, c, u) : -1;
        }
    }
    // Inverse, given every client's phase (op_count - 1, described with the actors).
    void undescribe(const i64* d, const u32* phases, u64& lo, u64& hi) const {
        lo = hi = 0;
        int k = 0;
        for (u32 c = 0; c < C; ++c) {
            put(lo, hi, 2 * c, 2, phases[c]);
            const i64 r = d[k++];
            if (r >= 0) put(lo, hi, ret_off(c), 3, (u64)r);
            for (u32 u = 0; u < C; ++u) {
                if (u == c) continue;
                const i64 l = d[k++];
                if (l >= 0) put(lo, hi, last_off(c, u), 2, (u64)l);
            }
        }
    }
};

using PaxosHist = PaxosHistT<0>;

// W = 11 holds the history of up to 4 clients in the 3 x 17 bits the servers leave free; W = 12
// adds a word for 5 or 6 clients. `linearizable` runs the search once per new state (its property
// check); caching its result in the state, computed at every client delivery, was no faster at 3
// clients and 9 % slower at 6 (profiles/r04_paxos_lin_ab.txt).
template <int WW, int CC = 0>
struct PaxosT {
    static constexpr int W = WW, MW = 1, NPROPS = 2;
    static constexpr int NET0 = W - px::SLOTS / 2;  // first network word
    static_assert(NET0 == 3 || NET0 == 4, "servers (+ one history word) then the network");
    static_assert(CC == 0 || (CC >= 1 && CC <= (WW == 11 ? 4 : px::MAX_CLIENTS)), "client count of this encoding");
    int C = 2;  // (= CC when CC > 0: the engines of the bench configurations, reg_paxos*.hip)

    static PaxosT make(int C) {
        if (C < 1 || C > max_clients()) throw Error(SR_ERR_UNSUPPORTED, "paxos: client_count out of this encoding's range");
        if (CC > 0 && C != CC) throw Error(SR_ERR_ARG, "paxos: this engine is compiled for another client count");
        PaxosT m;
        m.C = C;
        return m;
    }
    static constexpr int max_clients() { return W == 11 ? 4 : px::MAX_CLIENTS; }
    SR_HD PaxosHistT<CC> hs() const {
        PaxosHistT<CC> h;
        h.C = (u32)C;
        return h;
    }
    // the history field: bits 47..63 of words 0, 1, 2 (then word 3 with W = 12)
    SR_HD static void hist_get(const u64* s, u64& lo, u64& hi) {
        constexpr u32 B = 64 - px::SBITS;  // 17
        lo = (s[0] >> px::SBITS) | (s[1] >> px::SBITS) << B | (s[2] >> px::SBITS) << (2 * B);
        hi = (s[2] >> px::SBITS) >> (64 - 2 * B);
        if constexpr (NET0 == 4) {
            lo |= s[3] << (3 * B);
            hi |= s[3] >> (64 - 3 * B);
        }
    }
    SR_HD static void hist_set(u64* s, u64 lo, u64 hi) {
        constexpr u32 B = 64 - px::SBITS;
        constexpr u64 M = (1ull << B) - 1;
        s[0] = (s[0] & px::SMASK) | (lo & M) << px::SBITS;
        s[1] = (s[1] & px::SMASK) | (lo >> B & M) << px::SBITS;
        s[2] = (s[2] & px::SMASK) | ((lo >> (2 * B) | hi << (64 - 2 * B)) & M) << px::SBITS;
        if constexpr (NET0 == 4) s[3] = lo >> (3 * B) | hi << (64 - 3 * B);
    }

    int max_actions() const { return px::SLOTS; }
    int max_out_degree() const { return px::SLOTS; }
    SR_HD static u32 slot(const u64* s, int k) { return (u32)(s[NET0 + k / 2] >> (32 * (k & 1))); }
    SR_HD u32 phase(const u64* s, int c) const { return (u32)(s[0] >> (px::SBITS + 2 * c)) & 3u; }
    SR_HD static u64 server_word(const u64* s, u32 i) { return s[i] & px::SMASK; }

    // Every envelope is deliverable (model.rs:238-257), but most deliveries are no-ops
    // (`next_state` = None, src/actor/model.rs:299-301: the actor ignores the message). The mask
    // keeps the slots whose delivery changes the state: the exact complement of apply's `false`
    // returns below, so the successors and their slot order are unchanged, and the load-balanced
    // expansion spends its lanes on real successors only.
    // phases: client c's phase in bits 2c, 2c+1
    SR_HD bool delivers(const u64* s, u32 e, u32 phases) const {
        const u32 dst = px::e_dst(e), kind = px::e_kind(e), bal = px::e_bal(e);
        if (dst >= 3) {  // (request ids are the client's own: e_req)
            const u32 ph = phases >> (2 * (dst - 3)) & 3;
            return (ph == 0 && kind == px::PUTOK) || (ph == 1 && kind == px::GETOK);
        }
        const u64 sw = server_word(s, dst);
        const u32 sbal = (u32)(sw & 15), sprop = (u32)(sw >> 4 & 15), decided = (u32)(sw >> 46 & 1);
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
        const u32 phases = (u32)(s[0] >> px::SBITS);  // the history field starts with the phases
        u64 mk = 0;
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) {
            const u32 e = slot(s, k);
            if (e != px::EMPTY && delivers(s, e, phases)) mk |= 1ull << k;
        }
        m[0] = mk;
    }
    // Bit k of enabled(s) alone (has_enabled_slot: one lane per parent and slot on the device).
    static constexpr int ESLOTS = px::SLOTS;
    SR_HD bool enabled_slot(const u64* s, int k) const {
        const u32 e = slot(s, k);
        return e != px::EMPTY && delivers(s, e, (u32)(s[0] >> px::SBITS));
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
        u64 w[4] = {s[0], s[1], s[2], NET0 == 4 ? s[3] : 0ull};
        if (dst < 3) {
            px::Srv sv = px::Srv::load(server_word(s, dst));
            const bool owned = px::server_on_msg(dst, sv, e, out, nout);
            if (!owned && nout == 0) return false;  // is_no_op (src/actor.rs:232-234)
            const u64 nw = sv.store();
#pragma unroll
            for (u32 i = 0; i < 3; ++i)
                if (i == dst) w[i] = (w[i] & ~px::SMASK) | nw;
        } else {  // RegisterActor::Client::on_msg (src/actor/register.rs:170-200), put_count = 1
            const u32 c = dst - 3, kind = px::e_kind(e);
            const PaxosHistT<CC> h = hs();
            u64 lo, hi;
            hist_get(s, lo, hi);
            const u32 ph = h.phase(lo, hi, c);
            if (ph == 0 && kind == px::PUTOK) {
                // record_returns (WriteOk), then the Get is sent and recorded by record_invocations
                out[nout++] = px::env(dst, (dst + 1) % 3, px::GET, 0, 0);  // request 2 * id
                h.record_get(lo, hi, c);
            } else if (ph == 1 && kind == px::GETOK) {
                PaxosHist::put(lo, hi, h.ret_off(c), 3, px::e_val(e));  // record_returns (ReadOk(v))
            } else {
                return false;
            }
            PaxosHist::put(lo, hi, 2 * c, 2, ph + 1);
            hist_set(w, lo, hi);
        }
        // remove the delivered envelope (DuplicatingNetwork::No), then insert what was sent
#pragma unroll
        for (int k = 0; k < px::SLOTS; ++k) net[k] = k < a ? net[k] : (k + 1 < px::SLOTS ? net[k + 1] : px::EMPTY);
#pragma unroll
        for (int j = 0; j < 3; ++j) {  // (unrolled: out[] and net[] stay in registers)
            if (j >= nout) break;
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
#pragma unroll
        for (int i = 0; i < NET0; ++i) o[i] = w[i];
#pragma unroll
        for (int k = 0; k < px::SLOTS / 2; ++k) o[NET0 + k] = (u64)net[2 * k] | (u64)net[2 * k + 1] << 32;
        return true;
    }

    SR_HD bool discovers(int p, const u64* s) const {
        if (p == 0) {  // always "linearizable" (examples/paxos.rs:251-254): once per new state
#ifdef SR_PX_NOLIN
            return false;  // (measurement build only: the test's cost)
#endif
            u64 lo, hi;
            hist_get(s, lo, hi);
            return !hs().linearizable(lo, hi);
        }
        bool any = false;  // sometimes "value chosen" (examples/paxos.rs:255-261)
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
            net[c] = px::env(id, id % 3, px::PUT, 0, 0);  // request id and value: the client's
        }
        std::sort(net, net + C);
        for (int i = 0; i < NET0; ++i) out[i] = 0;  // every Put in flight: all phases 0
        for (int k = 0; k < px::SLOTS / 2; ++k) out[NET0 + k] = (u64)net[2 * k] | (u64)net[2 * k + 1] << 32;
        return 1;
    }
    int expectation(int p) const { return p == 0 ? ALWAYS : SOMETIMES; }
    const char* prop_name(int p) const { return p == 0 ? "linearizable" : "value chosen"; }
    // The oracle's canonical description (oracle/paxos.hpp describe).
    int describe_width() const { return 3 * 9 + C + 16 + hs().width(); }
    void describe(const u64* s, i64* d) const {
        int k = 0;
        for (int i = 0; i < 3; ++i) {
            const px::Srv v = px::Srv::load(server_word(s, (u32)i));
            d[k++] = v.bal >> 2;
            d[k++] = v.bal & 3;
            d[k++] = v.prop ? (i64)v.prop : -1;
            for (int j = 0; j < 3; ++j) d[k++] = (v.prep[j] >> 8) ? px::acc_code(v.prep[j] & 255) : -1;
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
        u64 lo, hi;
        hist_get(s, lo, hi);
        hs().describe(lo, hi, d + k);
    }
    // The state of a description (sr_model_fingerprint): the inverse of describe.
    void undescribe(const i64* d, u64* s) const {
        u64 w[4] = {0, 0, 0, 0};
        int k = 0;
        for (int i = 0; i < 3; ++i) {
            px::Srv v{};
            v.bal = (u32)(d[k] << 2 | d[k + 1]);
            k += 2;
            v.prop = d[k] < 0 ? 0u : (u32)d[k];
            ++k;
            for (int j = 0; j < 3; ++j, ++k) v.prep[j] = d[k] < 0 ? 0u : 256u | px::acc_decode(d[k]);
            v.accepts = (u32)d[k++];
            v.accepted = px::acc_decode(d[k++]);
            v.decided = (u32)d[k++];
            w[i] = v.store();
        }
        u32 phases[px::MAX_CLIENTS];
        for (int c = 0; c < C; ++c) phases[c] = (u32)(d[k++] - 1);
        u32 net[px::SLOTS];
        int n = 0;
        for (int j = 0; j < 16; ++j, ++k)
            if (d[k] >= 0) net[n++] = px::env_decode(d[k]);
        std::sort(net, net + n);
        for (int j = n; j < px::SLOTS; ++j) net[j] = px::EMPTY;
        u64 lo, hi;
        hs().undescribe(d + k, phases, lo, hi);
        hist_set(w, lo, hi);
        for (int i = 0; i < NET0; ++i) s[i] = w[i];
        for (int j = 0; j < px::SLOTS / 2; ++j) s[NET0 + j] = (u64)net[2 * j] | (u64)net[2 * j + 1] << 32;
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
using Paxos = PaxosT<11>;      // up to 4 clients
using PaxosWide = PaxosT<12>;  // 5 or 6 clients

}  // namespace sr
