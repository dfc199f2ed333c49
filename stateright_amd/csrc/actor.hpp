// GpuModels for Stateright's ActorModel (src/actor/model.rs:176-327): a generic encoding of the
// actor system's state and transition rules, `ActorGpu<Sys>`, over a system description Sys (the
// actors' `on_start` / `on_msg` / `on_timeout`, the history's `record_msg_in` / `record_msg_out`,
// the boundary and the properties), with the reference's actor fixtures on top:
//   PingPongSysT  ping-pong (src/actor/actor_test_util.rs:4-96), lossy / duplicating options
//   FixtureSys    the undeliverable-message and timer fixtures (src/actor/model.rs:697-733)
//   AbdSys        the ABD linearizable register (examples/linearizable-register.rs)
//   SingleCopySys the single-copy register (examples/single-copy-register.rs)
// The CPU restatement the encodings are tested against is oracle/actor.hpp.
//
// State: W = AW + K/2 words.
//   words [0, AW)     the system's fields (Sys), with word 0 bits 52..63 reserved here:
//                       [52, 56) length of `is_timer_set` (a Vec that grows on demand, so its
//                                length is part of the state, model.rs:189-198)
//                       [56, 64) its bits
//   words [AW, W)     the network: K u32 envelope codes, ascending, unused = 0xffffffff. The code
//                     src << 29 | dst << 22 | msg orders envelopes as the oracle's std::set of
//                     (src, dst, msg), so action slots enumerate `actions()` in the oracle's order
//                     (the reference iterates a HashSet: its order is parity unpinned).
// Action slots: 2k = Drop(envelope k) (lossy networks), 2k + 1 = Deliver(envelope k) (dst among
// the actors), 2K + i = Timeout(i) (timer i set).
#pragma once
#include "paxos.hpp"

namespace sr {
namespace act {

constexpr u32 EMPTY = 0xffffffffu;
constexpr u32 MSG_BITS = 22;
SR_HD u32 env(u32 src, u32 dst, u32 msg) { return src << 29 | dst << MSG_BITS | msg; }
SR_HD u32 e_src(u32 e) { return e >> 29; }
SR_HD u32 e_dst(u32 e) { return e >> MSG_BITS & 127; }
SR_HD u32 e_msg(u32 e) { return e & ((1u << MSG_BITS) - 1); }

// `Out` (src/actor.rs:163-201): the commands one actor emits, in order.
enum CmdKind : u32 { SEND = 0, SET_TIMER = 1, CANCEL_TIMER = 2 };
struct Out {
    static constexpr int MAX = 4;
    int n = 0;
    u32 kind[MAX];
    u32 dst[MAX];
    u32 msg[MAX];
    SR_HD void send(u32 d, u32 m) {
        kind[n] = SEND;
        dst[n] = d;
        msg[n] = m;
        ++n;
    }
    SR_HD void set_timer() { kind[n] = SET_TIMER, dst[n] = 0, msg[n] = 0, ++n; }
    SR_HD void cancel_timer() { kind[n] = CANCEL_TIMER, dst[n] = 0, msg[n] = 0, ++n; }
};

constexpr u64 OVERFLOW_BIT = 1ull << 51;  // a network past its K slots (refused at make(); never set)

template <class Sys>
struct ActorGpu : Sys {
    static constexpr int K = Sys::K, AW = Sys::AW, W = AW + K / 2, NPROPS = Sys::NPROPS;
    static constexpr int MW = (2 * K + 8 + 63) / 64;
    static_assert(K % 2 == 0 && Sys::NACT <= 8, "actor model layout");

    SR_HD static u32 slot(const u64* s, int k) { return (u32)(s[AW + k / 2] >> (32 * (k & 1))); }
    SR_HD static u32 tlen(const u64* s) { return (u32)(s[0] >> 52 & 15); }
    SR_HD static u32 tmask(const u64* s) { return (u32)(s[0] >> 56 & 255); }

    int max_actions() const { return 2 * K + 8; }
    int max_out_degree() const { return 2 * K + (int)this->nact(); }

    // `actions` (model.rs:238-257)
    SR_HD void enabled(const u64* s, u64* m) const {
        for (int w = 0; w < MW; ++w) m[w] = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u32 e = slot(s, k);
            if (e == EMPTY) continue;
            if (this->lossy) m[(2 * k) >> 6] |= 1ull << ((2 * k) & 63);
            if (e_dst(e) < this->nact()) m[(2 * k + 1) >> 6] |= 1ull << ((2 * k + 1) & 63);
        }
        const u32 len = tlen(s), mask = tmask(s);
        for (u32 i = 0; i < len; ++i)
            if (mask >> i & 1) m[(2 * K + i) >> 6] |= 1ull << ((2 * K + i) & 63);
    }

    // process_commands (model.rs:176-202): record_msg_out, then the set insert; timers
    SR_HD void process(u64* o, u32* net, u32 id, const Out& out) const {
        for (int c = 0; c < out.n; ++c) {
            if (out.kind[c] == SET_TIMER) {
                const u32 len = tlen(o) > id + 1 ? tlen(o) : id + 1;
                o[0] = (o[0] & ~(15ull << 52)) | (u64)len << 52 | 1ull << (56 + id);
                continue;
            }
            if (out.kind[c] == CANCEL_TIMER) {
                if (id >= tlen(o)) o[0] |= OVERFLOW_BIT;  // the reference panics
                o[0] &= ~(1ull << (56 + id));
                continue;
            }
            this->record_out(o, id, out.dst[c], out.msg[c]);
            const u32 x = env(id, out.dst[c], out.msg[c]);
            bool dup = false;
#pragma unroll
            for (int k = 0; k < K; ++k) dup |= net[k] == x;
            if (dup) continue;
            if (net[K - 1] != EMPTY) o[0] |= OVERFLOW_BIT;
            u32 prev = 0;  // sorted insert
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const u32 cur = net[k];
                net[k] = cur < x ? cur : ((k == 0 || prev < x) ? x : prev);
                prev = cur;
            }
        }
    }
    SR_HD static void remove(u32* net, int k0) {
#pragma unroll
        for (int k = 0; k < K; ++k) net[k] = k < k0 ? net[k] : (k + 1 < K ? net[k + 1] : EMPTY);
    }
    SR_HD static void pack(u64* o, const u32* net) {
#pragma unroll
        for (int k = 0; k < K / 2; ++k) o[AW + k] = (u64)net[2 * k] | (u64)net[2 * k + 1] << 32;
    }

    // `next_state` (model.rs:259-327) AND `within_boundary`.
    SR_HD bool apply(const u64* s, int a, u64* o) const {
        u32 net[K];
#pragma unroll
        for (int k = 0; k < K; ++k) net[k] = slot(s, k);
#pragma unroll
        for (int w = 0; w < AW; ++w) o[w] = s[w];
        if (a < 2 * K) {
            const int k = a >> 1;
            u32 e = 0;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (j == k) e = net[j];
            if ((a & 1) == 0) {  // Drop
                remove(net, k);
            } else {  // Deliver
                const u32 dst = e_dst(e);
                if (dst >= this->nact()) return false;
                Out out;
                const bool owned = this->on_msg(o, dst, e_src(e), e_msg(e), out);
                if (!owned && out.n == 0) return false;  // is_no_op (src/actor.rs:232-234)
                this->record_in(o, e_src(e), dst, e_msg(e));
                if (!this->duplicating) remove(net, k);
                process(o, net, dst, out);
            }
        } else {  // Timeout
            const u32 id = (u32)(a - 2 * K);
            Out out;
            const bool owned = this->on_timeout(o, id, out);
            bool keep = false;
            for (int c = 0; c < out.n; ++c) keep |= out.kind[c] == SET_TIMER;
            if (!owned && out.n == 0 && keep) return false;
            o[0] &= ~(1ull << (56 + id));
            process(o, net, id, out);
        }
        pack(o, net);
        return this->within_boundary(o);
    }

    SR_HD bool discovers(int p, const u64* s) const {
        u32 net[K];
#pragma unroll
        for (int k = 0; k < K; ++k) net[k] = slot(s, k);
        return Sys::discovers(p, s, net);
    }

    // init: the init network, then every actor's on_start in index order (model.rs:215-242)
    int init_count() const { return 1; }
    int init_states(u64* out) const {
        for (int w = 0; w < W; ++w) out[w] = 0;
        u32 net[K];
        for (int k = 0; k < K; ++k) net[k] = EMPTY;
        Out o0;
        u32 src0 = 0;
        this->init_network(o0, src0);
        for (int c = 0; c < o0.n; ++c) {  // the init network is inserted as is (no record_msg_out)
            const u32 x = env(src0, o0.dst[c], o0.msg[c]);
            int p = 0;
            while (p < K && net[p] < x) ++p;
            if (p < K && net[p] == x) continue;
            for (int q = K - 1; q > p; --q) net[q] = net[q - 1];
            if (p < K) net[p] = x;
        }
        for (u32 id = 0; id < this->nact(); ++id) {
            Out o;
            this->on_start(out, id, o);
            process(out, net, id, o);
        }
        pack(out, net);
        if (out[0] & OVERFLOW_BIT) throw Error(SR_ERR_UNSUPPORTED, "actor model: the init network exceeds its capacity");
        return this->within_boundary(out) ? 1 : 0;
    }

    // Canonical description (oracle/actor.hpp describe): the actors' and the history's fields, the
    // timer vector (length, bits), then the network as NET descriptive envelope codes (msg code *
    // 128 + dst) * 16 + src, ascending, padded with -1.
    int describe_width() const { return this->actors_width() + this->history_width() + 2 + Sys::NET; }
    static i64 desc_env(const Sys& sy, u32 e) { return (sy.msg_code(e_msg(e)) * 128 + (i64)e_dst(e)) * 16 + (i64)e_src(e); }
    static_assert(Sys::NET >= K, "the description holds every envelope");
    void describe(const u64* s, i64* d) const {
        if (s[0] & OVERFLOW_BIT) throw Error(SR_ERR_UNSUPPORTED, "actor model: a network exceeded its capacity");
        int k = this->describe_fields(s, d);
        d[k++] = tlen(s);
        d[k++] = tmask(s);
        std::vector<i64> net;
        for (int j = 0; j < K; ++j)
            if (slot(s, j) != EMPTY) net.push_back(desc_env(*this, slot(s, j)));
        std::sort(net.begin(), net.end());
        net.resize(Sys::NET, -1);
        for (i64 v : net) d[k++] = v;
    }
    // The state of a description (sr_model_fingerprint): the inverse of describe.
    void undescribe(const i64* d, u64* s) const {
        for (int w = 0; w < W; ++w) s[w] = 0;
        int k = this->undescribe_fields(d, s);
        s[0] |= (u64)(d[k] & 15) << 52 | (u64)(d[k + 1] & 255) << 56;
        k += 2;
        u32 net[K];
        int n = 0;
        for (int j = 0; j < Sys::NET; ++j, ++k) {
            if (d[k] < 0) continue;
            if (n >= K) throw Error(SR_ERR_ARG, "actor model: the described network exceeds the encoding's capacity");
            const i64 c = d[k];
            net[n++] = env((u32)(c % 16), (u32)(c / 16 % 128), this->msg_decode(c / 2048));
        }
        std::sort(net, net + n);
        for (int j = n; j < K; ++j) net[j] = EMPTY;
        pack(s, net);
    }
    // Action ids (oracle/actor.hpp action_id): Deliver = code * 4 + 1, Drop = code * 4 + 2,
    // Timeout(i) = i * 4 + 3.
    i64 action_id(const u64* s, int a) const {
        if (a >= 2 * K) return (i64)(a - 2 * K) * 4 + 3;
        return desc_env(*this, slot(s, a >> 1)) * 4 + ((a & 1) ? 1 : 2);
    }
    i64 action_id_bound() const { return 0; }  // sparse ids
    std::string action_name(i64 id) const {
        const i64 kind = id & 3, code = id >> 2;
        if (kind == 3) return "Timeout(Id(" + std::to_string(code) + "))";
        const i64 src = code % 16, dst = (code / 16) % 128, msg = code / 2048;
        const std::string env = "src: Id(" + std::to_string(src) + "), dst: Id(" + std::to_string(dst) + "), msg: " +
                                this->format_msg(msg);
        return kind == 1 ? "Deliver { " + env + " }" : "Drop(Envelope { " + env + " })";
    }
};

// ---------------------------------------------------------------------------------------------
// Ping-pong (src/actor/actor_test_util.rs:4-96). Word 0: actor counts (4 bits each), history
// (#in, #out) 8 bits each. Message: pong << 8 | value (the oracle's key order (pong, value)).
// The duplicating network keeps every Ping(v) and Pong(v) ever sent, 2 * (max_nat + 1) envelopes
// within the boundary: KK = 16 slots hold max_nat <= 7, KK = 32 slots (17-word states) max_nat
// <= 14 (a count reaches max_nat + 1 <= 15 in its 4 bits before the boundary drops the state).
// ---------------------------------------------------------------------------------------------
template <int KK>
struct PingPongSysT {
    static constexpr int K = KK, AW = 1, NACT = 2, NPROPS = 6, NET = KK;
    static constexpr u32 MAX_NAT = KK / 2 - 1 < 14 ? KK / 2 - 1 : 14;
    u32 max_nat = 1;
    bool lossy = false, duplicating = true, maintains_history = false;
    SR_HD u32 nact() const { return 2; }

    static SR_HD u32 count(const u64* s, u32 i) { return (u32)(s[0] >> (4 * i) & 15); }
    SR_HD void init_network(Out&, u32&) const {}
    SR_HD void on_start(u64*, u32 id, Out& o) const {
        if (id == 0) o.send(1, 0);  // Ping(0) to actor 1
    }
    SR_HD bool on_msg(u64* o, u32 id, u32 src, u32 msg, Out& out) const {
        const u32 pong = msg >> 8, v = msg & 255, c = count(o, id);
        if (c != v) return false;
        out.send(src, pong ? (v + 1) : (1u << 8 | v));  // Pong(v) -> Ping(v + 1); Ping(v) -> Pong(v)
        o[0] = (o[0] & ~(15ull << (4 * id))) | (u64)(c + 1) << (4 * id);
        return true;
    }
    SR_HD bool on_timeout(u64*, u32, Out&) const { return false; }
    SR_HD void record_in(u64* o, u32, u32, u32) const {
        if (maintains_history) o[0] += 1ull << 8;
    }
    SR_HD void record_out(u64* o, u32, u32, u32) const {
        if (maintains_history) o[0] += 1ull << 16;
    }
    SR_HD bool within_boundary(const u64* s) const { return count(s, 0) <= max_nat && count(s, 1) <= max_nat; }
    SR_HD bool discovers(int p, const u64* s, const u32*) const {
        const u32 a = count(s, 0), b = count(s, 1), hi = a > b ? a : b, lo = a > b ? b : a;
        const u32 hin = (u32)(s[0] >> 8 & 255), hout = (u32)(s[0] >> 16 & 255);
        switch (p) {
            case 0: return !(hi - lo <= 1);                    // always "delta within 1"
            case 1: return a == max_nat || b == max_nat;        // sometimes "can reach max"
            case 2: return a == max_nat || b == max_nat;        // eventually "must reach max"
            case 3: return a == max_nat + 1 || b == max_nat + 1;  // eventually "must exceed max"
            case 4: return !(hin <= hout);                      // always "#in <= #out"
            default: return hout <= hin + 1;                    // eventually "#out <= #in + 1"
        }
    }
    u32 emask() const { return 1u << 2 | 1u << 3 | 1u << 5; }
    int expectation(int p) const { return p == 0 || p == 4 ? ALWAYS : p == 1 ? SOMETIMES : EVENTUALLY; }
    const char* prop_name(int p) const {
        static const char* n[] = {"delta within 1", "can reach max", "must reach max", "must exceed max", "#in <= #out",
                                  "#out <= #in + 1"};
        return n[p];
    }
    i64 msg_code(u32 msg) const { return (i64)(msg & 255) * 2 + (msg >> 8); }
    u32 msg_decode(i64 code) const { return (u32)(code & 1) << 8 | (u32)(code / 2); }
    std::string format_msg(i64 code) const { return std::string(code & 1 ? "Pong(" : "Ping(") + std::to_string(code / 2) + ")"; }
    static int actors_width() { return 2; }
    static int history_width() { return 2; }
    int describe_fields(const u64* s, i64* d) const {
        d[0] = count(s, 0);
        d[1] = count(s, 1);
        d[2] = (i64)(s[0] >> 8 & 255);
        d[3] = (i64)(s[0] >> 16 & 255);
        return 4;
    }
    int undescribe_fields(const i64* d, u64* s) const {
        s[0] = (u64)(d[0] & 15) | (u64)(d[1] & 15) << 4 | (u64)(d[2] & 255) << 8 | (u64)(d[3] & 255) << 16;
        return 4;
    }
};

// ---------------------------------------------------------------------------------------------
// Unit-actor fixtures (src/actor/model.rs:697-733): kind 0 = one `Actor for ()` and an init
// envelope to Id 99 (undeliverable); kind 1 = an actor that sets its timer on start.
// ---------------------------------------------------------------------------------------------
struct FixtureSys {
    static constexpr int K = 4, AW = 1, NACT = 1, NPROPS = 1, NET = 4;
    int kind = 0;
    bool lossy = false, duplicating = true;
    SR_HD u32 nact() const { return 1; }
    SR_HD void init_network(Out& o, u32& src) const {
        src = 0;
        if (kind == 0) o.send(99, 0);
    }
    SR_HD void on_start(u64*, u32, Out& o) const {
        if (kind == 1) o.set_timer();
    }
    SR_HD bool on_msg(u64*, u32, u32, u32, Out&) const { return false; }
    SR_HD bool on_timeout(u64*, u32, Out&) const { return false; }
    SR_HD void record_in(u64*, u32, u32, u32) const {}
    SR_HD void record_out(u64*, u32, u32, u32) const {}
    SR_HD bool within_boundary(const u64*) const { return true; }
    SR_HD bool discovers(int, const u64*, const u32*) const { return false; }  // always "unused": true
    int expectation(int) const { return ALWAYS; }
    const char* prop_name(int) const { return "unused"; }
    i64 msg_code(u32) const { return 0; }
    u32 msg_decode(i64) const { return 0; }
    std::string format_msg(i64) const { return "()"; }
    static int actors_width() { return 1; }
    static int history_width() { return 0; }
    int describe_fields(const u64*, i64* d) const {
        d[0] = 0;
        return 1;
    }
    int undescribe_fields(const i64*, u64*) const { return 1; }
};

// ---------------------------------------------------------------------------------------------
// ABD linearizable register (examples/linearizable-register.rs): S AbdActor servers (ids 0..S-1)
// wrapped by RegisterActor::Server, C RegisterActor clients (ids S..S+C-1, put_count 1), a
// non-duplicating lossless network, a LinearizabilityTester<Id, Register<char>> history.
//   word 0     history index (16 bits: the host-interned closure of the clients' register events,
//              px::Tables — the same client protocol as paxos'), then per client c at 16 + 7c:
//              awaiting present (1), awaiting request id (4), op_count (2)
//   word 1 + i server i: seq clock [0,3), seq id [3,5), val [5,7) ('\0' 0, 'A'.. 1..), phase
//              [7,9), request id [9,13), requester [13,16), write/read [16,19) (0 None, else val
//              + 1), response of server j at [19 + 8j, 27 + 8j) (present, clock 3, id 2, val 2),
//              acks mask [19 + 8S, 19 + 9S)
// Message (22 bits, the oracle's key order (kind, req, seq, val)): kind << 12 | req << 8 | clock
// << 5 | id << 2 | val.
// ---------------------------------------------------------------------------------------------
struct AbdSys {
    static constexpr int K = 8, AW = 4, NACT = 6, NPROPS = 2, NET = 16;
    enum Kind : u32 { PUT, GET, PUTOK, GETOK, QUERY, ACKQUERY, RECORD, ACKRECORD };
    u32 S = 2, C = 2;
    bool lossy = false, duplicating = false;
    int nev = 0;
    const u16* h_next_d = nullptr;
    const u8* h_lin_d = nullptr;
    const u16* h_next_h = nullptr;
    const u8* h_lin_h = nullptr;

    static AbdSys make(int clients, int servers, int device) {
        if (clients < 1 || clients > 3 || servers < 1 || servers > 3)
            throw Error(SR_ERR_UNSUPPORTED, "abd: client_count and server_count in 1..=3");
        px::Tables& t = px::tables(clients, device);
        if (t.init_hist != 0) throw Error(SR_ERR_ARG, "abd: the history closure must start at index 0");
        AbdSys m;
        m.C = (u32)clients;
        m.S = (u32)servers;
        m.nev = t.nev;
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
    static SR_HD u32 msg(u32 kind, u32 req, u32 clock, u32 id, u32 val) { return kind << 12 | req << 8 | clock << 5 | id << 2 | val; }
    static SR_HD u32 getf(u64 w, int off, int n) { return (u32)(w >> off & ((1ull << n) - 1)); }
    static SR_HD u64 setf(u64 w, int off, int n, u32 v) { return (w & ~(((1ull << n) - 1) << off)) | (u64)v << off; }
    SR_HD u32 majority() const { return S / 2 + 1; }
    SR_HD u32 nact() const { return S + C; }

    SR_HD void init_network(Out&, u32&) const {}
    SR_HD void on_start(u64* o, u32 id, Out& out) const {
        if (id < S) {  // AbdActor::on_start: seq (0, id), val '\0', phase None
            o[1 + id] = setf(0, 3, 2, id);
            return;
        }
        if (id >= S + C) return;
        // RegisterActor::Client::on_start, put_count 1 (src/actor/register.rs:130-160)
        const u32 c = id - S, req = id;
        out.send(id % S, msg(PUT, req, 0, 0, c + 1));  // Put(1 x index, 'A' + index - S)
        o[0] = setf(o[0], 16 + 7 * (int)c, 7, 1u | req << 1 | 1u << 5);  // awaiting Some(req), op_count 1
    }
    SR_HD bool on_msg(u64* o, u32 id, u32 src, u32 m, Out& out) const {
        const u32 kind = m >> 12, req = m >> 8 & 15, mclock = m >> 5 & 7, mid = m >> 2 & 7, mval = m & 3;
        if (id >= S) {  // RegisterActor::Client::on_msg (src/actor/register.rs:170-200)
            const int off = 16 + 7 * (int)(id - S);
            const u32 f = getf(o[0], off, 7), await_some = f & 1, awaiting = f >> 1 & 15, ops = f >> 5;
            if (!await_some || req != awaiting) return false;
            if (kind == PUTOK) {  // op_count 1 < put_count? no: Get((op_count + 1) x index)
                const u32 nreq = (ops + 1) * id;
                out.send((id + ops) % S, msg(GET, nreq, 0, 0, 0));
                o[0] = setf(o[0], off, 7, 1u | nreq << 1 | (ops + 1) << 5);
                return true;
            }
            if (kind == GETOK) {
                o[0] = setf(o[0], off, 7, (ops + 1) << 5);
                return true;
            }
            return false;
        }
        // AbdActor::on_msg (examples/linearizable-register.rs:66-173)
        u64 w = o[1 + id];
        const u32 clock = getf(w, 0, 3), sid = getf(w, 3, 2), val = getf(w, 5, 2), phase = getf(w, 7, 2);
        const u32 preq = getf(w, 9, 4), requester = getf(w, 13, 3), wr = getf(w, 16, 3);
        const int RSP = 19, ACK = 19 + 8 * (int)S;
        switch (kind) {
            case PUT:
            case GET: {
                if (phase != 0) return false;
                for (u32 p = 0; p < S; ++p)
                    if (p != id) out.send(p, msg(QUERY, req, 0, 0, 0));
                w = setf(w, 7, 2, 1);
                w = setf(w, 9, 4, req);
                w = setf(w, 13, 3, src);
                w = setf(w, 16, 3, kind == PUT ? mval + 1 : 0);
                for (u32 j = 0; j < S; ++j) w = setf(w, RSP + 8 * (int)j, 8, 0);
                w = setf(w, RSP + 8 * (int)id, 8, 1u | clock << 1 | sid << 4 | val << 6);
                w = setf(w, ACK, (int)S, 0);
                o[1 + id] = w;
                return true;
            }
            case QUERY:
                out.send(src, msg(ACKQUERY, req, clock, sid, val));
                return false;
            case ACKQUERY: {
                if (!(phase == 1 && preq == req)) return false;
                w = setf(w, RSP + 8 * (int)src, 8, 1u | mclock << 1 | mid << 4 | mval << 6);
                u32 count = 0, bclock = 0, bid = 0, bval = 0;
                bool first = true;
                for (u32 j = 0; j < S; ++j) {
                    const u32 r = getf(w, RSP + 8 * (int)j, 8);
                    if (!(r & 1)) continue;
                    ++count;
                    const u32 rc = r >> 1 & 7, ri = r >> 4 & 3, rv = r >> 6 & 3;
                    if (first || rc > bclock || (rc == bclock && ri > bid)) bclock = rc, bid = ri, bval = rv;  // max seq
                    first = false;
                }
                if (count == majority()) {
                    u32 nclock = bclock, nid = bid, nval = bval, read = 0;
                    if (wr) {  // write: seq = (seq.0 + 1, id), the written value
                        nclock = bclock + 1;
                        nid = id;
                        nval = wr - 1;
                    } else {
                        read = bval + 1;
                    }
                    for (u32 p = 0; p < S; ++p)
                        if (p != id) out.send(p, msg(RECORD, preq, nclock, nid, nval));
                    if (nclock > clock || (nclock == clock && nid > sid)) {  // self Record
                        w = setf(w, 0, 3, nclock);
                        w = setf(w, 3, 2, nid);
                        w = setf(w, 5, 2, nval);
                    }
                    w = setf(w, 7, 2, 2);
                    w = setf(w, 16, 3, read);
                    for (u32 j = 0; j < S; ++j) w = setf(w, RSP + 8 * (int)j, 8, 0);
                    w = setf(w, ACK, (int)S, 1u << id);  // self AckRecord
                }
                o[1 + id] = w;
                return true;  // `state.to_mut()` before the quorum test
            }
            case RECORD:
                out.send(src, msg(ACKRECORD, req, 0, 0, 0));
                if (mclock > clock || (mclock == clock && mid > sid)) {
                    w = setf(w, 0, 3, mclock);
                    w = setf(w, 3, 2, mid);
                    w = setf(w, 5, 2, mval);
                    o[1 + id] = w;
                    return true;
                }
                return false;
            case ACKRECORD: {
                const u32 acks = getf(w, ACK, (int)S);
                if (!(phase == 2 && preq == req && !(acks >> src & 1))) return false;
                const u32 nacks = acks | 1u << src;
                w = setf(w, ACK, (int)S, nacks);
                if ((u32)__builtin_popcount(nacks) == majority()) {
                    if (wr) out.send(requester, msg(GETOK, preq, 0, 0, wr - 1));
                    else out.send(requester, msg(PUTOK, preq, 0, 0, 0));
                    w = setf(w, 7, 2, 0);
                    w = setf(w, 9, 4, 0);
                    w = setf(w, 13, 3, 0);
                    w = setf(w, 16, 3, 0);
                    w = setf(w, ACK, (int)S, 0);
                }
                o[1 + id] = w;
                return true;
            }
            default:
                return false;
        }
    }
    SR_HD bool on_timeout(u64*, u32, Out&) const { return false; }
    // RegisterMsg::record_returns / record_invocations (src/actor/register.rs:37-87) on the
    // interned history: PutOk returns WriteOk and the client's Get invocation follows in the same
    // delivery (one px event); GetOk(v) returns ReadOk(v).
    SR_HD void record_in(u64* o, u32, u32 dst, u32 m) const {
        const u32 kind = m >> 12;
        if (dst < S || (kind != PUTOK && kind != GETOK)) return;
        const u32 c = dst - S;
        const u32 ev = c * px::NEV_PER_CLIENT + (kind == PUTOK ? 0u : 1u + (m & 3));
        const u64 h = h_next()[(size_t)(o[0] & 0xffff) * nev + ev];
        o[0] = (o[0] & ~0xffffull) | h;
    }
    SR_HD void record_out(u64*, u32, u32, u32) const {}  // folded into record_in (see above)
    SR_HD bool within_boundary(const u64*) const { return true; }
    SR_HD bool discovers(int p, const u64* s, const u32* net) const {
        if (p == 0) return !h_lin()[s[0] & 0xffff];  // always "linearizable"
        bool any = false;                             // sometimes "value chosen"
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u32 e = net[k];
            any |= e != EMPTY && (e_msg(e) >> 12) == GETOK && (e & 3) != 0;
        }
        return any;
    }
    int expectation(int p) const { return p == 0 ? ALWAYS : SOMETIMES; }
    const char* prop_name(int p) const { return p == 0 ? "linearizable" : "value chosen"; }
    // the oracle's msg code: ((((req * 8 + clock) * 8 + id) * 8 + val) * 8 + kind)
    i64 msg_code(u32 m) const {
        const i64 kind = m >> 12, req = m >> 8 & 15, clock = m >> 5 & 7, id = m >> 2 & 7, val = m & 3;
        return (((req * 8 + clock) * 8 + id) * 8 + val) * 8 + kind;
    }
    u32 msg_decode(i64 code) const {
        return msg((u32)(code % 8), (u32)(code / 4096), (u32)(code / 512 % 8), (u32)(code / 64 % 8), (u32)(code / 8 % 8));
    }
    std::string format_msg(i64 code) const {
        const i64 kind = code % 8, val = code / 8 % 8, id = code / 64 % 8, clock = code / 512 % 8, req = code / 4096;
        auto ch = [](i64 v) { return v ? std::string("'") + (char)('A' + v - 1) + "'" : std::string("'\\u{0}'"); };
        const std::string seq = "(" + std::to_string(clock) + ", Id(" + std::to_string(id) + "))", r = std::to_string(req);
        switch (kind) {
            case PUT: return "Put(" + r + ", " + ch(val) + ")";
            case GET: return "Get(" + r + ")";
            case PUTOK: return "PutOk(" + r + ")";
            case GETOK: return "GetOk(" + r + ", " + ch(val) + ")";
            case QUERY: return "Internal(Query(" + r + "))";
            case ACKQUERY: return "Internal(AckQuery(" + r + ", " + seq + ", " + ch(val) + "))";
            case RECORD: return "Internal(Record(" + r + ", " + seq + ", " + ch(val) + "))";
            default: return "Internal(AckRecord(" + r + "))";
        }
    }
    int actors_width() const { return (int)((S + C) * (8 + S)); }
    int history_width() const { return (int)(C * C); }
    // oracle/actor.hpp AbdSys::describe_actor, per actor (8 + S values), then the history
    // (oracle/paxos.hpp describe_register_history) of the interned index's history
    int describe_fields(const u64* s, i64* d) const {
        int k = 0;
        const int width = 8 + (int)S;
        for (u32 id = 0; id < S + C; ++id) {
            const int base = k;
            if (id < S) {
                const u64 w = s[1 + id];
                const u32 phase = getf(w, 7, 2), wr = getf(w, 16, 3);
                d[k++] = getf(w, 0, 3);
                d[k++] = getf(w, 3, 2);
                d[k++] = getf(w, 5, 2);
                d[k++] = phase;
                d[k++] = phase ? getf(w, 9, 4) : 0;
                d[k++] = phase ? getf(w, 13, 3) : 0;
                d[k++] = phase && wr ? (i64)wr - 1 : -1;
                for (u32 j = 0; j < S; ++j) {
                    const u32 r = getf(w, 19 + 8 * (int)j, 8);
                    d[k++] = phase != 1 || !(r & 1) ? -1 : (i64)(r >> 1 & 7) * 64 + (i64)(r >> 4 & 3) * 8 + (r >> 6 & 3);
                }
                d[k++] = phase == 2 ? getf(w, 19 + 8 * (int)S, (int)S) : 0;
            } else {
                const u32 f = getf(s[0], 16 + 7 * (int)(id - S), 7);
                d[k++] = (f & 1) ? (i64)(f >> 1 & 15) : -1;
                d[k++] = f >> 5;
            }
            while (k < base + width) d[k++] = 0;
        }
        px::Tables& t = px::tables((int)C, -1);
        const u32 h = (u32)(s[0] & 0xffff);
        if (h >= t.hists.size()) throw Error(SR_ERR_ARG, "abd: history index out of range");
        px::describe_hist(t.hists[h], (int)C, d + k);
        return k + history_width();
    }
    int undescribe_fields(const i64* d, u64* s) const {
        int k = 0;
        const int width = 8 + (int)S;
        for (u32 id = 0; id < S + C; ++id) {
            const int base = k;
            if (id < S) {
                u64 w = 0;
                const u32 phase = (u32)d[k + 3];
                w = setf(w, 0, 3, (u32)d[k]);
                w = setf(w, 3, 2, (u32)d[k + 1]);
                w = setf(w, 5, 2, (u32)d[k + 2]);
                w = setf(w, 7, 2, phase);
                if (phase) {
                    w = setf(w, 9, 4, (u32)d[k + 4]);
                    w = setf(w, 13, 3, (u32)d[k + 5]);
                    if (d[k + 6] >= 0) w = setf(w, 16, 3, (u32)d[k + 6] + 1);
                }
                for (u32 j = 0; j < S; ++j) {
                    const i64 r = d[k + 7 + (int)j];
                    if (r >= 0) w = setf(w, 19 + 8 * (int)j, 8, 1u | (u32)(r / 64) << 1 | (u32)(r / 8 % 8) << 4 | (u32)(r % 8) << 6);
                }
                if (phase == 2) w = setf(w, 19 + 8 * (int)S, (int)S, (u32)d[k + 7 + (int)S]);
                s[1 + id] = w;
            } else {
                const i64 aw = d[k], ops = d[k + 1];
                s[0] = setf(s[0], 16 + 7 * (int)(id - S), 7, (aw >= 0 ? 1u | (u32)aw << 1 : 0u) | (u32)ops << 5);
            }
            k = base + width;
        }
        px::Tables& t = px::tables((int)C, -1);
        s[0] |= t.hist_index(d + k);
        return k + history_width();
    }
};

// ---------------------------------------------------------------------------------------------
// Single-copy register (examples/single-copy-register.rs): S SingleCopyActor servers (ids 0..S-1,
// one register value each, no consensus) wrapped by RegisterActor::Server, C RegisterActor clients
// (ids S..S+C-1, put_count 1), a non-duplicating lossless network, a LinearizabilityTester<Id,
// Register<char>> history. A client's state follows from its history phase (0: awaiting PutOk(id),
// 1: awaiting GetOk(2 id), 2: done), so the history holds the clients' whole state:
//   word 0     server i's value at [3i, 3i + 3) ('\0' 0, 'A'.. 1..)
//   words 1-2  the history (paxos.hpp PaxosHist: phases, returned values, Get `last` vectors;
//              the same client protocol as paxos', so its device-side linearizability search)
// Message (the oracle's key order (kind, req, val)): kind << 12 | req << 4 | val. Each client has
// at most one message in flight, so K = 6 slots hold up to 6 clients.
// ---------------------------------------------------------------------------------------------
struct SingleCopySys {
    static constexpr int K = 6, AW = 3, NACT = 8, NPROPS = 2, NET = 8;
    enum Kind : u32 { PUT, GET, PUTOK, GETOK };
    u32 S = 1, C = 2;
    bool lossy = false, duplicating = false;

    static SingleCopySys make(int clients, int servers) {
        if (clients < 1 || clients > 6 || servers < 1 || clients + servers > NACT)
            throw Error(SR_ERR_UNSUPPORTED, "single-copy register: client_count in 1..=6, client_count + server_count <= 8");
        SingleCopySys m;
        m.C = (u32)clients;
        m.S = (u32)servers;
        return m;
    }
    SR_HD u32 nact() const { return S + C; }
    SR_HD PaxosHist hs() const {
        PaxosHist h;
        h.C = C;
        return h;
    }
    static SR_HD u32 msg(u32 kind, u32 req, u32 val) { return kind << 12 | req << 4 | val; }
    static SR_HD u32 value(const u64* s, u32 i) { return (u32)(s[0] >> (3 * i)) & 7u; }

    SR_HD void init_network(Out&, u32&) const {}
    SR_HD void on_start(u64*, u32 id, Out& out) const {
        // servers: Value::default(); clients: RegisterActor::Client::on_start (register.rs:130-160)
        if (id >= S && id < S + C) out.send(id % S, msg(PUT, id, id - S + 1));  // Put(1 x id, 'A' + index)
    }
    SR_HD bool on_msg(u64* o, u32 id, u32 src, u32 m, Out& out) const {
        const u32 kind = m >> 12, req = m >> 4 & 255;
        if (id >= S) {  // RegisterActor::Client::on_msg (register.rs:170-200): the phase is the awaited reply
            const u32 ph = hs().phase(o[1], o[2], id - S);
            if (ph == 0 && kind == PUTOK && req == id) {
                out.send((id + 1) % S, msg(GET, 2 * id, 0));  // Get((op_count + 1) x id) to (id + op_count) % S
                return true;
            }
            return ph == 1 && kind == GETOK && req == 2 * id;
        }
        // SingleCopyActor::on_msg (examples/single-copy-register.rs:26-37)
        if (kind == PUT) {
            o[0] = (o[0] & ~(7ull << (3 * id))) | (u64)(m & 7) << (3 * id);  // `*state.to_mut() = value`
            out.send(src, msg(PUTOK, req, 0));
            return true;
        }
        if (kind == GET) {
            out.send(src, msg(GETOK, req, value(o, id)));
            return false;
        }
        return false;
    }
    SR_HD bool on_timeout(u64*, u32, Out&) const { return false; }
    // RegisterMsg::record_returns / record_invocations (src/actor/register.rs:37-87) on the history
    // field: PutOk returns WriteOk and the client's Get invocation follows in the same delivery (its
    // `last` vector: every other client's completed ops); GetOk(v) returns ReadOk(v).
    SR_HD void record_in(u64* o, u32, u32 dst, u32 m) const {
        const u32 kind = m >> 12;
        if (dst < S || (kind != PUTOK && kind != GETOK)) return;
        const u32 c = dst - S;
        const PaxosHist h = hs();
        u64 lo = o[1], hi = o[2];
        const u32 ph = h.phase(lo, hi, c);
        if (kind == PUTOK) {
            h.record_get(lo, hi, c);
        } else {
            PaxosHist::put(lo, hi, h.ret_off(c), 3, m & 7);
        }
        PaxosHist::put(lo, hi, 2 * c, 2, ph + 1);
        o[1] = lo;
        o[2] = hi;
    }
    SR_HD void record_out(u64*, u32, u32, u32) const {}  // the Puts at start: phase 0; Gets: in record_in
    SR_HD bool within_boundary(const u64*) const { return true; }
    SR_HD bool discovers(int p, const u64* s, const u32* net) const {
        if (p == 0) return !hs().linearizable(s[1], s[2]);  // always "linearizable"
        bool any = false;                                   // sometimes "value chosen"
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u32 e = net[k];
            any |= e != EMPTY && (e_msg(e) >> 12) == GETOK && (e & 7) != 0;
        }
        return any;
    }
    int expectation(int p) const { return p == 0 ? ALWAYS : SOMETIMES; }
    const char* prop_name(int p) const { return p == 0 ? "linearizable" : "value chosen"; }
    // the oracle's msg code (AbdSys::msg_code with seq (0, Id(0))): ((req * 512 + val) * 8 + kind)
    i64 msg_code(u32 m) const { return ((i64)(m >> 4 & 255) * 512 + (i64)(m & 7)) * 8 + (i64)(m >> 12); }
    u32 msg_decode(i64 code) const { return msg((u32)(code % 8), (u32)(code / 4096), (u32)(code / 8 % 512)); }
    std::string format_msg(i64 code) const { return AbdSys{}.format_msg(code); }
    int actors_width() const { return (int)(2 * (S + C)); }
    int history_width() const { return hs().width(); }
    // oracle/actor.hpp SingleCopySys::describe_actor: server [value, 0]; client [awaiting, op_count]
    int describe_fields(const u64* s, i64* d) const {
        int k = 0;
        for (u32 id = 0; id < S + C; ++id) {
            if (id < S) {
                d[k++] = value(s, id);
                d[k++] = 0;
            } else {
                const u32 ph = hs().phase(s[1], s[2], id - S);
                d[k++] = ph == 0 ? (i64)id : ph == 1 ? (i64)(2 * id) : -1;
                d[k++] = (i64)ph + 1;
            }
        }
        hs().describe(s[1], s[2], d + k);
        return k + history_width();
    }
    int undescribe_fields(const i64* d, u64* s) const {
        int k = 0;
        u32 phases[px::MAX_CLIENTS];
        for (u32 id = 0; id < S + C; ++id, k += 2) {
            if (id < S) s[0] |= (u64)(d[k] & 7) << (3 * id);
            else phases[id - S] = (u32)(d[k + 1] - 1);
        }
        hs().undescribe(d + k, phases, s[1], s[2]);
        return k + history_width();
    }
};

}  // namespace act

using PingPong = act::ActorGpu<act::PingPongSysT<16>>;      // max_nat <= 7
using PingPongWide = act::ActorGpu<act::PingPongSysT<32>>;  // max_nat 8..=14
using ActorFixture = act::ActorGpu<act::FixtureSys>;
using AbdRegister = act::ActorGpu<act::AbdSys>;
using SingleCopyRegister = act::ActorGpu<act::SingleCopySys>;

}  // namespace sr
