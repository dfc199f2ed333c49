// GpuModel for the reference's test fixture `DGraph` (src/test_util.rs:47-116): a directed graph
// over u8 states given as paths from initial states, with ONE property "odd" (s % 2 == 1) whose
// expectation is a parameter — the fixture the reference uses for `eventually` properties
// (src/checker.rs:349-414).
//
// Encoding: the state is the node (W = 1). `actions(s)` is the BTreeSet of s's successors in
// ascending order, so action slot a IS the destination node a: enabled(s) = the 256-bit
// adjacency row of s (MW = 4) and apply(s, a) = a (`next_state` is always Some(action)).
// Params (shared with the CPU oracle, oracle/capi.cpp make_dgraph):
//   [expectation (0 always, 1 eventually, 2 sometimes), len0, v.., len1, v.., ...]
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/stateright_gpu.h"
#include "device.hpp"
#include "models.hpp"

namespace sr {
namespace dg {

struct Tables {
    int expectation = EVENTUALLY;
    std::vector<u64> adj;    // [256][4] adjacency bitsets
    std::vector<u8> inits;   // ascending (BTreeSet)
    std::map<int, u64*> dev;  // device copies of adj (process lifetime)
};

inline Tables parse(const i64* p, int np) {
    if (np < 1) throw Error(SR_ERR_ARG, "dgraph: needs (expectation, paths...)");
    Tables t;
    if (p[0] < 0 || p[0] > 2) throw Error(SR_ERR_ARG, "dgraph: expectation must be 0, 1 or 2");
    t.expectation = p[0] == 0 ? ALWAYS : p[0] == 1 ? EVENTUALLY : SOMETIMES;
    t.adj.assign(256 * 4, 0);
    bool init[256] = {};
    for (int i = 1; i < np;) {  // DGraph::with_path (src/test_util.rs:68-86)
        const i64 len = p[i++];
        if (len < 1 || i + len > np) throw Error(SR_ERR_ARG, "dgraph: malformed path list");
        for (i64 k = 0; k < len; ++k)
            if (p[i + k] < 0 || p[i + k] > 255) throw Error(SR_ERR_ARG, "dgraph: nodes are u8");
        u32 src = (u32)p[i];
        init[src] = true;
        for (i64 k = 1; k < len; ++k) {
            const u32 dst = (u32)p[i + k];
            t.adj[src * 4 + dst / 64] |= 1ull << (dst % 64);
            src = dst;
        }
        i += (int)len;
    }
    for (int v = 0; v < 256; ++v)
        if (init[v]) t.inits.push_back((u8)v);
    return t;
}

inline Tables& tables(const i64* p, int np, int device) {
    static std::mutex mu;
    static std::map<std::vector<i64>, std::unique_ptr<Tables>> cache;
    std::lock_guard<std::mutex> g(mu);
    auto& t = cache[std::vector<i64>(p, p + np)];
    if (!t) t = std::make_unique<Tables>(parse(p, np));
    if (device >= 0 && !t->dev.count(device)) {
        int prev = 0;
        SR_HIP(hipGetDevice(&prev));
        SR_HIP(hipSetDevice(device));
        u64* d = nullptr;
        SR_HIP(hipMalloc(&d, t->adj.size() * sizeof(u64)));
        SR_HIP(hipMemcpy(d, t->adj.data(), t->adj.size() * sizeof(u64), hipMemcpyHostToDevice));
        SR_HIP(hipSetDevice(prev));
        t->dev[device] = d;
    }
    return *t;
}

}  // namespace dg

struct DGraph {
    static constexpr int W = 1, MW = 4, NPROPS = 1;
    int expect = EVENTUALLY;
    int max_deg = 0;
    const u64* adj_d = nullptr;
    const u64* adj_h = nullptr;
    const dg::Tables* host = nullptr;

    static DGraph make(const i64* p, int np, int device) {
        dg::Tables& t = dg::tables(p, np, device);
        DGraph m;
        m.expect = t.expectation;
        m.adj_d = device >= 0 ? t.dev.at(device) : nullptr;
        m.adj_h = t.adj.data();
        m.host = &t;
        for (int v = 0; v < 256; ++v) {
            int d = 0;
            for (int w = 0; w < 4; ++w) d += __builtin_popcountll(t.adj[v * 4 + w]);
            m.max_deg = std::max(m.max_deg, d);
        }
        return m;
    }
    SR_HD const u64* adj() const {
#if defined(__HIP_DEVICE_COMPILE__)
        return adj_d;
#else
        return adj_h;
#endif
    }
    int max_actions() const { return 256; }
    int max_out_degree() const { return std::max(1, max_deg); }
    u32 emask() const { return expect == EVENTUALLY ? 1u : 0u; }
    SR_HD void enabled(const u64* s, u64* m) const {
        const u64* row = adj() + (s[0] & 255) * 4;
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] = row[w];
    }
    SR_HD bool apply(const u64*, int a, u64* o) const {
        o[0] = (u64)a;
        return true;
    }
    // always: a violation; sometimes: an example; eventually: the condition holds here (clears
    // the property's bit on the path, src/checker/bfs.rs:212-222).
    SR_HD bool discovers(int, const u64* s) const {
        const bool odd = (s[0] & 1) != 0;
        return expect == ALWAYS ? !odd : odd;
    }
    int init_states(u64* out) const {
        int k = 0;
        for (u8 v : host->inits) out[k++] = v;
        return k;
    }
    int expectation(int) const { return expect; }
    const char* prop_name(int) const { return "odd"; }
    int describe_width() const { return 1; }
    void describe(const u64* s, i64* d) const { d[0] = (i64)(s[0] & 255); }
    i64 action_id(const u64*, int a) const { return a; }
    i64 action_id_bound() const { return 256; }
    std::string action_name(i64 id) const { return std::to_string(id); }
};

}  // namespace sr
