// The partitioned search's host protocol run WITHOUT a GPU: every rank is a
// process on the shared-memory transport (ShmComm in host mode), and the host code the pipelined
// engine runs between its kernels -- the level rows (RowField), their error precedence
// (throw_row_errors), the bucket plan (LevelPlan), the outcome vote (outcome_of,
// decide_after_vote) and the transport's collectives -- is driven by a CPU stand-in for the
// device side: each rank expands the frontier it owns (2pc, the GpuModel's own host-callable
// enabled / apply / part_of), routes the successors it does not own as records to their owner
// through the transport's exchange, with the direct exchange's per-slot checksum, and publishes
// its row of the level. tests/test_dist_host_protocol.py runs it in two processes.
//
// Faults are injected where the device would raise them: a bucket over the planned capacity
// (ERR_FRONTIER_OVERFLOW in the sender's row), a record altered after its source checksummed it
// (ERR_EXCHANGE in the owner's row one level later, or, for the last exchange, in the owner's own
// check only), and a capacity or other error that one rank alone sees at the end of a check.
#pragma once
#include <unordered_set>

#include "dist.hpp"

namespace sr {

struct DistHostRun {
    ShmComm& comm;
    TwoPhase m;
    sr_dist_host_opts o;
    sr_dist_host_result r{};
    u32 T, me;
    bool synchronous = false;  // after a capacity restart: exact bucket sizes (no plan)
    bool direct = true;        // the direct exchange (checksummed slots); false after a fallback
    int injected_corrupt = 0, injected_capacity = 0, injected_error = 0;  // each fault fires once

    DistHostRun(ShmComm& c, const sr_dist_host_opts& opts) : comm(c), o(opts) {
        m.n = o.rm_count;
        T = (u32)c.world;
        me = (u32)c.rank;
    }

    static u64 mix(u64 h, u64 v) { return fmix64(h ^ (v + 0x9E3779B97F4A7C15ull)); }

    // One check: the level loop of the pipelined engine with the CPU stand-in for its kernels.
    void run_once() {
        constexpr u32 NP = TwoPhase::NPROPS;
        const size_t RW = row_words(T, NP);
        std::unordered_set<u64> visited;  // this partition's share of the visited set
        std::vector<u64> frontier;
        LevelPlan lp;
        lp.n_last.assign(T, 1);
        lp.n_hi.assign(T, 1);
        lp.growth = (double)std::min(m.max_out_degree(), 32);
        u64 unique = 0, state_count = 0;
        u32 depth = 0, level = 0;
        std::vector<u64> row(RW, 0), all(RW * T, 0);
        // level 0: the init states this partition owns
        u64 init[1];
        m.init_states(init);
        if (part_of(m, init, state_fp<TwoPhase>(init), T) == me && visited.insert(init[0]).second) frontier.push_back(init[0]);
        row[T + ROW_N] = row[T + ROW_ROOTS] = frontier.size();
        // The owner's check of an exchange reaches the rows one level later (the insert's err word
        // persists into the NEXT level's rows, which every rank reads); the last exchange's check is
        // in no row and is read by its owner alone where the search ends.
        u64 pending = 0;
        for (;; ++level) {
            for (u32 p = 0; p < NP; ++p) row[T + ROW_DISC + p] = ~0ull;
            comm.all_gather(row.data(), all.data(), RW, nullptr);
            const LevelPlan::Sums sm = LevelPlan::sums(all.data(), T, RW);
            throw_row_errors(sm.err, level);
            lp.absorb(all.data(), T, RW, sm);
            if (level == 0) unique = state_count = sm.roots;  // init states are counted (bfs.rs:43-66)
            else unique += sm.n, state_count += sm.succ;
            if (sm.n == 0) {
                throw_row_errors(pending & ERR_EXCHANGE, level);  // the owner's own check
                break;
            }
            depth = level;
            // ---- the level's expansion (expand_route's work on this partition) ----
            const u64 C = synchronous ? ~0ull : lp.bucket_cap(lp.have_rows ? 2 : 1, o.cmin) / (u64)std::max(1, o.plan_div);
            r.plan_digest = mix(r.plan_digest, synchronous ? 0 : C);
            std::vector<std::vector<u64>> rec(T);
            std::vector<u64> next;
            u64 succ = 0, enabled = 0, local = 0, err = 0;
            for (u64 s : frontier) {
                u64 mk[TwoPhase::MW];
                m.enabled(&s, mk);
                for (int w = 0; w < TwoPhase::MW; ++w)
                    for (u64 bits = mk[w]; bits; bits &= bits - 1) {
                        u64 ns;
                        ++enabled;
                        if (!m.apply(&s, w * 64 + __builtin_ctzll(bits), &ns)) continue;
                        ++succ;
                        if (ns == s) continue;  // a self-loop: counted, never routed
                        const u32 q = part_of(m, &ns, state_fp<TwoPhase>(&ns), T);
                        if (q == me) {
                            if (visited.insert(ns).second) next.push_back(ns), ++local;
                        } else if (rec[q].size() < C) {
                            rec[q].push_back(ns);
                        } else {
                            err |= ERR_FRONTIER_OVERFLOW;  // the bucket is full: the record is lost
                        }
                    }
            }
            // ---- the exchange: records and their per-slot checksums ----
            std::vector<u64> scount(T), sums(T), rcount(T);
            for (u32 q = 0; q < T; ++q) {
                scount[q] = rec[q].size();
                u64 x = 0;
                for (u64 v : rec[q]) x += v;
                sums[q] = x;
            }
            std::vector<u64> all_counts((size_t)T * T), all_sums((size_t)T * T);
            comm.all_gather(scount.data(), all_counts.data(), T, nullptr);
            comm.all_gather(sums.data(), all_sums.data(), T, nullptr);
            for (u32 q = 0; q < T; ++q) rcount[q] = all_counts[(size_t)q * T + me];
            std::vector<std::vector<u64>> got(T);
            std::vector<const u64*> sp(T);
            std::vector<u64*> rp(T);
            for (u32 q = 0; q < T; ++q) {
                got[q].resize(rcount[q] + 1);
                sp[q] = rec[q].data();
                rp[q] = got[q].data();
            }
            comm.exchange(sp, scount, rp, rcount, nullptr);
            // a record altered in transit after its source summed it (SR_DX_CORRUPT_LEVEL's analogue)
            const bool corrupt_here = direct && !injected_corrupt && (int)level == o.corrupt_level;
            u64 exchange_err = 0;
            for (u32 q = 0; q < T; ++q) {
                if (corrupt_here && q != me && !injected_corrupt) {
                    // a record, or (a slot without records) the header's checksum word, read stale
                    if (rcount[q]) got[q][0] ^= 1ull << 3;
                    else all_sums[(size_t)q * T + me] ^= 1;
                    injected_corrupt = 1;
                }
                u64 x = 0;
                for (u64 i = 0; i < rcount[q]; ++i) x += got[q][i];
                if (direct && x != all_sums[(size_t)q * T + me]) exchange_err |= ERR_EXCHANGE;
                for (u64 i = 0; i < rcount[q]; ++i)
                    if (visited.insert(got[q][i]).second) next.push_back(got[q][i]);
            }
            // ---- this partition's row of the next level; the owner reports its exchange check
            // there, so every rank acts on it at the same level ----
            for (u32 q = 0; q < T; ++q) row[q] = scount[q];
            row[T + ROW_N] = next.size();
            row[T + ROW_SUCC] = succ;
            row[T + ROW_LOCAL] = local;
            row[T + ROW_ERR] = err | pending;
            pending = exchange_err;
            row[T + ROW_ENABLED] = enabled;
            row[T + ROW_ROOTS] = 0;
            if (err && r.overflow_level == ~0u) r.overflow_level = level;
            frontier.swap(next);
        }
        r.unique = unique;
        r.state_count = state_count;
        r.max_depth = depth;
        r.levels = level;
        r.local_unique = visited.size();
        // faults that one rank alone sees once its search has ended
        if (!injected_capacity && o.capacity_fail_at_end) {
            injected_capacity = 1;
            throw Error(SR_ERR_CAPACITY, "injected: this rank's arena ran out at the end of the check");
        }
        if (!injected_error && o.fail_at_end) {
            injected_error = 1;
            throw Error(SR_ERR_ARG, "injected: this rank failed at the end of the check");
        }
    }

    // DistEngine::run's attempt loop: every rank votes on the outcome of each attempt.
    int run() {
        r.overflow_level = ~0u;
        for (int attempt = 0;; ++attempt) {
            int code = OUT_OK, ecode = 0;
            std::string what;
            try {
                r.plan_digest = 0;
                run_once();
            } catch (const Error& e) {
                code = outcome_of(e.code);
                ecode = e.code;
                what = e.what();
            }
            if (attempt == 0) r.first_outcome = (u32)code;
            u64 v[2] = {(u64)code, ~(u64)code};  // max and min of the ranks' outcomes
            comm.all_reduce(v, 2, RedOp::Max, nullptr);
            ++r.attempts;
            const VoteDecision d = decide_after_vote(code, (int)v[0], (int)~v[1], attempt, ecode, what);
            if (d.act == VoteAction::Done) return SR_OK;
            if (d.act == VoteAction::Fail) throw Error(d.code, d.why);
            if (d.act == VoteAction::Fallback) {
                ++r.fallbacks;
                direct = false;  // the collective exchange from now on
                continue;
            }
            ++r.restarts;
            if (d.disagree) ++r.disagreements;
            if (!synchronous) synchronous = true;  // the plan under-estimated: exact buckets
        }
    }
};

}  // namespace sr
