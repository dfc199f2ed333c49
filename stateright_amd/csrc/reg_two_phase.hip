// Registry family: 2pc and its canonical (symmetry) reduction (registry.hpp).
#include "registry.hpp"

namespace sr {
// 2pc's owner key for the partitioned search (TwoPhase::okey_rms): the tuples of this many RMs.
// More RMs balance the partitions better, fewer keep more successors local (DESIGN.md §6 measures
// the trade-off). SR_OWNER_RMS overrides it; 0 owns states by fingerprint.
// Round 6 (multiplicative owner hash, profiles/r06_config4_stages.txt), config 4 per-rank critical
// path: T = 8: 4 RMs 10.85 ms, 3: 13.24, 5: 11.66; T = 4: 4 RMs 18.73, 5: 19.63; T = 2: 4 RMs 35.03,
// 5: 33.45 (two partitions need the finer key for balance).
static int two_phase_owner_rms(int n, int parts) {
    if (const char* e = std::getenv("SR_OWNER_RMS")) return std::max(0, std::min(n, std::atoi(e)));
    if (n <= 7) return (n + 1) / 2;
    return parts == 2 ? std::min(n, 5) : 4;
}

std::unique_ptr<EngineBase> reg_two_phase(const EngineArgs& a) {
    a.need(1);
    const i64 n = a.p[0];
    if (n < 1 || n > 14) throw Error(SR_ERR_UNSUPPORTED, "2pc: rm_count must be in 1..=14 (4n+4 <= 63 bits)");
    const int parts = !a.dist ? 1 : a.comm ? a.comm->world : a.vparts;
    const TwoPhase m{(int)n, two_phase_owner_rms((int)n, parts)};
    if (a.o->symmetry) return make_for(Canon<TwoPhase>(m), a);
    // The engines of the bench configurations with the rm count compiled in (TwoPhaseT<NC>: the
    // per-rm loops unroll with constant shifts): BASELINE configs[2] (N = 9, 10) on one GPU and
    // partitioned (the multi-GPU headline), configs[3] (N = 11) partitioned and on one GPU.
    // SR_2PC_GENERIC=1: the runtime-n engine (A/B).
    if (!std::getenv("SR_2PC_GENERIC")) {
        if (n == 9) return make_for(TwoPhaseT<9>{9, m.okey_rms}, a);
        if (n == 10 && !a.dist) return make_for(TwoPhaseT<10>{10, m.okey_rms}, a);
        if (n == 11) return make_for(TwoPhaseT<11>{11, m.okey_rms}, a);
    }
    return make_for(m, a);
}
}  // namespace sr
