// Registry family: paxos with 5-6 clients, W = 12 (registry.hpp). The client count stays a runtime
// value here: compiled in (PaxosT<12, 6>) the unrolled per-client loops spill ~150 VGPRs to scratch
// and bench.sh's `paxos check 6` took 4.44 ms instead of 3.01 (profiles/r05_compiled_params.txt).
#include "registry.hpp"
#include "paxos.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_paxos_wide(const EngineArgs& a) {
#ifdef SR_PX6_CC
    if (a.p[0] == 6 && !std::getenv("SR_PAXOS_GENERIC")) return make_for(PaxosT<12, 6>::make(6), a);
#endif
    return make_for(PaxosWide::make((int)a.p[0]), a);
}
}  // namespace sr
