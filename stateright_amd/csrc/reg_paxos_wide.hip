// Registry family: paxos with 5-6 clients, W = 12 (registry.hpp).
#include "registry.hpp"
#include "paxos.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_paxos_wide(const EngineArgs& a) {
    // The engine of the bench configuration (the reference's bench.sh `paxos check 6`) with the
    // client count compiled in (PaxosT<W, CC>); SR_PAXOS_GENERIC=1: the runtime-count engine (A/B).
    if (a.p[0] == 6 && !std::getenv("SR_PAXOS_GENERIC")) return make_for(PaxosT<12, 6>::make(6), a);
    return make_for(PaxosWide::make((int)a.p[0]), a);
}
}  // namespace sr
