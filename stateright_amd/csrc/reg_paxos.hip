// Registry family: paxos with 1-4 clients, W = 11 (registry.hpp).
#include "registry.hpp"
#include "paxos.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_paxos(const EngineArgs& a) {
    // The engine of the bench configuration (BASELINE configs[4], `paxos check 3`) with the client
    // count compiled in (PaxosT<W, CC>); SR_PAXOS_GENERIC=1: the runtime-count engine (A/B).
    if (a.p[0] == 3 && !std::getenv("SR_PAXOS_GENERIC")) return make_for(PaxosT<11, 3>::make(3), a);
    return make_for(Paxos::make((int)a.p[0]), a);
}
}  // namespace sr
