// Registry family: paxos with 5-6 clients, W = 12 (registry.hpp).
#include "registry.hpp"
#include "paxos.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_paxos_wide(const EngineArgs& a) { return make_for(PaxosWide::make((int)a.p[0]), a); }
}  // namespace sr
