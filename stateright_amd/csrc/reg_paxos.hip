// Registry family: paxos with 1-4 clients, W = 11 (registry.hpp).
#include "registry.hpp"
#include "paxos.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_paxos(const EngineArgs& a) { return make_for(Paxos::make((int)a.p[0]), a); }
}  // namespace sr
