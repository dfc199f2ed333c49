// Registry family: LinearEquation, BinaryClock, DGraph and the one-actor fixtures (registry.hpp).
#include "registry.hpp"
#include "dgraph.hpp"
#include "actor.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_basic(const EngineArgs& a) {
    const i64* p = a.p;
    switch (a.model) {
        case SR_MODEL_LINEAR_EQUATION:
            a.need(3);
            return make_for(LinearEquation{(u32)(p[0] & 0xff), (u32)(p[1] & 0xff), (u32)(p[2] & 0xff)}, a);
        case SR_MODEL_BINARY_CLOCK:
            return make_for(BinaryClock{}, a);
        case SR_MODEL_DGRAPH:
            return make_for<DGraph, true>(DGraph::make(p, a.np, a.o->device), a);
        case SR_MODEL_ACTOR_FIXTURE: {
            a.need(1);
            if (p[0] < 0 || p[0] > 1) throw Error(SR_ERR_ARG, "actor fixture: kind 0 (undeliverable) or 1 (timer)");
            ActorFixture m;
            m.kind = (int)p[0];
            return make_for(m, a);
        }
    }
    return nullptr;
}
}  // namespace sr
