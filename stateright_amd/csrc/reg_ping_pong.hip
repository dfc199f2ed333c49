// Registry family: the ping-pong actor system (registry.hpp).
#include "registry.hpp"
#include "actor.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_ping_pong(const EngineArgs& a) {
    a.need(1);
    const i64* p = a.p;
    if (p[0] < 0 || p[0] > (i64)PingPongWide::MAX_NAT)
        throw Error(SR_ERR_UNSUPPORTED, "ping-pong: max_nat must be in 0..=14 (32 network slots)");
    auto fill = [&](auto& m) {
        m.max_nat = (u32)p[0];
        m.lossy = a.np > 1 && p[1] != 0;
        m.duplicating = a.np > 2 ? p[2] != 0 : true;
        m.maintains_history = a.np > 3 && p[3] != 0;
    };
    if (p[0] <= (i64)PingPong::MAX_NAT) {  // 16 slots, 9-word states
        PingPong m;
        fill(m);
        return make_for<PingPong, true>(m, a);
    }
    PingPongWide m;  // 32 slots, 17-word states
    fill(m);
    return make_for<PingPongWide, true>(m, a);
}
}  // namespace sr
