// Registry family: increment (registry.hpp).
#include "registry.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_increment(const EngineArgs& a) {
    a.need(1);
    const i64 n = a.p[0];
    if (n < 1 || n > 15) throw Error(SR_ERR_UNSUPPORTED, "increment: threads must be in 1..=15");
    if (n <= 9) return make_for(Increment<1>{(int)n}, a);
    return make_for(Increment<2>{(int)n}, a);
}
}  // namespace sr
