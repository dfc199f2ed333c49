// Registry family: increment_lock (registry.hpp).
#include "registry.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_increment_lock(const EngineArgs& a) {
    a.need(1);
    const i64 n = a.p[0];
    if (n < 1 || n > 12) throw Error(SR_ERR_UNSUPPORTED, "increment_lock: threads must be in 1..=12");
    if (n <= 8) return make_for(IncrementLock<1>{(int)n}, a);
    return make_for(IncrementLock<2>{(int)n}, a);
}
}  // namespace sr
