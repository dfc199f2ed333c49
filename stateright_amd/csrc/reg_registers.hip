// Registry family: the ABD linearizable register and the single-copy register (registry.hpp).
#include "registry.hpp"
#include "actor.hpp"

namespace sr {
std::unique_ptr<EngineBase> reg_registers(const EngineArgs& a) {
    a.need(1);
    const i64* p = a.p;
    if (a.model == SR_MODEL_ABD) {
        AbdRegister m;
        static_cast<act::AbdSys&>(m) = act::AbdSys::make((int)p[0], a.np > 1 ? (int)p[1] : 2, a.o->device);
        return make_for(m, a);
    }
    SingleCopyRegister m;
    static_cast<act::SingleCopySys&>(m) = act::SingleCopySys::make((int)p[0], a.np > 1 ? (int)p[1] : 1);
    return make_for(m, a);
}
}  // namespace sr
