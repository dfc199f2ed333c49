// The compiled-in GpuModel registry, split into families that compile as separate translation units
// (reg_*.hip, built in parallel by stateright_amd/build.py and linked into libstateright_gpu.so).
// Each family instantiates the single-GPU Engine<M> and the partitioned DistEngine<M> for its
// models; engine.hip maps a model id (SR_MODEL_*) to its family.
#pragma once
#include <memory>

#include "engine.hpp"
#include "dist.hpp"

namespace sr {

// What a spawn asks for: the model's integer parameters and options, and for the partitioned
// search its communicator (or none) and virtual partitions.
struct EngineArgs {
    int model;
    const i64* p;
    int np;
    const sr_opts* o;
    bool dist;
    Comm* comm;
    int vparts;
    void need(int k) const {
        if (np < k) throw Error(SR_ERR_ARG, "model " + std::to_string(model) + " needs " + std::to_string(k) + " params");
    }
};

// Engine<M> or DistEngine<M>. EV: a model with `eventually` properties runs partitioned as
// EvBits<M> (models.hpp).
template <class M, bool EV = false>
std::unique_ptr<EngineBase> make_for(const M& m, const EngineArgs& a) {
    if (!a.dist) return std::make_unique<Engine<M>>(m, *a.o);
    if constexpr (EV && has_emask<M>::value) {
        if (model_emask(m)) return std::make_unique<DistEngine<EvBits<M>>>(EvBits<M>(m), *a.o, a.comm, a.vparts);
    }
    return std::make_unique<DistEngine<M>>(m, *a.o, a.comm, a.vparts);
}

// One function per family (reg_<family>.hip): the engine of a.model.
std::unique_ptr<EngineBase> reg_basic(const EngineArgs& a);           // LinearEquation, BinaryClock, DGraph, actor fixtures
std::unique_ptr<EngineBase> reg_two_phase(const EngineArgs& a);       // 2pc (and its canonical reduction)
std::unique_ptr<EngineBase> reg_increment(const EngineArgs& a);       // increment
std::unique_ptr<EngineBase> reg_increment_lock(const EngineArgs& a);  // increment_lock
std::unique_ptr<EngineBase> reg_paxos(const EngineArgs& a);           // paxos, 1-4 clients (W = 11)
std::unique_ptr<EngineBase> reg_paxos_wide(const EngineArgs& a);      // paxos, 5-6 clients (W = 12)
std::unique_ptr<EngineBase> reg_ping_pong(const EngineArgs& a);       // ping-pong
std::unique_ptr<EngineBase> reg_registers(const EngineArgs& a);       // ABD and the single-copy register

}  // namespace sr
