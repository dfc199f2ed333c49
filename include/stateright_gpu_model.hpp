/*
 * stateright_gpu_model.hpp — write a GpuModel and build it into a plugin for the MI355X engine.
 *
 * The reference checks any `impl Model` (src/lib.rs:155-237). Device code cannot call host
 * closures, so a model for the GPU engine is a C++ struct, the GpuModel concept, compiled with
 * hipcc together with the engine templates this header brings in; the result is a shared library
 * that the engine library (include/stateright_gpu.h, sr_gpu_bfs_spawn_plugin) runs like a
 * registered model. A GpuModel M provides (models in stateright_amd/csrc/models.hpp):
 *
 *   static constexpr int W, MW, NPROPS;      words per state, 64-bit words of the action mask, properties
 *   int max_actions(), max_out_degree();     action slots (`actions()` positions), max successors
 *   SR_HD void enabled(const u64* s, u64* m);           bit a: slot a is listed by `actions(s)`
 *   SR_HD bool apply(const u64* s, int a, u64* out);    `next_state(s, a)` is Some and within boundary
 *   SR_HD bool discovers(int p, const u64* s);           always: !condition; sometimes/eventually: condition
 *   host: init_states(u64*) -> count, expectation(p), prop_name(p), describe_width(), describe(s, i64*),
 *         action_id(s, a), action_name(id), action_id_bound()
 *         init_states writes at most 256 states (sr::MAX_INIT_STATES) unless the model reports its
 *         count with init_count(); the engine checks the count once at spawn (SR_ERR_ARG)
 *   optional: init_count()                    the number of init states (any count; the engine sizes
 *                                             its host buffers from it)
 *             undescribe(const i64*, u64*)    (sr_plugin.fingerprint)
 *             emask()                         (the mask of `eventually` properties)
 *             qkey_bits(), SR_HD qkey(s)      (exact quotient visited set for multi-word states)
 *             SR_HD self_loops(s, enabled, out)   out = enabled slots whose next_state is s itself:
 *                                             FAST expansion counts them (state_count) without
 *                                             generating them. Every slot reported must be a
 *                                             self-loop; an unreported one is still detected
 *                                             (2pc reports all of them: 37% of successors)
 *             SR_HD canonical(s, out)         a canonical representative under the model's symmetry
 *                                             (the opt-in symmetry_canonical reduction)
 *
 * Equal states must have equal words (the words ARE the state), and slots are enumerated in the
 * reference's `actions()` order, so FIFO runs reproduce the reference's visit order and paths.
 *
 *   #include "stateright_gpu_model.hpp"
 *   struct MyModel { ... };
 *   MyModel make_my_model(const int64_t* params, int32_t nparams, int device) { ... }
 *   SR_GPU_PLUGIN(my_model, MyModel, make_my_model)
 *
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I<repo>/include my_model.hip \
 *         -o libmy_model.so -L/opt/rocm/lib -lrccl
 *
 * `make` builds the model from integer parameters (device < 0: host-only use, e.g. fingerprints)
 * and may throw sr::Error(SR_ERR_ARG, "...") for bad parameters. examples/plugins/sliding_puzzle.hip
 * is a complete example (the sliding puzzle of the reference's crate documentation, src/lib.rs:40-116).
 */
#ifndef STATERIGHT_GPU_MODEL_HPP
#define STATERIGHT_GPU_MODEL_HPP

#include "stateright_gpu.h"
#include "../stateright_amd/csrc/engine.hpp"

#define SR_GPU_PLUGIN(NAME, MODEL, MAKE)                                                                    \
    extern "C" const sr_plugin* sr_plugin_##NAME(void) {                                                    \
        static const sr_plugin p = {                                                                        \
            SR_PLUGIN_ABI, (uint32_t)sizeof(sr_opts), #NAME,                                                \
            [](const int64_t* a, int32_t n, const sr_opts* o, void* c, int32_t v, char* e, int32_t cap) -> void* { \
                return ::sr::plugin_create<MODEL>(MAKE, a, n, o, c, v, e, cap);                           \
            },                                                                                              \
            [](const int64_t* a, int32_t n, const int64_t* d, int32_t w, uint64_t* fp) -> int32_t {         \
                return ::sr::plugin_fingerprint<MODEL>(MAKE, a, n, d, w, fp);                             \
            }};                                                                                             \
        return &p;                                                                                          \
    }

#endif /* STATERIGHT_GPU_MODEL_HPP */
