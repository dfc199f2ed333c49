/*
 * stateright_gpu.h — C ABI of the MI355X breadth-first model-checking engine.
 *
 * This is the drop-in boundary for Stateright's `CheckerBuilder::spawn_bfs` path. Each entry point
 * replaces one piece of the reference's Rust interface (crate `stateright` 0.28.0, paths relative to
 * the reference repository):
 *
 *   sr_gpu_bfs_spawn              <- CheckerBuilder::spawn_bfs        src/checker.rs:124-129
 *                                    BfsChecker::spawn                src/checker/bfs.rs:36-163
 *                                    (builder options threads/target_state_count/visitor:
 *                                     src/checker.rs:35-51,162-177, mirrored by sr_opts)
 *   sr_gpu_bfs_join               <- Checker::join                    src/checker/bfs.rs:300-305
 *   sr_gpu_bfs_is_done            <- Checker::is_done                 src/checker/bfs.rs:307-311
 *   sr_gpu_bfs_state_count        <- Checker::state_count             src/checker/bfs.rs:283-285
 *   sr_gpu_bfs_unique_state_count <- Checker::unique_state_count      src/checker/bfs.rs:287
 *   sr_gpu_bfs_max_depth          <- (new: BFS depth metric, SURVEY.md §5 "no depth metric")
 *   sr_gpu_bfs_property_*         <- Model::properties / Property     src/lib.rs:214-300
 *   sr_gpu_bfs_discovery          <- discoveries() + reconstruct_path src/checker/bfs.rs:289-298,314-342
 *   sr_gpu_bfs_discovery_path     <- Path::from_fingerprints          src/checker/path.rs:20-86
 *   sr_gpu_bfs_replay             <- Path::from_actions (assert_discovery) src/checker/path.rs:90-112,
 *                                                                     src/checker.rs:292-337
 *   sr_gpu_bfs_visits             <- StateRecorder visitor            src/checker/visitor.rs:70-99
 *   sr_gpu_bfs_visit_tree         <- PathRecorder / Fn(Path) visitors src/checker/visitor.rs:19-66,
 *                                                                     src/checker/bfs.rs:187-189
 *   sr_gpu_bfs_free               <- Drop of the checker (join(self) consumes it in Rust)
 *   sr_last_error                 <- the reference panics; see "Errors" below
 *   sr_dist_* / sr_gpu_bfs_spawn_partitioned <- new: the visited set partitioned over GPUs
 *
 * Models: device code cannot call host function pointers, so `impl Model` becomes a registry of
 * compiled-in GpuModel encodings selected by `model_id` + integer parameters (SR_MODEL_*). Each
 * encoding packs one state into fixed-width 64-bit words and enumerates the reference's
 * `actions()` in order as action slots.
 *
 * Errors: the reference panics (zero fingerprint src/lib.rs:310, path nondeterminism
 * src/checker/path.rs:35-79, worker panics src/checker/bfs.rs:302). Here every call returns a
 * status (SR_OK or a negative SR_ERR_*) and sr_last_error() describes the last failure on the
 * calling thread.
 *
 * Threading: spawn returns immediately; the level loop runs on a host driver thread bound to one
 * HIP device. Counters are readable while it runs (like the reference's atomics).
 */
#ifndef STATERIGHT_GPU_H
#define STATERIGHT_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Model registry (params in parentheses). */
enum sr_model_id {
    SR_MODEL_LINEAR_EQUATION = 1, /* (a, b, c)      src/test_util.rs:140-188            */
    SR_MODEL_BINARY_CLOCK = 2,    /* ()             src/test_util.rs:4-45               */
    SR_MODEL_2PC = 3,             /* (rm_count<=14) examples/2pc.rs:10-121              */
    SR_MODEL_INCREMENT = 4,       /* (threads<=15)  examples/increment.rs:109-197       */
    SR_MODEL_INCREMENT_LOCK = 5,  /* (threads<=12)  examples/increment_lock.rs:3-107    */
    SR_MODEL_DGRAPH = 6,          /* (expectation, len, v.., len, v..) src/test_util.rs:47-116 */
    SR_MODEL_PAXOS = 7,           /* (client_count<=6) examples/paxos.rs:93-263 + src/actor/model.rs */
    /* ActorModel fixtures (src/actor/model.rs:176-327 over stateright_amd/csrc/actor.hpp): */
    SR_MODEL_PINGPONG = 9,        /* (max_nat<=14, lossy, duplicating, maintains_history)
                                     src/actor/actor_test_util.rs:4-96                     */
    SR_MODEL_ACTOR_FIXTURE = 10,  /* (kind: 0 undeliverable envelope, 1 timer) src/actor/model.rs:697-733 */
    SR_MODEL_ABD = 11,            /* (client_count<=3, server_count<=3) examples/linearizable-register.rs */
    SR_MODEL_SINGLE_COPY = 12     /* (client_count<=6, server_count; <=8 actors) examples/single-copy-register.rs */
};

/* Visit order inside a BFS level. */
enum sr_order {
    SR_ORDER_AUTO = 0, /* FAST; rerun as FIFO if an early exit makes counts order-dependent */
    SR_ORDER_FIFO = 1, /* exactly the single-threaded reference order (pop_back/push_front)   */
    SR_ORDER_FAST = 2  /* any order inside a level: wave-aggregated append, no ordering pass  */
};

enum sr_expectation { SR_ALWAYS = 0, SR_EVENTUALLY = 1, SR_SOMETIMES = 2 }; /* src/lib.rs:293-300 */

enum sr_status {
    SR_OK = 0,
    SR_ERR_ARG = -1,
    SR_ERR_HIP = -2,
    SR_ERR_CAPACITY = -3,
    SR_ERR_UNSUPPORTED = -4,
    SR_ERR_NO_DEVICE = -5,
    SR_ERR_NONDETERMINISM = -6
};

typedef struct sr_opts {
    uint32_t struct_size;        /* sizeof(sr_opts)                                              */
    int32_t device;              /* HIP device ordinal                                           */
    uint64_t target_state_count; /* 0 = None; `CheckerBuilder::target_state_count` checker.rs:164 */
    int32_t order;               /* enum sr_order                                                */
    int32_t record_visits;       /* keep every visited state (a StateRecorder visitor)           */
    uint64_t capacity_hint;      /* expected unique states; 0 = grow the visited table on demand */
    int32_t profile;             /* time every expand launch with HIP events                     */
    int32_t verbose;             /* per-level log lines on stderr                                */
    int32_t counters;            /* count visited-set probes and CAS attempts (sr_stats.probes/cas)
                                    with a counting variant of the expand kernel (slower)        */
    int32_t defer_paths;         /* partitioned search: 0 = at join, every rank gathers the states
                                    of every discovery path (collectively), so sr_gpu_bfs_discovery*
                                    work on any single rank afterwards; 1 = skip that at join and
                                    reconstruct on demand (then collective: every rank must call
                                    sr_gpu_bfs_discovery* for the same property in the same order).
                                    The reference's join reconstructs nothing either
                                    (src/checker/bfs.rs:289-298 builds paths in discoveries()). */
    int32_t symmetry;            /* 1 = canonical symmetry reduction (models with a canonical form:
                                    2pc, plugins with `canonical`): one state per orbit, order-
                                    independent counts; NOT the reference's DFS count, whose
                                    representatives are not canonical (src/checker/dfs.rs:258-283) */
} sr_opts;

/* Timing/throughput counters of a finished run (sr_gpu_bfs_stats / sr_gpu_bfs_stats_sized).
 * Layout of SR_PLUGIN_ABI 4 (ABI 3 plus exchange_fallbacks and owner_key). */
typedef struct sr_stats {
    double level_loop_sec;       /* first expand launch .. last level synchronised              */
    double total_sec;            /* spawn .. done, excluding one-time device allocation          */
    double expand_kernel_ms;     /* sum of expand-kernel HIP-event durations (profile=1)         */
    uint64_t expand_launches;
    uint64_t levels;
    uint64_t table_capacity;     /* visited-set slots                                            */
    uint64_t rehashes;
    uint64_t algorithmic_bytes;  /* 8 B per successor probe + 16 B per insert +
                                    8*W B frontier write + 8*W B frontier read per state         */
    uint64_t successors;         /* == state_count - init states                                 */
    uint32_t words_per_state;
    uint32_t order_used;         /* enum sr_order actually used for the reported counts          */
    uint32_t restarts;           /* capacity restarts of this check (larger buffers / synchronous) */
    uint32_t pipelined;          /* partitioned search: 1 = levels pipelined, no host wait inside;
                                    2 = pipelined with the direct exchange (records stored into the
                                    owners' buffers through peer pointers, device flags per level) */
    uint64_t records_routed;     /* partitioned search: successor records sent between partitions (all ranks) */
    uint64_t head_levels;        /* partitioned search: levels run replicated before partitioning */
    uint64_t probes;             /* visited-set slots loaded by the expand kernels (first probe + linear steps) */
    uint64_t cas;                /* 64-bit atomicCAS claims attempted on the visited set */
    uint64_t max_displacement;   /* longest linear-probe displacement (slots past home) of any entry
                                    of the final visited set; measured with counters=1, else 0    */
    uint32_t displacement_limit; /* probe limit of the final table's slot encoding (quotient mode:
                                    2^dbits - 2; fingerprint mode: 65536)                          */
    uint32_t table_doublings;    /* quotient mode: in-check doublings after a level overflowed the
                                    probe limit (the level is finished on the larger table)       */
    uint32_t exchange_fallbacks; /* partitioned search: checks redone on the collective exchange after
                                    the direct exchange failed its per-slot sequence tag / checksum
                                    or a peer's flag timed out (the result is then still exact)    */
    uint32_t owner_key;          /* partitioned search: 1 = states are owned by the model's owner key
                                    (a projection most actions keep), 0 = by fingerprint          */
} sr_stats;

typedef struct sr_bfs sr_bfs;

void sr_opts_init(sr_opts* opts);
/* The same for a caller whose sr_opts mirror has `size` bytes (a binding written against an older
 * header): writes at most `size` bytes and sets struct_size to what it wrote. Bindings in other
 * languages should call this with their own struct size rather than sr_opts_init. */
void sr_opts_init_sized(sr_opts* opts, uint32_t size);
const char* sr_last_error(void);
int sr_device_count(void);

/* Spawns the checker; returns NULL on error (see sr_last_error). Non-blocking. */
sr_bfs* sr_gpu_bfs_spawn(int32_t model_id, const int64_t* params, int32_t nparams, const sr_opts* opts);
int32_t sr_gpu_bfs_join(sr_bfs* bfs);
int32_t sr_gpu_bfs_is_done(const sr_bfs* bfs);
/* 1 while the driver thread is still searching (for `report`'s polling loop, src/checker.rs:223). */
int32_t sr_gpu_bfs_is_running(const sr_bfs* bfs);
uint64_t sr_gpu_bfs_state_count(const sr_bfs* bfs);
uint64_t sr_gpu_bfs_unique_state_count(const sr_bfs* bfs);
uint32_t sr_gpu_bfs_max_depth(const sr_bfs* bfs);
int32_t sr_gpu_bfs_stats(const sr_bfs* bfs, sr_stats* out);
/* The same for a caller whose sr_stats mirror has `size` bytes (a binding written against another
 * header): copies at most `size` bytes; returns the engine's sizeof(sr_stats). */
int32_t sr_gpu_bfs_stats_sized(const sr_bfs* bfs, sr_stats* out, uint32_t size);
/* profile=1: HIP-event duration (ms) of every expand launch in launch order and the frontier size
 * it expanded (0 if unknown); returns the number of launches (FAST pipelined order: launch i
 * expands level i, a last launch past the end expands nothing). */
int64_t sr_gpu_bfs_launch_profile(const sr_bfs* bfs, double* kernel_ms, uint64_t* frontier, int64_t cap);
/* Visited-set probes and CAS claims of every expand launch of the pipelined FAST loop, in launch
 * order (sr_opts.counters = 1; zeros otherwise). Returns the number of launches. */
int64_t sr_gpu_bfs_launch_counters(const sr_bfs* bfs, uint64_t* probes, uint64_t* cas, int64_t cap);

int32_t sr_gpu_bfs_property_count(const sr_bfs* bfs);
/* Copies the property name (NUL-terminated) and its expectation; returns the name length. */
int32_t sr_gpu_bfs_property(const sr_bfs* bfs, int32_t prop, char* name, int32_t cap, int32_t* expectation);

/* Discovery of property `prop`: writes the fingerprint chain init..discovered state (the
 * reference's `reconstruct_path` input) and returns its length; 0 = no discovery. */
int32_t sr_gpu_bfs_discovery(const sr_bfs* bfs, int32_t prop, uint64_t* fp_chain, uint32_t cap);
/* Replays that chain on the host model (`Path::from_fingerprints`): canonical action ids
 * (len = chain-1) and states (chain * describe_width int64s). Returns the number of actions,
 * -1 if no discovery, or a negative SR_ERR_*. */
int32_t sr_gpu_bfs_discovery_path(const sr_bfs* bfs, int32_t prop, int64_t* action_ids, int32_t cap_actions,
                                  int64_t* states, int64_t cap_states);
int32_t sr_gpu_bfs_describe_width(const sr_bfs* bfs);
/* Reference `Debug` text of a canonical action id (e.g. "RmPrepare(3)"). */
int32_t sr_gpu_bfs_action_name(const sr_bfs* bfs, int64_t action_id, char* buf, int32_t cap);
/* Upper bound (exclusive) on canonical action ids of the model, for name lookups. */
int64_t sr_gpu_bfs_action_id_bound(const sr_bfs* bfs);
/* Number of init states (`Model::init_states`, src/lib.rs:163). */
int32_t sr_gpu_bfs_init_count(const sr_bfs* bfs);
/* `Path::from_actions` (src/checker/path.rs:90-112) from init state `init_index` on the host copy
 * of the model: writes the states (describe_width int64s each) and, per property, whether its
 * CONDITION holds on the last state. Returns the number of actions applied, or -1 if an action is
 * not enabled along the way (the reference returns None). */
int32_t sr_gpu_bfs_replay(const sr_bfs* bfs, int32_t init_index, const int64_t* action_ids, int32_t n_actions,
                          int64_t* states, int64_t cap_states, int32_t* conditions, int32_t cap_conditions);
/* `Path::from_actions` as above, reporting each property's condition on EVERY state of the path
 * (conditions[i * property_count + p], i = 0..n) and whether the last state is terminal (its
 * `actions()` list is empty): what `assert_discovery` needs for an `eventually` property
 * (src/checker.rs:306-323). Returns n, or -1 if an action is not enabled along the way. */
int32_t sr_gpu_bfs_replay_trace(const sr_bfs* bfs, int32_t init_index, const int64_t* action_ids, int32_t n_actions,
                                int32_t* conditions, int64_t cap, int32_t* terminal);
/* Explorer's `states` route (src/checker/explorer.rs:159-240), host-only: n == 0 lists the init
 * states (action -1); otherwise the state reached by the fingerprint path (`Path::final_state`,
 * src/checker/path.rs:115-136) and, per action its `actions()` lists (in order), the canonical
 * action id, whether `next_state` is Some (has_state), the next state's fingerprint and its
 * description (describe_width int64s per view). Returns the number of views (at most cap are
 * written), or -1 if no state follows the fingerprints. */
int32_t sr_gpu_bfs_explore(const sr_bfs* bfs, const uint64_t* fingerprints, int32_t n, int64_t* action_ids,
                           int32_t* has_state, uint64_t* fingerprints_out, int64_t* states, int32_t cap);
/* Visited states in visit order (record_visits=1), describe_width int64s each; returns count*width. */
int64_t sr_gpu_bfs_visits(const sr_bfs* bfs, int64_t* out, int64_t cap);
/* The visitor's paths (`CheckerVisitor::visit` gets `Path::from_fingerprints` of every popped
 * state, src/checker/bfs.rs:187-189, src/checker/visitor.rs:19-66): per visit, in the order of
 * sr_gpu_bfs_visits, the visit index of its BFS-tree parent and the canonical id of the first
 * action leading from that parent to it (-1 and -1 for init states). Returns the visit count,
 * or SR_ERR_UNSUPPORTED when the check kept no visit record (record_visits=0). The partitioned
 * search gathers every rank's records at join, so its tree is global on every rank. */
int64_t sr_gpu_bfs_visit_tree(const sr_bfs* bfs, int64_t* parent, int64_t* action, int64_t cap);
void sr_gpu_bfs_free(sr_bfs* bfs);

/* ---- Partitioned search over several GPUs (no counterpart in the reference,
 * which is single-process shared-memory: src/checker/bfs.rs:70-152) ----
 * One process per GPU. Rank 0 creates a unique id, every rank receives it out of band (e.g. a
 * torch.distributed broadcast) and calls sr_dist_init with its rank. The first small levels run
 * replicated on every rank with no collective. After them every level is exchanged DIRECTLY: each
 * rank's expand kernel stores its successor records (8*W bytes each) into the owners' receive
 * buffers through peer pointers (IPC handles across processes, shared once through the
 * communicator) and raises a device flag per level in every owner; owners wait for the flags on
 * the device. No collective and no host step runs inside a level. If a one-off
 * collective probe finds the peer path unusable on any rank (or SR_DIRECT=0), RCCL instead carries
 * ONE all-to-all of fixed-capacity buckets per level, every rank's row in the bucket headers.
 * Counts reported by every rank are global. Discovery paths are gathered on every rank at join
 * (sr_opts.defer_paths = 0, the default), so any rank may ask for them alone. */
#define SR_DIST_ID_BYTES 128
typedef struct sr_dist sr_dist;
int32_t sr_dist_unique_id(uint8_t* id_out);
/* An RCCL communicator (one process per GPU). */
sr_dist* sr_dist_init(int32_t rank, int32_t world, const uint8_t* id, int32_t device);
/* `world` communicators whose ranks are threads of THIS process (rank r on devices[r], or device 0
 * when devices is NULL): the same stream-ordered collectives as RCCL, carried by device copies
 * across the ranks' streams, with a host rendezvous per call that rejects ranks issuing different
 * collectives, and the direct exchange through raw device pointers. Runs the partitioned engine's
 * multi-rank code path on one GPU (tests). Ranks that share a device each need a hardware queue of
 * their own for the direct exchange's device-side waits (GPU_MAX_HW_QUEUES >= world + 2). */
int32_t sr_dist_local_group(int32_t world, const int32_t* devices, sr_dist** comms_out);
/* `world` PROCESSES of one host whose host-side transport is the POSIX shared-memory segment `name`
 * (created by the first rank to open it; rank 0 unlinks it when freed): synchronous staged
 * collectives through per-rank slots of slot_bytes, a barrier in the segment, and the direct
 * exchange through IPC handles. Lets the one-process-per-GPU code path run as separate processes on
 * ONE GPU, where RCCL refuses two ranks on one device (tests, bench rehearsals).
 * devices_distinct = 1 when every rank has its own GPU. */
sr_dist* sr_dist_shm_init(int32_t rank, int32_t world, const char* name, int32_t device, int64_t slot_bytes,
                          int32_t devices_distinct);
int32_t sr_dist_rank(const sr_dist* comm);
int32_t sr_dist_world(const sr_dist* comm);
/* Ranks the transport reports (RCCL: ncclCommCount). */
int32_t sr_dist_nranks(const sr_dist* comm);
/* "rccl", "local" or "shm". */
int32_t sr_dist_kind(const sr_dist* comm, char* buf, int32_t cap);
/* Device synchronisation of this rank, then a collective barrier (bench timing brackets). */
int32_t sr_dist_barrier(sr_dist* comm);
/* Element-wise min (op 0) or max (op 1) of n doubles over the ranks, in place. */
int32_t sr_dist_allreduce_f64(sr_dist* comm, double* values, int32_t n, int32_t op);
void sr_dist_free(sr_dist* comm);

/* The partitioned search's HOST protocol without a GPU (tests): `world` processes on the
 * shared-memory segment `name` (as sr_dist_shm_init, host buffers only) run a 2pc check whose
 * device side is a CPU stand-in (expansion, routing by part_of, the direct exchange's per-slot
 * checksum, one row per partition and level), while the level rows, their error precedence, the
 * pipelined bucket plan and the outcome vote are the engine's own code (dist.hpp). Faults are
 * injected where the device would raise them. Returns SR_OK with *out filled, or the error every
 * rank agreed to fail with (sr_last_error). */
typedef struct sr_dist_host_opts {
    uint32_t struct_size;
    int32_t rm_count;               /* 2pc resource managers (1..=7) */
    uint64_t cmin;                  /* minimum planned bucket capacity (records per pair) */
    int32_t corrupt_level;          /* >= 0: a record this rank receives at that level is altered after
                                       its source checksummed it (once); -1: none */
    int32_t capacity_fail_at_end;   /* this rank alone fails with a capacity error at the end (once) */
    int32_t fail_at_end;            /* this rank alone fails with another error at the end (once) */
    int32_t plan_div;               /* > 1: the planned capacities divided by it (an under-estimate) */
} sr_dist_host_opts;
typedef struct sr_dist_host_result {
    uint64_t unique, state_count, local_unique;  /* global counts; states this rank's partition holds */
    uint32_t max_depth, levels;
    uint32_t attempts, restarts, fallbacks, disagreements;
    uint32_t overflow_level;        /* first level with a bucket over its planned capacity (~0: none) */
    uint32_t first_outcome;         /* this rank's outcome of the first attempt: 0 ok, 1 capacity,
                                       2 exchange, 3 other error (dist.hpp Outcome) */
    uint64_t plan_digest;           /* hash of the planned bucket capacities (equal on every rank) */
} sr_dist_host_result;
int32_t sr_dist_host_protocol(const char* name, int32_t rank, int32_t world, const sr_dist_host_opts* opts,
                              sr_dist_host_result* out);

/* Versions: runtime = what the loaded library reports, compiled = the headers the engine was built
 * against (RCCL: NCCL_VERSION_CODE; HIP: HIP_VERSION). A mismatch means another process-wide copy
 * of the runtime (e.g. one bundled with a Python framework) was loaded first. */
int32_t sr_rccl_version(int32_t* runtime, int32_t* compiled);
int32_t sr_hip_runtime_version(int32_t* runtime, int32_t* compiled);
int32_t sr_device_synchronize(int32_t device);
/* The source digest this library was compiled from (16 hex digits: sha256 over the engine's sources
 * and headers, stateright_amd/build.py `source_digest`). The Python loader refuses a library whose
 * digest differs from the sources beside it, so a stale binary never tests or benches old code. */
const char* sr_build_digest(void);
/* Host-only self-test of the visited set's quotient encoding (kernels.hpp): the key permutation is
 * a bijection and slot values decode to their keys. SR_OK or SR_ERR_ARG (sr_last_error). */
int32_t sr_selftest_tables(void);
/* Host-only self-check of the compiled-in model encodings: every slot a model's optional
 * `self_loops` reports (counted by the FAST expansion without being generated) is enabled and
 * returns the state itself, over every reachable state of 2pc N=1..7 (and its canonical form);
 * and the register clients' linearizability test (paxos, single-copy register) agrees with the
 * tester's serialization search on random histories of 1..6 clients.
 * SR_OK or SR_ERR_ARG (sr_last_error says where). */
int32_t sr_selftest_models(void);
/* comm == NULL: `virtual_partitions` partitions in this process on opts->device (same protocol;
 * the partitions store into each other's receive buffers). FAST order only. */
sr_bfs* sr_gpu_bfs_spawn_partitioned(sr_dist* comm, int32_t virtual_partitions, int32_t model_id,
                                     const int64_t* params, int32_t nparams, const sr_opts* opts);

/* ---- GpuModel plugins: `impl Model` outside the registry (src/lib.rs:155-237) ----
 * A user writes a GpuModel (the encoding concept of stateright_amd/csrc/models.hpp) and builds it
 * with hipcc into its own shared library, instantiating the engine from
 * include/stateright_gpu_model.hpp; the macro SR_GPU_PLUGIN(name, Model, make) there exports
 * `const sr_plugin* sr_plugin_<name>(void)`. The engine library then runs it like a registered
 * model. The plugin must be built from the same headers (abi). */
#define SR_PLUGIN_ABI 4
typedef struct sr_plugin {
    uint32_t abi;         /* SR_PLUGIN_ABI of the headers the plugin was built with */
    uint32_t opts_size;   /* sizeof(sr_opts) in that build */
    const char* name;
    /* Creates an engine object (comm = NULL and virtual_parts <= 1: one GPU; else partitioned). */
    void* (*create)(const int64_t* params, int32_t nparams, const sr_opts* opts, void* comm, int32_t virtual_parts,
                    char* err, int32_t errcap);
    /* Fingerprint of a state given by its canonical description (needs the model's `undescribe`). */
    int32_t (*fingerprint)(const int64_t* params, int32_t nparams, const int64_t* described, int32_t width,
                           uint64_t* fp_out);
} sr_plugin;

sr_bfs* sr_gpu_bfs_spawn_plugin(const sr_plugin* plugin, const int64_t* params, int32_t nparams, const sr_opts* opts);
sr_bfs* sr_gpu_bfs_spawn_plugin_partitioned(const sr_plugin* plugin, sr_dist* comm, int32_t virtual_partitions,
                                            const int64_t* params, int32_t nparams, const sr_opts* opts);

/* The engine's fingerprint of a state of a registered model, given by its canonical description
 * (the integers sr_gpu_bfs_discovery_path / sr_gpu_bfs_visits return, describe_width of them):
 * what a host-side `Path::from_fingerprints` (src/checker/path.rs:20-86) compares with the chain of
 * sr_gpu_bfs_discovery. Host-only (no device needed). Every registered model but DGraph: the
 * register models (paxos, ABD, single-copy) describe their LinearizabilityTester history
 * canonically (per client the Get's returned value and its real-time predecessors), so their
 * description determines the state. SR_ERR_UNSUPPORTED for DGraph. */
int32_t sr_model_fingerprint(int32_t model_id, const int64_t* params, int32_t nparams, const int64_t* described,
                             int32_t width, uint64_t* fp_out);
/* Host-only self-test of sr_model_fingerprint: a host BFS over up to max_states reachable states of
 * the model; every state's description must give the state back and the engine's fingerprint of
 * it. Returns the states checked, or SR_ERR_* (sr_last_error says which state failed). */
int64_t sr_selftest_describe(int32_t model_id, const int64_t* params, int32_t nparams, int64_t max_states);

#ifdef __cplusplus
}
#endif
#endif /* STATERIGHT_GPU_H */
