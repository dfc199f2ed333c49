"""ctypes binding to the MI355X engine's C ABI (include/stateright_gpu.h).

The shared library `stateright_amd/libstateright_gpu.so` is built in-tree by
`stateright_amd.build.build()` (hipcc --offload-arch=gfx950). There is no fallback: if the library
is missing, or no HIP device is visible, every checker call raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SR_LIB_PATH") or os.path.join(HERE, "libstateright_gpu.so")

SR_MODEL_LINEAR_EQUATION = 1
SR_MODEL_BINARY_CLOCK = 2
SR_MODEL_2PC = 3
SR_MODEL_INCREMENT = 4
SR_MODEL_INCREMENT_LOCK = 5
SR_MODEL_DGRAPH = 6
SR_MODEL_PAXOS = 7
SR_MODEL_PINGPONG = 9
SR_MODEL_ACTOR_FIXTURE = 10
SR_MODEL_ABD = 11
SR_MODEL_SINGLE_COPY = 12

SR_ORDER_AUTO, SR_ORDER_FIFO, SR_ORDER_FAST = 0, 1, 2
SR_ALWAYS, SR_EVENTUALLY, SR_SOMETIMES = 0, 1, 2


class sr_opts(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("target_state_count", ctypes.c_uint64),
        ("order", ctypes.c_int32),
        ("record_visits", ctypes.c_int32),
        ("capacity_hint", ctypes.c_uint64),
        ("profile", ctypes.c_int32),
        ("verbose", ctypes.c_int32),
        ("counters", ctypes.c_int32),
        ("defer_paths", ctypes.c_int32),
        ("symmetry", ctypes.c_int32),
    ]


class sr_stats(ctypes.Structure):
    _fields_ = [
        ("level_loop_sec", ctypes.c_double),
        ("total_sec", ctypes.c_double),
        ("expand_kernel_ms", ctypes.c_double),
        ("expand_launches", ctypes.c_uint64),
        ("levels", ctypes.c_uint64),
        ("table_capacity", ctypes.c_uint64),
        ("rehashes", ctypes.c_uint64),
        ("algorithmic_bytes", ctypes.c_uint64),
        ("successors", ctypes.c_uint64),
        ("words_per_state", ctypes.c_uint32),
        ("order_used", ctypes.c_uint32),
        ("restarts", ctypes.c_uint32),
        ("pipelined", ctypes.c_uint32),
        ("records_routed", ctypes.c_uint64),
        ("head_levels", ctypes.c_uint64),
        ("probes", ctypes.c_uint64),
        ("cas", ctypes.c_uint64),
        ("max_displacement", ctypes.c_uint64),
        ("displacement_limit", ctypes.c_uint32),
        ("table_doublings", ctypes.c_uint32),
        ("exchange_fallbacks", ctypes.c_uint32),
        ("owner_key", ctypes.c_uint32),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class sr_dist_host_opts(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("rm_count", ctypes.c_int32),
        ("cmin", ctypes.c_uint64),
        ("corrupt_level", ctypes.c_int32),
        ("capacity_fail_at_end", ctypes.c_int32),
        ("fail_at_end", ctypes.c_int32),
        ("plan_div", ctypes.c_int32),
    ]


class sr_dist_host_result(ctypes.Structure):
    _fields_ = [
        ("unique", ctypes.c_uint64),
        ("state_count", ctypes.c_uint64),
        ("local_unique", ctypes.c_uint64),
        ("max_depth", ctypes.c_uint32),
        ("levels", ctypes.c_uint32),
        ("attempts", ctypes.c_uint32),
        ("restarts", ctypes.c_uint32),
        ("fallbacks", ctypes.c_uint32),
        ("disagreements", ctypes.c_uint32),
        ("overflow_level", ctypes.c_uint32),
        ("first_outcome", ctypes.c_uint32),
        ("plan_digest", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# (name, restype, argtypes) of every exported entry point; tests check this list against the header.
_P = ctypes.c_void_p
_I64P = ctypes.POINTER(ctypes.c_int64)
SIGNATURES = [
    ("sr_opts_init", None, [ctypes.POINTER(sr_opts)]),
    ("sr_opts_init_sized", None, [ctypes.POINTER(sr_opts), ctypes.c_uint32]),
    ("sr_last_error", ctypes.c_char_p, []),
    ("sr_device_count", ctypes.c_int, []),
    ("sr_gpu_bfs_spawn", _P, [ctypes.c_int32, _I64P, ctypes.c_int32, ctypes.POINTER(sr_opts)]),
    ("sr_gpu_bfs_join", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_is_done", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_is_running", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_state_count", ctypes.c_uint64, [_P]),
    ("sr_gpu_bfs_unique_state_count", ctypes.c_uint64, [_P]),
    ("sr_gpu_bfs_max_depth", ctypes.c_uint32, [_P]),
    ("sr_gpu_bfs_stats", ctypes.c_int32, [_P, ctypes.POINTER(sr_stats)]),
    ("sr_gpu_bfs_stats_sized", ctypes.c_int32, [_P, ctypes.POINTER(sr_stats), ctypes.c_uint32]),
    ("sr_gpu_bfs_launch_counters", ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                                    ctypes.c_int64]),
    ("sr_gpu_bfs_launch_profile", ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                                   ctypes.c_int64]),
    ("sr_gpu_bfs_property_count", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_property", ctypes.c_int32, [_P, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_int32)]),
    ("sr_gpu_bfs_discovery", ctypes.c_int32, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]),
    ("sr_gpu_bfs_discovery_path", ctypes.c_int32, [_P, ctypes.c_int32, _I64P, ctypes.c_int32, _I64P, ctypes.c_int64]),
    ("sr_gpu_bfs_describe_width", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_action_name", ctypes.c_int32, [_P, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int32]),
    ("sr_gpu_bfs_action_id_bound", ctypes.c_int64, [_P]),
    ("sr_gpu_bfs_init_count", ctypes.c_int32, [_P]),
    ("sr_gpu_bfs_replay", ctypes.c_int32, [_P, ctypes.c_int32, _I64P, ctypes.c_int32, _I64P, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    ("sr_gpu_bfs_replay_trace", ctypes.c_int32, [_P, ctypes.c_int32, _I64P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                                 ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]),
    ("sr_gpu_bfs_explore", ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32, _I64P,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64), _I64P,
                                            ctypes.c_int32]),
    ("sr_gpu_bfs_visits", ctypes.c_int64, [_P, _I64P, ctypes.c_int64]),
    ("sr_gpu_bfs_visit_tree", ctypes.c_int64, [_P, _I64P, _I64P, ctypes.c_int64]),
    ("sr_gpu_bfs_free", None, [_P]),
    ("sr_dist_unique_id", ctypes.c_int32, [ctypes.c_char_p]),
    ("sr_dist_init", _P, [ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32]),
    ("sr_dist_local_group", ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_P)]),
    ("sr_dist_shm_init", _P, [ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64,
                              ctypes.c_int32]),
    ("sr_dist_rank", ctypes.c_int32, [_P]),
    ("sr_dist_world", ctypes.c_int32, [_P]),
    ("sr_dist_nranks", ctypes.c_int32, [_P]),
    ("sr_dist_kind", ctypes.c_int32, [_P, ctypes.c_char_p, ctypes.c_int32]),
    ("sr_dist_barrier", ctypes.c_int32, [_P]),
    ("sr_dist_allreduce_f64", ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_double), ctypes.c_int32, ctypes.c_int32]),
    ("sr_dist_free", None, [_P]),
    ("sr_dist_host_protocol", ctypes.c_int32, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.POINTER(sr_dist_host_opts), ctypes.POINTER(sr_dist_host_result)]),
    ("sr_rccl_version", ctypes.c_int32, [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    ("sr_hip_runtime_version", ctypes.c_int32, [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    ("sr_device_synchronize", ctypes.c_int32, [ctypes.c_int32]),
    ("sr_build_digest", ctypes.c_char_p, []),
    ("sr_selftest_tables", ctypes.c_int32, []),
    ("sr_selftest_models", ctypes.c_int32, []),
    ("sr_gpu_bfs_spawn_plugin", _P, [_P, _I64P, ctypes.c_int32, ctypes.POINTER(sr_opts)]),
    ("sr_gpu_bfs_spawn_plugin_partitioned", _P, [_P, _P, ctypes.c_int32, _I64P, ctypes.c_int32,
                                                 ctypes.POINTER(sr_opts)]),
    ("sr_model_fingerprint", ctypes.c_int32, [ctypes.c_int32, _I64P, ctypes.c_int32, _I64P, ctypes.c_int32,
                                              ctypes.POINTER(ctypes.c_uint64)]),
    ("sr_selftest_describe", ctypes.c_int64, [ctypes.c_int32, _I64P, ctypes.c_int32, ctypes.c_int64]),
    ("sr_gpu_bfs_spawn_partitioned", _P, [_P, ctypes.c_int32, ctypes.c_int32, _I64P, ctypes.c_int32,
                                          ctypes.POINTER(sr_opts)]),
]

SR_DIST_ID_BYTES = 128

_lib = None


def load():
    """Loads the engine library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"MI355X engine library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        ab = os.environ.get("SR_LIB_DIGEST_CHECK", "1") == "0"
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name, None)
            if fn is None and ab:  # an A/B build of older sources: entry points it lacks stay unbound
                continue
            if fn is None:
                raise ImportError(f"{LIB_PATH} lacks {name}: rebuild it")
            fn.restype = res
            fn.argtypes = args
        check_digest(lib)
        _lib = lib
    return _lib


class StaleLibraryError(ImportError):
    pass


def check_digest(lib, sources_root=None):
    """Refuses a library compiled from other sources than the ones beside it: sr_build_digest()
    must equal build.source_digest() (stateright_amd/build.py). SR_LIB_DIGEST_CHECK=0 turns the
    check off; only scripts/gpu_lib_ab.sh does that, to time a saved build of older sources against
    the current one (bench.py still records both digests in its line)."""
    if os.environ.get("SR_LIB_DIGEST_CHECK", "1") == "0":
        return
    from . import build
    want = build.source_digest() if sources_root is None else build.source_digest_at(sources_root)
    got = lib.sr_build_digest().decode()
    if got != want:
        raise StaleLibraryError(
            f"{LIB_PATH} was built from sources with digest {got}, but the sources here have digest {want}; "
            "rebuild it (`python -c 'import __graft_entry__ as g; g.build()'`)")


def build_digest():
    """The source digest compiled into the loaded library ("unstamped" for an A/B build of
    sources older than the stamp)."""
    lib = load()
    return lib.sr_build_digest().decode() if hasattr(lib, "sr_build_digest") else "unstamped"


def last_error():
    return load().sr_last_error().decode(errors="replace")


def runtime_versions():
    """{"hip": (runtime, compiled), "rccl": (runtime, compiled)} as the engine library sees them."""
    lib = load()
    out = {}
    for key, fn in (("hip", lib.sr_hip_runtime_version), ("rccl", lib.sr_rccl_version)):
        r, c = ctypes.c_int32(), ctypes.c_int32()
        out[key] = (r.value, c.value) if fn(ctypes.byref(r), ctypes.byref(c)) == 0 else (None, None)
    return out


def loaded_runtime_paths():
    """Paths of the HIP runtime and RCCL libraries mapped into this process (Linux)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.count(" ") >= 5 else ""
                if "libamdhip64" in p or "librccl" in p:
                    paths.add(p)
    except OSError:
        pass
    return sorted(paths)
