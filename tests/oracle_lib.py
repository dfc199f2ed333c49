"""ctypes binding to the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

The oracle is a C++ restatement of Stateright's `src/checker/bfs.rs`; it is the checker for the
MI355X engine, never part of the product path.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

# Model ids shared with include/stateright_gpu.h (SR_MODEL_*).
LINEAR_EQUATION, BINARY_CLOCK, TWO_PHASE, INCREMENT, INCREMENT_LOCK, DGRAPH, PAXOS = 1, 2, 3, 4, 5, 6, 7
SYM_TOY = 8  # oracle only: the symmetry fixture of src/checker/dfs.rs:393-476

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(LIB_PATH)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.oracle_spawn_bfs.restype = ctypes.c_void_p
        L.oracle_spawn_bfs.argtypes = [ctypes.c_int, i64p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
        L.oracle_spawn_dfs.restype = ctypes.c_void_p
        L.oracle_spawn_dfs.argtypes = [ctypes.c_int, i64p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.c_int]
        L.oracle_join.argtypes = [ctypes.c_void_p]
        for f in ("oracle_state_count", "oracle_unique_state_count"):
            getattr(L, f).restype = ctypes.c_uint64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.oracle_max_depth.restype = ctypes.c_uint32
        L.oracle_max_depth.argtypes = [ctypes.c_void_p]
        L.oracle_is_done.argtypes = [ctypes.c_void_p]
        L.oracle_width.argtypes = [ctypes.c_void_p]
        L.oracle_elapsed_sec.restype = ctypes.c_double
        L.oracle_elapsed_sec.argtypes = [ctypes.c_void_p]
        L.oracle_discovery_count.argtypes = [ctypes.c_void_p]
        L.oracle_discovery_name.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.oracle_discovery_actions.argtypes = [ctypes.c_void_p, ctypes.c_char_p, i64p, ctypes.c_int64]
        L.oracle_discovery_states.argtypes = [ctypes.c_void_p, ctypes.c_char_p, i64p, ctypes.c_int64]
        L.oracle_visits.restype = ctypes.c_int64
        L.oracle_visits.argtypes = [ctypes.c_void_p, i64p, ctypes.c_int64]
        L.oracle_report.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.oracle_visit_path.argtypes = [ctypes.c_void_p, ctypes.c_int64, i64p, ctypes.c_int64]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_replay.argtypes = [ctypes.c_int, i64p, ctypes.c_int, i64p, ctypes.c_int, i64p, ctypes.c_int64,
                                    ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.oracle_fingerprint_i8.restype = ctypes.c_uint64
        L.oracle_fingerprint_i8.argtypes = [ctypes.c_int8]
        _lib = L
    return _lib


def _arr(vals):
    vals = list(vals) or [0]
    return (ctypes.c_int64 * len(vals))(*vals)


class OracleRun:
    """Runs the restated `spawn_bfs().join()` and exposes the `Checker` surface."""

    def __init__(self, model, params=(), threads=1, target=0, record_visits=False, dfs=False, symmetry=False):
        """`spawn_bfs` (default) or `spawn_dfs` (dfs=True, optionally with `symmetry()`)."""
        L = lib()
        self.model, self.params = model, list(params)
        p = _arr(self.params)
        if dfs:
            self.h = L.oracle_spawn_dfs(model, p, len(self.params), threads, target, int(record_visits), int(symmetry))
        else:
            self.h = L.oracle_spawn_bfs(model, p, len(self.params), threads, target, int(record_visits))
        if not self.h:
            raise RuntimeError(L.oracle_last_error().decode())
        if L.oracle_join(self.h) != 0:
            raise RuntimeError(L.oracle_last_error().decode())
        self.state_count = L.oracle_state_count(self.h)
        self.unique_state_count = L.oracle_unique_state_count(self.h)
        self.max_depth = L.oracle_max_depth(self.h)
        self.is_done = bool(L.oracle_is_done(self.h))
        self.width = L.oracle_width(self.h)
        self.elapsed = L.oracle_elapsed_sec(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_free(self.h)
            self.h = None

    def discovery_names(self):
        L = lib()
        out = []
        buf = ctypes.create_string_buffer(256)
        for i in range(L.oracle_discovery_count(self.h)):
            L.oracle_discovery_name(self.h, i, buf, 256)
            out.append(buf.value.decode())
        return sorted(out)

    def discovery_actions(self, name):
        L = lib()
        buf = (ctypes.c_int64 * 4096)()
        n = L.oracle_discovery_actions(self.h, name.encode(), buf, 4096)
        if n == -1:
            return None
        if n < 0:
            raise RuntimeError(L.oracle_last_error().decode())
        return list(buf[:n])

    def discovery_states(self, name):
        L = lib()
        buf = (ctypes.c_int64 * 65536)()
        n = L.oracle_discovery_states(self.h, name.encode(), buf, 65536)
        if n < 0:
            return None
        flat = list(buf[:n])
        return [tuple(flat[i:i + self.width]) for i in range(0, n, self.width)]

    def visits(self):
        L = lib()
        n = L.oracle_visits(self.h, None, 0)
        buf = (ctypes.c_int64 * max(n, 1))()
        L.oracle_visits(self.h, buf, n)
        flat = list(buf[:n])
        return [tuple(flat[i:i + self.width]) for i in range(0, n, self.width)]

    def visits_array(self):
        """The visits as an int64 numpy array (count x width), without Python tuples."""
        import numpy as np
        L = lib()
        n = L.oracle_visits(self.h, None, 0)
        out = np.empty(max(n, 1), dtype=np.int64)
        L.oracle_visits(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n)
        return out[:n].reshape(-1, self.width)

    def visit_paths(self):
        """Action ids of the path the reference's visitor receives at each pop, in visit order."""
        L = lib()
        buf = (ctypes.c_int64 * 65536)()
        out = []
        i = 0
        while True:
            n = L.oracle_visit_path(self.h, i, buf, 65536)
            if n == -1:
                return out
            if n < 0:
                raise RuntimeError(L.oracle_last_error().decode())
            out.append(list(buf[:n]))
            i += 1

    def report(self):
        buf = ctypes.create_string_buffer(1 << 16)
        lib().oracle_report(self.h, buf, 1 << 16)
        return buf.value.decode()


def replay(model, params, action_ids, n_props=8):
    """Replays canonical action ids on the CPU model (`Path::from_actions`).

    Returns (states, holds) — the descriptions of every state on the path and, per property,
    whether its condition holds on the last state — or None if some action is not enabled.
    """
    L = lib()
    p = _arr(params)
    a = _arr(action_ids)
    out = (ctypes.c_int64 * 65536)()
    holds = (ctypes.c_int * n_props)()
    n = L.oracle_replay(model, p, len(list(params)), a, len(list(action_ids)), out, 65536, holds, n_props)
    if n == -1:
        return None
    if n < 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return list(out[:n]), list(holds)


def dgraph_params(expectation, paths):
    """Encodes a DGraph (src/test_util.rs:47-116): expectation 0 always / 1 eventually / 2 sometimes."""
    p = [expectation]
    for path in paths:
        p.append(len(path))
        p.extend(path)
    return p
