"""Host-side mirror of Stateright's checker API over the MI355X engine.

Mirrors, name for name, the reference's `CheckerBuilder` (src/checker.rs:35-178), the `Checker`
trait (src/checker.rs:184-338) and `Path` (src/checker/path.rs), so that code written against
`model.checker().spawn_bfs().join()` reads the same. Every call goes through the C ABI in
include/stateright_gpu.h; there is no CPU fallback.
"""
import ctypes
import enum
import sys
import time

from . import _native as N


class Expectation(enum.IntEnum):
    """`Expectation` (src/lib.rs:293-300)."""
    Always = N.SR_ALWAYS
    Eventually = N.SR_EVENTUALLY
    Sometimes = N.SR_SOMETIMES


class CheckerError(RuntimeError):
    """A failed engine call (the reference panics in these cases)."""

    def __init__(self, what, code=None):
        super().__init__(f"{what}: {N.last_error()}" + (f" (status {code})" if code is not None else ""))
        self.code = code


class Path:
    """`Path<State, Action>` (src/checker/path.rs:16): states with the action taken from each.

    States are the canonical integer descriptions shared with the CPU oracle; actions are their
    `Debug` text (e.g. "RmPrepare(3)"), with the canonical ids in `action_ids`.
    """

    def __init__(self, states, action_ids, action_names):
        self.states = [tuple(s) for s in states]
        self.action_ids = list(action_ids)
        self.action_names = list(action_names)

    def last_state(self):
        return self.states[-1]

    def into_states(self):
        return list(self.states)

    def into_actions(self):
        return list(self.action_names)

    def into_vec(self):
        acts = self.action_names + [None]
        return list(zip(self.states, acts))

    def __len__(self):
        return len(self.action_ids)

    def __str__(self):  # `impl Display for Path` (src/checker/path.rs:174-187)
        return f"Path[{len(self.action_ids)}]:\n" + "".join(f"- {a}\n" for a in self.action_names)

    def __repr__(self):
        return f"Path({self.action_names!r})"

    def __eq__(self, other):
        return isinstance(other, Path) and (self.states, self.action_ids) == (other.states, other.action_ids)

    def __hash__(self):
        return hash((tuple(self.states), tuple(self.action_ids)))


class StateRecorder:
    """`StateRecorder` visitor (src/checker/visitor.rs:70-99): records every visited state."""

    def __init__(self):
        self.states = []

    @classmethod
    def new_with_accessor(cls):
        r = cls()
        return r, (lambda: list(r.states))


class PathRecorder:
    """`PathRecorder` visitor (src/checker/visitor.rs:32-66): records the path to every visited
    state (as a set, like the reference's `HashSet<Path>`)."""

    def __init__(self):
        self.paths = set()

    @classmethod
    def new_with_accessor(cls):
        r = cls()
        return r, (lambda: set(r.paths))

    def visit(self, path):
        self.paths.add(path)


class CheckerBuilder:
    """`CheckerBuilder` (src/checker.rs:35-178) for a registered GpuModel."""

    def __init__(self, model):
        self._model = model
        self._opts = N.sr_opts()
        self._opts.struct_size = ctypes.sizeof(N.sr_opts)
        self._threads = 1
        self._visitor = None
        self._partitions = 1
        self._comm = None
        self._symmetry = False

    # --- options mirrored from the reference ---------------------------------------------------
    def threads(self, thread_count):
        """`threads` (src/checker.rs:170-172). The engine runs one host driver thread per GPU;
        the value is kept for API compatibility and does not change results."""
        self._threads = int(thread_count)
        return self

    def target_state_count(self, count):
        """`target_state_count` (src/checker.rs:164-166): stop at the first 1500-pop block
        boundary of the single-threaded reference order at which state_count >= count."""
        self._opts.target_state_count = int(count)
        return self

    def visitor(self, visitor):
        """`visitor` (src/checker.rs:175-177): a `StateRecorder`, a `PathRecorder`, or any callable
        taking a `Path` (`impl Fn(Path)`, src/checker/visitor.rs:23-30). The GPU explores a whole
        level per launch, so the visits are exported in bulk after the run and handed to the
        visitor in visit order (the reference's order in FIFO mode); a visitor cannot steer the
        search in the reference either."""
        if not (isinstance(visitor, (StateRecorder, PathRecorder)) or callable(visitor)):
            raise TypeError("visitor must be a StateRecorder, a PathRecorder or a callable taking a Path")
        self._visitor = visitor
        self._opts.record_visits = 1
        return self

    def symmetry(self):
        """`symmetry` (src/checker.rs:145-160). The BFS checker ignores it, as the reference's does
        (src/checker/bfs.rs:36-74 never reads options.symmetry); `spawn_dfs` rejects it (see there)."""
        self._symmetry = True
        return self

    def symmetry_canonical(self):
        """Engine opt-in: canonical symmetry reduction. Visited states, frontier and BFS tree hold one
        representative per orbit (2pc: RMs sorted by their full (rm_state, tm_prepared, Prepared msg)
        tuple), so `unique_state_count` is the number of reachable orbits, the same in every visit
        order; discovery paths are concrete paths of the original model. This is deliberately NOT the
        reference's `symmetry().spawn_dfs()` count (665 for 2pc N=5), whose representatives sort by
        rm_state alone and make the count depend on the DFS order (src/checker/dfs.rs:258-283)."""
        self._opts.symmetry = 1
        return self

    # --- engine-specific options ---------------------------------------------------------------
    def order(self, order):
        """"auto" (default), "fifo" (exact reference visit order) or "fast"."""
        self._opts.order = {"auto": N.SR_ORDER_AUTO, "fifo": N.SR_ORDER_FIFO, "fast": N.SR_ORDER_FAST}[order]
        return self

    def capacity_hint(self, unique_states):
        self._opts.capacity_hint = int(unique_states)
        return self

    def device(self, ordinal):
        self._opts.device = int(ordinal)
        return self

    def partitions(self, n):
        """Partition the visited set into `n` virtual partitions on one GPU (the multi-GPU protocol
        with a device-copy exchange; FAST order)."""
        self._partitions = int(n)
        return self

    def comm(self, communicator):
        """Partition the search over the GPUs of a `stateright_amd.distributed.Communicator`
        (one process per GPU, RCCL all-to-all per level; FAST order)."""
        self._comm = communicator
        return self

    def defer_paths(self, on=True):
        """Partitioned search: skip gathering the discovery paths at join (they are then built on
        demand, collectively: every rank must ask for the same property in the same order)."""
        self._opts.defer_paths = int(bool(on))
        return self

    def counters(self, on=True):
        """Count visited-set probes and CAS claims (stats()["probes"], ["cas"]) with a counting
        variant of the expand kernel (slower; for measurement passes only)."""
        self._opts.counters = int(bool(on))
        return self

    def profile(self, on=True):
        self._opts.profile = int(bool(on))
        return self

    def verbose(self, on=True):
        self._opts.verbose = int(bool(on))
        return self

    # --- spawn ---------------------------------------------------------------------------------
    def spawn_bfs(self):
        """`spawn_bfs` (src/checker.rs:124-129): non-blocking; call `join()`."""
        if self._comm is not None or self._partitions > 1:
            # (a visitor's record is gathered from every partition at join, collectively: every
            # rank of a communicator passes a visitor)
            return GpuBfsChecker(self._model, self._opts, self._visitor, comm=self._comm, partitions=self._partitions)
        return GpuBfsChecker(self._model, self._opts, self._visitor)

    spawn_gpu_bfs = spawn_bfs

    def spawn_dfs(self):
        """`spawn_dfs` (src/checker.rs:131-136, src/checker/dfs.rs) on the GPU engine.

        A check that runs to completion (no early exit) visits the same reachable set whatever the
        traversal, so `unique_state_count`, `state_count`, `is_done` and the set of discovered
        properties equal the reference DFS's; the engine explores level by level (FAST order) and
        its discovery paths are BFS-tree paths (valid, and shortest). When every property gets
        discovered, the reference stops at an order-dependent point of its depth-first order, and
        the counts then differ. `symmetry()` is refused: the reference's representatives
        (e.g. examples/2pc.rs:164-182) are not canonical forms, so the reduced count depends on the
        DFS visit order itself (2pc N=5: 665 in DFS order, tests/test_oracle_dfs.py), which a
        level-synchronous search cannot reproduce."""
        if self._symmetry:
            raise NotImplementedError(
                "symmetry().spawn_dfs(): the symmetry-reduced count depends on the reference's "
                "depth-first visit order (non-canonical representatives); not reproducible on the GPU. "
                "symmetry_canonical() gives an order-independent reduction (one state per orbit)")
        self._opts.order = N.SR_ORDER_FAST
        return self.spawn_bfs()

    def serve(self, address=("127.0.0.1", 3000), block=True):
        """`serve` (src/checker.rs:107-113, src/checker/explorer.rs:71-129): spawns the GPU check and
        serves the Explorer's JSON routes (`/.status`, `/.states/<fp>/<fp>/...`) and a small UI over
        it. Blocks like the reference unless block=False, which returns the running
        `stateright_amd.explorer.Explorer` (its `.checker`, `.url`, `.shutdown()`)."""
        from .explorer import Explorer
        ex = Explorer(self.spawn_bfs(), address)
        if not block:
            return ex.start()
        try:
            ex.serve_forever()
        finally:
            ex.shutdown()
        return ex.checker


class GpuBfsChecker:
    """The `Checker` trait (src/checker.rs:184-338) implemented by the MI355X engine."""

    def __init__(self, model, opts, visitor=None, comm=None, partitions=1):
        lib = N.load()
        self._lib = lib
        self._model = model
        self._visitor = visitor
        self._comm = comm
        params = list(model.params())
        arr = (ctypes.c_int64 * max(1, len(params)))(*params)
        plugin = getattr(model, "plugin", None)
        if plugin is not None:  # a GpuModel compiled into its own library (stateright_amd.plugin)
            if comm is not None or partitions > 1:
                self._h = lib.sr_gpu_bfs_spawn_plugin_partitioned(plugin.handle, comm.handle if comm is not None else None,
                                                                  partitions, arr, len(params), ctypes.byref(opts))
            else:
                self._h = lib.sr_gpu_bfs_spawn_plugin(plugin.handle, arr, len(params), ctypes.byref(opts))
        elif comm is not None or partitions > 1:
            self._h = lib.sr_gpu_bfs_spawn_partitioned(comm.handle if comm is not None else None, partitions,
                                                       model.MODEL_ID, arr, len(params), ctypes.byref(opts))
        else:
            self._h = lib.sr_gpu_bfs_spawn(model.MODEL_ID, arr, len(params), ctypes.byref(opts))
        if not self._h:
            raise CheckerError("sr_gpu_bfs_spawn")
        self._joined = False
        self._props = None
        self._names = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.sr_gpu_bfs_free(h)
            self._h = None

    # --- Checker trait -------------------------------------------------------------------------
    def model(self):
        return self._model

    def state_count(self):
        return self._lib.sr_gpu_bfs_state_count(self._h)

    def unique_state_count(self):
        return self._lib.sr_gpu_bfs_unique_state_count(self._h)

    def max_depth(self):
        return self._lib.sr_gpu_bfs_max_depth(self._h)

    def join(self):
        if not self._joined:
            st = self._lib.sr_gpu_bfs_join(self._h)
            self._joined = True
            if st != 0:
                raise CheckerError("sr_gpu_bfs_join", st)
            if isinstance(self._visitor, StateRecorder):
                self._visitor.states.extend(self.visits())
            elif self._visitor is not None:
                visit = self._visitor.visit if isinstance(self._visitor, PathRecorder) else self._visitor
                for path in self.visit_paths():
                    visit(path)
        return self

    def is_done(self):
        return bool(self._lib.sr_gpu_bfs_is_done(self._h))

    def properties(self):
        if self._props is None:
            out = []
            buf = ctypes.create_string_buffer(256)
            exp = ctypes.c_int32()
            for i in range(self._lib.sr_gpu_bfs_property_count(self._h)):
                self._lib.sr_gpu_bfs_property(self._h, i, buf, 256, ctypes.byref(exp))
                out.append((buf.value.decode(), Expectation(exp.value)))
            self._props = out
        return self._props

    def _prop_index(self, name):
        for i, (n, _) in enumerate(self.properties()):
            if n == name:
                return i
        raise KeyError(f"Unknown property. requested={name}, available={[n for n, _ in self.properties()]}")

    def action_name(self, action_id):
        if action_id not in self._names:
            buf = ctypes.create_string_buffer(256)
            self._lib.sr_gpu_bfs_action_name(self._h, action_id, buf, 256)
            self._names[action_id] = buf.value.decode()
        return self._names[action_id]

    def action_id(self, action):
        if isinstance(action, int):
            return action
        for i in range(self._lib.sr_gpu_bfs_action_id_bound(self._h)):
            if self.action_name(i) == action:
                return i
        raise KeyError(f"unknown action {action!r}")

    def discovery_fingerprints(self, name):
        """The fingerprint chain init..discovery (`reconstruct_path` input, bfs.rs:314-342)."""
        i = self._prop_index(name)
        buf = (ctypes.c_uint64 * 65536)()
        n = self._lib.sr_gpu_bfs_discovery(self._h, i, buf, 65536)
        if n < 0:
            raise CheckerError("sr_gpu_bfs_discovery", n)
        return list(buf[:n])

    def discovery(self, name):
        """`discovery` (src/checker.rs:211-213): the Path for `name`, or None."""
        i = self._prop_index(name)
        acts = (ctypes.c_int64 * 65536)()
        width = self._lib.sr_gpu_bfs_describe_width(self._h)
        states = (ctypes.c_int64 * (65536 * max(1, width)))()
        n = self._lib.sr_gpu_bfs_discovery_path(self._h, i, acts, 65536, states, 65536 * max(1, width))
        if n == -1:
            return None
        if n < 0:
            raise CheckerError("sr_gpu_bfs_discovery_path", n)
        flat = list(states[:(n + 1) * width])
        st = [tuple(flat[k:k + width]) for k in range(0, len(flat), width)]
        ids = list(acts[:n])
        return Path(st, ids, [self.action_name(a) for a in ids])

    def discoveries(self):
        """`discoveries` (src/checker/bfs.rs:289-298): property name -> Path."""
        out = {}
        for name, _ in self.properties():
            p = self.discovery(name)
            if p is not None:
                out[name] = p
        return out

    def visits(self):
        width = self._lib.sr_gpu_bfs_describe_width(self._h)
        n = self._lib.sr_gpu_bfs_visits(self._h, None, 0)
        buf = (ctypes.c_int64 * max(1, n))()
        self._lib.sr_gpu_bfs_visits(self._h, buf, n)
        flat = list(buf[:n])
        return [tuple(flat[k:k + width]) for k in range(0, n, width)]

    def explore(self, fingerprints):
        """Explorer's `states` view (src/checker/explorer.rs:159-240): [(action name or None, state
        description or None, fingerprint or None)] of the init states (no fingerprints) or of the
        steps following the state the fingerprint path leads to; None if no state follows."""
        n = len(fingerprints)
        fps = (ctypes.c_uint64 * max(1, n))(*fingerprints)
        width = self._lib.sr_gpu_bfs_describe_width(self._h)
        cap = 64
        while True:  # re-called with room for every view when the first buffer is too small
            acts = (ctypes.c_int64 * cap)()
            has = (ctypes.c_int32 * cap)()
            fpo = (ctypes.c_uint64 * cap)()
            st = (ctypes.c_int64 * (cap * max(1, width)))()
            v = self._lib.sr_gpu_bfs_explore(self._h, fps, n, acts, has, fpo, st, cap)
            if v == -1:
                return None
            if v < 0:
                raise CheckerError("sr_gpu_bfs_explore", v)
            if v <= cap:
                break
            cap = v
        out = []
        for i in range(v):
            name = None if acts[i] < 0 else self.action_name(acts[i])
            if has[i]:
                out.append((name, tuple(st[i * width:(i + 1) * width]), fpo[i]))
            else:
                out.append((name, None, None))
        return out

    def visit_paths(self):
        """The path to every visited state, in visit order (what the reference hands to its
        visitor at each pop, src/checker/bfs.rs:187-189)."""
        n = self._lib.sr_gpu_bfs_visit_tree(self._h, None, None, 0)
        if n < 0:
            raise CheckerError("sr_gpu_bfs_visit_tree", n)
        parent = (ctypes.c_int64 * max(1, n))()
        action = (ctypes.c_int64 * max(1, n))()
        self._lib.sr_gpu_bfs_visit_tree(self._h, parent, action, n)
        states = self.visits()
        out = []
        for i in range(n):
            chain = []
            j = i
            while j >= 0:
                chain.append(j)
                j = parent[j]
            chain.reverse()
            ids = [action[k] for k in chain[1:]]
            out.append(Path([states[k] for k in chain], ids, [self.action_name(a) for a in ids]))
        return out

    def stats(self):
        s = N.sr_stats()
        self._lib.sr_gpu_bfs_stats_sized(self._h, ctypes.byref(s), ctypes.sizeof(s))
        return s.as_dict()

    def launch_profile(self):
        """profile(): [(kernel_ms, frontier)] of every expand launch, in launch order."""
        n = self._lib.sr_gpu_bfs_launch_profile(self._h, None, None, 0)
        ms = (ctypes.c_double * max(1, n))()
        fr = (ctypes.c_uint64 * max(1, n))()
        self._lib.sr_gpu_bfs_launch_profile(self._h, ms, fr, n)
        return [(ms[i], fr[i]) for i in range(n)]

    def launch_counters(self):
        """[(probes, cas)] of every expand launch (builder.counters(); zeros otherwise)."""
        n = self._lib.sr_gpu_bfs_launch_counters(self._h, None, None, 0)
        pr = (ctypes.c_uint64 * max(1, n))()
        cs = (ctypes.c_uint64 * max(1, n))()
        self._lib.sr_gpu_bfs_launch_counters(self._h, pr, cs, n)
        return [(pr[i], cs[i]) for i in range(n)]

    # --- report / asserts (src/checker.rs:216-337) ---------------------------------------------
    def discovery_classification(self, name):
        exp = dict(self.properties())[name]
        return "example" if exp == Expectation.Sometimes else "counterexample"

    def report(self, w=None):
        w = w or sys.stdout
        start = time.monotonic()
        # `report` polls once per second while checking (src/checker.rs:223-228).
        while not self._joined and not self.is_done():
            w.write(f"Checking. states={self.state_count()}, unique={self.unique_state_count()}\n")
            for _ in range(100):
                if not self._lib.sr_gpu_bfs_is_running(self._h):
                    break
                time.sleep(0.01)
            if not self._lib.sr_gpu_bfs_is_running(self._h):
                break
        self.join()
        w.write(f"Done. states={self.state_count()}, unique={self.unique_state_count()}, "
                f"sec={int(time.monotonic() - start)}\n")
        for name, path in self.discoveries().items():
            w.write(f'Discovered "{name}" {self.discovery_classification(name)} {path}')
        return self

    def assert_properties(self):
        for name, exp in self.properties():
            if exp == Expectation.Sometimes:
                self.assert_any_discovery(name)
            else:
                self.assert_no_discovery(name)

    def assert_any_discovery(self, name):
        found = self.discovery(name)
        if found is not None:
            return found
        assert self.is_done(), f'Discovery for "{name}" not found, but model checking is incomplete.'
        raise AssertionError(f'Discovery for "{name}" not found.')

    def assert_no_discovery(self, name):
        found = self.discovery(name)
        if found is not None:
            raise AssertionError(f'Unexpected "{name}" {self.discovery_classification(name)} {found}'
                                 f"Last state: {found.last_state()}\n")
        assert self.is_done(), f'Discovery for "{name}" not found, but model checking is incomplete.'

    def replay(self, actions, init_index=0):
        """`Path::from_actions` on the host copy of the model: (states, conditions) or None."""
        ids = [self.action_id(a) for a in actions]
        arr = (ctypes.c_int64 * max(1, len(ids)))(*ids)
        width = self._lib.sr_gpu_bfs_describe_width(self._h)
        states = (ctypes.c_int64 * ((len(ids) + 1) * width))()
        conds = (ctypes.c_int32 * 64)()
        n = self._lib.sr_gpu_bfs_replay(self._h, init_index, arr, len(ids), states, (len(ids) + 1) * width, conds, 64)
        if n < 0:
            return None
        flat = list(states)
        return [tuple(flat[k:k + width]) for k in range(0, len(flat), width)], list(conds[:len(self.properties())])

    def replay_trace(self, actions, init_index=0):
        """`Path::from_actions`: (per-state conditions [[cond of property p] per state], last state
        terminal?) or None if an action is not enabled along the way."""
        ids = [self.action_id(a) for a in actions]
        arr = (ctypes.c_int64 * max(1, len(ids)))(*ids)
        n_props = len(self.properties())
        conds = (ctypes.c_int32 * max(1, (len(ids) + 1) * n_props))()
        term = ctypes.c_int32()
        n = self._lib.sr_gpu_bfs_replay_trace(self._h, init_index, arr, len(ids), conds, len(conds), ctypes.byref(term))
        if n < 0:
            return None
        flat = list(conds)
        return [flat[k * n_props:(k + 1) * n_props] for k in range(len(ids) + 1)], bool(term.value)

    def assert_discovery(self, name, actions):
        """`assert_discovery` (src/checker.rs:292-337): the actions, from some init state, lead to a
        state violating an `always` / satisfying a `sometimes` property, or along a path on which
        an `eventually` property never holds and that ends at a terminal state."""
        found = self.assert_any_discovery(name)
        i = self._prop_index(name)
        exp = self.properties()[i][1]
        info = []
        for init in range(self._lib.sr_gpu_bfs_init_count(self._h)):
            r = self.replay_trace(actions, init)
            if r is None:
                continue
            per_state, terminal = r
            last = per_state[-1][i]
            if exp == Expectation.Always and not last:
                return
            if exp == Expectation.Sometimes and last:
                return
            if exp == Expectation.Eventually:
                satisfied = any(s[i] for s in per_state)
                if not satisfied and terminal:
                    return
                if satisfied:
                    info.append("incorrect counterexample satisfies eventually property")
                if not terminal:
                    info.append("incorrect counterexample is nonterminal")
        extra = f" ({'; '.join(info)})" if info else ""
        raise AssertionError(f'Invalid discovery for "{name}"{extra}, but a valid one was found. '
                             f"found={found.into_actions()}")
