"""Opt-in canonical symmetry reduction (CheckerBuilder.symmetry_canonical) on 2pc: one
representative per orbit of the resource-manager permutations. Expected values come from the CPU
oracle's FULL visit list: the orbits are the distinct canonical forms of its reachable states, and
state_count is the init state plus every representative's out-degree (examples/2pc.rs:56-104 lists
the actions; every one returns Some). This is NOT the reference's `symmetry().spawn_dfs()` count
(665 at N=5, order-dependent: tests/test_symmetry_order.py); see DESIGN.md §7."""
import pytest

from oracle_lib import TWO_PHASE, OracleRun, replay

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")


def split(d, n):
    return d[:n], d[n], d[n + 1:2 * n + 1], d[2 * n + 1:3 * n + 1], d[3 * n + 1], d[3 * n + 2]


def canon(d, n):
    rm, tm, prep, msg, commit, abort = split(d, n)
    keys = sorted(rm[i] | prep[i] << 2 | msg[i] << 3 for i in range(n))
    return tuple([k & 3 for k in keys] + [tm] + [k >> 2 & 1 for k in keys] + [k >> 3 & 1 for k in keys] + [commit, abort])


def outdeg(d, n):
    rm, tm, prep, msg, commit, abort = split(d, n)
    k = (tm == 0 and all(prep)) + (tm == 0)
    for i in range(n):
        k += (tm == 0 and msg[i]) + 2 * (rm[i] == 0) + commit + abort
    return k


_orbits = {}


def orbits(n):
    if n not in _orbits:
        o = OracleRun(TWO_PHASE, [n], record_visits=True)
        reps = {canon(v, n) for v in o.visits()}
        _orbits[n] = (o, reps, 1 + sum(outdeg(r, n) for r in reps))
    return _orbits[n]


@pytest.mark.parametrize("order", ["fifo", "fast"])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7])
def test_orbit_counts(n, order):
    o, reps, sc = orbits(n)
    c = sr.TwoPhaseSys(n).checker().symmetry_canonical().order(order).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (len(reps), sc, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()
    for name, path in c.discoveries().items():  # concrete paths of the original model, shortest
        r = replay(TWO_PHASE, [n], path.action_ids, n_props=3)
        assert r is not None and r[1][["abort agreement", "commit agreement", "consistent"].index(name)] == 1
        assert len(path) == len(o.discovery_actions(name))


def test_visits_are_the_representatives():
    n = 4
    _, reps, _ = orbits(n)
    rec = sr.StateRecorder()
    sr.TwoPhaseSys(n).checker().symmetry_canonical().order("fifo").visitor(rec).spawn_bfs().join()
    assert len(rec.states) == len(reps) and set(rec.states) == reps


def test_partitioned_with_symmetry():
    n = 6
    o, reps, sc = orbits(n)
    c = sr.TwoPhaseSys(n).checker().symmetry_canonical().partitions(3).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (len(reps), sc, o.max_depth)


def test_symmetry_requires_a_canonical_form():
    with pytest.raises(sr.CheckerError):
        sr.IncrementLock(3).checker().symmetry_canonical().spawn_bfs()


@pytest.mark.parametrize("partitions", [1, 3])
@pytest.mark.parametrize("n", [2, 3, 4, 5])
def test_discoveries_replay_through_the_engine(n, partitions):
    # The engine's own replay, chain and Explorer walk concrete states of the original model under
    # the canonical reduction: assert_discovery(name, into_actions()) holds for every discovery
    # (RmPrepare(0) then RmPrepare(1) is valid although the representative after the first step
    # has RM 1 prepared), the fingerprint chain has one fingerprint per path state, and the
    # Explorer's `Path::final_state` follows it to the discovered state.
    b = sr.TwoPhaseSys(n).checker().symmetry_canonical().order("fast")
    c = (b.partitions(partitions) if partitions > 1 else b).spawn_bfs().join()
    found = c.discoveries()
    assert found
    for name, path in found.items():
        c.assert_discovery(name, path.into_actions())
        chain = c.discovery_fingerprints(name)
        assert len(chain) == len(path) + 1
        views = c.explore(chain)
        assert views is not None  # the chain is a walk of concrete states
        # the state the chain leads to is the path's last (concrete) state: its successors' views
        # are those of the original model from there
        for action, state, fp in views:
            if state is not None:
                assert len(state) == len(path.last_state())
