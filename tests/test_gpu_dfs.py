"""`spawn_dfs` on the MI355X engine against the oracle's restatement of src/checker/dfs.rs.

Checks that run to completion must match the reference DFS exactly (unique_state_count,
state_count, is_done, discovered properties): the reachable set and the successors generated do
not depend on the traversal. When every property is discovered the reference stops at a point of
its depth-first order; then only the discovered set and `is_done` are compared, and every
discovery path must replay on the CPU model. `symmetry()` is refused (tests/test_symmetry_order.py)."""
import pytest

from oracle_lib import (BINARY_CLOCK, INCREMENT, INCREMENT_LOCK, LINEAR_EQUATION, PAXOS, TWO_PHASE, OracleRun,
                        replay)

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")

MODELS = {
    LINEAR_EQUATION: lambda p: sr.LinearEquation(*p),
    BINARY_CLOCK: lambda p: sr.BinaryClock(),
    TWO_PHASE: lambda p: sr.TwoPhaseSys(*p),
    INCREMENT: lambda p: sr.Increment(*p),
    INCREMENT_LOCK: lambda p: sr.IncrementLock(*p),
    PAXOS: lambda p: sr.Paxos(*p),
}
CASES = [(LINEAR_EQUATION, [2, 4, 7]), (LINEAR_EQUATION, [2, 10, 14]), (BINARY_CLOCK, [])] + \
    [(TWO_PHASE, [n]) for n in range(1, 8)] + [(INCREMENT, [n]) for n in (2, 3, 6)] + \
    [(INCREMENT_LOCK, [n]) for n in (2, 4, 6)] + [(PAXOS, [1]), (PAXOS, [2])]


def ids(c):
    return {LINEAR_EQUATION: "lineq", BINARY_CLOCK: "clock", TWO_PHASE: "2pc", INCREMENT: "inc",
            INCREMENT_LOCK: "inclock", PAXOS: "paxos"}[c[0]] + "-" + "-".join(map(str, c[1]))


@pytest.mark.parametrize("case", CASES, ids=ids)
def test_spawn_dfs_matches_reference_dfs(case):
    model, params = case
    o = OracleRun(model, params, dfs=True)
    c = MODELS[model](params).checker().spawn_dfs().join()
    props = [n for n, _ in c.properties()]
    assert sorted(c.discoveries()) == o.discovery_names()
    assert c.is_done() == o.is_done
    if len(o.discovery_names()) < len(props):  # ran to completion: traversal-independent counts
        assert (c.unique_state_count(), c.state_count()) == (o.unique_state_count, o.state_count)
    for name, path in c.discoveries().items():
        _, holds = replay(model, params, path.action_ids, n_props=len(props))
        assert holds[props.index(name)] == (1 if dict(c.properties())[name] == sr.Expectation.Sometimes else 0)


def test_2pc_5_dfs_golden():
    # examples/2pc.rs:131-134
    c = sr.TwoPhaseSys(5).checker().spawn_dfs().join()
    assert c.unique_state_count() == 8_832
    c.assert_properties()


def test_symmetry_dfs_refused():
    with pytest.raises(NotImplementedError):
        sr.TwoPhaseSys(5).checker().symmetry().spawn_dfs()
    # BFS ignores symmetry, as the reference's does
    assert sr.TwoPhaseSys(3).checker().symmetry().spawn_bfs().join().unique_state_count() == 288
