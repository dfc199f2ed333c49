"""Pins the oracle's depth-first checker (oracle/dfs.hpp, a restatement of src/checker/dfs.rs) to
the reference's own DFS goldens, and shows why symmetry reduction is order-dependent.

Every expected value is quoted from /root/reference (cited per test)."""
from oracle_lib import LINEAR_EQUATION, SYM_TOY, TWO_PHASE, OracleRun, replay

INCREASE_X, INCREASE_Y = 0, 1


def test_visits_states_in_dfs_order():
    # src/checker/dfs.rs:349-363
    r = OracleRun(LINEAR_EQUATION, [2, 10, 14], dfs=True, record_visits=True)
    assert r.visits() == [(0, y) for y in range(28)]


def test_can_complete_by_enumerating_all_states():
    # src/checker/dfs.rs:365-372
    r = OracleRun(LINEAR_EQUATION, [2, 4, 7], dfs=True)
    assert r.is_done and r.discovery_names() == [] and r.unique_state_count == 256 * 256


def test_can_complete_by_eliminating_properties():
    # src/checker/dfs.rs:374-391
    r = OracleRun(LINEAR_EQUATION, [2, 10, 14], dfs=True)
    assert r.unique_state_count == 55
    assert r.discovery_actions("solvable") == [INCREASE_Y] * 27
    states, holds = replay(LINEAR_EQUATION, [2, 10, 14], [INCREASE_X, INCREASE_Y, INCREASE_X])
    assert holds[0] == 1


def test_2pc_dfs_and_symmetry_goldens():
    # examples/2pc.rs:131-139
    assert OracleRun(TWO_PHASE, [5], dfs=True).unique_state_count == 8_832
    sym = OracleRun(TWO_PHASE, [5], dfs=True, symmetry=True)
    assert sym.unique_state_count == 665
    assert sym.discovery_names() == ["abort agreement", "commit agreement"]  # assert_properties


def test_symmetry_fixture_goldens():
    # src/checker/dfs.rs:470-481: 9 states without reduction (DFS and BFS), 6 with.
    assert OracleRun(SYM_TOY, [], dfs=True).unique_state_count == 9
    assert OracleRun(SYM_TOY, []).unique_state_count == 9
    r = OracleRun(SYM_TOY, [], dfs=True, symmetry=True, record_visits=True)
    assert r.unique_state_count == 6
    # PathRecorder in that test panics on an invalid path: every visit's path must replay.
    for actions, state in zip(r.visit_paths(), r.visits()):
        states, _ = replay(SYM_TOY, [], actions, n_props=2)
        assert tuple(states[-2:]) == state


def test_full_exploration_counts_are_traversal_independent():
    # What the GPU engine's spawn_dfs relies on: without an early exit, DFS and BFS visit the same
    # reachable set and generate the same successors.
    for n in range(1, 6):
        d, b = OracleRun(TWO_PHASE, [n], dfs=True), OracleRun(TWO_PHASE, [n])
        assert (d.unique_state_count, d.state_count, d.discovery_names()) == \
               (b.unique_state_count, b.state_count, b.discovery_names())


def test_symmetry_reduction_depends_on_visit_order():
    # The 2pc representative sorts RMs by rm_state only (examples/2pc.rs:164-182 via
    # RewritePlan::from_values_to_sort, src/checker/rewrite_plan.rs:36-49), so RMs with equal
    # rm_state keep their index order and symmetric states can have different representatives.
    # Which of them get generated depends on which originals are expanded first: the reduced counts
    # grow differently from the unreduced ones in DFS order and are not a function of the state
    # space alone (a level-synchronous search keyed by the same representative reaches 508 at
    # N = 5, not 665). Pinned here: the reference-order values.
    got = [OracleRun(TWO_PHASE, [n], dfs=True, symmetry=True).unique_state_count for n in range(1, 7)]
    assert got == [12, 38, 107, 276, 665, 1521]
