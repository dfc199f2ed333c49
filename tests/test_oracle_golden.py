"""Pins the CPU oracle (oracle/) to the reference's own BFS goldens.

Every expected value here is quoted from a test or doc in /root/reference (cited per test).
"""
import pytest

from oracle_lib import (BINARY_CLOCK, DGRAPH, INCREMENT, INCREMENT_LOCK, LINEAR_EQUATION, PAXOS, TWO_PHASE,
                        OracleRun, dgraph_params, replay)
from paxos_golden import PAXOS_VALUE_CHOSEN_PATH

INCREASE_X, INCREASE_Y = 0, 1


def test_visits_states_in_bfs_order():
    # src/checker/bfs.rs:351-364
    r = OracleRun(LINEAR_EQUATION, [2, 10, 14], record_visits=True)
    assert r.visits() == [(0, 0), (1, 0), (0, 1), (2, 0), (1, 1), (0, 2), (3, 0), (2, 1)]


def test_can_complete_by_enumerating_all_states():
    # src/checker/bfs.rs:367-372
    r = OracleRun(LINEAR_EQUATION, [2, 4, 7])
    assert r.is_done
    assert r.discovery_names() == []
    assert r.unique_state_count == 256 * 256


def test_can_complete_by_eliminating_properties():
    # src/checker/bfs.rs:375-388
    r = OracleRun(LINEAR_EQUATION, [2, 10, 14])
    assert r.unique_state_count == 12
    assert r.discovery_actions("solvable") == [INCREASE_X, INCREASE_X, INCREASE_Y]
    # assert_discovery("solvable", vec![IncreaseY; 27]) is also a valid discovery.
    states, holds = replay(LINEAR_EQUATION, [2, 10, 14], [INCREASE_Y] * 27)
    assert states[-2:] == [0, 27] and holds[0] == 1


def test_report_bfs():
    # src/checker.rs:449-468
    r = OracleRun(LINEAR_EQUATION, [2, 10, 14])
    out = r.report()
    assert out.startswith("Done. states=15, unique=12, sec=")
    assert out.endswith('Discovered "solvable" example Path[3]:\n- IncreaseX\n- IncreaseX\n- IncreaseY\n')


def test_2pc_bfs_288():
    # examples/2pc.rs:127-129: BFS unique 288 + assert_properties.
    r = OracleRun(TWO_PHASE, [3])
    assert r.unique_state_count == 288
    assert r.is_done
    # sometimes: abort/commit agreement discovered; always: consistent not discovered.
    assert r.discovery_names() == ["abort agreement", "commit agreement"]


def test_2pc_5_8832():
    # examples/2pc.rs:132-134 (full exploration: the unique count is traversal independent).
    r = OracleRun(TWO_PHASE, [5])
    assert r.unique_state_count == 8832


@pytest.mark.parametrize("threads", [2, 4])
def test_2pc_multithreaded_counts_match(threads):
    # Full-exploration counts do not depend on the job market's interleaving.
    r1 = OracleRun(TWO_PHASE, [5])
    rt = OracleRun(TWO_PHASE, [5], threads=threads)
    assert (rt.unique_state_count, rt.state_count, rt.max_depth) == (r1.unique_state_count, r1.state_count, r1.max_depth)


@pytest.mark.parametrize("n", range(1, 7))
def test_2pc_closed_forms(n):
    # SURVEY.md §0.5 closed forms, fitted on the restatement and anchored at 288 / 8 832.
    r = OracleRun(TWO_PHASE, [n])
    assert r.unique_state_count == 6 ** n + 4 ** n + 2 ** n
    assert 3 * r.state_count == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert r.max_depth == 3 * n + 1


@pytest.mark.parametrize("n", range(1, 7))
def test_increment_lock_closed_form(n):
    from math import factorial
    r = OracleRun(INCREMENT_LOCK, [n])
    expect = 1 + 4 * sum(factorial(n) // factorial(n - k) for k in range(1, n + 1))
    assert r.unique_state_count == r.state_count == expect
    assert r.max_depth == 4 * n
    assert r.discovery_names() == []


@pytest.mark.parametrize("n,unique,states", [(8, 1158, 1774), (10, 2379, 3867), (12, 4293, 7340)])
def test_increment_early_exit(n, unique, states):
    # BASELINE.md §3 (single-thread FIFO order); `fin` found at depth 4.
    r = OracleRun(INCREMENT, [n])
    assert (r.unique_state_count, r.state_count) == (unique, states)
    assert r.discovery_names() == ["fin"]
    assert len(r.discovery_actions("fin")) == 4


def test_binary_clock():
    # src/test_util.rs:4-45 / src/checker/explorer.rs:249-255: two init states, both visited.
    # `pending` is built in init order and popped from the BACK (bfs.rs:61-66,183), so the init
    # states are visited in reverse order.
    r = OracleRun(BINARY_CLOCK, [], record_visits=True)
    assert r.unique_state_count == 2 and r.visits() == [(1,), (0,)]
    assert r.discovery_names() == []


EVENTUALLY = 1


def _odd(*paths):
    return OracleRun(DGRAPH, dgraph_params(EVENTUALLY, paths))


def test_eventually_can_validate():
    # src/checker.rs:358-376
    assert _odd([1], [2, 3], [2, 6, 7], [4, 9, 10]).discovery_names() == []
    for p in ([1], [2, 3], [2, 6, 7], [4, 9, 10]):
        assert _odd(p).discovery_names() == []


def test_eventually_can_discover_counterexample():
    # src/checker.rs:378-398
    assert _odd([0, 1], [0, 2]).discovery_states("odd") == [(0,), (2,)]
    assert _odd([0, 1], [2, 4]).discovery_states("odd") == [(2,), (4,)]
    assert _odd([0, 1, 4, 6], [2, 4, 8]).discovery_states("odd") == [(2,), (4,), (6,)]


def test_eventually_fixme_misses_counterexample_when_revisiting():
    # src/checker.rs:400-413 (known false negatives are part of the reference semantics)
    assert _odd([0, 2, 4, 2]).discovery_states("odd") is None
    assert _odd([0, 2, 4], [1, 4, 6]).discovery_states("odd") is None


@pytest.mark.slow
def test_2pc_7_counts():
    r = OracleRun(TWO_PHASE, [7], threads=4)
    assert r.unique_state_count == 6 ** 7 + 4 ** 7 + 2 ** 7


def test_paxos_2_clients_golden():
    # examples/paxos.rs:268-290 (BFS half): assert_properties, the "value chosen" example path and
    # unique_state_count 16_668. The reference's own discovery depends on its HashSet iteration
    # order; the golden path must be a valid discovery (assert_discovery replays it) and every BFS
    # discovery is a shortest path of the same length.
    r = OracleRun(PAXOS, [2])
    assert r.unique_state_count == 16_668
    assert r.discovery_names() == ["value chosen"]  # "linearizable" holds everywhere
    states, holds = replay(PAXOS, [2], PAXOS_VALUE_CHOSEN_PATH, n_props=2)
    assert holds == [1, 1]
    assert len(r.discovery_actions("value chosen")) == len(PAXOS_VALUE_CHOSEN_PATH)


def test_paxos_golden_path_prefix_is_no_discovery():
    # The 7-step prefix of the golden path leaves no GetOk in flight: "value chosen" is false there.
    _, holds = replay(PAXOS, [2], PAXOS_VALUE_CHOSEN_PATH[:-1], n_props=2)
    assert holds == [1, 0]


def test_paxos_multithreaded_counts_match():
    a = OracleRun(PAXOS, [2], threads=1)
    b = OracleRun(PAXOS, [2], threads=4)
    assert (a.unique_state_count, a.state_count, a.max_depth) == (b.unique_state_count, b.state_count, b.max_depth)


@pytest.mark.slow
def test_paxos_3_clients_counts():
    # BASELINE.json config 5 (`paxos check 3`); counts pinned by the oracle (parity for C = 3 is
    # anchored on the C = 2 reference golden above).
    r = OracleRun(PAXOS, [3], threads=8)
    assert (r.unique_state_count, r.state_count, r.max_depth) == (1_194_428, 2_420_477, 27)
