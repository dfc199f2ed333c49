"""`eventually` properties on the MI355X engine (src/checker/bfs.rs:52-60,212-222,265-272) against
the reference's own tests (src/checker.rs:349-414) and the CPU oracle on random graphs.

The GPU keeps one EventuallyBits word per frontier state, finds each level's terminal states, and
reproduces the reference's overwrite-at-terminal semantics in its FIFO order (the default for
eventually models). An explicit FAST order gives each state the bits of the generator that claims
it, one of the reference's multi-threaded orders: its discoveries are valid counterexamples, and
on graphs without joins (where no order can lose one) the same as the oracle's. The partitioned
search carries the bits in an extra word of every state and record (models.hpp EvBits), with the
same claiming-generator rule.
"""
import random

import pytest

from oracle_lib import DGRAPH, OracleRun, dgraph_params

pytestmark = pytest.mark.gpu

sr = pytest.importorskip("stateright_amd")

ALWAYS, EVENTUALLY, SOMETIMES = 0, 1, 2


def odd(*paths, expectation=EVENTUALLY):
    g = sr.DGraph.with_property(expectation)
    for p in paths:
        g = g.with_path(p)
    return g.checker().spawn_bfs().join()


def test_can_validate():
    # src/checker.rs:358-376
    odd([1], [2, 3], [2, 6, 7], [4, 9, 10]).assert_properties()
    for p in ([1], [2, 3], [2, 6, 7], [4, 9, 10]):
        odd(p).assert_properties()


def test_can_discover_counterexample():
    # src/checker.rs:378-398
    assert odd([0, 1], [0, 2]).discovery("odd").into_states() == [(0,), (2,)]
    assert odd([0, 1], [2, 4]).discovery("odd").into_states() == [(2,), (4,)]
    assert odd([0, 1, 4, 6], [2, 4, 8]).discovery("odd").into_states() == [(2,), (4,), (6,)]


def test_fixme_can_miss_counterexample_when_revisiting_a_state():
    # src/checker.rs:400-413: known false negatives are part of the reference semantics
    assert odd([0, 2, 4, 2]).discovery("odd") is None
    assert odd([0, 2, 4], [1, 4, 6]).discovery("odd") is None


def test_report_says_counterexample():
    import io
    w = io.StringIO()
    g = sr.DGraph.with_property(EVENTUALLY).with_path([0, 1]).with_path([0, 2])
    g.checker().spawn_bfs().report(w)
    assert 'Discovered "odd" counterexample Path[1]:\n- 2\n' in w.getvalue()


def _random_graph(rng):
    paths = []
    for _ in range(rng.randint(1, 6)):
        n = rng.randint(1, 7)
        paths.append([rng.randrange(0, 24) for _ in range(n)])
    return paths


@pytest.mark.parametrize("expectation", [ALWAYS, EVENTUALLY, SOMETIMES])
def test_random_graphs_match_oracle(expectation):
    rng = random.Random(1234 + expectation)
    for _ in range(60):
        paths = _random_graph(rng)
        o = OracleRun(DGRAPH, dgraph_params(expectation, paths))
        c = odd(*paths, expectation=expectation)
        assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (
            o.unique_state_count, o.state_count, o.max_depth), paths
        assert sorted(c.discoveries()) == o.discovery_names(), paths
        assert c.is_done() == o.is_done, paths
        if o.discovery_names():
            assert c.discovery("odd").into_states() == o.discovery_states("odd"), paths


def _graph(paths):
    g = sr.DGraph.with_property(EVENTUALLY)
    for p in paths:
        g = g.with_path(p)
    return g


@pytest.mark.parametrize("head", ["0", "65536"])
@pytest.mark.parametrize("parts", [2, 3])
def test_partitioned_eventually_matches_oracle_without_joins(parts, head, monkeypatch):
    # The partitioned search carries each state's EventuallyBits in an extra word of its records
    # (models.hpp EvBits): the claiming generator's bits, as in FAST order on one GPU. On graphs
    # without joins every order finds the oracle's discoveries; a check without one explores
    # everything, with the oracle's counts.
    monkeypatch.setenv("SR_HEAD_MAX", head)
    rng = random.Random(99 + parts)
    for _ in range(40):
        paths = _chains(rng)
        o = OracleRun(DGRAPH, dgraph_params(EVENTUALLY, paths))
        c = _graph(paths).checker().partitions(parts).spawn_bfs().join()
        assert sorted(c.discoveries()) == o.discovery_names(), paths
        for name, path in c.discoveries().items():
            c.assert_discovery(name, path.action_ids)
        if not o.discovery_names():
            assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (
                o.unique_state_count, o.state_count, o.max_depth), paths


def test_partitioned_eventually_reference_cases(monkeypatch):
    # src/checker.rs:358-398 on 2 and 3 partitions, from level 0 (no replicated head)
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    for parts in (2, 3):
        _graph([[1], [2, 3], [2, 6, 7], [4, 9, 10]]).checker().partitions(parts).spawn_bfs().join().assert_properties()
        for paths, last in ([[[0, 1], [0, 2]], 2], [[[0, 1], [2, 4]], 4]):
            c = _graph(paths).checker().partitions(parts).spawn_bfs().join()
            assert c.discovery("odd").last_state() == (last,)
            c.assert_discovery("odd", c.discovery("odd").action_ids)
        c = _graph([[0, 1, 4, 6], [2, 4, 8]]).checker().partitions(parts).spawn_bfs().join()
        assert c.discovery("odd").last_state() in ((6,), (8,))
        c.assert_discovery("odd", c.discovery("odd").action_ids)


@pytest.mark.parametrize("parts", [2, 4])
def test_partitioned_eventually_discoveries_are_valid(parts, monkeypatch):
    # graphs with joins: whatever the partitioned order reports is a valid counterexample
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    rng = random.Random(2024 + parts)
    for _ in range(40):
        paths = _random_graph(rng)
        c = _graph(paths).checker().partitions(parts).spawn_bfs().join()
        for name, path in c.discoveries().items():
            c.assert_discovery(name, path.action_ids)


def test_partitioned_eventually_ranks(monkeypatch):
    # in-process ranks (the exchange between ranks carries the bit word with the state)
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    from stateright_amd.distributed import Communicator
    paths = [[0, 2, 4, 6], [1, 3], [8, 10, 12]]
    o = OracleRun(DGRAPH, dgraph_params(EVENTUALLY, paths))
    comms = Communicator.local_group(2)
    try:
        cs = [_graph(paths).checker().comm(cm).spawn_bfs() for cm in comms]
        for c in cs:
            c.join()
        for c in cs:
            assert sorted(c.discoveries()) == o.discovery_names()
            c.assert_discovery("odd", c.discovery("odd").action_ids)
        cs.clear()
    finally:
        for cm in comms:
            cm.close()


def test_assert_discovery_eventually():
    # src/checker.rs:306-323: an `eventually` counterexample is valid when the condition holds on
    # no state of the path and the path ends at a terminal state (no actions)
    c = odd([0, 1], [0, 2])
    c.assert_discovery("odd", [2])
    with pytest.raises(AssertionError, match="satisfies eventually property"):
        c.assert_discovery("odd", [1])
    c = odd([0, 1, 4, 6], [2, 4, 8])
    c.assert_discovery("odd", [4, 6])       # 2 -> 4 -> 6, terminal, never odd
    c.assert_discovery("odd", [4, 8])       # 2 -> 4 -> 8 as well
    with pytest.raises(AssertionError, match="is nonterminal"):
        c.assert_discovery("odd", [4])      # 2 -> 4 has successors
    with pytest.raises(AssertionError, match="Invalid discovery"):
        c.assert_discovery("odd", [7])      # not an action anywhere


def test_replay_trace_conditions_every_state():
    c = odd([0, 1, 4, 6], [2, 4, 8])
    per_state, terminal = c.replay_trace([1, 4, 6], init_index=0)  # 0 -> 1 -> 4 -> 6
    assert [s[0] for s in per_state] == [0, 1, 0, 0] and terminal


def _chains(rng):
    # disjoint chains: no state has two generators, so no visit order can lose a counterexample
    labels = rng.sample(range(0, 200), 40)
    paths, k = [], 0
    for _ in range(rng.randint(1, 6)):
        n = rng.randint(1, 6)
        paths.append(labels[k:k + n])
        k += n
    return paths


def test_fast_order_eventually_matches_oracle_without_joins():
    rng = random.Random(77)
    for _ in range(60):
        paths = _chains(rng)
        o = OracleRun(DGRAPH, dgraph_params(EVENTUALLY, paths))
        g = sr.DGraph.with_property(EVENTUALLY)
        for p in paths:
            g = g.with_path(p)
        c = g.checker().order("fast").spawn_bfs().join()
        assert c.stats()["order_used"] == 2, paths  # FAST honoured
        assert sorted(c.discoveries()) == o.discovery_names(), paths
        for name, path in c.discoveries().items():
            c.assert_discovery(name, path.action_ids)


def test_fast_order_eventually_discoveries_are_valid():
    # graphs with joins (the reference's known false negatives depend on the order): whatever FAST
    # reports is a valid counterexample (never satisfied along the path, ending at a terminal state)
    rng = random.Random(4321)
    for _ in range(60):
        paths = _random_graph(rng)
        g = sr.DGraph.with_property(EVENTUALLY)
        for p in paths:
            g = g.with_path(p)
        c = g.checker().order("fast").spawn_bfs().join()
        for name, path in c.discoveries().items():
            c.assert_discovery(name, path.action_ids)
