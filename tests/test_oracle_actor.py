"""Pins the oracle's generic ActorModel restatement (oracle/actor.hpp) to the reference's actor
goldens (ping-pong 14 / 4 094 / 11, undeliverable 1, timer 2, Explorer status 5/5,
ABD register 544). Every expected value is quoted from the reference (cited per test)."""
from actor_golden import (ABD, ABD_VALUE_CHOSEN_PATH, ACTOR_FIXTURE, PINGPONG, PINGPONG_14, PINGPONG_DROP_FIRST_PING,
                          PINGPONG_PROPS, pingpong_params)
from oracle_lib import OracleRun, replay


def prop(name):
    return PINGPONG_PROPS.index(name)


def test_pingpong_visits_expected_states():
    # src/actor/model.rs:515-610: lossy + duplicating network, max_nat 1 -> 14 states, this set
    r = OracleRun(PINGPONG, pingpong_params(1, lossy=True), record_visits=True)
    assert r.unique_state_count == 14
    v = r.visits()
    assert len(v) == 14 and set(v) == PINGPONG_14


def test_pingpong_maintains_fixed_delta_despite_lossy_duplicating_network():
    # src/actor/model.rs:612-623
    r = OracleRun(PINGPONG, pingpong_params(5, lossy=True))
    assert r.unique_state_count == 4_094
    assert "delta within 1" not in r.discovery_names()


def test_pingpong_may_never_reach_max_on_lossy_network():
    # src/actor/model.rs:625-642: assert_discovery("must reach max", [Drop(Ping(0) 0 -> 1)]): the
    # path never satisfies the eventually property and ends at a terminal state
    params = pingpong_params(5, lossy=True)
    r = OracleRun(PINGPONG, params)
    assert r.unique_state_count == 4_094
    assert "must reach max" in r.discovery_names()
    states, holds = replay(PINGPONG, params, PINGPONG_DROP_FIRST_PING)
    w = len(states) // 2
    init, last = states[:w], states[w:]
    assert init[:2] == [0, 0] and last[:2] == [0, 0]  # never reaches max_nat 5
    assert holds[prop("must reach max")] == 0
    assert all(c == -1 for c in last[6:])  # empty network, no timer: terminal


def test_pingpong_eventually_reaches_max_on_perfect_delivery_network():
    # src/actor/model.rs:644-656
    r = OracleRun(PINGPONG, pingpong_params(5, lossy=False, duplicating=False))
    assert r.unique_state_count == 11
    assert "must reach max" not in r.discovery_names()


def test_pingpong_can_reach_max():
    # src/actor/model.rs:658-671: last state of "can reach max" has actor states [4, 5]
    r = OracleRun(PINGPONG, pingpong_params(5, lossy=False))
    assert r.unique_state_count == 11
    assert r.discovery_states("can reach max")[-1][:2] == (4, 5)


def test_pingpong_might_never_reach_beyond_max():
    # src/actor/model.rs:673-694: "must exceed max" discovered at actor states [5, 5]
    r = OracleRun(PINGPONG, pingpong_params(5, lossy=False, duplicating=False))
    assert r.unique_state_count == 11
    assert r.discovery_states("must exceed max")[-1][:2] == (5, 5)


def test_handles_undeliverable_messages():
    # src/actor/model.rs:697-707
    assert OracleRun(ACTOR_FIXTURE, [0]).unique_state_count == 1


def test_resets_timer():
    # src/actor/model.rs:709-733: init state with the timer set, then one without
    r = OracleRun(ACTOR_FIXTURE, [1], record_visits=True)
    assert r.unique_state_count == 2
    assert [v[1:3] for v in r.visits()] == [(1, 1), (1, 0)]  # is_timer_set [true] then [false]


def test_explorer_status_pingpong():
    # src/checker/explorer.rs:370-416: max_nat 2, history kept, no duplication, lossless
    r = OracleRun(PINGPONG, pingpong_params(2, lossy=False, duplicating=False, maintains_history=True))
    assert r.is_done
    assert (r.state_count, r.unique_state_count) == (5, 5)
    assert r.discovery_names() == ["can reach max", "must exceed max"]


def test_abd_linearizable_register():
    # examples/linearizable-register.rs:236-258: 2 clients, 2 servers, BFS
    params = [2, 2]
    r = OracleRun(ABD, params)
    assert r.unique_state_count == 544
    assert r.discovery_names() == ["value chosen"]  # assert_properties: linearizable holds
    states, holds = replay(ABD, params, ABD_VALUE_CHOSEN_PATH, n_props=2)
    assert holds == [1, 1]  # linearizable, and the value is chosen at the end of the golden path


def test_single_copy_register():
    # examples/single-copy-register.rs:80-118. One server: linearizable, 93 states (DFS and, with no
    # early exit, BFS) and the golden "value chosen" path. Two servers: not linearizable, both
    # golden paths are discoveries (the reference's BFS count of 20 stops early in its HashSet
    # order: parity unpinned).
    from actor_golden import (SINGLE_COPY, SINGLE_COPY_NOT_LINEARIZABLE_2, SINGLE_COPY_VALUE_CHOSEN_1,
                              SINGLE_COPY_VALUE_CHOSEN_2)
    r = OracleRun(SINGLE_COPY, [2, 1], dfs=True)
    assert r.unique_state_count == 93
    assert r.discovery_names() == ["value chosen"]
    assert OracleRun(SINGLE_COPY, [2, 1]).unique_state_count == 93
    _, holds = replay(SINGLE_COPY, [2, 1], SINGLE_COPY_VALUE_CHOSEN_1, n_props=2)
    assert holds == [1, 1]
    _, holds = replay(SINGLE_COPY, [2, 2], SINGLE_COPY_NOT_LINEARIZABLE_2, n_props=2)
    assert holds[0] == 0  # "linearizable" does not hold: an `always` discovery
    _, holds = replay(SINGLE_COPY, [2, 2], SINGLE_COPY_VALUE_CHOSEN_2, n_props=2)
    assert holds[1] == 1
    assert sorted(OracleRun(SINGLE_COPY, [2, 2]).discovery_names()) == ["linearizable", "value chosen"]
