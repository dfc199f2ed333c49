"""Visitors on the MI355X engine (src/checker/visitor.rs): StateRecorder, PathRecorder and plain
callables. The reference hands `Path::from_fingerprints(reconstruct_path(fp))` of every popped
state to the visitor (src/checker/bfs.rs:187-189); the engine exports the BFS tree after the run
(sr_gpu_bfs_visit_tree) and replays the same paths in visit order. In FIFO order the paths must be
exactly the oracle's; in FAST order every path must replay on the CPU model to its state with the
BFS depth of that state."""
import pytest

from oracle_lib import BINARY_CLOCK, INCREMENT, LINEAR_EQUATION, PAXOS, TWO_PHASE, OracleRun, replay

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")

MODELS = {
    LINEAR_EQUATION: lambda p: sr.LinearEquation(*p),
    BINARY_CLOCK: lambda p: sr.BinaryClock(),
    TWO_PHASE: lambda p: sr.TwoPhaseSys(*p),
    INCREMENT: lambda p: sr.Increment(*p),
    PAXOS: lambda p: sr.Paxos(*p),
}
CASES = [(LINEAR_EQUATION, [2, 10, 14]), (BINARY_CLOCK, []), (TWO_PHASE, [2]), (TWO_PHASE, [3]),
         (INCREMENT, [3]), (PAXOS, [1])]


def ids(c):
    return {LINEAR_EQUATION: "lineq", BINARY_CLOCK: "clock", TWO_PHASE: "2pc", INCREMENT: "inc", PAXOS: "paxos"}[c[0]] + \
        "-" + "-".join(map(str, c[1]))


@pytest.mark.parametrize("case", CASES, ids=ids)
def test_fifo_visitor_paths_equal_oracle(case):
    model, params = case
    o = OracleRun(model, params, record_visits=True)
    seen = []
    MODELS[model](params).checker().order("fifo").visitor(seen.append).spawn_bfs().join()
    assert [p.action_ids for p in seen] == o.visit_paths()
    assert [p.last_state() for p in seen] == o.visits()


@pytest.mark.parametrize("case", CASES, ids=ids)
def test_path_recorder_matches_oracle(case):
    model, params = case
    o = OracleRun(model, params, record_visits=True)
    recorder, accessor = sr.PathRecorder.new_with_accessor()
    MODELS[model](params).checker().order("fifo").visitor(recorder).spawn_bfs().join()
    got = {(tuple(p.action_ids), p.last_state()) for p in accessor()}
    want = {(tuple(a), s) for a, s in zip(o.visit_paths(), o.visits())}
    assert got == want


def test_fast_visitor_paths_replay():
    n = 4
    seen = []
    c = sr.TwoPhaseSys(n).checker().order("fast").visitor(seen.append).spawn_bfs().join()
    assert len(seen) == c.unique_state_count()
    assert len({p.last_state() for p in seen}) == len(seen)
    for p in seen:
        states, _ = replay(TWO_PHASE, [n], p.action_ids, n_props=3)
        width = len(p.last_state())
        assert tuple(states[-width:]) == p.last_state()
        assert [tuple(states[k:k + width]) for k in range(0, len(states), width)] == p.into_states()
    # BFS-tree paths are shortest paths: each state's path length is its BFS level
    o = OracleRun(TWO_PHASE, [n], record_visits=True)
    depth = {s: len(a) for s, a in zip(o.visits(), o.visit_paths())}
    assert all(len(p) == depth[p.last_state()] for p in seen)


@pytest.mark.parametrize("head", ["0", "65536"])
@pytest.mark.parametrize("parts", [2, 3])
def test_partitioned_visitors(parts, head, monkeypatch):
    # The partitioned search gathers every partition's visited states at join (visit order: level
    # by level, partitions in turn, FAST order inside): the StateRecorder sees exactly the oracle's
    # visited set, and every PathRecorder path replays on the CPU model with its BFS depth.
    monkeypatch.setenv("SR_HEAD_MAX", head)
    n = 5
    o = OracleRun(TWO_PHASE, [n], record_visits=True)
    rec = sr.StateRecorder()
    c = sr.TwoPhaseSys(n).checker().partitions(parts).visitor(rec).spawn_bfs().join()
    assert len(rec.states) == c.unique_state_count() == len(o.visits())
    assert set(rec.states) == set(o.visits())
    seen = []
    sr.TwoPhaseSys(n).checker().partitions(parts).visitor(seen.append).spawn_bfs().join()
    depth = {s: len(a) for s, a in zip(o.visits(), o.visit_paths())}
    assert len(seen) == len(o.visits())
    for p in seen:
        states, _ = replay(TWO_PHASE, [n], p.action_ids, n_props=3)
        width = len(p.last_state())
        assert tuple(states[-width:]) == p.last_state()
        assert len(p) == depth[p.last_state()]


def test_partitioned_visitors_ranks():
    # the same on in-process ranks (collective gathering at join; any rank holds the record)
    from stateright_amd.distributed import Communicator
    n = 4
    o = OracleRun(TWO_PHASE, [n], record_visits=True)
    comms = Communicator.local_group(2)
    try:
        recs = [sr.StateRecorder() for _ in comms]
        cs = [sr.TwoPhaseSys(n).checker().comm(cm).visitor(r).spawn_bfs() for cm, r in zip(comms, recs)]
        for ch in cs:
            ch.join()
        for r in recs:
            assert sorted(r.states) == sorted(o.visits())
        cs.clear()
    finally:
        for cm in comms:
            cm.close()


@pytest.mark.parametrize("parts", [2, 3])
def test_partitioned_target_stop_visits_popped_states_only(parts, monkeypatch):
    # A target_state_count stop ends the partitioned search at a level boundary: the
    # last level's states were generated, never popped, and the reference calls the visitor at a
    # pop (src/checker/bfs.rs:188). So the StateRecorder sees every state of the levels before the
    # last one, and none of the last level.
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    n, target = 7, 20_000
    o = OracleRun(TWO_PHASE, [n], record_visits=True)
    depth = {s: len(a) for s, a in zip(o.visits(), o.visit_paths())}
    rec = sr.StateRecorder()
    c = sr.TwoPhaseSys(n).checker().partitions(parts).target_state_count(target).visitor(rec).spawn_bfs().join()
    assert not c.is_done()
    last = c.max_depth()
    want = {s for s, d in depth.items() if d < last}
    assert set(rec.states) == want
    assert len(rec.states) == len(want)
