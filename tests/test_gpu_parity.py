"""Parity of the MI355X engine (through the C ABI) with the CPU oracle and the reference goldens.

Bar: bit-exact unique_state_count, state_count, max depth and discovered-property set on every
config; in FIFO order also the exact visit order and the exact discovery paths of the
single-threaded reference; in FAST order every discovery path replays on the CPU oracle model and
has the reference's (shortest) length.
"""
import math

import os

import pytest

from oracle_lib import (BINARY_CLOCK, INCREMENT, INCREMENT_LOCK, LINEAR_EQUATION, PAXOS, TWO_PHASE, OracleRun,
                        replay)
from paxos_golden import PAXOS_VALUE_CHOSEN_PATH

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

CASES = [
    (LINEAR_EQUATION, [2, 10, 14]),
    (LINEAR_EQUATION, [2, 4, 7]),
    (LINEAR_EQUATION, [1, 1, 0]),
    (BINARY_CLOCK, []),
] + [(TWO_PHASE, [n]) for n in range(1, 8)] + [
    (INCREMENT, [n]) for n in (1, 2, 3, 4, 6, 8, 9, 10, 11, 12)
] + [(INCREMENT_LOCK, [n]) for n in (1, 2, 3, 5, 7, 8, 9)] + [(PAXOS, [1]), (PAXOS, [2])]


def ids(c):
    names = {LINEAR_EQUATION: "lineq", BINARY_CLOCK: "clock", TWO_PHASE: "2pc", INCREMENT: "inc",
             INCREMENT_LOCK: "inclock", PAXOS: "paxos"}
    return names[c[0]] + "-" + "-".join(map(str, c[1]))


_oracle_cache = {}


def oracle(model, params, **kw):
    key = (model, tuple(params), tuple(sorted(kw.items())))
    if key not in _oracle_cache:
        _oracle_cache[key] = OracleRun(model, params, **kw)
    return _oracle_cache[key]


def gpu(model, params, order, **kw):
    b = MODELS[model](params).checker().order(order)
    rec = None
    if kw.get("record_visits"):
        rec = sr.StateRecorder()
        b = b.visitor(rec)
    if kw.get("target"):
        b = b.target_state_count(kw["target"])
    if kw.get("counters"):
        b = b.counters()
    if kw.get("hint"):
        b = b.capacity_hint(kw["hint"])
    c = b.spawn_bfs().join()
    return c, rec


@pytest.mark.parametrize("order", ["fifo", "fast", "auto"])
@pytest.mark.parametrize("case", CASES, ids=ids)
def test_counts_match_oracle(case, order):
    model, params = case
    o = oracle(model, params)
    c, _ = gpu(model, params, order)
    assert sorted(c.discoveries()) == o.discovery_names()
    n_props = len(c.properties())
    if order == "fast" and n_props and len(o.discovery_names()) == n_props:
        # Early exit inside a level: the counts depend on the visit order, which FAST does not
        # reproduce by design (AUTO re-runs such checks in FIFO order).
        assert c.unique_state_count() <= c.state_count()
        return
    assert c.unique_state_count() == o.unique_state_count
    assert c.state_count() == o.state_count
    assert c.max_depth() == o.max_depth
    assert sorted(c.discoveries()) == o.discovery_names()
    assert c.is_done() == o.is_done


@pytest.mark.parametrize("case", [c for c in CASES if c[0] != BINARY_CLOCK or True], ids=ids)
def test_fifo_paths_identical(case):
    model, params = case
    o = oracle(model, params)
    c, _ = gpu(model, params, "fifo")
    for name in o.discovery_names():
        p = c.discovery(name)
        assert p.action_ids == o.discovery_actions(name), name
        assert p.into_states() == o.discovery_states(name), name


@pytest.mark.parametrize("case", CASES, ids=ids)
def test_fast_paths_replay_on_cpu_model(case):
    model, params = case
    o = oracle(model, params)
    c, _ = gpu(model, params, "fast")
    props = c.properties()
    for name, path in c.discoveries().items():
        r = replay(model, params, path.action_ids, n_props=len(props))
        assert r is not None, f"{name}: path does not replay on the CPU model"
        states, holds = r
        width = len(path.states[0])
        assert [tuple(states[i:i + width]) for i in range(0, len(states), width)] == path.into_states()
        i = [n for n, _ in props].index(name)
        exp = props[i][1]
        assert holds[i] == (1 if exp == sr.Expectation.Sometimes else 0)
        assert len(path) == len(o.discovery_actions(name)), "BFS discoveries are shortest paths"


@pytest.mark.parametrize("case", [(LINEAR_EQUATION, [2, 10, 14]), (BINARY_CLOCK, []), (TWO_PHASE, [3]),
                                  (INCREMENT, [4]), (INCREMENT, [10]), (INCREMENT_LOCK, [3]),
                                  (INCREMENT_LOCK, [9]), (PAXOS, [2])], ids=ids)
def test_fifo_visit_order_identical(case):
    # Generalises `visits_states_in_bfs_order` (src/checker/bfs.rs:351-364).
    model, params = case
    o = oracle(model, params, record_visits=True)
    _, rec = gpu(model, params, "fifo", record_visits=True)
    assert rec.states == o.visits()


def test_visits_states_in_bfs_order_golden():
    # src/checker/bfs.rs:351-364 verbatim.
    rec, accessor = sr.StateRecorder.new_with_accessor()
    sr.LinearEquation(2, 10, 14).checker().order("fifo").visitor(rec).spawn_bfs().join()
    assert accessor() == [(0, 0), (1, 0), (0, 1), (2, 0), (1, 1), (0, 2), (3, 0), (2, 1)]


def test_fast_visits_same_set():
    o = oracle(TWO_PHASE, [4], record_visits=True)
    _, rec = gpu(TWO_PHASE, [4], "fast", record_visits=True)
    assert sorted(rec.states) == sorted(o.visits())


def test_can_complete_by_eliminating_properties_golden():
    # src/checker/bfs.rs:375-388
    c = sr.LinearEquation(2, 10, 14).checker().spawn_bfs().join()
    c.assert_properties()
    assert c.unique_state_count() == 12
    assert c.discovery("solvable").into_actions() == ["IncreaseX", "IncreaseX", "IncreaseY"]
    c.assert_discovery("solvable", ["IncreaseY"] * 27)


def test_can_complete_by_enumerating_all_states_golden():
    # src/checker/bfs.rs:367-372
    c = sr.LinearEquation(2, 4, 7).checker().spawn_bfs().join()
    assert c.is_done()
    c.assert_no_discovery("solvable")
    assert c.unique_state_count() == 256 * 256


def test_report_golden():
    # src/checker.rs:449-468 (the timing-dependent "Checking." lines are not compared)
    import io
    w = io.StringIO()
    sr.LinearEquation(2, 10, 14).checker().spawn_bfs().report(w)
    out = w.getvalue()
    assert "Done. states=15, unique=12, sec=" in out
    assert out.endswith('Discovered "solvable" example Path[3]:\n- IncreaseX\n- IncreaseX\n- IncreaseY\n')


def test_2pc_golden():
    # examples/2pc.rs:127-134
    c = sr.TwoPhaseSys(3).checker().spawn_bfs().join()
    assert c.unique_state_count() == 288
    c.assert_properties()
    c = sr.TwoPhaseSys(5).checker().spawn_bfs().join()
    assert c.unique_state_count() == 8832
    c.assert_properties()


@pytest.mark.parametrize("target", [1, 2, 100, 1499, 1500, 5000, 20000, 50000])
@pytest.mark.parametrize("case", [(TWO_PHASE, [4]), (INCREMENT_LOCK, [5]), (INCREMENT, [8])], ids=ids)
def test_target_state_count_matches_oracle(case, target):
    model, params = case
    o = OracleRun(model, params, target=target)
    c, _ = gpu(model, params, "auto", target=target)
    assert (c.unique_state_count(), c.state_count()) == (o.unique_state_count, o.state_count)
    assert c.is_done() == o.is_done


@pytest.mark.parametrize("n", [8, 9, 10, 11, 12])
def test_2pc_large_closed_form(n):
    # n = 11 is BASELINE.json configs[3] (367 M states); n = 12 (2.2 G states, a 64 GB visited set
    # and a 26 GB arena) is the largest size one MI355X holds with this layout.
    # Full sizes: BASELINE.md §3 (closed forms anchored at the reference goldens 288 / 8 832).
    c = sr.TwoPhaseSys(n).checker().capacity_hint(6 ** n + 4 ** n + 2 ** n).spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert c.max_depth() == 3 * n + 1
    assert sorted(c.discoveries()) == ["abort agreement", "commit agreement"]
    c.assert_properties()


@pytest.mark.parametrize("n", [9, 10, 11])
def test_increment_lock_large_closed_form(n):
    c = sr.IncrementLock(n).checker().spawn_bfs().join()
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    assert c.unique_state_count() == c.state_count() == expect
    assert c.max_depth() == 4 * n
    assert c.discoveries() == {}


def test_increment_lock_12_exact_on_one_gpu():
    # BASELINE.json configs[1] at its top (increment_lock, 12 threads): 5 208 245 377 states, depth
    # 48, on ONE MI355X. An 89-bit state: a 64-bit fingerprint would expect ~0.74 colliding pairs
    # at this size (n^2 / 2^65); the quotient visited set is exact (kernels.hpp TableView). Sized
    # for 288 GB: 2^33 slots x 8 B = 64 GiB of table + ~6.8e9 x 20 B of BFS-tree arena.
    n = 12
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    assert expect == 5_208_245_377
    c = sr.IncrementLock(n).checker().capacity_hint(expect).spawn_bfs().join()
    assert c.unique_state_count() == c.state_count() == expect
    assert c.max_depth() == 4 * n
    assert c.discoveries() == {}
    assert c.stats()["table_capacity"] == 1 << 33


@pytest.mark.parametrize("order", ["fifo", "fast"])
def test_increment_lock_quotient_table_grows(order):
    # A two-word state in a quotient-mode table that starts small (no hint) and doubles: the rehash
    # decodes every slot back to its key (exact counts in both orders; FIFO also remaps the level's
    # candidate slots).
    n = 9
    o = oracle(INCREMENT_LOCK, [n])
    c = sr.IncrementLock(n).checker().order(order).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert c.stats()["rehashes"] > 0


def test_increment_lock_grows_through_x5_levels():
    # No hint, increment_lock N=10 (39 M states): every fourth level has five times the states of
    # the one before, so a speculative launch planned from the last level's growth meets a frontier
    # five times larger than planned. It must expand nothing (ERR_DEFERRED) and run again on a grown
    # table, not overfill a small quotient table (kernels.hpp SlotWork.room); counts stay exact.
    n = 10
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    c = sr.IncrementLock(n).checker().order("fast").spawn_bfs().join()
    assert c.unique_state_count() == c.state_count() == expect
    assert c.max_depth() == 4 * n
    assert c.stats()["rehashes"] > 0


def test_2pc_10_fifo_matches_fast():
    # The exact-order pipeline at a BASELINE size: same counts as FAST, same closed forms.
    n = 10
    a = sr.TwoPhaseSys(n).checker().order("fifo").capacity_hint(6 ** n + 4 ** n + 2 ** n).spawn_bfs().join()
    assert a.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * a.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert a.max_depth() == 3 * n + 1


def test_2pc_8_fifo_matches_fast():
    a = sr.TwoPhaseSys(8).checker().order("fifo").spawn_bfs().join()
    b = sr.TwoPhaseSys(8).checker().order("fast").spawn_bfs().join()
    assert (a.unique_state_count(), a.state_count(), a.max_depth()) == (b.unique_state_count(), b.state_count(), b.max_depth())


@pytest.mark.parametrize("step", ["2", "8"])
def test_growth_from_small_table(step, monkeypatch):
    # No capacity hint (the path a reference user gets): the visited set and the arena grow during
    # the check, in steps of SR_GROW_STEP (default 8; 2 = doublings, several rehashes), and the
    # counts stay exact.
    monkeypatch.setenv("SR_GROW_STEP", step)
    n = 9
    c = sr.TwoPhaseSys(n).checker().order("fast").spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert c.stats()["rehashes"] >= (2 if step == "2" else 1)


@pytest.mark.parametrize("ranges", ["0", "1"])
@pytest.mark.parametrize("step", ["2", "8", "64"])
def test_rehash_by_ranges(step, ranges, monkeypatch):
    # Growth of a quotient table range by range (kernels.hpp rehash_ranges: no clear, LDS insertion,
    # entries past a range's end spilled and inserted afterwards) against the CAS rehash: steps of 2
    # leave the new table at up to half load (many spills), 64 at a few percent. One-word keys in
    # 4-byte slots (2pc) and two-word keys in 8-byte slots (increment_lock); exact counts.
    monkeypatch.setenv("SR_GROW_STEP", step)
    monkeypatch.setenv("SR_REHASH_RANGES", ranges)
    n = 9
    c = sr.TwoPhaseSys(n).checker().order("fast").spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert c.stats()["rehashes"] >= 1
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    c = sr.IncrementLock(n).checker().order("fast").spawn_bfs().join()
    assert c.unique_state_count() == c.state_count() == expect
    assert c.max_depth() == 4 * n
    assert c.stats()["rehashes"] >= 1


def test_rehash_by_ranges_probe_limit(monkeypatch):
    # A probe limit of 6 slots (SR_DISP_LIMIT): range rebuilds that meet it report a full table and
    # the growth goes on to a larger table; counts stay exact.
    monkeypatch.setenv("SR_DISP_LIMIT", "6")
    monkeypatch.setenv("SR_GROW_STEP", "2")
    n = 7
    c = sr.TwoPhaseSys(n).checker().order("fast").spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6


def test_paxos_golden():
    # examples/paxos.rs:268-290 (BFS): assert_properties, assert_discovery of the reference's
    # "value chosen" path, unique_state_count 16_668.
    for order in ("fifo", "fast", "auto"):
        c = sr.Paxos(2, 3).checker().order(order).spawn_bfs().join()
        c.assert_properties()
        c.assert_discovery("value chosen", PAXOS_VALUE_CHOSEN_PATH)
        assert c.unique_state_count() == 16_668
        assert len(c.discovery("value chosen")) == len(PAXOS_VALUE_CHOSEN_PATH)
        assert c.discovery("value chosen").into_actions()[0].startswith("Deliver { src: Id(")


@pytest.mark.parametrize("order", ["fifo", "fast"])
def test_paxos_3_clients_matches_oracle(order):
    # BASELINE.json config 5 (`paxos check 3`) at full size.
    o = oracle(PAXOS, [3])
    c, _ = gpu(PAXOS, [3], order)
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (1_194_428, 2_420_477, 27)
    assert sorted(c.discoveries()) == ["value chosen"]
    if order == "fifo":
        assert c.discovery("value chosen").action_ids == o.discovery_actions("value chosen")


@pytest.mark.parametrize("clients,order", [(4, "fifo"), (4, "fast"), (5, "fast"), (6, "fast"), (6, "fifo")])
def test_paxos_more_clients(clients, order):
    # The reference's parameter space (bench.sh:27 checks 6 clients): the encoding keeps the
    # linearizability history in the state (no precomputed table, whose closure has 558 385
    # histories at 4 clients), W = 11 up to 4 clients and 12 for 5-6. Counts against the oracle's
    # (tests/golden/paxos_counts.json), the discovery path replays on the CPU model, and at 4
    # clients the FIFO path equals the single-threaded oracle's.
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "paxos_counts.json")) as f:
        want = next(r for r in json.load(f)["cases"] if r["client_count"] == clients)
    c, _ = gpu(PAXOS, [clients], order)
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == \
        (want["unique_state_count"], want["state_count"], want["max_depth"])
    assert sorted(c.discoveries()) == want["discoveries"]
    c.assert_properties()
    path = c.discovery("value chosen")
    r = replay(PAXOS, [clients], path.action_ids, n_props=2)
    assert r is not None and r[1][1] == 1
    if clients == 4 and order == "fifo":
        o = oracle(PAXOS, [4])
        assert path.action_ids == o.discovery_actions("value chosen")


@pytest.mark.parametrize("grid", ["1", "2"])
@pytest.mark.parametrize("case", [(TWO_PHASE, [5]), (TWO_PHASE, [8]), (PAXOS, [2])], ids=ids)
def test_small_grid_strides(case, grid, monkeypatch):
    # A one- or two-block grid strides over every chunk of every level, with and without level
    # pipelining (dev_n = 1 / 0): the LDS duplicate filter and the stage persist across chunks and
    # the stage overflows into direct appends. Counts and discoveries must not change.
    monkeypatch.setenv("SR_GRID_MAX", grid)
    model, params = case
    o = oracle(model, params)
    for pipe in ("1", "0"):
        monkeypatch.setenv("SR_PIPELINE", pipe)
        c, _ = gpu(model, params, "fast")
        assert (c.unique_state_count(), c.state_count(), c.max_depth()) == \
            (o.unique_state_count, o.state_count, o.max_depth)
        assert sorted(c.discoveries()) == o.discovery_names()


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("order", ["fifo", "fast"])
@pytest.mark.parametrize("case", [(INCREMENT_LOCK, [9]), (TWO_PHASE, [7])], ids=ids)
def test_probe_limit_overflow_doubles_the_table(case, order, pipe, monkeypatch):
    # SR_DISP_LIMIT lowers the probe limit to a few slots, so levels overflow it. The engine doubles
    # the visited set in the middle of the check (quotient mode: one more displacement bit) and
    # finishes the level on it (repair pass: the missing successors are claimed, none is counted
    # twice), instead of restarting the check; counts stay exact in both orders, with and without
    # level pipelining, in 8-byte quotient slots (increment_lock, 2 words) and 32-bit ones (2pc, one
    # word: its 296 448 states in the default 2^22 slots displace at most 5 slots, so its limit is 3).
    model, params = case
    limit = 3 if model == TWO_PHASE else 6
    monkeypatch.setenv("SR_DISP_LIMIT", str(limit))
    monkeypatch.setenv("SR_PIPELINE", pipe)
    o = oracle(model, params)
    c, _ = gpu(model, params, order, counters=True)
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()
    st = c.stats()
    assert st["table_doublings"] > 0 and st["restarts"] == 0
    assert st["displacement_limit"] == limit and 0 < st["max_displacement"] < limit


def test_displacement_stats_increment_lock_10():
    # The quotient key of increment_lock (6 bits per thread) leaves a probe limit far above the
    # longest run; counters() measures the longest displacement of the final table.
    n = 10
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    c = sr.IncrementLock(n).checker().capacity_hint(expect).counters().spawn_bfs().join()
    st = c.stats()
    assert c.unique_state_count() == expect
    assert st["displacement_limit"] >= 4094 and 0 < st["max_displacement"] < st["displacement_limit"] // 4
    assert st["table_doublings"] == 0
