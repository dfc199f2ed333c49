"""The partitioned (multi-GPU) search protocol on one MI355X: T virtual partitions exchanging
successor records by device copies, and a one-rank RCCL communicator (the RCCL code path with a
self-exchange). Counts must equal the oracle's on every full-exploration config; every discovery
path must replay on the CPU oracle model."""
import math

import pytest

from oracle_lib import BINARY_CLOCK, INCREMENT_LOCK, LINEAR_EQUATION, TWO_PHASE, OracleRun, replay

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")

MODELS = {
    LINEAR_EQUATION: lambda p: sr.LinearEquation(*p),
    BINARY_CLOCK: lambda p: sr.BinaryClock(),
    TWO_PHASE: lambda p: sr.TwoPhaseSys(*p),
    INCREMENT_LOCK: lambda p: sr.IncrementLock(*p),
}
CASES = [(LINEAR_EQUATION, [2, 4, 7]), (BINARY_CLOCK, [])] + [(TWO_PHASE, [n]) for n in (1, 2, 3, 5, 7)] + [
    (INCREMENT_LOCK, [n]) for n in (2, 5, 7, 9)]


def ids(c):
    return {LINEAR_EQUATION: "lineq", BINARY_CLOCK: "clock", TWO_PHASE: "2pc", INCREMENT_LOCK: "inclock"}[c[0]] + \
        "-" + "-".join(map(str, c[1]))


_cache = {}


def oracle(model, params):
    k = (model, tuple(params))
    if k not in _cache:
        _cache[k] = OracleRun(model, params)
    return _cache[k]


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("case", CASES, ids=ids)
def test_partitioned_counts_match_oracle(case, parts):
    model, params = case
    o = oracle(model, params)
    c = MODELS[model](params).checker().partitions(parts).spawn_bfs().join()
    assert c.unique_state_count() == o.unique_state_count
    assert c.state_count() == o.state_count
    assert c.max_depth() == o.max_depth
    assert sorted(c.discoveries()) == o.discovery_names()
    assert c.is_done() == o.is_done  # explored everything, or discovered every property


@pytest.mark.parametrize("parts", [2, 3, 8])
@pytest.mark.parametrize("case", [(TWO_PHASE, [3]), (TWO_PHASE, [7]), (INCREMENT_LOCK, [5]), (INCREMENT_LOCK, [8])],
                         ids=ids)
def test_batched_insert_counts_match_oracle(case, parts, monkeypatch):
    # SR_INSERT_BATCH_MIN=0: every level's insert takes the batched form (four records per thread,
    # probes and claims issued back to back, the large grid), which otherwise runs only on inserts
    # of more than 8 M planned records (2pc N=11); one- and two-word states.
    monkeypatch.setenv("SR_INSERT_BATCH_MIN", "0")
    model, params = case
    o = oracle(model, params)
    c = MODELS[model](params).checker().partitions(parts).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()


def test_partitioned_target_state_count():
    # `target_state_count` (src/checker/bfs.rs:113-135): the partitioned search stops at the first
    # LEVEL boundary at which state_count >= target (the reference's single order has 1500-pop
    # blocks; the partitions have no single pop order). Level-synchronous, so the counts do not
    # depend on the partition count; the stop is past the target and short of the full check.
    n, target = 7, 20_000
    full = oracle(TWO_PHASE, [n])
    seen = set()
    for parts in (2, 3, 5):
        c = sr.TwoPhaseSys(n).checker().partitions(parts).target_state_count(target).spawn_bfs().join()
        assert c.state_count() >= target
        assert c.unique_state_count() < full.unique_state_count
        assert not c.is_done()
        seen.add((c.unique_state_count(), c.state_count(), c.max_depth()))
    assert len(seen) == 1, seen


@pytest.mark.parametrize("parts", [2, 5])
def test_partitioned_paths_replay(parts):
    c = sr.TwoPhaseSys(5).checker().partitions(parts).spawn_bfs().join()
    o = oracle(TWO_PHASE, [5])
    props = [n for n, _ in c.properties()]
    for name, path in c.discoveries().items():
        states, holds = replay(TWO_PHASE, [5], path.action_ids, n_props=len(props))
        assert holds[props.index(name)] == 1
        assert len(path) == len(o.discovery_actions(name))


def test_partitioned_large_closed_form():
    n = 9
    c = sr.TwoPhaseSys(n).checker().partitions(8).capacity_hint(6 ** n + 4 ** n + 2 ** n).spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert c.max_depth() == 3 * n + 1


def test_partitioned_restart_on_overflow():
    # A tiny capacity hint forces the optimistic buffers to overflow; the check restarts and stays exact.
    c = sr.IncrementLock(8).checker().partitions(4).capacity_hint(10).spawn_bfs().join()
    n = 8
    expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
    assert c.unique_state_count() == expect


@pytest.mark.parametrize("direct,fused", [("1", "1"), ("1", "0"), ("0", "1")])
def test_rccl_single_rank(direct, fused, monkeypatch):
    # the RCCL communicator's code path with one rank: the direct exchange (its flag protocol with
    # this rank as the only source and owner; RCCL ranks have distinct devices, so the insert grid
    # polls the flags itself unless SR_FUSED_WAIT=0 keeps the one-wave wait kernel), or RCCL's
    # all-to-all (SR_DIRECT=0)
    monkeypatch.setenv("SR_DIRECT", direct)
    monkeypatch.setenv("SR_FUSED_WAIT", fused)
    from stateright_amd.distributed import Communicator
    comm = Communicator(0, 1, Communicator.unique_id(), 0)
    c = sr.TwoPhaseSys(6).checker().comm(comm).spawn_bfs().join()
    o = oracle(TWO_PHASE, [6])
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()
    assert c.stats()["pipelined"] == (2 if direct == "1" else 1)
    del c
    comm.close()


@pytest.mark.parametrize("parts", [2, 3, 8])
@pytest.mark.parametrize("case", [(TWO_PHASE, [5]), (TWO_PHASE, [7]), (INCREMENT_LOCK, [7]), (LINEAR_EQUATION, [2, 4, 7])],
                         ids=ids)
def test_exchange_by_copies_matches_oracle(case, parts, monkeypatch):
    # SR_DIRECT=0: the buckets of every partition are exchanged by device copies (the all-to-all's
    # stand-in) instead of being stored straight into the owners' receive buffers
    monkeypatch.setenv("SR_DIRECT", "0")
    model, params = case
    o = oracle(model, params)
    c = MODELS[model](params).checker().partitions(parts).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()
    assert c.stats()["pipelined"] == 1


@pytest.mark.parametrize("parts", [2, 4, 8])
def test_pipelined_plan_holds_on_bench_config(parts):
    # The bench configuration (2pc N=9) must run pipelined without a capacity restart: the bucket
    # plan depends only on the rows every rank sees, so T virtual partitions make exactly the
    # decisions T RCCL ranks would make.
    n = 9
    want = 6 ** n + 4 ** n + 2 ** n
    c = sr.TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want).spawn_bfs().join()
    st = c.stats()
    assert c.unique_state_count() == want
    assert st["pipelined"] == (2 if parts > 1 else 1) and st["restarts"] == 0, st


@pytest.mark.parametrize("sync", [False, True])
def test_pipelined_and_synchronous_agree(sync, monkeypatch):
    if sync:
        monkeypatch.setenv("SR_DIST_SYNC", "1")
    else:
        monkeypatch.delenv("SR_DIST_SYNC", raising=False)
    monkeypatch.setenv("SR_HEAD_MAX", "0")  # every level partitioned (the head would explore it all)
    o = oracle(INCREMENT_LOCK, [7])
    c = sr.IncrementLock(7).checker().partitions(3).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert c.stats()["pipelined"] == (0 if sync else 2)


@pytest.mark.parametrize("head", ["0", "64", "65536"])
@pytest.mark.parametrize("case", [(TWO_PHASE, [5]), (INCREMENT_LOCK, [6]), (LINEAR_EQUATION, [2, 4, 7])], ids=ids)
def test_replicated_head_counts_and_paths(case, head, monkeypatch):
    # The replicated head (SR_HEAD_MAX: largest frontier run on every rank before partitioning;
    # 0 = none): counts equal the oracle's whatever the hand-over level, and discovery paths that
    # cross from the partitioned levels into the head replay on the CPU model.
    monkeypatch.setenv("SR_HEAD_MAX", head)
    model, params = case
    o = oracle(model, params)
    c = MODELS[model](params).checker().partitions(3).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    assert sorted(c.discoveries()) == o.discovery_names()
    props = c.properties()
    names = [n for n, _ in props]
    for name, path in c.discoveries().items():
        r = replay(model, params, path.action_ids, n_props=len(props))
        assert r is not None  # every action of the path is enabled where it is taken
        want = 1 if props[names.index(name)][1] == sr.Expectation.Sometimes else 0
        assert r[1][names.index(name)] == want
        assert len(path) == len(o.discovery_actions(name))  # a shortest path, as BFS reports
    if head == "0":
        assert c.stats()["head_levels"] == 0


def test_ipc_direct_exchange_across_processes():
    # The direct exchange across processes (one process per GPU under the bench) rests on IPC
    # handles of pool buffers, stores into another process's memory from every workgroup of a
    # kernel, and a flag raised after a system-scope release: scripts/ipc_selftest runs exactly that
    # between two processes on this GPU, each checking every word the other stored.
    import os
    import subprocess
    from stateright_amd import build
    assert os.path.exists(build.IPC_SELFTEST), "built by __graft_entry__.build()"
    r = subprocess.run([build.IPC_SELFTEST, str(1 << 20)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ipc selftest ok" in r.stdout and r.stdout.count(": 0 wrong") == 2, r.stdout


def test_direct_virtual_partitions_change_between_checks():
    # Virtual partitions share the pooled context's direct-exchange buffers: a different partition
    # count between checks sets them up again, the same count reuses them.
    for parts, n in [(8, 5), (2, 6), (8, 7), (8, 5)]:
        o = oracle(TWO_PHASE, [n])
        c = sr.TwoPhaseSys(n).checker().partitions(parts).spawn_bfs().join()
        assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
