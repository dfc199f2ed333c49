"""The partitioned engine's MULTI-RANK code path (dist.hpp with a communicator: one rank-local
partition per rank, every collective issued in its order by every rank) run with world = 2, 3 and
8 on one MI355X. The ranks are threads of this process on the in-process transport
(sr_dist_local_group), which keeps RCCL's contract: stream-ordered collectives that every rank
issues in the same sequence; a rank that issues a different collective or size makes every rank
fail (RCCL would hang). Counts must equal the oracle's, every rank reports the same global counts,
and discovery paths are available from ANY single rank after join (gathered at join), replaying on
the CPU oracle model. Plus the BASELINE configuration 4 at its full size: 2pc N=11 partitioned 8
ways (virtual partitions) against the closed forms of BASELINE.md §3."""
import json
import os
import time
import subprocess
import sys

import pytest

from oracle_lib import INCREMENT_LOCK, LINEAR_EQUATION, TWO_PHASE, OracleRun, replay

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")
from stateright_amd.distributed import Communicator  # noqa: E402

MODELS = {
    LINEAR_EQUATION: lambda p: sr.LinearEquation(*p),
    TWO_PHASE: lambda p: sr.TwoPhaseSys(*p),
    INCREMENT_LOCK: lambda p: sr.IncrementLock(*p),
}
_cache = {}


def oracle(model, params):
    k = (model, tuple(params))
    if k not in _cache:
        _cache[k] = OracleRun(model, params)
    return _cache[k]


def run_ranks(model, params, world, hint=0, defer=False):
    comms = Communicator.local_group(world)
    checkers = []
    for c in comms:
        b = MODELS[model](params).checker().comm(c)
        if hint:
            b = b.capacity_hint(hint)
        if defer:
            b = b.defer_paths()
        checkers.append(b.spawn_bfs())
    for ch in checkers:
        ch.join()
    return comms, checkers


def close(comms, checkers):
    checkers.clear()
    for c in comms:
        c.close()


@pytest.mark.parametrize("direct", ["1", "0"], ids=["direct", "alltoall"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", [(TWO_PHASE, [3]), (TWO_PHASE, [5]), (TWO_PHASE, [7]), (INCREMENT_LOCK, [7]),
                                  (LINEAR_EQUATION, [2, 4, 7])],
                         ids=lambda c: f"{c[0]}-{'-'.join(map(str, c[1]))}")
def test_ranks_match_oracle(case, world, direct, monkeypatch):
    # direct: every rank stores its records straight into the owners' receive buffers and raises
    # a per-level flag there; the owners' streams wait for the flags on the device (no collective
    # per level). alltoall: the collective exchange of buckets (SR_DIRECT=0).
    monkeypatch.setenv("SR_DIRECT", direct)
    if direct == "1":  # every level partitioned (the replicated head would explore the small cases)
        monkeypatch.setenv("SR_HEAD_MAX", "0")
    model, params = case
    o = oracle(model, params)
    comms, cs = run_ranks(model, params, world)
    try:
        assert all(c.kind() == "local" and c.nranks() == world for c in comms)
        for ch in cs:  # every rank reports the global counts
            assert (ch.unique_state_count(), ch.state_count(), ch.max_depth()) == \
                (o.unique_state_count, o.state_count, o.max_depth)
            assert ch.stats()["pipelined"] == (2 if direct == "1" else 1)
        # discovery paths from ONE rank alone (no collective after join), valid on the CPU model
        last = cs[-1]
        assert sorted(last.discoveries()) == o.discovery_names()
        props = last.properties()
        names = [n for n, _ in props]
        for name, path in last.discoveries().items():
            r = replay(model, params, path.action_ids, n_props=len(props))
            assert r is not None
            want = 1 if props[names.index(name)][1] == sr.Expectation.Sometimes else 0
            assert r[1][names.index(name)] == want
            assert len(path) == len(o.discovery_actions(name))
        # every rank gathered the same paths
        assert cs[0].discoveries() == last.discoveries()
    finally:
        close(comms, cs)


@pytest.mark.parametrize("sync", [False, True])
@pytest.mark.parametrize("head", ["0", "65536"])
def test_ranks_protocol_modes(sync, head, monkeypatch):
    # the pipelined loop (one all-to-all per level, plan from the rows every rank holds) and the
    # synchronous one (all-gather of rows + grouped exact-size exchange), with and without the
    # replicated head
    if sync:
        monkeypatch.setenv("SR_DIST_SYNC", "1")
    else:
        monkeypatch.delenv("SR_DIST_SYNC", raising=False)
    monkeypatch.setenv("SR_HEAD_MAX", head)
    o = oracle(TWO_PHASE, [6])
    comms, cs = run_ranks(TWO_PHASE, [6], 2)
    try:
        for ch in cs:
            assert (ch.unique_state_count(), ch.state_count(), ch.max_depth()) == \
                (o.unique_state_count, o.state_count, o.max_depth)
            # (2pc N=6 fits the 65536-state head entirely: no partitioned level is exchanged)
            assert ch.stats()["pipelined"] == (0 if sync else 2 if head == "0" else 1)
        assert sorted(cs[1].discoveries()) == o.discovery_names()
    finally:
        close(comms, cs)


def test_ranks_deferred_paths_are_collective():
    # defer_paths(): nothing gathered at join; every rank must then ask for the same property in
    # the same order (threads here, as separate processes would)
    import threading
    o = oracle(TWO_PHASE, [5])
    comms, cs = run_ranks(TWO_PHASE, [5], 2, defer=True)
    out = [None, None]
    try:
        ts = [threading.Thread(target=lambda i=i: out.__setitem__(i, cs[i].discoveries())) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        # the walk through the replicated head is rank-local (each rank's head arena orders a
        # level differently), so deferred paths may differ between ranks: all valid and shortest
        assert out[0] is not None and out[1] is not None
        for res in out:
            assert sorted(res) == o.discovery_names()
            for name, path in res.items():
                r = replay(TWO_PHASE, [5], path.action_ids, n_props=3)
                assert r is not None and r[1][["abort agreement", "commit agreement", "consistent"].index(name)] == 1
                assert len(path) == len(o.discovery_actions(name))
    finally:
        close(comms, cs)


def test_ranks_overflow_restart_is_collective():
    # A tiny capacity hint: buffers overflow, every rank sees it in the rows and all restart together.
    import math
    n = 8
    comms, cs = run_ranks(INCREMENT_LOCK, [n], 2, hint=10)
    try:
        expect = 1 + 4 * sum(math.factorial(n) // math.factorial(n - k) for k in range(1, n + 1))
        assert [ch.unique_state_count() for ch in cs] == [expect, expect]
    finally:
        close(comms, cs)


@pytest.mark.parametrize("world,direct", [(2, "1"), (8, "1"), (8, "0")])
def test_ranks_bench_config(world, direct, monkeypatch):
    # BASELINE config 3 (2pc N=9) on `world` ranks: closed forms, pipelined, no restart; the direct
    # exchange (default) and the collective all-to-all
    monkeypatch.setenv("SR_DIRECT", direct)
    n = 9
    want = 6 ** n + 4 ** n + 2 ** n
    comms, cs = run_ranks(TWO_PHASE, [n], world, hint=want)
    try:
        for ch in cs:
            assert ch.unique_state_count() == want
            assert 3 * ch.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
            assert ch.max_depth() == 3 * n + 1
            st = ch.stats()
            assert st["pipelined"] == (2 if direct == "1" else 1) and st["restarts"] == 0, st
        assert sorted(cs[0].discoveries()) == ["abort agreement", "commit agreement"]
    finally:
        close(comms, cs)


def test_config4_2pc11_partitioned_8_full_size():
    # BASELINE configs[3]: 2pc N=11 partitioned 8 ways, at its full size (366 993 408 unique /
    # 5 371 377 666 generated states, depth 34; BASELINE.md §3 closed forms).
    n = 11
    want = 6 ** n + 4 ** n + 2 ** n
    c = sr.TwoPhaseSys(n).checker().partitions(8).capacity_hint(want).spawn_bfs().join()
    assert c.unique_state_count() == want == 366_993_408
    assert c.state_count() == 5_371_377_666
    assert 3 * c.state_count() == 4 * n * 6 ** n + 3 * (n + 1) * 4 ** n + 3 * n * 2 ** n + 6
    assert c.max_depth() == 3 * n + 1
    assert sorted(c.discoveries()) == ["abort agreement", "commit agreement"]
    for name, path in c.discoveries().items():
        r = replay(TWO_PHASE, [n], path.action_ids, n_props=3)
        assert r is not None and r[1][["abort agreement", "commit agreement", "consistent"].index(name)] == 1


def test_direct_state_reused_across_checks(monkeypatch):
    # The direct exchange keeps its flag words, receive buffers and address tables in the pooled
    # per-device context across the checks of one communicator (flags are monotonic sequence
    # numbers, never cleared). Consecutive checks of different sizes on the same ranks: the second
    # grows the buffers, the third reuses them; every count equals the oracle's.
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    comms = Communicator.local_group(3)
    try:
        for model, params in [(TWO_PHASE, [4]), (TWO_PHASE, [7]), (INCREMENT_LOCK, [6]), (TWO_PHASE, [5])]:
            o = oracle(model, params)
            cs = [MODELS[model](params).checker().comm(c).spawn_bfs() for c in comms]
            for ch in cs:
                ch.join()
            for ch in cs:
                assert (ch.unique_state_count(), ch.state_count(), ch.max_depth()) == \
                    (o.unique_state_count, o.state_count, o.max_depth)
                assert ch.stats()["pipelined"] == 2
            cs.clear()
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("head", ["0", "65536"])
def test_direct_repeated_checks_same_ranks(head, monkeypatch):
    # The bench's pattern: the same in-process ranks run several checks of 2pc N=7 back to back,
    # with and without the replicated head.
    monkeypatch.setenv("SR_HEAD_MAX", head)
    n = 7
    want = 6 ** n + 4 ** n + 2 ** n
    comms = Communicator.local_group(2)
    try:
        for _ in range(4):
            cs = [sr.TwoPhaseSys(n).checker().comm(c).capacity_hint(want).defer_paths().spawn_bfs() for c in comms]
            for ch in cs:
                ch.join()
            assert [ch.unique_state_count() for ch in cs] == [want, want]
            cs.clear()
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("level", [1, 3])
def test_corrupt_slot_falls_back_to_collective(level, monkeypatch):
    # The exchange check: a record (or a header row word, at a level where no source
    # sent records to rank 0) flipped after its source checksummed the slot makes the owner's insert
    # report ERR_EXCHANGE; the ranks vote, and the check is redone on the collective exchange with
    # exact counts. The communicator then keeps the collective exchange.
    # Every rank throws at the same level: with SR_PEER_TIMEOUT_MS at its default (20 s)
    # the fallback must not wait for an unanswered peer flag.
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    monkeypatch.setenv("SR_DX_CORRUPT_LEVEL", str(level))
    monkeypatch.delenv("SR_PEER_TIMEOUT_MS", raising=False)
    o = oracle(TWO_PHASE, [6])
    comms = Communicator.local_group(2)
    try:
        for k in range(2):
            t0 = time.monotonic()
            cs = [sr.TwoPhaseSys(6).checker().comm(c).spawn_bfs() for c in comms]
            for ch in cs:
                ch.join()
            assert time.monotonic() - t0 < 5.0, "the fallback stalled (a peer waited for its timeout)"
            for ch in cs:
                assert (ch.unique_state_count(), ch.state_count(), ch.max_depth()) == \
                    (o.unique_state_count, o.state_count, o.max_depth)
                st = ch.stats()
                assert st["exchange_fallbacks"] == (1 if k == 0 else 0), st
                assert st["pipelined"] == 1, st
            cs.clear()
    finally:
        for c in comms:
            c.close()


def test_corrupt_slot_virtual_partitions(monkeypatch):
    # the same check between virtual partitions of one process (no vote: the engine itself redoes
    # the check on the device-copy exchange)
    monkeypatch.setenv("SR_HEAD_MAX", "0")
    monkeypatch.setenv("SR_DX_CORRUPT_LEVEL", "4")
    o = oracle(TWO_PHASE, [7])
    c = sr.TwoPhaseSys(7).checker().partitions(4).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth()) == (o.unique_state_count, o.state_count, o.max_depth)
    st = c.stats()
    assert st["exchange_fallbacks"] == 1 and st["pipelined"] == 1, st


def test_exchange_check_passes_without_corruption(monkeypatch):
    # the checksum of every slot agrees on a full 2pc N=9 partitioned search (no fallback)
    monkeypatch.delenv("SR_DX_CORRUPT_LEVEL", raising=False)
    n = 9
    c = sr.TwoPhaseSys(n).checker().partitions(3).spawn_bfs().join()
    assert c.unique_state_count() == 6 ** n + 4 ** n + 2 ** n
    st = c.stats()
    assert st["exchange_fallbacks"] == 0 and st["pipelined"] == 2, st


_QUEUE_SCRIPT = """
import json, sys
sys.path.insert(0, {root!r})
import stateright_amd as sr
from stateright_amd.distributed import Communicator
comms = Communicator.local_group(8)
cs = [sr.TwoPhaseSys(7).checker().comm(c).spawn_bfs() for c in comms]
for ch in cs:
    ch.join()
print(json.dumps([[ch.unique_state_count(), ch.state_count(), ch.max_depth(), ch.stats()["pipelined"]] for ch in cs]))
"""


def test_world8_one_device_default_queues():
    # Eight in-process ranks on ONE device with HIP's default of 4 hardware queues, set before the
    # runtime starts (a fresh interpreter): the library itself must avoid the direct exchange's
    # device-side waits (a wait queued in front of the expand it waits for), so the check completes
    # on the collective exchange with exact counts and no timeout.
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4", SR_HEAD_MAX="0", SR_PEER_TIMEOUT_MS="5000")
    r = subprocess.run([sys.executable, "-c", _QUEUE_SCRIPT.format(root=root)], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("[")][-1])
    o = oracle(TWO_PHASE, [7])
    for unique, states, depth, pipelined in rows:
        assert (unique, states, depth) == (o.unique_state_count, o.state_count, o.max_depth)
        assert pipelined == 1
