"""The visited set handed from one check to the next (engine.hpp `release_table`, device.hpp
`DBuf::release_zero` / `DevicePool::alloc_zeroed`): a FAST check returns its table to the pool
zeroed on its stream behind its last level, and the next check of the same table size takes it
without a clear. Every check below must still count exactly what the oracle counts, whatever
model used the table before it, in FAST and FIFO order, with and without recycling
(SR_TABLE_RECYCLE is read when a checker is created), and with a counting run (which keeps its
table for the displacement scan) in between.
"""
import pytest

from oracle_lib import INCREMENT_LOCK, TWO_PHASE, OracleRun

pytestmark = pytest.mark.gpu

sr = pytest.importorskip("stateright_amd")

HINT = 200_000  # one table size for every check below


def counts(c):
    # (as in test_gpu_parity: a FAST check whose every property is discovered stops inside a
    # level, and its counts then depend on the visit order; only the discoveries are compared)
    early = c.properties() and len(c.discoveries()) == len(c.properties())
    return (None, None, sorted(c.discoveries())) if early else (c.unique_state_count(), c.state_count(),
                                                                 sorted(c.discoveries()))


def check(model, order="fast", counters=False):
    b = model.checker().capacity_hint(HINT).order(order)
    if counters:
        b = b.counters()
    return counts(b.spawn_bfs().join())


@pytest.fixture(scope="module")
def expected():
    out = {}
    for name, kind, p in (("2pc5", TWO_PHASE, [5]), ("2pc6", TWO_PHASE, [6]), ("lock5", INCREMENT_LOCK, [5])):
        o = OracleRun(kind, p)
        out[name] = (o.unique_state_count, o.state_count, o.discovery_names())
    return out


def same(got, want):
    return got[2] == want[2] and (got[0] is None or got[:2] == want[:2])


def models():
    return {"2pc5": sr.TwoPhaseSys(5), "2pc6": sr.TwoPhaseSys(6), "lock5": sr.IncrementLock(5)}


@pytest.mark.parametrize("recycle", ["1", "0"])
def test_back_to_back_checks_share_a_table(monkeypatch, expected, recycle):
    monkeypatch.setenv("SR_TABLE_RECYCLE", recycle)
    m = models()
    # alternate models over the same table size, FAST (releases its table) and FIFO (keeps it)
    seq = [("2pc6", "fast"), ("2pc5", "fast"), ("lock5", "fast"), ("2pc6", "fifo"), ("2pc6", "fast"),
           ("lock5", "fifo"), ("2pc5", "fast"), ("2pc6", "fast")]
    for name, order in seq:
        assert same(check(m[name], order), expected[name]), (name, order, recycle)


def test_counting_run_between_recycled_checks(expected):
    m = models()
    assert same(check(m["2pc6"]), expected["2pc6"])
    assert same(check(m["lock5"], counters=True), expected["lock5"])  # keeps its table for the scan
    assert same(check(m["2pc5"]), expected["2pc5"])
    assert same(check(m["2pc6"]), expected["2pc6"])


def test_checker_alive_while_the_next_runs(expected):
    """A finished checker that is still referenced no longer holds its table: a second check
    can take it while the first one's results (counts, discovery paths) stay readable."""
    m = models()
    first = m["2pc6"].checker().capacity_hint(HINT).spawn_bfs().join()
    second = m["2pc5"].checker().capacity_hint(HINT).spawn_bfs().join()
    assert same(counts(first), expected["2pc6"])
    assert same(counts(second), expected["2pc5"])
    for c in (first, second):
        for name in c.discoveries():
            assert c.discovery(name) is not None
