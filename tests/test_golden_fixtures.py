"""The committed golden table (tests/golden/bfs_goldens.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every row, and the rows agree with the reference's own goldens
(src/checker/bfs.rs:351-388, examples/2pc.rs:127-134, examples/paxos.rs:268-290).
GPU: the engine, through the C ABI, reproduces every row in the reference's FIFO order — counts,
depth, `is_done`, discovered properties and the exact discovery action paths.
"""
import json
import os

import pytest

from oracle_lib import OracleRun

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "bfs_goldens.json")) as f:
    CASES = json.load(f)["cases"]
with open(os.path.join(HERE, "golden", "paxos_counts.json")) as f:
    PAXOS_COUNTS = json.load(f)["cases"]


def cid(c):
    return c["model"] + "-" + "-".join(map(str, c["params"]))


def _by(model, params):
    return next(c for c in CASES if c["model"] == model and c["params"] == params)


def test_table_agrees_with_reference_goldens():
    assert _by("linear_equation", [2, 10, 14])["unique_state_count"] == 12        # bfs.rs:375-388
    assert _by("linear_equation", [2, 10, 14])["discoveries"]["solvable"] == [0, 0, 1]
    assert _by("linear_equation", [2, 4, 7])["unique_state_count"] == 65536       # bfs.rs:367-372
    assert _by("2pc", [3])["unique_state_count"] == 288                            # 2pc.rs:127-129
    assert _by("2pc", [5])["unique_state_count"] == 8832                           # 2pc.rs:132-134
    assert _by("paxos", [2])["unique_state_count"] == 16668                        # paxos.rs:268-290
    assert _by("linear_equation", [2, 10, 14])["state_count"] == 15                # checker.rs:449-468


@pytest.mark.parametrize("case", CASES, ids=cid)
def test_oracle_reproduces_table(case):
    r = OracleRun(case["model_id"], case["params"])
    assert (r.unique_state_count, r.state_count, r.max_depth, r.is_done) == (
        case["unique_state_count"], case["state_count"], case["max_depth"], case["is_done"])
    assert {n: r.discovery_actions(n) for n in r.discovery_names()} == case["discoveries"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=cid)
def test_gpu_reproduces_table(case):
    import stateright_amd as sr
    make = {
        "linear_equation": lambda p: sr.LinearEquation(*p),
        "binary_clock": lambda p: sr.BinaryClock(),
        "2pc": lambda p: sr.TwoPhaseSys(*p),
        "increment": lambda p: sr.Increment(*p),
        "increment_lock": lambda p: sr.IncrementLock(*p),
        "paxos": lambda p: sr.Paxos(*p),
    }[case["model"]]
    c = make(case["params"]).checker().order("fifo").spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count(), c.max_depth(), c.is_done()) == (
        case["unique_state_count"], case["state_count"], case["max_depth"], case["is_done"])
    assert sorted(c.discoveries()) == sorted(case["discoveries"])
    for name, actions in case["discoveries"].items():
        assert c.discovery(name).action_ids == actions


def test_paxos_counts_fixture_agrees():
    # tests/golden/paxos_counts.json (oracle/bfs_cli, client_count 1..6): the rows the FIFO table
    # also holds agree, the reference's own golden (examples/paxos.rs:268-290) holds, and the
    # single-threaded oracle reproduces the small rows here (4..6 take minutes on the CPU; the GPU
    # tests compare against them).
    by = {r["client_count"]: r for r in PAXOS_COUNTS}
    assert sorted(by) == [1, 2, 3, 4, 5, 6]
    assert by[2]["unique_state_count"] == 16668
    # only the C=2 row is pinned by the reference; the others say they are oracle-derived
    assert by[2]["pinning"].startswith("pinned") and all(by[c]["pinning"].startswith("oracle-derived") for c in by if c != 2)
    for c in (1, 2):
        t = _by("paxos", [c])
        assert (by[c]["unique_state_count"], by[c]["state_count"], by[c]["max_depth"]) == \
            (t["unique_state_count"], t["state_count"], t["max_depth"])
    for c in (1, 2, 3):
        r = OracleRun(7, [c])
        assert (r.unique_state_count, r.state_count, r.max_depth, r.discovery_names()) == (
            by[c]["unique_state_count"], by[c]["state_count"], by[c]["max_depth"], by[c]["discoveries"])
