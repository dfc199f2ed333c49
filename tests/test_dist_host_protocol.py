"""The partitioned engine's host protocol in C++, two PROCESSES, no GPU.

sr_dist_host_protocol runs a 2pc check per rank over the shared-memory transport in host mode: a
CPU stand-in does the device's work (expansion, routing by part_of, the direct exchange's per-slot
checksum, one row per partition and level), while the rows' error precedence (throw_row_errors),
the pipelined bucket plan (LevelPlan) and the outcome vote (outcome_of, decide_after_vote) are
the code the engine itself runs between its kernels (stateright_amd/csrc/dist.hpp). Each case
checks what every rank decided and that the counts equal the single-process oracle's."""
import ctypes
import multiprocessing as mp
import os
import sys
import uuid

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_lib import TWO_PHASE, OracleRun  # noqa: E402


def _rank(rank, world, name, kw, out):
    from stateright_amd import _native as N
    lib = N.load()
    o = N.sr_dist_host_opts()
    o.struct_size = ctypes.sizeof(o)
    o.rm_count = kw.get("n", 4)
    o.cmin = kw.get("cmin", 8192)
    o.corrupt_level = kw.get("corrupt", {}).get(rank, -1)
    o.capacity_fail_at_end = int(rank in kw.get("capacity_at_end", ()))
    o.fail_at_end = int(rank in kw.get("fail_at_end", ()))
    o.plan_div = kw.get("plan_div", 1)
    r = N.sr_dist_host_result()
    st = lib.sr_dist_host_protocol(name.encode(), rank, world, ctypes.byref(o), ctypes.byref(r))
    out[rank] = (st, N.last_error() if st else "", r.as_dict())


def run(world=2, **kw):
    ctx = mp.get_context("spawn")
    name = f"/sr_host_proto_{uuid.uuid4().hex[:12]}"
    with ctx.Manager() as mgr:
        out = mgr.dict()
        ps = [ctx.Process(target=_rank, args=(r, world, name, kw, out)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
            assert p.exitcode == 0, f"rank process exit code {p.exitcode}"
        return [out[r] for r in range(world)]


def oracle(n):
    o = OracleRun(TWO_PHASE, [n])
    return o.unique_state_count, o.state_count, o.max_depth


def assert_counts(res, n):
    want = oracle(n)
    for st, err, r in res:
        assert st == 0, err
        assert (r["unique"], r["state_count"], r["max_depth"]) == want
    # the partitions are disjoint and hold every state; every rank planned the same buckets
    assert sum(r["local_unique"] for _, _, r in res) == want[0]
    assert len({r["plan_digest"] for _, _, r in res}) == 1


@pytest.mark.parametrize("n,world", [(3, 2), (5, 2), (4, 3)])
def test_clean_run(n, world):
    res = run(world, n=n)
    assert_counts(res, n)
    for _, _, r in res:
        assert (r["attempts"], r["restarts"], r["fallbacks"]) == (1, 0, 0)
        assert r["overflow_level"] == 0xFFFFFFFF


def test_bucket_overflow_restarts_every_rank_at_the_same_level():
    # the plan under-estimates (capacities / 16): a sender's row carries ERR_FRONTIER_OVERFLOW,
    # every rank throws at the same level (no disagreement), and the check is redone with exact
    # buckets
    res = run(2, n=5, cmin=4, plan_div=16)
    assert_counts(res, 5)
    levels = {r["overflow_level"] for _, _, r in res if r["overflow_level"] != 0xFFFFFFFF}
    assert len(levels) >= 1
    for _, _, r in res:
        assert (r["attempts"], r["restarts"], r["fallbacks"], r["disagreements"]) == (2, 1, 0, 0)
        assert r["first_outcome"] == 1  # every rank saw the capacity error itself


def test_exchange_error_in_the_rows_falls_back_on_every_rank():
    # rank 1 receives an altered record at level 2: its check reaches the rows of a later level, on
    # every rank, and every rank redoes the check on the collective exchange
    res = run(2, n=4, corrupt={1: 2})
    assert_counts(res, 4)
    for _, _, r in res:
        assert (r["attempts"], r["restarts"], r["fallbacks"]) == (2, 0, 1)
        assert r["first_outcome"] == 2  # both ranks read the error in the rows


def test_exchange_error_seen_by_its_owner_only_falls_back_on_every_rank():
    # the LAST exchange's check is in no row: only its owner sees it, at the end (here a slot
    # without records whose checksum word was read stale), and the vote makes the other rank,
    # which finished cleanly, fall back too
    clean = run(2, n=4)
    last = clean[0][2]["levels"] - 1  # the expansion of the last frontier
    res = run(2, n=4, corrupt={0: last})
    assert_counts(res, 4)
    for _, _, r in res:
        assert (r["attempts"], r["restarts"], r["fallbacks"]) == (2, 0, 1)
    assert [r["first_outcome"] for _, _, r in res] == [2, 0]


def test_capacity_error_on_one_rank_restarts_every_rank():
    # a capacity error that did not travel in the rows: the vote's max is a capacity restart, its
    # min a clean finish, so every rank notes the disagreement and restarts
    res = run(2, n=4, capacity_at_end=(0,))
    assert_counts(res, 4)
    for _, _, r in res:
        assert (r["attempts"], r["restarts"], r["fallbacks"], r["disagreements"]) == (2, 1, 0, 1)
    assert [r["first_outcome"] for _, _, r in res] == [1, 0]


def test_other_error_on_one_rank_fails_every_rank():
    res = run(2, n=3, fail_at_end=(1,))
    (s0, e0, _), (s1, e1, _) = res
    assert s1 == -1 and "injected" in e1          # the failing rank reports its own error
    assert s0 == -2 and "another rank failed" in e0  # the other one, that a rank failed
