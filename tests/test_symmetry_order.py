"""Why symmetry reduction is not reproducible by a level-synchronous search — a pure-Python
restatement of 2pc (examples/2pc.rs:10-121) and its representative (examples/2pc.rs:164-182) for
small N, TEST INFRASTRUCTURE ONLY.

The reference's DFS with symmetry keys its visited set by fingerprint(representative(s)) but keeps
exploring the ORIGINAL states (src/checker/dfs.rs:258-267). The 2pc representative sorts RMs by
rm_state with ties kept in index order, which is not a canonical form, so the set of generated
representatives depends on which originals are expanded first. The same reduction in BFS order
gives a different count; the DFS-order count reproduces the reference golden 665
(examples/2pc.rs:137-138) and agrees with the C++ oracle (oracle/dfs.hpp)."""
from collections import deque

from oracle_lib import TWO_PHASE, OracleRun

WORKING, PREPARED, COMMITTED, ABORTED = range(4)  # derived Ord of RmState


def _init(n):
    return (tuple([WORKING] * n), 0, tuple([False] * n), frozenset())


def _successors(s, n):
    rm, tm, prep, msgs = s
    acts = []
    if tm == 0 and all(prep):
        acts.append(("TmCommit", 0))
    if tm == 0:
        acts.append(("TmAbort", 0))
    for r in range(n):
        if tm == 0 and ("P", r) in msgs:
            acts.append(("TmRcvPrepared", r))
        if rm[r] == WORKING:
            acts += [("RmPrepare", r), ("RmChooseToAbort", r)]
        if ("C", 0) in msgs:
            acts.append(("RmRcvCommitMsg", r))
        if ("A", 0) in msgs:
            acts.append(("RmRcvAbortMsg", r))
    for k, r in acts:
        rm2, tm2, prep2, msgs2 = list(rm), tm, list(prep), set(msgs)
        if k == "TmRcvPrepared":
            prep2[r] = True
        elif k == "TmCommit":
            tm2 = 1
            msgs2.add(("C", 0))
        elif k == "TmAbort":
            tm2 = 2
            msgs2.add(("A", 0))
        elif k == "RmPrepare":
            rm2[r] = PREPARED
            msgs2.add(("P", r))
        elif k == "RmChooseToAbort":
            rm2[r] = ABORTED
        elif k == "RmRcvCommitMsg":
            rm2[r] = COMMITTED
        else:
            rm2[r] = ABORTED
        yield (tuple(rm2), tm2, tuple(prep2), frozenset(msgs2))


def _representative(s):
    rm, tm, prep, msgs = s
    order = [i for _, i in sorted((v, i) for i, v in enumerate(rm))]  # reindex: new -> old
    new = {old: k for k, old in enumerate(order)}                      # rewrite: old -> new
    return (tuple(rm[i] for i in order), tm, tuple(prep[i] for i in order),
            frozenset((k, new[r]) if k == "P" else (k, r) for k, r in msgs))


def _reduced_count(n, depth_first):
    s0 = _init(n)
    seen = {_representative(s0)}
    pending = deque([s0])
    while pending:
        s = pending.pop()
        for ns in _successors(s, n):
            key = _representative(ns)
            if key in seen:
                continue
            seen.add(key)
            if depth_first:
                pending.append(ns)      # Vec push / pop (dfs.rs:290)
            else:
                pending.appendleft(ns)  # VecDeque push_front / pop_back (bfs.rs:263)
    return len(seen)


def test_dfs_order_reproduces_reference_golden():
    assert _reduced_count(5, depth_first=True) == 665
    for n in range(1, 5):
        assert _reduced_count(n, True) == OracleRun(TWO_PHASE, [n], dfs=True, symmetry=True).unique_state_count


def test_bfs_order_gives_a_different_reduced_count():
    assert [_reduced_count(n, depth_first=False) for n in range(1, 6)] == [12, 36, 94, 225, 508]
