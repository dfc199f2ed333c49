"""BASELINE.json configs[4] asks for `paxos check 3` "+ symmetry reduction". This file records, with
evidence, why no symmetry reduction applies to the paxos model, so that the check runs unreduced
(1 194 428 states, like the reference's own `spawn_bfs`).

The reference itself never reduces paxos: `examples/paxos.rs:325-330` checks with `spawn_dfs()`
and no `.symmetry()`, the BFS checker ignores symmetry (src/checker/bfs.rs:36-74), and
`ActorModelState::representative` (src/actor/model_state.rs:103-118) needs `Rewrite<Id>` on the
history, which `LinearizabilityTester` does not implement. A reduction would therefore have to be
a symmetry of the model: a permutation g of the actors (servers 0..2, clients 3..2+C) that maps
the init state to itself and commutes with the transition relation. Then g maps the reachable set R
onto itself. The tests below try every candidate g and show g(R) != R for every g but the identity,
on the oracle's full reachable set (oracle/paxos.hpp, pinned by 16 668 at C = 2 and the GPU's
1 194 428 at C = 3):

* `ids`: g renames actor Ids wherever an Id occurs (envelope src/dst, ballot ids, proposal
  requesters, the prepares map's keys, the accepts set), as `Rewrite<Id>` would; request ids and
  values are data and stay.
* `ids+data`: g also renames what the reference derives from a client's id (request ids 1 x index
  and 2 x index, value 'A' + index - server_count: src/actor/register.rs:144-188), the most
  permissive reading.

Why they fail: every server starts with ballot (0, Id(0)) (examples/paxos.rs:98-110), so g must fix
server 0; a client's id fixes its Put target (index % server_count), its request ids and its value,
so g must move clients with their servers; and the remaining candidate at C = 3, (1 2)(4 5) with
B <-> C, breaks the tie-break of ballots by server id (examples/paxos.rs:60, `Ballot = (Round, Id)`
compared lexicographically) and the Get routing ((index + op_count) % server_count). The refuted
candidate is exhibited by a reachable state whose image is not reachable.

The only symmetry the paxos encoding keeps is the order-independence of the network SET
(src/actor/model.rs:69, `HashableHashSet`): the GPU encoding stores it as a sorted list of envelope
codes (stateright_amd/csrc/paxos.hpp), one word sequence per set.
"""
import itertools

import numpy as np
import pytest

from oracle_lib import PAXOS, OracleRun

SERVERS = 3
PREPARE, PREPARED, ACCEPT, ACCEPTED, DECIDED, PUT, GET, PUTOK, GETOK = range(9)


def _reachable(c):
    o = OracleRun(PAXOS, [c], threads=8, record_visits=True)
    v = o.visits_array()
    assert v.shape[0] == o.unique_state_count
    return v


_cache = {}


def reachable(c):
    if c not in _cache:
        _cache[c] = _reachable(c)
    return _cache[c]


def apply_g(v, c, ps, pc, data):
    """g on described states (oracle/paxos.hpp describe): ps maps server i -> ps[i], pc maps client
    index k (id 3 + k) -> pc[k]; data=True also renames request ids and values with the client."""
    v = np.asarray(v, dtype=np.int64)
    ps = np.asarray(ps, dtype=np.int64)
    pc = np.asarray(pc, dtype=np.int64)
    actor = np.concatenate([ps, SERVERS + pc, np.arange(SERVERS + c, 16)])  # id -> id

    def acc(a):  # acc code: 0 None, -1 absent, else 1 + round*64 + id*8 + requester
        x = a - 1
        out = 1 + (x // 64) * 64 + ps[np.clip((x % 64) // 8, 0, 2)] * 8 + actor[np.clip(x % 8, 0, 15)]
        return np.where(a > 0, out, a)

    def bal(b):  # round * 8 + id
        return (b // 8) * 8 + ps[np.clip(b % 8, 0, 2)]

    out = np.empty_like(v)
    for i in range(SERVERS):
        blk = v[:, 9 * i:9 * i + 9]
        j = int(ps[i])
        nb = out[:, 9 * j:9 * j + 9]
        nb[:, 0] = blk[:, 0]
        nb[:, 1] = ps[np.clip(blk[:, 1], 0, 2)]
        nb[:, 2] = np.where(blk[:, 2] >= 0, actor[np.clip(blk[:, 2], 0, 15)], -1)
        for q in range(SERVERS):
            nb[:, 3 + int(ps[q])] = acc(blk[:, 3 + q])
        mask = np.zeros(len(v), dtype=np.int64)
        for q in range(SERVERS):
            mask |= ((blk[:, 6] >> q) & 1) << ps[q]
        nb[:, 6] = mask
        nb[:, 7] = acc(blk[:, 7])
        nb[:, 8] = blk[:, 8]
    for k in range(c):
        out[:, 27 + int(pc[k])] = v[:, 27 + k]
    net = v[:, 27 + c:27 + c + 16]
    code = np.where(net >= 0, net, 0)
    src, dst, kind, f = code % 16, (code // 16) % 16, (code // 256) % 16, code // 4096
    nsrc, ndst = actor[src], actor[dst]
    nf = f.copy()
    m = (kind == PREPARE) | (kind == ACCEPTED)
    nf[m] = bal(f[m])
    m = kind == PREPARED
    nf[m] = bal(f[m] // 4096) * 4096 + acc(f[m] % 4096)
    m = (kind == ACCEPT) | (kind == DECIDED)
    nf[m] = bal(f[m] // 16) * 16 + actor[f[m] % 16]
    if data:  # request ids k * index and values 'A' + index - servers follow the client
        m = (kind == PUT) | (kind == PUTOK)
        nf[m] = actor[np.clip(f[m], 0, 15)]
        m = kind == GET
        nf[m] = 2 * actor[np.clip(f[m] // 2, 0, 15)]
        m = kind == GETOK
        req, ch = f[m] // 256, f[m] % 256
        nch = np.where(ch >= ord("A"), ord("A") + actor[np.clip(ch - ord("A") + SERVERS, 0, 15)] - SERVERS, ch)
        nf[m] = 2 * actor[np.clip(req // 2, 0, 15)] * 256 + nch
    ncode = (((nf * 16) + kind) * 16 + ndst) * 16 + nsrc
    ncode = np.where(net >= 0, ncode, np.iinfo(np.int64).max)
    ncode.sort(axis=1)
    out[:, 27 + c:27 + c + 16] = np.where(ncode == np.iinfo(np.int64).max, -1, ncode)
    # the register history (oracle/paxos.hpp describe_register_history): per client k its Get's
    # returned value, then its `last` entries for the other clients in ascending order
    h0 = 27 + c + 16
    for k in range(c):
        nk = int(pc[k])
        ret = v[:, h0 + k * c]
        if data:  # a value is a client's letter: it follows the client
            ret = np.where(ret > 0, 1 + pc[np.clip(ret - 1, 0, c - 1)], ret)
        out[:, h0 + nk * c] = ret
        others, nothers = [u for u in range(c) if u != k], [u for u in range(c) if u != nk]
        for i, u in enumerate(others):
            out[:, h0 + nk * c + 1 + nothers.index(int(pc[u]))] = v[:, h0 + k * c + 1 + i]
    return out


def rows(a):
    """One 64-bit key per described state (a multiply-xorshift hash of its columns). A collision
    could only make an unreachable image look reachable, i.e. hide a refutation, never invent one;
    the exhibited counterexample is checked exactly."""
    a = np.asarray(a, dtype=np.int64).view(np.uint64)
    h = np.full(a.shape[0], 0x9E3779B97F4A7C15, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(a.shape[1]):
            h = (h ^ a[:, j]) * np.uint64(0xBF58476D1CE4E5B9)
            h ^= h >> np.uint64(31)
    return h


def candidates(c):
    for ps in itertools.permutations(range(SERVERS)):
        for pc in itertools.permutations(range(c)):
            for data in (False, True):
                yield ps, pc, data


def identity(ps, pc):
    return list(ps) == list(range(SERVERS)) and list(pc) == list(range(len(pc)))


@pytest.mark.parametrize("c", [2, 3])
def test_identity_maps_reachable_set_onto_itself(c):
    v = reachable(c)
    assert np.array_equal(apply_g(v, c, range(SERVERS), range(c), True), v)
    assert np.array_equal(apply_g(v, c, range(SERVERS), range(c), False), v)
    # g is an action: an involution applied twice gives every state back
    g = ((0, 2, 1), tuple(range(c))[:1] + tuple(reversed(range(1, c))) if c == 3 else tuple(range(c)))
    for data in (False, True):
        assert np.array_equal(apply_g(apply_g(v, c, *g, data), c, *g, data), v)


@pytest.mark.parametrize("c", [2, 3])
def test_no_actor_permutation_is_a_symmetry(c):
    v = reachable(c)
    init = v[:1]  # the first visit is the init state (one init state, src/actor/model.rs:215-242)
    r = np.sort(rows(v))
    passing_init = []
    for ps, pc, data in candidates(c):
        if identity(ps, pc):
            continue
        g_init = apply_g(init, c, ps, pc, data)
        if not np.array_equal(g_init, init):
            continue  # g moves the init state: not a symmetry
        passing_init.append((ps, pc, data))
        img = rows(apply_g(v, c, ps, pc, data))
        outside = ~np.isin(img, r)
        assert outside.any(), f"g = {ps}, {pc}, data={data} maps the reachable set onto itself"
    # Only (1 2)(4 5) with its data (request ids, values B <-> C) fixes the init state, at C = 3:
    # ballots start at (0, Id(0)), so server 0 is fixed; each client's Put target, request ids and
    # value are functions of its id. It is refuted above by a reachable state with no reachable image.
    assert passing_init == ([((0, 2, 1), (0, 2, 1), True)] if c == 3 else [])


def test_refuted_candidate_counterexample():
    # The exhibit for the record: the first reachable state of C = 3, in visit
    # order, whose image under (1 2)(4 5) is unreachable, and what tells them apart.
    c = 3
    v = reachable(c)
    img = apply_g(v, c, (0, 2, 1), (0, 2, 1), True)
    bad = np.flatnonzero(~np.isin(rows(img), np.sort(rows(v))))
    assert bad.size > 0
    first = int(bad[0])
    # exactly: the image differs from every reachable state although the state itself is reachable
    assert not (v == img[first]).all(axis=1).any()
