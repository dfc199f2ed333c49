"""sr_model_fingerprint for every registered model: a state's canonical description
determines the state, so a host holding the reference's state can compute the engine's fingerprint
of it (`Path::from_fingerprints`, /root/reference/src/checker/path.rs:20-86). CPU only: the
self-test walks the reachable states on the host (describe -> undescribe -> fingerprint)."""
import ctypes
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stateright_amd import _native as N  # noqa: E402

CASES = [
    # (model, params, states checked (None: every reachable state))
    (N.SR_MODEL_PAXOS, [1], 265),
    (N.SR_MODEL_PAXOS, [2], 16668),               # examples/paxos.rs:289
    (N.SR_MODEL_PAXOS, [3], None),                # first 200 000 of 1 194 428
    (N.SR_MODEL_PAXOS, [5], None),                # W = 12 encoding
    (N.SR_MODEL_ABD, [2, 2], 544),                # examples/linearizable-register.rs:256
    (N.SR_MODEL_ABD, [1, 1], None),
    (N.SR_MODEL_SINGLE_COPY, [2, 1], 93),         # examples/single-copy-register.rs:91-97
    (N.SR_MODEL_SINGLE_COPY, [3, 2], None),
    (N.SR_MODEL_SINGLE_COPY, [4, 1], 400233),     # bench.sh's `check 4`
    (N.SR_MODEL_PINGPONG, [5], None),
    (N.SR_MODEL_PINGPONG, [3, 1, 0, 1], None),
    (N.SR_MODEL_PINGPONG, [8, 1], 262142),        # 32-slot encoding: the oracle's count (4^9 - 2)
    (N.SR_MODEL_PINGPONG, [9, 1], 1048574),       # 32-slot encoding: 4^10 - 2
    (N.SR_MODEL_PINGPONG, [10, 1, 0, 1], 42),     # 32-slot encoding: the oracle's count
    (N.SR_MODEL_PINGPONG, [14, 0, 1, 1], 29),    # 32-slot encoding, max_nat 14
    (N.SR_MODEL_ACTOR_FIXTURE, [0], 1),
    (N.SR_MODEL_ACTOR_FIXTURE, [1], 2),
    (N.SR_MODEL_2PC, [5], 8832),                  # examples/2pc.rs:127-134
    (N.SR_MODEL_INCREMENT_LOCK, [4], None),
    (N.SR_MODEL_INCREMENT, [3], None),
]


@pytest.mark.parametrize("model,params,want", CASES)
def test_describe_roundtrip(model, params, want):
    lib = N.load()
    p = (ctypes.c_int64 * len(params))(*params)
    cap = max(200000, (want or 0) + 1)  # one past the count: the walk ended by itself
    n = lib.sr_selftest_describe(model, p, len(params), cap)
    assert n > 0, N.last_error()
    if want is not None:
        assert n == want


def test_paxos_description_carries_the_history():
    # two paxos states that differ only in a client's Get `last` vector describe differently, and
    # each description gives its own fingerprint back
    from stateright_amd import Paxos
    from stateright_amd.plugin import model_fingerprint
    m = Paxos(2)
    # widths: 3 servers x 9, C op counts, 16 envelopes, C x C history values
    # history per client c: its Get's return value (-1: not returned; op count 2 = Get invoked),
    # then how many ops of the other client had completed at that Get
    base = [0] * 27 + [2, 2] + [-1] * 16 + [-1, 0, -1, 0]
    for i in range(3):
        base[i * 9 + 2] = -1
        base[i * 9 + 3:i * 9 + 6] = [-1, -1, -1]
    a = list(base)
    b = list(base)
    b[-3] = 1  # client 0's Get saw 1 op of client 1 completed (not 0)
    assert model_fingerprint(m, a) != model_fingerprint(m, b)


def test_dgraph_has_no_inverse():
    from stateright_amd.plugin import model_fingerprint
    from stateright_amd.models import DGraph
    with pytest.raises(ValueError):
        model_fingerprint(DGraph.with_property(N.SR_EVENTUALLY).with_path([0, 1]), [0])


def test_malformed_description_is_rejected():
    # undescribe masks its fields, so a description that is not a state's canonical one
    # (here a 2pc rm_state of 7, masked to 3) must not yield a plausible fingerprint
    from stateright_amd import TwoPhaseSys
    from stateright_amd.plugin import model_fingerprint
    m = TwoPhaseSys(3)
    good = [0] * (3 * 3 + 3)
    assert model_fingerprint(m, good) != 0
    bad = list(good)
    bad[0] = 7
    with pytest.raises(ValueError, match="canonical"):
        model_fingerprint(m, bad)
