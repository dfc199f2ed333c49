"""The engine's discovery fingerprint chains (sr_gpu_bfs_discovery, the input of the reference's
`reconstruct_path` / `Path::from_fingerprints`, /root/reference/src/checker/bfs.rs:314-342 and
src/checker/path.rs:20-86) equal sr_model_fingerprint of the described path states, for the actor
and register models: a host that holds the reference's states can match them."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stateright_amd as sr  # noqa: E402
from stateright_amd.plugin import model_fingerprint  # noqa: E402

MODELS = [
    ("paxos2", lambda: sr.Paxos(2)),
    ("paxos3", lambda: sr.Paxos(3)),
    ("paxos5", lambda: sr.Paxos(5)),
    ("abd", lambda: sr.AbdRegister(2, 2)),
    ("single_copy2", lambda: sr.SingleCopyRegister(2, 2)),
    ("single_copy3", lambda: sr.SingleCopyRegister(3, 1)),
    ("pingpong", lambda: sr.PingPong(5, maintains_history=True)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["fifo", "fast"])
@pytest.mark.parametrize("name,make", MODELS, ids=[m[0] for m in MODELS])
def test_discovery_chain_is_model_fingerprint(name, make, order):
    if name == "paxos5" and order == "fifo":
        pytest.skip("paxos C=5 in FIFO order: covered in FAST order (9 M states)")
    m = make()
    c = m.checker().order(order).spawn_bfs().join()
    found = c.discoveries()
    assert found, "every model here has a discovery"
    for prop, path in found.items():
        chain = c.discovery_fingerprints(prop)
        want = [model_fingerprint(m, list(st)) for st in path.into_states()]
        assert chain == want, (prop, len(chain), len(want))
