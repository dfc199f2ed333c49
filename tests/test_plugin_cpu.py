"""The user-model plugin boundary on the CPU (no GPU calls): the example plugin library loads and
exports `sr_plugin_sliding_puzzle` built against the engine's headers, and both fingerprint entry
points (the plugin's and sr_model_fingerprint for registered models) return the engine's
fingerprint of a described state. Plus the Python bfs.rs restatement against the reference's
sliding-puzzle doc test (src/lib.rs:89-115)."""
import os

import pytest

from oracle_lib import TWO_PHASE  # noqa: F401  (makes tests/ importable like the other oracle tests)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pybfs  # noqa: E402

MASK = (1 << 64) - 1


def fmix64(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & MASK
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & MASK
    k ^= k >> 33
    return k


def fp1(word):  # models.hpp fingerprint<1>
    return fmix64(word ^ (1 << 63))


def test_puzzle_doc_test_on_the_restatement():
    r = pybfs.puzzle_bfs([1, 4, 2, 3, 5, 8, 6, 7, 0])
    assert "solved" in r["discoveries"]
    states = pybfs.puzzle_replay([1, 4, 2, 3, 5, 8, 6, 7, 0], ["Down", "Right", "Down", "Right"])
    assert states[-1] == pybfs.SOLVED  # the doc test's assert_discovery path (src/lib.rs:94-115)
    assert len(r["discoveries"]["solved"]) == 5  # a shortest discovery: 4 actions


def test_plugin_library_exports_and_fingerprints():
    from stateright_amd import build
    from stateright_amd.plugin import Plugin
    path = build.plugin_path("sliding_puzzle")
    assert os.path.exists(path), "build() compiles the example plugin"
    pl = Plugin(path, "sliding_puzzle")
    cells = [1, 4, 2, 3, 5, 8, 6, 7, 0]
    word = sum(c << (4 * i) for i, c in enumerate(cells))
    assert pl.fingerprint(cells, cells) == fp1(word)
    with pytest.raises(ValueError):
        pl.fingerprint(cells, cells[:5])  # wrong description width


def test_model_fingerprint_registered_models():
    from stateright_amd import TwoPhaseSys, LinearEquation
    from stateright_amd.plugin import model_fingerprint
    # 2pc N=2 description: rm_state[2], tm_state, tm_prepared[2], msgs Prepared[2], Commit, Abort
    d = [1, 0, 0, 1, 0, 1, 0, 0, 0]
    n = 2
    word = (1 << 0) | (1 << (2 * n + 2)) | (1 << (3 * n + 2))
    assert model_fingerprint(TwoPhaseSys(2), d) == fp1(word)
    assert model_fingerprint(LinearEquation(2, 4, 7), [3, 5]) == fp1(3 | 5 << 8)
    from stateright_amd import Paxos
    with pytest.raises(ValueError):
        model_fingerprint(Paxos(2), [0] * 45)  # a description of the wrong width (paxos C=2: 49)
