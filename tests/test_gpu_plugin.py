"""A GpuModel OUTSIDE the engine's registry, compiled into its own plugin library against
include/stateright_gpu_model.hpp (examples/plugins/sliding_puzzle.hip: the sliding puzzle of the
reference crate's documentation, src/lib.rs:40-116), run through the engine library's C ABI
(sr_gpu_bfs_spawn_plugin). Parity against the reference's doc test and against oracle/pybfs.py,
the Python restatement of single-threaded bfs.rs."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pybfs  # noqa: E402
from stateright_amd import build  # noqa: E402
from stateright_amd.plugin import Plugin  # noqa: E402

DOC = [1, 4, 2, 3, 5, 8, 6, 7, 0]
UNSOLVABLE = [1, 2, 3, 4, 5, 6, 8, 7, 0]  # odd permutation: the whole 9!/2 component, never solved


@pytest.fixture(scope="module")
def puzzle():
    return Plugin(build.plugin_path("sliding_puzzle"), "sliding_puzzle")


_full = {}


def full_space():
    if "r" not in _full:
        _full["r"] = pybfs.puzzle_bfs(UNSOLVABLE)
    return _full["r"]


def test_doc_test(puzzle):
    # src/lib.rs:89-115: spawn_bfs().join(); assert_properties(); assert_discovery("solved", [...])
    c = puzzle.model(*DOC).checker().spawn_bfs().join()
    c.assert_properties()
    c.assert_discovery("solved", ["Down", "Right", "Down", "Right"])


def test_fifo_early_exit_matches_reference_order(puzzle):
    o = pybfs.puzzle_bfs(DOC)
    rec = sr.StateRecorder()
    c = puzzle.model(*DOC).checker().order("fifo").visitor(rec).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count()) == (o["unique"], o["state_count"])
    assert rec.states == [tuple(s) for s in o["visits"]]
    assert [tuple(s) for s in c.discovery("solved").into_states()] == o["discoveries"]["solved"]


@pytest.mark.parametrize("order", ["fast", "fifo"])
def test_full_exploration(puzzle, order):
    o = full_space()
    assert o["unique"] == 181440 and o["discoveries"] == {}
    c = puzzle.model(*UNSOLVABLE).checker().order(order).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count()) == (o["unique"], o["state_count"])
    assert c.is_done() and c.discoveries() == {}
    assert c.max_depth() == o["max_depth"]


def test_partitioned(puzzle):
    o = full_space()
    c = puzzle.model(*UNSOLVABLE).checker().partitions(3).spawn_bfs().join()
    assert (c.unique_state_count(), c.state_count()) == (o["unique"], o["state_count"])


def test_discovery_fingerprints_match_plugin_fingerprint(puzzle):
    c = puzzle.model(*DOC).checker().spawn_bfs().join()
    path = c.discovery("solved")
    fps = c.discovery_fingerprints("solved")
    assert fps == [puzzle.fingerprint(DOC, list(s)) for s in path.into_states()]


def test_bad_params_fail_loudly(puzzle):
    with pytest.raises(sr.CheckerError):
        puzzle.model(1, 1, 2, 3, 4, 5, 6, 7, 8).checker().spawn_bfs()
