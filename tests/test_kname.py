"""scripts/kname.py: which rocprofv3 kernel names are timed expand_fast dispatches (the roofline's and
the PMC passes' filter). The counting pass (STATS = true) is excluded, whatever the number of trailing
template arguments (NOPF, DYN)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scripts"))

from kname import is_counting, is_expand_fast, is_timed_expand  # noqa: E402

TAIL = "(sr::TwoPhaseT<9>, unsigned long const*, unsigned int, unsigned int, sr::TableView)"


def test_timed_and_counting_dispatches():
    for args, counting in [("1, 0, false", False), ("1, 0, true", True), ("-4, 0, false, true", False),
                           ("1, 0, true, false", True), ("1, 0, false, false, true", False),
                           ("-4, 0, true, false, false", True), ("1, 0, false, true, false", False)]:
        name = f"void sr::expand_fast<sr::TwoPhaseT<9>, {args}>{TAIL}"
        assert is_expand_fast(name)
        assert is_counting(name) == counting, name
        assert is_timed_expand(name) == (not counting), name


def test_nested_model_templates():
    name = f"void sr::expand_fast<sr::PaxosT<11, 3>, 1, 0, false, true, false>{TAIL}"
    assert is_timed_expand(name)
    name = "void sr::expand_fast<sr::act::ActorGpu<sr::act::FixtureSys>, -4, 0, true, false, true>"
    assert is_counting(name) and not is_timed_expand(name)


def test_other_kernels():
    for name in ["void sr::rehash_ranges<unsigned int>(sr::TableView, unsigned long)", "__amd_rocclr_fillBufferAligned",
                 "void sr::expand_route<sr::TwoPhaseT<9>, 1, false>(sr::TwoPhaseT<9>)"]:
        assert not is_expand_fast(name) and not is_timed_expand(name) and not is_counting(name)
