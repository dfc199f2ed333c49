"""Kernel-name helpers for the rocprofv3 CSV tools: expand_fast<M, PB, POL, STATS, NOPF, DYN> dispatches of
the counting pass (STATS = true, bench.py's last check) are excluded from rates and traffic."""
import re

_ARGS = re.compile(r"expand_fast<.*?, (-?\d+), (\d+), (true|false)((?:, (?:true|false))*)>(?:\(|$)")


def is_expand_fast(name):
    return "expand_fast<" in name


def is_counting(name):
    """expand_fast's STATS instantiation (the counting pass)."""
    m = _ARGS.search(name)
    return bool(m) and m.group(3) == "true"


def is_timed_expand(name):
    """An expand_fast dispatch of a timed (non-counting) check."""
    return is_expand_fast(name) and not is_counting(name)
