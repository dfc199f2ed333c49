#!/usr/bin/env python3
"""Regenerates tests/golden/bfs_goldens.json from the CPU oracle (oracle/liboracle.so).

The oracle is the C++ restatement of the reference's single-threaded `spawn_bfs`
(src/checker/bfs.rs), pinned by the reference's own goldens in tests/test_oracle_golden.py. This
table freezes its outputs per (model, params) in the reference's FIFO order: unique and total state
counts, max depth, `is_done`, the discovered property names and each discovery's action path (as
canonical action ids) — the §8c "build-generated goldens". Fixture only: data, no reference source.

    python tests/golden/make_golden.py        # rewrites the JSON next to this script
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle_lib import (BINARY_CLOCK, INCREMENT, INCREMENT_LOCK, LINEAR_EQUATION, PAXOS,  # noqa: E402
                        TWO_PHASE, OracleRun)

CASES = (
    [("linear_equation", LINEAR_EQUATION, p) for p in ([2, 10, 14], [2, 4, 7], [1, 1, 3], [3, 5, 11])]
    + [("binary_clock", BINARY_CLOCK, [])]
    + [("2pc", TWO_PHASE, [n]) for n in range(1, 8)]
    + [("increment", INCREMENT, [n]) for n in (1, 2, 3, 4, 8, 10, 12)]
    + [("increment_lock", INCREMENT_LOCK, [n]) for n in range(1, 8)]
    + [("paxos", PAXOS, [c]) for c in (1, 2)]
)


def entry(name, model, params):
    r = OracleRun(model, params)
    names = r.discovery_names()
    return {
        "model": name,
        "model_id": model,
        "params": params,
        "unique_state_count": r.unique_state_count,
        "state_count": r.state_count,
        "max_depth": r.max_depth,
        "is_done": r.is_done,
        "discoveries": {n: r.discovery_actions(n) for n in names},
    }


def main():
    rows = [entry(*c) for c in CASES]
    out = os.path.join(HERE, "bfs_goldens.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (CPU oracle, single-thread FIFO order)",
                   "cases": rows}, f, indent=1)
        f.write("\n")
    print(f"wrote {len(rows)} cases to {out}")


if __name__ == "__main__":
    main()
