#!/usr/bin/env python3
"""Regenerates tests/golden/paxos_counts.json: the CPU oracle's `spawn_bfs` counts of the paxos
example (examples/paxos.rs:223-263) for client_count 1..6 (bench.sh:27 checks 6), from the
multi-threaded restatement oracle/bfs_cli (counts are order-independent: paxos explores its whole
state space). Fixture only: data, no reference source.

    python tests/golden/make_paxos_counts.py     # rewrites the JSON next to this script
"""
import json
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "bfs_cli")


def run(c):
    out = subprocess.run([CLI, "paxos", str(c), str(os.cpu_count() or 1)], capture_output=True, text=True,
                         check=True).stdout
    r = dict(kv.split("=") for kv in re.search(r"^RESULT (.*)$", out, re.M).group(1).split())
    return {"client_count": c, "unique_state_count": int(r["unique"]), "state_count": int(r["state_count"]),
            "max_depth": int(r["max_depth"]), "discoveries": sorted(re.findall(r'^Discovered "([^"]+)"', out, re.M)),
            "pinning": PIN.get(c, "oracle-derived (CPU restatement only; parity unpinned beyond the C=2 golden)")}


# Only C = 2 has a reference golden; every other row is the CPU restatement's own.
PIN = {2: "pinned: the reference's own golden, examples/paxos.rs:289 (unique_state_count 16668)"}


def main():
    rows = [run(c) for c in range(1, 7)]
    with open(os.path.join(HERE, "paxos_counts.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_paxos_counts.py (oracle/bfs_cli, CPU restatement); only the C=2 row "
                                "is pinned by a reference golden", "cases": rows},
                  f, indent=1)
        f.write("\n")
    print(rows)


if __name__ == "__main__":
    main()
