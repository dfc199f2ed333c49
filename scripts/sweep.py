"""Tuning sweep for the expand kernel (internal knobs SR_PROBE_BATCH / SR_TABLE_LOAD)."""
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stateright_amd import IncrementLock, TwoPhaseSys  # noqa: E402


def run(make, expect, reps=5, warm=2):
    for _ in range(warm):
        make().spawn_bfs().join()
    torch.cuda.synchronize()
    ts, ks = [], []
    for _ in range(reps):
        t = time.perf_counter()
        c = make().profile().spawn_bfs().join()
        ts.append(time.perf_counter() - t)
        st = c.stats()
        ks.append(st["expand_kernel_ms"])
        assert c.unique_state_count() == expect, (c.unique_state_count(), expect)
    return min(ts) * 1e3, sorted(ts)[len(ts) // 2] * 1e3, min(ks), st["table_capacity"], st["expand_launches"]


def main():
    n = int(os.environ.get("N", "9"))
    exp = 6 ** n + 4 ** n + 2 ** n
    out = []
    for pb, load in itertools.product([1, 2, 4], [0.25, 0.5, 0.7]):
        os.environ["SR_PROBE_BATCH"] = str(pb)
        os.environ["SR_TABLE_LOAD"] = str(load)
        r = run(lambda: TwoPhaseSys(n).checker().order("fast").capacity_hint(exp), exp)
        line = {"model": f"2pc{n}", "pb": pb, "load": load, "best_ms": r[0], "med_ms": r[1], "kernel_ms": r[2],
                "cap": r[3], "launches": r[4], "unique_per_s": exp / r[0] * 1e3}
        print(json.dumps(line), flush=True)
        out.append(line)
    os.environ["SR_PROBE_BATCH"] = "4"
    os.environ["SR_TABLE_LOAD"] = "0.5"
    il = 39456401
    r = run(lambda: IncrementLock(10).checker().order("fast").capacity_hint(il), il, reps=3, warm=1)
    print(json.dumps({"model": "inclock10", "best_ms": r[0], "kernel_ms": r[2], "unique_per_s": il / r[0] * 1e3}), flush=True)


if __name__ == "__main__":
    main()
