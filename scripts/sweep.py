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
    for pb, load, pol, ppw in itertools.product([1, 2], [0.5], [0], [-1, 6]):
        os.environ["SR_PROBE_BATCH"] = str(pb)
        os.environ["SR_TABLE_LOAD"] = str(load)
        os.environ["SR_PROBE_LOAD"] = str(pol)
        os.environ["SR_PPW_LOG2"] = str(ppw)
        r = run(lambda: TwoPhaseSys(n).checker().order("fast").capacity_hint(exp), exp)
        line = {"model": f"2pc{n}", "lib": os.environ.get("SR_LIB_PATH", "default")[-12:], "pb": pb, "load": load, "pol": pol, "ppw": ppw, "best_ms": r[0], "med_ms": r[1], "kernel_ms": r[2],
                "cap": r[3], "launches": r[4], "unique_per_s": exp / r[0] * 1e3}
        print(json.dumps(line), flush=True)
        out.append(line)
    os.environ["SR_PROBE_BATCH"] = "1"
    os.environ["SR_TABLE_LOAD"] = "0.5"
    os.environ["SR_PROBE_LOAD"] = "0"
    il = 39456401
    r = run(lambda: IncrementLock(10).checker().order("fast").capacity_hint(il), il, reps=3, warm=1)
    print(json.dumps({"model": "inclock10", "best_ms": r[0], "kernel_ms": r[2], "unique_per_s": il / r[0] * 1e3}), flush=True)


if __name__ == "__main__":
    main()
