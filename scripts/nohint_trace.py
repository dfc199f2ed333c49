"""Time model checks without a capacity hint, the last one with the engine's per-level verbose log:
    python scripts/nohint_trace.py inclock 11 [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import stateright_amd as sr  # noqa: E402

kind, n = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
make = {"inclock": sr.IncrementLock, "2pc": sr.TwoPhaseSys}[kind]
for rep in range(reps):
    t = time.perf_counter()
    c = make(n).checker().order("fast").verbose(rep == reps - 1).spawn_bfs().join()
    el = time.perf_counter() - t
    print(f"rep {rep}: {el * 1e3:.1f} ms unique {c.unique_state_count()} stats {c.stats()}", flush=True)
