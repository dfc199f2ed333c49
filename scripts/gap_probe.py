"""A/B of one 2pc check with and without per-launch HIP events (profile), wall clock per check."""
import sys, time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from stateright_amd import TwoPhaseSys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
mode = sys.argv[2] if len(sys.argv) > 2 else "both"
exp = 6 ** n + 4 ** n + 2 ** n
def run(profile):
    b = TwoPhaseSys(n).checker().capacity_hint(exp).device(0)
    if profile:
        b = b.profile()
    c = b.spawn_bfs().join()
    assert c.unique_state_count() == exp
for prof in ([False, True] if mode == "both" else [mode == "prof"]):
    for _ in range(3):
        run(prof)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter(); run(prof); ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"profile={prof}: best {ts[0]*1e3:.3f} ms  median {ts[5]*1e3:.3f} ms", flush=True)
