"""Sweep of the block-local duplicate filter size (SR_FILTER_LOG2) on a 2pc check, profile off."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from stateright_amd import TwoPhaseSys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
exp = 6 ** n + 4 ** n + 2 ** n
def run(verbose=False):
    b = TwoPhaseSys(n).checker().capacity_hint(exp).device(0)
    if verbose:
        b = b.verbose()
    c = b.spawn_bfs().join()
    assert c.unique_state_count() == exp
run(verbose=True)
for f in sys.argv[2].split(","):
    os.environ["SR_FILTER_LOG2"] = f
    for _ in range(3):
        run()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter(); run(); ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"filter_log2={f}: best {ts[0]*1e3:.3f} ms  median {ts[5]*1e3:.3f} ms", flush=True)
