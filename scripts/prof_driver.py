"""Small driver for rocprofv3 PMC passes: 2pc N (default 9) in FAST order, warmup + 2 checks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stateright_amd import TwoPhaseSys  # noqa: E402

n = int(os.environ.get("N", "9"))
exp = 6 ** n + 4 ** n + 2 ** n
for i in range(int(os.environ.get("REPS", "3"))):
    c = TwoPhaseSys(n).checker().order(os.environ.get("ORDER", "fast")).capacity_hint(exp).spawn_bfs().join()
    assert c.unique_state_count() == exp
print("ok", c.stats())
