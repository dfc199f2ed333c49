"""One traced partitioned check (SR_DIST_TRACE per-level host timeline) on one GPU."""
import os
import sys

sys.path.insert(0, ".")
os.environ["SR_DIST_TRACE"] = "1"
from stateright_amd import TwoPhaseSys  # noqa: E402
from stateright_amd.distributed import Communicator  # noqa: E402

n, parts = int(sys.argv[1]), int(sys.argv[2])
want = 6 ** n + 4 ** n + 2 ** n
if parts == 0:
    comm = Communicator(0, 1, Communicator.unique_id(), 0)
    mk = lambda: TwoPhaseSys(n).checker().comm(comm).capacity_hint(want)  # noqa: E731
else:
    mk = lambda: TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want)  # noqa: E731
for _ in range(2):
    print("---- run", flush=True)
    c = mk().spawn_bfs().join()
    assert c.unique_state_count() == want
