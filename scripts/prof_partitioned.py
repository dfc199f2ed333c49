"""Driver for a rocprofv3 kernel trace of the partitioned search on one GPU:
    python scripts/prof_partitioned.py <local|virtual|rccl1> <world> [N] [reps]
runs `reps` full checks of 2pc N (default 9) after one warmup."""
import sys

sys.path.insert(0, ".")
from stateright_amd import TwoPhaseSys  # noqa: E402
from stateright_amd.distributed import Communicator  # noqa: E402

kind, world = sys.argv[1], int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 9
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
want = 6 ** n + 4 ** n + 2 ** n
comms = (Communicator.local_group(world) if kind == "local"
         else [Communicator(0, 1, Communicator.unique_id(), 0)] if kind == "rccl1" else [None])
for _ in range(reps + 1):
    cs = []
    for c in comms:
        b = TwoPhaseSys(n).checker().capacity_hint(want).defer_paths()
        b = b.comm(c) if c is not None else b.partitions(world)
        cs.append(b.spawn_bfs())
    recs = 0
    for c in cs:
        c.join()
        assert c.unique_state_count() == want
        recs = c.stats()["records_routed"]
    del cs
for c in comms:
    if c is not None:
        c.close()
print("ok", kind, world, n, reps, "records_routed", recs)
