"""Partitioned-search timing (2pc N=9, one GPU) over route-kernel knobs: record stage words and the
block filter. Virtual partitions and a one-rank RCCL communicator; best of 5 full checks."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stateright_amd import TwoPhaseSys  # noqa: E402
from stateright_amd.distributed import Communicator  # noqa: E402

n = 9
want = 6 ** n + 4 ** n + 2 ** n
comm = Communicator(0, 1, Communicator.unique_id(), 0)


def best(make, reps=5):
    t = 1e9
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        c = make().spawn_bfs().join()
        t = min(t, time.perf_counter() - t0)
        assert c.unique_state_count() == want
    return t * 1e3, c.stats()


for head in ["0", "65536"]:
    os.environ["SR_HEAD_MAX"] = head
    line = [f"head_max={head}:"]
    for parts in (2, 4, 8):
        ms, st = best(lambda: TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want))
        line.append(f"T{parts} {ms:.2f}ms rec={st['records_routed'] / 1e6:.1f}M head={st['head_levels']} "
                    f"restarts={st['restarts']}")
    ms, st = best(lambda: TwoPhaseSys(n).checker().comm(comm).capacity_hint(want))
    line.append(f"rccl1 {ms:.2f}ms head={st['head_levels']} restarts={st['restarts']}")
    print("  ".join(line), flush=True)
comm.close()
