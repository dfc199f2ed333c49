"""One rank of tests/test_gpu_shm_ranks.py: a separate process on the GPU, joined to the other ranks
through the shared-memory communicator (Communicator.shm). Runs the checks named on the command
line and prints one JSON line per check: global counts and how the levels were exchanged.

    python tests/shm_rank_worker.py <rank> <world> <shm name> <distinct 0|1> <model:param>...
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world, name, distinct = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4] == "1"
    import stateright_amd as sr
    from stateright_amd.distributed import Communicator
    comm = Communicator.shm(rank, world, name, device=0, slot_bytes=32 << 20, devices_distinct=distinct)
    make = {"2pc": lambda n: sr.TwoPhaseSys(n), "inclock": lambda n: sr.IncrementLock(n),
            # ping-pong on a lossy duplicating network: three `eventually` properties, so the
            # records carry their EventuallyBits word (models.hpp EvBits)
            "pingpong": lambda n: sr.PingPong(n, lossy=True)}
    try:
        for spec in sys.argv[5:]:
            model, n = spec.split(":")
            c = make[model](int(n)).checker().comm(comm).spawn_bfs().join()
            st = c.stats()
            print(json.dumps({"rank": rank, "check": spec, "unique": c.unique_state_count(), "states": c.state_count(),
                              "depth": c.max_depth(), "discoveries": sorted(c.discoveries()),
                              "pipelined": st["pipelined"], "restarts": st["restarts"],
                              "exchange_fallbacks": st["exchange_fallbacks"]}), flush=True)
            c = None
    finally:
        comm.close()


if __name__ == "__main__":
    main()
