"""Times the partitioned search on one GPU, best of `reps` full checks of 2pc N (default 9):
T virtual partitions of one engine, world in-process ranks (LocalComm, one stream each), and a
one-rank RCCL communicator, beside the single-GPU engine.
    python scripts/time_partitioned.py [N] [modes: pipelined,sync,nocache]"""
import os
import sys
import time

sys.path.insert(0, ".")
from stateright_amd import TwoPhaseSys  # noqa: E402
from stateright_amd.distributed import Communicator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["pipelined"]
reps = int(os.environ.get("REPS", "5"))
want = 6 ** n + 4 ** n + 2 ** n


def timed(make, reps=reps):
    best = 1e9
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        cs = make()
        for c in cs:
            c.join()
        dt = time.perf_counter() - t0
        for c in cs:
            assert c.unique_state_count() == want, c.unique_state_count()
        best = min(best, dt)
        s = cs[0].stats()
        del cs
    return best, s


def st(s):
    return f"levels={s['levels']} head={s.get('head_levels')} restarts={s['restarts']} records={s['records_routed']}"


def line(name, dt, s):
    print(f"{name}: {dt * 1e3:.2f} ms  {want / dt / 1e9:.3f} G unique/s  {st(s)}", flush=True)


for mode in modes:
    os.environ.pop("SR_DIST_SYNC", None)
    os.environ.pop("SR_SEND_CACHE", None)
    if mode == "sync":
        os.environ["SR_DIST_SYNC"] = "1"
    if mode == "nocache":
        os.environ["SR_SEND_CACHE"] = "0"
    print(f"== {mode}", flush=True)
    for parts in (1, 2, 4, 8):
        line(f"virtual parts={parts}", *timed(lambda: [TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want).defer_paths().spawn_bfs()]))
    for world in (2, 4, 8):
        comms = Communicator.local_group(world)
        line(f"local ranks world={world}", *timed(lambda: [TwoPhaseSys(n).checker().comm(c).capacity_hint(want).defer_paths().spawn_bfs() for c in comms]))
        for c in comms:
            c.close()
    comm = Communicator(0, 1, Communicator.unique_id(), 0)
    line("rccl world=1", *timed(lambda: [TwoPhaseSys(n).checker().comm(comm).capacity_hint(want).defer_paths().spawn_bfs()]))
    comm.close()
dt, s = timed(lambda: [TwoPhaseSys(n).checker().order("fast").capacity_hint(want).spawn_bfs()])
print(f"single-GPU engine: {dt * 1e3:.2f} ms  {want / dt / 1e9:.3f} G unique/s", flush=True)
