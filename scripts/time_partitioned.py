"""Times the partitioned search on one GPU: T virtual partitions and a one-rank RCCL communicator."""
import os
import sys
import time

sys.path.insert(0, ".")
from stateright_amd import TwoPhaseSys  # noqa: E402
from stateright_amd.distributed import Communicator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
want = 6 ** n + 4 ** n + 2 ** n


def timed(make, reps=5):
    best = 1e9
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        c = make().spawn_bfs().join()
        dt = time.perf_counter() - t0
        assert c.unique_state_count() == want, c.unique_state_count()
        best = min(best, dt)
    return best, c


def st(c):
    s = c.stats()
    return f"pipelined={s['pipelined']} restarts={s['restarts']} records={s['records_routed']}"


for mode in ("pipelined", "sync", "nocache"):
    if mode == "sync":
        os.environ["SR_DIST_SYNC"] = "1"
    else:
        os.environ.pop("SR_DIST_SYNC", None)
    if mode == "nocache":
        os.environ["SR_SEND_CACHE"] = "0"
    print(f"== {mode}", flush=True)
    for parts in (1, 2, 4, 8):
        dt, c = timed(lambda: TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want))
        print(f"virtual parts={parts}: {dt * 1e3:.2f} ms  levels={c.stats()['levels']}  {want / dt / 1e9:.3f} G unique/s  {st(c)}", flush=True)
    comm = Communicator(0, 1, Communicator.unique_id(), 0)
    dt, c = timed(lambda: TwoPhaseSys(n).checker().comm(comm).capacity_hint(want))
    print(f"rccl world=1: {dt * 1e3:.2f} ms  {want / dt / 1e9:.3f} G unique/s  {st(c)}", flush=True)
    del c
    comm.close()
dt, c = timed(lambda: TwoPhaseSys(n).checker().capacity_hint(want))
print(f"single-GPU engine: {dt * 1e3:.2f} ms  {want / dt / 1e9:.3f} G unique/s", flush=True)
