"""Partitioned-search timing (2pc N=9, one GPU, T virtual partitions) over the route kernel's knobs:
record-stage words (SR_RSTAGE_WORDS), parents per wave (SR_ROUTE_PPW_LOG2, -1 = the host rule)
and the sent cache (SR_SEND_CACHE). Best of REPS full checks per point."""
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stateright_amd import TwoPhaseSys  # noqa: E402

n = int(os.environ.get("N", "9"))
want = 6 ** n + 4 ** n + 2 ** n
reps = int(os.environ.get("REPS", "3"))


def best(parts):
    t = 1e9
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        c = TwoPhaseSys(n).checker().partitions(parts).capacity_hint(want).defer_paths().spawn_bfs().join()
        t = min(t, time.perf_counter() - t0)
        assert c.unique_state_count() == want
        st = c.stats()
        del c
    return t * 1e3, st


grid = itertools.product(os.environ.get("PARTS", "2,8").split(","), os.environ.get("RSTAGE", "1024,2048,4096").split(","),
                         os.environ.get("PPW", "-1,5,6").split(","), os.environ.get("CACHE", "1,0").split(","))
for parts, rs, ppw, cache in grid:
    os.environ["SR_RSTAGE_WORDS"] = rs
    os.environ["SR_SEND_CACHE"] = cache
    if ppw == "-1":
        os.environ.pop("SR_ROUTE_PPW_LOG2", None)
    else:
        os.environ["SR_ROUTE_PPW_LOG2"] = ppw
    ms, st = best(int(parts))
    print(f"T={parts} rstage={rs} ppw_log2={ppw} cache={cache}: {ms:.2f} ms  records={st['records_routed'] / 1e6:.1f}M "
          f"restarts={st['restarts']}", flush=True)
