"""Times consecutive 2pc N=11 single-GPU checks with per-level engine logs (stderr)."""
import sys
import time

sys.path.insert(0, ".")
from stateright_amd import TwoPhaseSys

n = int(sys.argv[1]) if len(sys.argv) > 1 else 11
want = 6 ** n + 4 ** n + 2 ** n
for i in range(3):
    t0 = time.perf_counter()
    b = TwoPhaseSys(n).checker().capacity_hint(want).order("fast")
    if i == 2:
        b = b.verbose()
    c = b.spawn_bfs().join()
    st = c.stats()
    print(f"check {i}: {1e3 * (time.perf_counter() - t0):.1f} ms wall, loop {st['level_loop_sec'] * 1e3:.1f} ms, "
          f"total {st['total_sec'] * 1e3:.1f} ms, rehashes {st['rehashes']}, unique ok {c.unique_state_count() == want}",
          flush=True)
