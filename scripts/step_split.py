"""Where a 2pc N=9 check's wall time goes outside the level loop: per check, the Python-side wall
time (builder, spawn, join, free), the engine's total_sec (run start -> end of the level loop) and
level_loop_sec, without per-launch events."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stateright_amd as sr  # noqa: E402

n, want = 9, 6 ** 9 + 4 ** 9 + 2 ** 9
rows = []
for i in range(25):
    t0 = time.perf_counter()
    b = sr.TwoPhaseSys(n).checker().capacity_hint(want).order("fast")
    t1 = time.perf_counter()
    c = b.spawn_bfs()
    t2 = time.perf_counter()
    c.join()
    t3 = time.perf_counter()
    st = c.stats()
    assert c.unique_state_count() == want
    c = None
    t4 = time.perf_counter()
    rows.append((t4 - t0, t1 - t0, t2 - t1, t3 - t2, t4 - t3, st["total_sec"], st["level_loop_sec"]))
rows = rows[5:]
avg = [sum(r[k] for r in rows) / len(rows) * 1e3 for k in range(7)]
print("ms per check: wall %.3f | builder %.3f spawn %.3f join %.3f free %.3f | engine total %.3f loop %.3f" % tuple(avg))
