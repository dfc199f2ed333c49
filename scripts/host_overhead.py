"""Splits one bench step into builder / spawn / join / engine time (2pc N=9)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from stateright_amd import TwoPhaseSys

torch.cuda.set_device(0)
n = 9
hint = 6 ** n + 4 ** n + 2 ** n
for i in range(12):
    t0 = time.perf_counter()
    b = TwoPhaseSys(n).checker().capacity_hint(hint).device(0).order("fast")
    t1 = time.perf_counter()
    c = b.spawn_bfs()
    t2 = time.perf_counter()
    c.join()
    t3 = time.perf_counter()
    st = c.stats()
    u = c.unique_state_count()
    t4 = time.perf_counter()
    del c
    t5 = time.perf_counter()
    if i >= 2:
        print(f"builder {1e3*(t1-t0):.3f} spawn {1e3*(t2-t1):.3f} join {1e3*(t3-t2):.3f} "
              f"engine_total {1e3*st['total_sec']:.3f} loop {1e3*st['level_loop_sec']:.3f} "
              f"query {1e3*(t4-t3):.3f} free {1e3*(t5-t4):.3f} unique {u}")
