import sys; sys.path.insert(0, '.')
from stateright_amd import TwoPhaseSys
for i in range(2):
    c = TwoPhaseSys(9).checker().verbose(True).spawn_bfs().join()
    print("unique", c.unique_state_count(), flush=True)
