"""Attribution of the expand launches' times of one bench line: per level, the event
time (levels.kernel_us), the frontier, the visited-set loads and the CAS claims of the counting pass
(levels.probes / levels.cas), and a least-squares fit

    t = t0 + a * parents + b * probes + c * claims        (us; over the levels of >= 20 K parents)

so that the ascending mid levels (more claims per parent) and the descending ones of similar size
can be split into the floor, the parents' expansion, the probes and the claims.
    python scripts/level_attribution.py <bench.json> [first_up last_up first_down last_down]"""
import json
import sys

import numpy as np

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lv = d["levels"]
t = np.array(lv["kernel_us"], float)
fr = np.array(lv["frontier"], float)
pr = np.array(lv["probes"], float)
cs = np.array(lv["cas"], float)
up = range(int(sys.argv[2]), int(sys.argv[3]) + 1) if len(sys.argv) > 5 else range(7, 11)
down = range(int(sys.argv[4]), int(sys.argv[5]) + 1) if len(sys.argv) > 5 else range(18, 22)
sel = fr >= 20000
X = np.stack([np.ones(sel.sum()), fr[sel], pr[sel], cs[sel]], axis=1)
coef, *_ = np.linalg.lstsq(X, t[sel], rcond=None)
t0, a, b, c = coef
pred = np.stack([np.ones_like(fr), fr, pr, cs], axis=1) @ coef
print(f"fit over {sel.sum()} levels of >= 20 K parents: t = {t0:.1f} us + {a * 1e3:.2f} ns/parent + "
      f"{b * 1e3:.3f} ns/probe + {c * 1e3:.3f} ns/claim (rms residual {np.sqrt(np.mean((pred[sel] - t[sel]) ** 2)):.1f} us)")
print("level  parents   probes    claims  claims/parent   us   fit: floor parents probes claims")
for i in range(len(t)):
    if fr[i] < 1000:
        continue
    print(f"{i:5d} {fr[i]:8.0f} {pr[i]:9.0f} {cs[i]:9.0f} {cs[i] / fr[i]:8.2f} {t[i]:10.1f}   "
          f"{t0:6.1f} {a * fr[i]:7.1f} {b * pr[i]:7.1f} {c * cs[i]:7.1f}")
for name, r in (("ascending", up), ("descending", down)):
    idx = [i for i in r if i < len(t)]
    tt, ff, pp, cc = t[idx].sum(), fr[idx].sum(), pr[idx].sum(), cs[idx].sum()
    print(f"{name} levels {idx[0]}-{idx[-1]}: {tt:.1f} us; parents {ff:.0f}, probes {pp:.0f}, claims {cc:.0f}; "
          f"fit: floor {t0 * len(idx):.1f}, parents {a * ff:.1f}, probes {b * pp:.1f}, claims {c * cc:.1f} us")
